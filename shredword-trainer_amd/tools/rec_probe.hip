// Device -> host hand-off of a merge's records (the tail of every k_word_loop merge), measured
// in isolation on one MI355X: the host posts command i into pinned memory; one device wave (the
// loop's flag wave) polls it, writes n 24-B records tagged with i, and raises a flag; the host
// times post -> flag seen (and, for the unfenced variants, -> every record tag seen), the device
// times its own store phase (s_memrealtime, 100 MHz).  Variants:
//   fence      records as 3 x 8-B stores, s_waitcnt vmcnt(0), system-scope release flag (the loop today)
//   fence_nc   the same into non-coherent pinned memory (hipHostMallocNonCoherent)
//   line       records staged in LDS and written as 16-B stores (4 lanes fill a 64-B line), release flag
//   relaxed    records + flag as plain stores back to back, then one system-scope release fence
//              (L2 write-back + drain) after both; the host checks every record's tag
//   nowait     records + flag as plain stores, no fence at all; host checks tags (shows whether the
//              stores leave the L2 by themselves)
// Build: hipcc -O3 --offload-arch=gfx950 -o rec_probe rec_probe.hip ; run: ./rec_probe [iters] [records]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define OK(x)                                                                 \
  do {                                                                        \
    hipError_t e = (x);                                                       \
    if (e != hipSuccess) {                                                    \
      std::fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e));      \
      std::exit(1);                                                           \
    }                                                                         \
  } while (0)

typedef unsigned long long u64;

__device__ __forceinline__ u64 ld_sys(const u64* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// variant: 0 fence, 1 line, 2 relaxed, 3 nowait
__global__ void k_rec(const u64* cmd, u64* recs, u64* flag, int iters, int n, int variant, u64* ticks) {
  __shared__ u64 stage[3 * 256];
  const int lane = threadIdx.x;
  for (int i = 1; i <= iters; ++i) {
    u64 v = 0;
    unsigned polls = 0;
    do {
      v = ld_sys(cmd);
      if (v < (u64)i) __builtin_amdgcn_s_sleep(1);
    } while (v < (u64)i && ++polls < (1u << 22));
    if (v != (u64)i) return;  // the host gave up (it posts iters + 1) or went away: leave
    const u64 t0 = __builtin_amdgcn_s_memrealtime();
    const u64 tag = (u64)i << 32;
    if (variant == 1) {
      for (int r = lane; r < n; r += 64) {
        stage[3 * r] = tag | (u64)r;
        stage[3 * r + 1] = tag | 7u;
        stage[3 * r + 2] = tag | 9u;
      }
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
      const int q16 = (3 * n + 1) / 2;     // 16-B chunks
      const int4* s4 = reinterpret_cast<const int4*>(stage);
      int4* d4 = reinterpret_cast<int4*>(recs);
      for (int c = lane; c < q16; c += 64) d4[c] = s4[c];
    } else {
      for (int r = lane; r < n; r += 64) {
        recs[3 * r] = tag | (u64)r;
        recs[3 * r + 1] = tag | 7u;
        recs[3 * r + 2] = tag | 9u;
      }
    }
    if (variant <= 1) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (lane == 0) __hip_atomic_store(flag, (u64)i, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    } else if (variant == 2) {
      if (lane == 0) *flag = (u64)i;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    } else {
      if (lane == 0) *flag = (u64)i;
    }
    const u64 t1 = __builtin_amdgcn_s_memrealtime();
    if (lane == 0) ticks[i] = t1 - t0;
  }
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? std::atoi(argv[1]) : 2000;
  const int n = argc > 2 ? std::atoi(argv[2]) : 48;
  struct V {
    const char* name;
    int variant;
    unsigned flags;
  } vs[] = {{"fence", 0, hipHostMallocMapped | hipHostMallocCoherent},
            {"fence_nc", 0, hipHostMallocMapped | hipHostMallocNonCoherent},
            {"line", 1, hipHostMallocMapped | hipHostMallocCoherent},
            {"relaxed", 2, hipHostMallocMapped | hipHostMallocCoherent},
            {"relaxed_nc", 2, hipHostMallocMapped | hipHostMallocNonCoherent},
            {"nowait", 3, hipHostMallocMapped | hipHostMallocCoherent}};
  u64* dticks;
  OK(hipMalloc((void**)&dticks, (iters + 1) * sizeof(u64)));
  std::printf("{\"iters\": %d, \"records\": %d", iters, n);
  for (const V& v : vs) {
    u64* hbuf;
    OK(hipHostMalloc((void**)&hbuf, 1 << 16, v.flags));
    std::fill(hbuf, hbuf + (1 << 13), 0ull);
    u64 *cmd = hbuf, *flag = hbuf + 64, *recs = hbuf + 128;
    u64 *dcmd, *dflag, *drecs;
    OK(hipHostGetDevicePointer((void**)&dcmd, cmd, 0));
    dflag = dcmd + 64;
    drecs = dcmd + 128;
    hipStream_t s;
    OK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    k_rec<<<1, 64, 0, s>>>(dcmd, drecs, dflag, iters, n, v.variant, dticks);
    std::vector<double> lat(iters), lat_all(iters);
    bool bad = false;
    for (int i = 1; i <= iters; ++i) {
      const auto t0 = std::chrono::steady_clock::now();
      __atomic_store_n(cmd, (u64)i, __ATOMIC_RELEASE);
      while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != (u64)i) {
        if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) {
          bad = true;
          break;
        }
      }
      const auto t1 = std::chrono::steady_clock::now();
      // every record carries tag i (the unfenced variants may still be landing)
      for (int r = 0; r < n && !bad; ++r)
        for (int k = 0; k < 3; ++k)
          while ((__atomic_load_n(&recs[3 * r + k], __ATOMIC_ACQUIRE) >> 32) != (u64)i) {
            if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) {
              bad = true;
              break;
            }
          }
      const auto t2 = std::chrono::steady_clock::now();
      lat[i - 1] = std::chrono::duration<double, std::micro>(t1 - t0).count();
      lat_all[i - 1] = std::chrono::duration<double, std::micro>(t2 - t0).count();
      if (bad) break;
    }
    if (bad) __atomic_store_n(cmd, (u64)iters + 1, __ATOMIC_RELEASE);  // the kernel leaves at once
    OK(hipStreamSynchronize(s));
    std::vector<u64> t(iters + 1);
    OK(hipMemcpy(t.data(), dticks, (iters + 1) * sizeof(u64), hipMemcpyDeviceToHost));
    double dsum = 0;
    for (int i = 1; i <= iters; ++i) dsum += 0.01 * (double)t[i];
    std::vector<double> a = lat, b = lat_all;
    std::sort(a.begin(), a.end());
    std::sort(b.begin(), b.end());
    double sa = 0, sb = 0;
    for (int i = 0; i < iters; ++i) {
      sa += lat[i];
      sb += lat_all[i];
    }
    std::printf(", \"%s\": {\"ok\": %s, \"device_store_phase_us\": %.3f, \"post_to_flag_us\": {\"mean\": %.3f, \"p50\": %.3f, "
                "\"p90\": %.3f}, \"post_to_all_records_us\": {\"mean\": %.3f, \"p50\": %.3f, \"p90\": %.3f}}",
                v.name, bad ? "false" : "true", dsum / iters, sa / iters, a[iters / 2], a[iters * 9 / 10], sb / iters,
                b[iters / 2], b[iters * 9 / 10]);
    std::fflush(stdout);
    OK(hipStreamDestroy(s));
    OK(hipHostFree(hbuf));
  }
  std::printf("}\n");
  return 0;
}
