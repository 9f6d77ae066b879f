// Host <-> device handshake latencies on one MI355X (the transport of the persistent merge loops):
//   read   : dependent system-scope loads of pinned host memory by one lane (PCIe round trip)
//   pp_*   : host posts seq i into pinned memory, one device wave polls it and answers i in another
//            pinned word; the host times post -> answer seen.  Variants of the device side:
//            sleep  = one poll in flight, s_sleep(1) between polls (k_word_loop's loop)
//            spin   = one poll in flight, no sleep
//            pipe   = 4 polls in flight, issued ~100 ns apart
//            fence  = the answer after a plain store + __threadfence_system (release)
//            wt     = the answer as a system-scope (write-through) store after s_waitcnt vmcnt(0)
//   The answer is a tagged 8-byte word, so the host reads it with no further ordering.
//   vram   : (./pingpong N vram) the command word in fine-grained device memory
//            (hipExtMallocWithFlags hipDeviceMallocFinegrained) written by the CPU through its
//            mapping; the device polls its own memory, so a poll costs no PCIe round trip.
// Build: hipcc -O3 --offload-arch=gfx950 -o pingpong pingpong.hip ; run: ./pingpong [iters]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
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

__global__ void k_read_lat(const u64* host, int n, u64* out) {
  if (threadIdx.x != 0) return;
  u64 idx = 0;
  const u64 t0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < n; ++i) idx = ld_sys(host + (idx & 7));
  const u64 t1 = __builtin_amdgcn_s_memrealtime();
  out[0] = t1 - t0;
  out[1] = idx;
}

// The shader clock one lone workgroup runs at: s_memtime (core clock) against s_memrealtime
// (100 MHz) over a dependent ALU loop.
__global__ void k_clock(int iters, u64* out) {
  const u64 c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  unsigned x = threadIdx.x;
  for (int i = 0; i < iters; ++i) x = x * 1664525u + 1013904223u;
  const u64 c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) {
    out[0] = c1 - c0;
    out[1] = r1 - r0;
    out[2] = x;
  }
}

// mode: 0 sleep, 1 spin, 2 pipe; ans: 0 fence, 1 wt
__global__ void k_pong(const u64* cmd, u64* ans, int iters, int mode, int wt, u64* dev_ticks) {
  if (threadIdx.x >= 64) return;
  const int lane = threadIdx.x;
  u64 polls = 0;
  for (int i = 1; i <= iters; ++i) {
    const u64 want = (u64)i;
    u64 v = 0;
    if (mode == 2) {
      u64 r0 = ld_sys(cmd), r1, r2, r3;
      __builtin_amdgcn_s_sleep(2);
      r1 = ld_sys(cmd);
      __builtin_amdgcn_s_sleep(2);
      r2 = ld_sys(cmd);
      __builtin_amdgcn_s_sleep(2);
      r3 = ld_sys(cmd);
      for (;;) {
        ++polls;
        if (r0 == want) break;
        r0 = ld_sys(cmd);
        if (r1 == want) break;
        r1 = ld_sys(cmd);
        if (r2 == want) break;
        r2 = ld_sys(cmd);
        if (r3 == want) break;
        r3 = ld_sys(cmd);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      for (;;) {
        v = ld_sys(cmd);
        ++polls;
        if (v == want) break;
        if (mode == 0) __builtin_amdgcn_s_sleep(1);
      }
    }
    if (lane == 0) {
      if (wt) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store(ans, want, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      } else {
        __threadfence_system();
        __hip_atomic_store(ans, want, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
  }
  if (lane == 0) dev_ticks[0] = polls;
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? std::atoi(argv[1]) : 20000;
  u64 *hbuf, *dbuf;
  OK(hipHostMalloc((void**)&hbuf, 4096, hipHostMallocMapped | hipHostMallocCoherent));
  for (int i = 0; i < 512; ++i) hbuf[i] = 0;
  u64* hdev;
  OK(hipHostGetDevicePointer((void**)&hdev, hbuf, 0));
  OK(hipMalloc(&dbuf, 64));
  // dependent reads
  const int nr = 2000;
  k_read_lat<<<1, 64>>>(hdev, nr, dbuf);
  OK(hipDeviceSynchronize());
  k_read_lat<<<1, 64>>>(hdev, nr, dbuf);
  OK(hipDeviceSynchronize());
  u64 r[2];
  OK(hipMemcpy(r, dbuf, 16, hipMemcpyDeviceToHost));
  std::printf("{\"read_rtt_us\": %.3f", 1e-2 * (double)r[0] / nr);
  for (int rep = 0; rep < 3; ++rep) {
    k_clock<<<1, 512>>>(20000000, dbuf);
    OK(hipDeviceSynchronize());
    u64 c[3];
    OK(hipMemcpy(c, dbuf, 24, hipMemcpyDeviceToHost));
    std::printf(", \"lone_wg_clock_mhz_%d\": %.0f", rep, 100.0 * (double)c[0] / (double)c[1]);
  }
  const char* names[3] = {"sleep", "spin", "pipe"};
  hipStream_t s;
  OK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  for (int wt = 0; wt < 2; ++wt) {
    for (int mode = 0; mode < 3; ++mode) {
      volatile u64* cmd = hbuf;
      volatile u64* ans = hbuf + 64;
      *cmd = 0;
      *ans = 0;
      k_pong<<<1, 64, 0, s>>>(hdev, hdev + 64, iters, mode, wt, dbuf);
      OK(hipGetLastError());
      std::vector<double> lat;
      lat.reserve(iters);
      for (int i = 1; i <= iters; ++i) {
        const double t0 = now_us();
        __atomic_store_n(const_cast<u64*>(cmd), (u64)i, __ATOMIC_RELEASE);
        while (__atomic_load_n(const_cast<u64*>(ans), __ATOMIC_ACQUIRE) != (u64)i) __builtin_ia32_pause();
        lat.push_back(now_us() - t0);
        // a short host pause, as the merge loop's host work between posts
        const double tw = now_us();
        while (now_us() - tw < 3.0) __builtin_ia32_pause();
      }
      OK(hipStreamSynchronize(s));
      std::sort(lat.begin(), lat.end());
      double sum = 0;
      for (double x : lat) sum += x;
      std::printf(", \"pp_%s_%s_us\": {\"mean\": %.3f, \"p50\": %.3f, \"p10\": %.3f, \"p90\": %.3f}", names[mode],
                  wt ? "wt" : "fence", sum / iters, lat[iters / 2], lat[iters / 10], lat[iters * 9 / 10]);
    }
  }
  if (argc > 2 && std::string(argv[2]) == "vram") {
    u64* vcmd = nullptr;
    OK(hipExtMallocWithFlags((void**)&vcmd, 4096, hipDeviceMallocFinegrained));
    hipPointerAttribute_t at;
    OK(hipPointerGetAttributes(&at, vcmd));
    std::printf(", \"vram_host_ptr\": \"%p\", \"vram_dev_ptr\": \"%p\"", at.hostPointer, at.devicePointer);
    volatile u64* hv = static_cast<volatile u64*>(at.hostPointer ? at.hostPointer : (void*)vcmd);
    *hv = 0;  // the CPU mapping (a fault here ends this mode only)
    std::fflush(stdout);
    k_read_lat<<<1, 64>>>(vcmd, nr, dbuf);
    OK(hipDeviceSynchronize());
    OK(hipMemcpy(r, dbuf, 16, hipMemcpyDeviceToHost));
    std::printf(", \"vram_read_rtt_us\": %.3f", 1e-2 * (double)r[0] / nr);
    for (int mode = 0; mode < 2; ++mode) {
      volatile u64* ans = hbuf + 64;
      *hv = 0;
      *ans = 0;
      k_pong<<<1, 64, 0, s>>>(vcmd, hdev + 64, iters, mode, 0, dbuf);
      OK(hipGetLastError());
      std::vector<double> lat;
      lat.reserve(iters);
      for (int i = 1; i <= iters; ++i) {
        const double t0 = now_us();
        __atomic_store_n(const_cast<u64*>(hv), (u64)i, __ATOMIC_RELEASE);
        while (__atomic_load_n(const_cast<u64*>(ans), __ATOMIC_ACQUIRE) != (u64)i) __builtin_ia32_pause();
        lat.push_back(now_us() - t0);
        const double tw = now_us();
        while (now_us() - tw < 3.0) __builtin_ia32_pause();
      }
      OK(hipStreamSynchronize(s));
      std::sort(lat.begin(), lat.end());
      double sum = 0;
      for (double x : lat) sum += x;
      std::printf(", \"pp_vram_%s_fence_us\": {\"mean\": %.3f, \"p50\": %.3f, \"p10\": %.3f, \"p90\": %.3f}",
                  names[mode], sum / iters, lat[iters / 2], lat[iters / 10], lat[iters * 9 / 10]);
    }
    OK(hipFree(vcmd));
  }
  std::printf("}\n");
  OK(hipHostFree(hbuf));
  OK(hipFree(dbuf));
  return 0;
}
