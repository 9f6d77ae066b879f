// resident_probe — round-trip latency of a persistent (LDS-resident) merge-loop skeleton on
// MI355X (diagnostic, not product code).
//
// One workgroup per CU stays resident; the host posts commands through a mailbox in pinned host
// memory, every workgroup (or a leader that re-broadcasts in device memory) picks the command
// up, scans `lds_kb` of LDS, publishes a region header, takes a per-XCD sharded ticket, and the
// last workgroup gathers the headers and raises a host-visible flag.  Timed host post -> flag.
//
//   hipcc --offload-arch=gfx950 -O3 -o resident_probe resident_probe.hip
//   ./resident_probe [commands] [lds_kb]
// Variants: 0 all poll host; 1 leader polls host + device broadcast; 2 all poll host, only 4
// participants (mask) do the work and the ticket.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstring>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                            \
  do {                                                                                   \
    hipError_t e = (x);                                                                  \
    if (e != hipSuccess) {                                                               \
      std::printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);               \
      std::exit(1);                                                                      \
    }                                                                                    \
  } while (0)

struct Mbox {
  uint32_t seq;   // command sequence number (host writes last)
  uint32_t op;    // 1 run, 2 stop
  uint32_t nparts;
  uint32_t pad;
};

struct P {
  const Mbox* mbox;          // host memory
  uint32_t* dev_go;          // device broadcast word (variant 1)
  uint32_t* done;            // [0..7] per-XCD-shard tickets, [8] top
  uint32_t* rhdr;            // per-WG header (sc1)
  uint32_t* hflag;           // host: [0] flag seq, [1] gathered sum, [2] status
  int variant;
  int lds_words;
  uint32_t max_polls;
};

constexpr int kT = 256;

__device__ __forceinline__ uint32_t sys_load(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ __launch_bounds__(kT) void k_resident(P p) {
  extern __shared__ uint32_t lds[];
  __shared__ uint32_t s_cmd[4];
  __shared__ uint32_t s_last;
  for (int i = threadIdx.x; i < p.lds_words; i += kT) lds[i] = i * 2654435761u;
  __syncthreads();
  const uint32_t G = gridDim.x;
  uint32_t expect = 1;
  for (;;) {
    if (p.variant >= 6) {
      // leader dispatch: WG 0 polls the host mailbox and writes each participant's go word
      // (its own 128-B line); every WG polls only its own word.
      if (blockIdx.x == 0 && threadIdx.x < 64) {
        uint32_t s = 0, polls = 0, op = 2, np = G;
        if (threadIdx.x == 0) {
          while ((s = sys_load(&p.mbox->seq)) < expect && ++polls < p.max_polls) __builtin_amdgcn_s_sleep(1);
          if (s >= expect) {
            op = sys_load(&p.mbox->op);
            np = p.variant == 7 ? sys_load(&p.mbox->nparts) : G;
          } else {
            op = 3;
          }
        }
        op = __shfl(op, 0, 64);
        np = __shfl(np, 0, 64);
        if (op != 1) np = G;
        const uint32_t word = (op << 28) | (np << 16) | (expect & 0xFFFFu);
        for (uint32_t w = threadIdx.x; w < np; w += 64)
          __hip_atomic_store(p.dev_go + w * 32, word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      if (threadIdx.x == 0) {
        uint32_t v = 0, polls = 0;
        while (((v = __hip_atomic_load(p.dev_go + blockIdx.x * 32, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) & 0xFFFFu) !=
                   (expect & 0xFFFFu) && ++polls < p.max_polls)
          __builtin_amdgcn_s_sleep(1);
        s_cmd[0] = (v & 0xFFFFu) == (expect & 0xFFFFu) ? (v >> 28) : 3u;
        s_cmd[1] = (v >> 16) & 0xFFFu;
      }
    } else if (threadIdx.x == 0) {
      uint32_t s = 0, polls = 0, op = 2, np = G;
      if (p.variant == 1 && blockIdx.x != 0) {
        while ((s = __hip_atomic_load(p.dev_go, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) < expect &&
               ++polls < p.max_polls)
          __builtin_amdgcn_s_sleep(1);
        if (s >= expect) {
          op = sys_load(&p.mbox->op);
          np = sys_load(&p.mbox->nparts);
        }
      } else {
        while ((s = sys_load(&p.mbox->seq)) < expect && ++polls < p.max_polls) __builtin_amdgcn_s_sleep(1);
        if (s >= expect) {
          op = sys_load(&p.mbox->op);
          np = sys_load(&p.mbox->nparts);
          if (p.variant == 1) __hip_atomic_store(p.dev_go, s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
      if (s < expect) op = 3;  // timeout
      s_cmd[0] = op;
      s_cmd[1] = np;
    }
    __syncthreads();
    if (p.variant == 7 && s_cmd[0] == 1 && blockIdx.x >= s_cmd[1]) {  // not a participant: never told
      ++expect;
      continue;
    }
    const uint32_t op = s_cmd[0], np = s_cmd[1];
    if (op != 1) {
      if (op == 3 && threadIdx.x == 0) __hip_atomic_store(&p.hflag[2], 3u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      return;
    }
    const bool part = (p.variant != 2 && p.variant != 7) || blockIdx.x < np;
    if (part) {
      // "work": scan the LDS words
      uint32_t acc = 0;
      for (int i = threadIdx.x; i < p.lds_words; i += kT) acc ^= lds[i] + expect;
      acc = acc == 0x12345u ? 1u : 0u;
      if (acc) lds[0] = acc;
      if (threadIdx.x == 0)
        __hip_atomic_store(p.rhdr + blockIdx.x * 8, expect, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      const uint32_t T = (p.variant == 2 || p.variant == 7) ? np : G;
      if (threadIdx.x == 0) {
        bool last;
        if (T <= 32) {
          last = atomicAdd(&p.done[8], 1u) == T - 1u;
        } else {
          const uint32_t g = blockIdx.x & 7u, in_group = (T - g + 7u) >> 3;
          last = false;
          if (atomicAdd(&p.done[g], 1u) == in_group - 1u) {
            atomicExch(&p.done[g], 0u);
            last = atomicAdd(&p.done[8], 1u) == 7u;
          }
        }
        s_last = last;
      }
      __syncthreads();
      if (s_last) {
        uint32_t v = threadIdx.x < T ? __hip_atomic_load(p.rhdr + threadIdx.x * 8, __ATOMIC_RELAXED,
                                                         __HIP_MEMORY_SCOPE_AGENT) : 0u;
        for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
        __shared__ uint32_t s_sum[4];
        if ((threadIdx.x & 63) == 0) s_sum[threadIdx.x >> 6] = v;
        __syncthreads();
        if (threadIdx.x == 0) {
          atomicExch(&p.done[8], 0u);
          p.hflag[1] = s_sum[0] + s_sum[1] + s_sum[2] + s_sum[3];
          __threadfence_system();
          __hip_atomic_store(&p.hflag[0], expect, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
      }
    }
    ++expect;
  }
}

int main(int argc, char** argv) {
  const int ncmd = argc > 1 ? std::atoi(argv[1]) : 2000;
  const int lds_kb = argc > 2 ? std::atoi(argv[2]) : 64;
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int G = prop.multiProcessorCount;
  Mbox* mbox;
  uint32_t* hflag;
  CK(hipHostMalloc((void**)&mbox, 4096, hipHostMallocMapped | hipHostMallocCoherent));
  CK(hipHostMalloc((void**)&hflag, 4096, hipHostMallocMapped | hipHostMallocCoherent));
  uint32_t *dgo, *done, *rhdr;
  CK(hipMalloc(&dgo, 256 * 128));
  CK(hipMalloc(&done, 256));
  CK(hipMalloc(&rhdr, G * 32));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  for (int variant = 0; variant < 8; ++variant) {
    if (variant < 3 && getenv("SKIP_SLOW")) continue;
    const int Gv = variant == 3 ? 1 : variant == 4 ? 8 : variant == 5 ? 64 : G;
    std::memset(mbox, 0, 4096);
    std::memset(hflag, 0, 4096);
    CK(hipMemset(dgo, 0, 256 * 128));
    CK(hipMemset(done, 0, 256));
    CK(hipMemset(rhdr, 0, G * 32));
    P p;
    CK(hipHostGetDevicePointer((void**)&p.mbox, mbox, 0));
    CK(hipHostGetDevicePointer((void**)&p.hflag, hflag, 0));
    p.dev_go = dgo;
    p.done = done;
    p.rhdr = rhdr;
    p.variant = variant;
    p.lds_words = lds_kb * 256;
    p.max_polls = 1u << 22;
    const size_t shm = (size_t)p.lds_words * 4;
    CK(hipFuncSetAttribute((const void*)k_resident, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm));
    p.variant = (variant >= 3 && variant < 6) ? 0 : variant;
    hipLaunchKernelGGL(k_resident, dim3(Gv), dim3(kT), shm, s, p);
    CK(hipGetLastError());
    volatile uint32_t* vf = hflag;
    std::atomic_thread_fence(std::memory_order_seq_cst);
    std::vector<double> us;
    bool ok = true;
    for (int c = 1; c <= ncmd && ok; ++c) {
      mbox->op = 1;
      mbox->nparts = 4;
      auto t0 = std::chrono::steady_clock::now();
      __atomic_store_n(&mbox->seq, (uint32_t)c, __ATOMIC_RELEASE);
      for (long spin = 0; vf[0] != (uint32_t)c; ++spin) {
        if ((spin & 0xFFFF) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::seconds(3)) {
          std::printf("variant %d: timeout at command %d (status %u)\n", variant, c, vf[2]);
          ok = false;
          break;
        }
      }
      auto t1 = std::chrono::steady_clock::now();
      us.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
    }
    mbox->op = 2;
    __atomic_store_n(&mbox->seq, (uint32_t)ncmd + 1, __ATOMIC_RELEASE);
    CK(hipStreamSynchronize(s));
    std::vector<double> v(us.begin() + (us.size() > 100 ? 100 : 0), us.end());
    std::sort(v.begin(), v.end());
    double sum = 0;
    for (double x : v) sum += x;
    if (!v.empty())
      std::printf("variant %d (G=%d, lds %d KB): mean %.2f us, p50 %.2f, p10 %.2f, p90 %.2f, sum check %u\n", variant, Gv,
                  lds_kb, sum / v.size(), v[v.size() / 2], v[v.size() / 10], v[v.size() * 9 / 10], hflag[1]);
  }
  return 0;
}
