// kbench — latency anatomy of k_merge's skeleton on MI355X (diagnostic, not product code).
//
// Variants, each timed as host launch -> host flag (and HIP events):
//   0  empty: every workgroup signals a ticket, the last raises the host flag
//   1  + each wave loads its 1024-token tile (4 x 16 B per lane) and votes
//   2  + LDS hash init/flush loop (512 slots) as in k_merge
//   3  variant 2 with grid-stride (fewer, fatter workgroups: 2 per CU)
//   4  variant 1, single global ticket instead of per-XCD shards
//   5  variant 1 without the host flag: hipStreamSynchronize instead
//
//   hipcc --offload-arch=gfx950 -O3 -o kbench kbench.hip && ./kbench [ntiles]
#include <hip/hip_runtime.h>

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

struct P {
  const int* tok;
  const unsigned* len;
  unsigned ntiles;
  unsigned* done;
  unsigned* hflag;
  unsigned seq;
  int variant;
  unsigned long long* sink;
};

__global__ __launch_bounds__(256) void kb(P p) {
  __shared__ unsigned hk[512];
  __shared__ unsigned long long hs[512], hf[512];
  __shared__ unsigned s_last;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (p.variant >= 2) {
    for (int i = threadIdx.x; i < 512; i += 256) {
      hk[i] = ~0u;
      hs[i] = 0;
      hf[i] = ~0ull;
    }
    __syncthreads();
  }
  int acc = 0;
  if (p.variant >= 1) {
    for (unsigned tile = blockIdx.x * 4 + wid; tile < p.ntiles; tile += gridDim.x * 4) {
      const unsigned len = p.len[tile];
      const int* base = p.tok + (size_t)tile * 1024;
      int4 v[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int idx = lane * 16 + 4 * q;
        v[q] = idx + 4 <= (int)len ? *reinterpret_cast<const int4*>(base + idx) : make_int4(0, 0, 0, 0);
      }
      bool any = false;
#pragma unroll
      for (int q = 0; q < 4; ++q) any |= (v[q].x == -7) | (v[q].y == -7) | (v[q].z == -7) | (v[q].w == -7);
      acc += __any(any);
    }
  }
  if (p.variant >= 2) {
    __syncthreads();
    for (int i = threadIdx.x; i < 512; i += 256)
      if (hk[i] != ~0u) atomicAdd(p.sink, hs[i] + hf[i]);
  }
  if (acc > 1000000) atomicAdd(p.sink, 1ull);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    bool last;
    if (p.variant == 4) {
      last = atomicAdd(&p.done[8], 1u) == gridDim.x - 1;
    } else {
      const unsigned g = blockIdx.x & 7u;
      const unsigned in_group = (gridDim.x - g + 7u) >> 3;
      last = false;
      if (atomicAdd(&p.done[g], 1u) == in_group - 1u) {
        atomicExch(&p.done[g], 0u);
        const unsigned groups = gridDim.x < 8u ? gridDim.x : 8u;
        last = atomicAdd(&p.done[8], 1u) == groups - 1u;
      }
    }
    s_last = last;
  }
  __syncthreads();
  if (!s_last || threadIdx.x != 0) return;
  atomicExch(&p.done[8], 0u);
  __threadfence_system();
  __hip_atomic_store(p.hflag, p.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Doorbell variant: the kernel is queued before the host knows the work.  Block 0 / lane 0
// polls a host-written mailbox, publishes a go word in device memory; every other workgroup
// polls the go word (bounded spins), then does variant-1 work and the usual tickets + flag.
struct D {
  const int* tok;
  const unsigned* len;
  unsigned ntiles;
  unsigned* done;
  unsigned* hflag;
  const unsigned* mailbox;  // host memory
  unsigned* go;             // device memory
  unsigned seq;
  unsigned long long* sink;
};

__global__ __launch_bounds__(256) void kd(D p) {
  __shared__ unsigned s_go, s_last;
  if (threadIdx.x == 0) {
    unsigned v = 0;
    if (blockIdx.x == 0) {
      for (long spin = 0; spin < 200000000L; ++spin) {
        v = __hip_atomic_load(p.mailbox, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
        if (v == p.seq) break;
        __builtin_amdgcn_s_sleep(1);
      }
      __hip_atomic_store(p.go, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      for (long spin = 0; spin < 200000000L; ++spin) {
        v = __hip_atomic_load(p.go, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
        if (v == p.seq) break;
        __builtin_amdgcn_s_sleep(2);
      }
    }
    s_go = v;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  int acc = 0;
  for (unsigned tile = blockIdx.x * 4 + wid; tile < p.ntiles; tile += gridDim.x * 4) {
    const unsigned len = p.len[tile];
    const int* base = p.tok + (size_t)tile * 1024;
    int4 v[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int idx = lane * 16 + 4 * q;
      v[q] = idx + 4 <= (int)len ? *reinterpret_cast<const int4*>(base + idx) : make_int4(0, 0, 0, 0);
    }
    bool any = false;
#pragma unroll
    for (int q = 0; q < 4; ++q) any |= (v[q].x == -7) | (v[q].y == -7) | (v[q].z == -7) | (v[q].w == -7);
    acc += __any(any);
  }
  if (acc > 1000000) atomicAdd(p.sink, 1ull);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned g = blockIdx.x & 7u;
    const unsigned in_group = (gridDim.x - g + 7u) >> 3;
    bool last = false;
    if (atomicAdd(&p.done[g], 1u) == in_group - 1u) {
      atomicExch(&p.done[g], 0u);
      const unsigned groups = gridDim.x < 8u ? gridDim.x : 8u;
      last = atomicAdd(&p.done[8], 1u) == groups - 1u;
    }
    s_last = last;
  }
  __syncthreads();
  if (!s_last || threadIdx.x != 0) return;
  atomicExch(&p.done[8], 0u);
  __threadfence_system();
  __hip_atomic_store(p.hflag, p.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Fat variant: BLOCK threads per workgroup, every wave walks tiles grid-stride with the next
// tile's loads issued before the current tile is voted on.
template <int BLOCK>
__global__ __launch_bounds__(BLOCK) void kf(P p) {
  __shared__ unsigned s_last;
  constexpr int W = BLOCK / 64;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  int acc = 0;
  const unsigned stride = gridDim.x * W;
  unsigned tile = blockIdx.x * W + wid;
  int4 cur[4];
  unsigned clen = 0;
  auto load = [&](unsigned t, int4 (&v)[4], unsigned& l) {
    l = p.len[t];
    const int* base = p.tok + (size_t)t * 1024;
#pragma unroll
    for (int q = 0; q < 4; ++q) v[q] = *reinterpret_cast<const int4*>(base + lane * 16 + 4 * q);
  };
  if (tile < p.ntiles) load(tile, cur, clen);
  while (tile < p.ntiles) {
    const unsigned nt = tile + stride;
    int4 nxt[4];
    unsigned nlen = 0;
    if (nt < p.ntiles) load(nt, nxt, nlen);
    bool any = false;
#pragma unroll
    for (int q = 0; q < 4; ++q)
      any |= ((lane * 16 + 4 * q) < (int)clen) & ((cur[q].x == -7) | (cur[q].y == -7) | (cur[q].z == -7) | (cur[q].w == -7));
    acc += __any(any);
#pragma unroll
    for (int q = 0; q < 4; ++q) cur[q] = nxt[q];
    clen = nlen;
    tile = nt;
  }
  if (acc > 1000000) atomicAdd(p.sink, 1ull);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned g = blockIdx.x & 7u;
    const unsigned in_group = (gridDim.x - g + 7u) >> 3;
    bool last = false;
    if (atomicAdd(&p.done[g], 1u) == in_group - 1u) {
      atomicExch(&p.done[g], 0u);
      const unsigned groups = gridDim.x < 8u ? gridDim.x : 8u;
      last = atomicAdd(&p.done[8], 1u) == groups - 1u;
    }
    s_last = last;
  }
  __syncthreads();
  if (!s_last || threadIdx.x != 0) return;
  atomicExch(&p.done[8], 0u);
  __threadfence_system();
  __hip_atomic_store(p.hflag, p.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

template <int BLOCK>
void run_fat(P base, unsigned grid, hipStream_t s, hipEvent_t e0, hipEvent_t e1, unsigned* hflag, unsigned& seq) {
  const int iters = 2000;
  double host = 0, ev = 0;
  for (int it = 0; it < iters + 50; ++it) {
    P p = base;
    p.seq = ++seq;
    CK(hipEventRecord(e0, s));
    auto t0 = std::chrono::steady_clock::now();
    kf<BLOCK><<<grid, BLOCK, 0, s>>>(p);
    CK(hipEventRecord(e1, s));
    while (__atomic_load_n(hflag, __ATOMIC_ACQUIRE) != seq) __builtin_ia32_pause();
    auto t1 = std::chrono::steady_clock::now();
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (it >= 50) {
      host += std::chrono::duration<double, std::micro>(t1 - t0).count();
      ev += ms * 1e3;
    }
  }
  std::printf("fat block %4d grid %4u: host launch->flag %7.2f us, event %7.2f us\n", BLOCK, grid, host / iters, ev / iters);
}

int main(int argc, char** argv) {
  const unsigned ntiles = argc > 1 ? (unsigned)std::atoi(argv[1]) : 4576;
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  std::vector<int> h((size_t)ntiles * 1024, 1);
  std::vector<unsigned> lens(ntiles, 1000);
  int* tok;
  unsigned *len, *done, *hflag;
  unsigned long long* sink;
  CK(hipMalloc(&tok, h.size() * 4));
  CK(hipMalloc(&len, ntiles * 4));
  CK(hipMalloc(&done, 64));
  CK(hipMalloc(&sink, 8));
  CK(hipMemcpy(tok, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(len, lens.data(), ntiles * 4, hipMemcpyHostToDevice));
  CK(hipMemset(done, 0, 64));
  CK(hipHostMalloc((void**)&hflag, 64, hipHostMallocMapped | hipHostMallocCoherent));
  unsigned* dflag;
  CK(hipHostGetDevicePointer((void**)&dflag, hflag, 0));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  unsigned seq = 0;
  for (int variant = 0; variant <= 5; ++variant) {
    for (int gmode = 0; gmode < 2; ++gmode) {
      const unsigned groups = (ntiles + 3) / 4;
      unsigned grid = gmode == 0 ? std::min<unsigned>(groups, cus * 4) : std::min<unsigned>(groups, cus * 2);
      if (variant == 3 && gmode == 0) continue;
      const int iters = 2000;
      double host = 0, ev = 0;
      for (int it = 0; it < iters + 50; ++it) {
        P p{tok, len, ntiles, done, dflag, ++seq, variant == 3 ? 2 : variant, sink};
        CK(hipEventRecord(e0, s));
        auto t0 = std::chrono::steady_clock::now();
        kb<<<grid, 256, 0, s>>>(p);
        CK(hipEventRecord(e1, s));
        if (variant == 5) {
          CK(hipStreamSynchronize(s));
        } else {
          while (__atomic_load_n(hflag, __ATOMIC_ACQUIRE) != seq) __builtin_ia32_pause();
        }
        auto t1 = std::chrono::steady_clock::now();
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (it >= 50) {
          host += std::chrono::duration<double, std::micro>(t1 - t0).count();
          ev += ms * 1e3;
        }
      }
      std::printf("variant %d grid %4u (%s): host launch->flag %7.2f us, event %7.2f us\n", variant, grid,
                  gmode ? "2/CU" : "4/CU", host / iters, ev / iters);
    }
  }
  {
    P base{tok, len, ntiles, done, dflag, 0, 1, sink};
    for (unsigned g : {32u, 64u, 128u, 256u, 512u}) run_fat<256>(base, g, s, e0, e1, hflag, seq);
    for (unsigned g : {32u, 64u, 128u, 256u}) run_fat<512>(base, g, s, e0, e1, hflag, seq);
    for (unsigned g : {16u, 32u, 64u, 128u, 256u}) run_fat<1024>(base, g, s, e0, e1, hflag, seq);
  }
  if (argc > 2) return 0;
  // doorbell: kernel for step i+1 is queued right after step i's; host "works" 8 us between
  unsigned* mbox;
  CK(hipHostMalloc((void**)&mbox, 64, hipHostMallocMapped | hipHostMallocCoherent));
  unsigned* dmbox;
  CK(hipHostGetDevicePointer((void**)&dmbox, mbox, 0));
  unsigned* go;
  CK(hipMalloc(&go, 64));
  CK(hipMemset(go, 0, 64));
  for (int gmode = 0; gmode < 3; ++gmode) {
    const unsigned groups = (ntiles + 3) / 4;
    const unsigned grid = gmode == 0 ? std::min<unsigned>(groups, cus * 4)
                        : gmode == 1 ? std::min<unsigned>(groups, cus * 2) : std::min<unsigned>(groups, 64);
    const int iters = 2000;
    double lat = 0;
    unsigned s0 = seq + 1;
    D d{tok, len, ntiles, done, dflag, dmbox, go, s0, sink};
    kd<<<grid, 256, 0, s>>>(d);
    for (int it = 0; it < iters + 50; ++it) {
      const unsigned cur = s0 + it;
      D dn{tok, len, ntiles, done, dflag, dmbox, go, cur + 1, sink};
      kd<<<grid, 256, 0, s>>>(dn);  // pre-launch the next one
      auto w0 = std::chrono::steady_clock::now();
      while (std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - w0).count() < 8.0) {}
      auto t0 = std::chrono::steady_clock::now();
      __atomic_store_n(mbox, cur, __ATOMIC_RELEASE);
      while (__atomic_load_n(hflag, __ATOMIC_ACQUIRE) != cur) __builtin_ia32_pause();
      auto t1 = std::chrono::steady_clock::now();
      if (it >= 50) lat += std::chrono::duration<double, std::micro>(t1 - t0).count();
    }
    const unsigned last = s0 + iters + 50;
    __atomic_store_n(mbox, last, __ATOMIC_RELEASE);  // release the final pre-launched kernel
    CK(hipStreamSynchronize(s));
    seq = last;
    std::printf("doorbell grid %4u: mailbox write -> flag %7.2f us\n", grid, lat / iters);
  }
  return 0;
}
