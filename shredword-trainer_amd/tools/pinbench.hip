// Host read cost of pinned memory the GPU just wrote (coherent vs non-coherent mapping), and
// launch -> flag latency for a kernel whose every workgroup raises its own flag.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { std::printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__global__ void kw(uint32_t* hdr, uint32_t* flag, uint32_t seq, int words) {
  // each workgroup writes a 64-byte header then its flag
  if (threadIdx.x < 16) hdr[blockIdx.x * 16 + threadIdx.x] = seq + threadIdx.x;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store(flag + blockIdx.x, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

int run(unsigned flags, const char* name, int grid) {
  uint32_t *h, *f;
  CK(hipHostMalloc((void**)&h, 4096 * 64, flags));
  CK(hipHostMalloc((void**)&f, 4096 * 4, flags));
  std::memset(h, 0, 4096 * 64);
  std::memset(f, 0, 4096 * 4);
  void *dh, *df;
  CK(hipHostGetDevicePointer(&dh, h, 0));
  CK(hipHostGetDevicePointer(&df, f, 0));
  double tl = 0, tw = 0, tr = 0;
  const int iters = 2000;
  uint64_t sink = 0;
  for (int it = 1; it <= iters + 50; ++it) {
    double t0 = now();
    kw<<<grid, 64>>>((uint32_t*)dh, (uint32_t*)df, (uint32_t)it, 16);
    double t1 = now();
    for (int g = 0; g < grid; ++g)
      while (__atomic_load_n((volatile uint32_t*)(f + g), __ATOMIC_ACQUIRE) != (uint32_t)it) __builtin_ia32_pause();
    double t2 = now();
    for (int g = 0; g < grid; ++g)
      for (int k = 0; k < 16; k += 4) sink += h[g * 16 + k];
    double t3 = now();
    if (it > 50) { tl += t1 - t0; tw += t2 - t1; tr += t3 - t2; }
  }
  CK(hipDeviceSynchronize());
  std::printf("%-12s grid %4d: launch %6.2f us  flags-wait %6.2f us  header-read %6.2f us (sink %llu)\n", name, grid,
              1e6 * tl / iters, 1e6 * tw / iters, 1e6 * tr / iters, (unsigned long long)(sink & 1));
  CK(hipHostFree(h));
  CK(hipHostFree(f));
  return 0;
}

int main() {
  for (int grid : {4, 64, 256, 1024}) {
    run(hipHostMallocMapped | hipHostMallocCoherent, "coherent", grid);
    run(hipHostMallocMapped | hipHostMallocNonCoherent, "noncoherent", grid);
    run(hipHostMallocMapped, "default", grid);
  }
  return 0;
}
