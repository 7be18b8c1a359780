// Ceiling of random 16 B gathers on this GPU: the access pattern of the
// decoders' feature-table probes (one 16 B slot per load, uniformly random
// slots of a table of T bytes), with as many loads in flight as the hardware
// takes -- every lane issues U independent loads per iteration, the grid fills
// every CU.  Prints one JSON line per (table size, loads in flight): loads/s
// and the bytes those loads name (16 B each), from HIP events around the
// timed launches (warm-up launch first).  The decoders' probe rates are read
// against the row of their table size (bench.py / profiles/).
//   hipcc --offload-arch=gfx950 -O3 tools/gather_ceiling.hip -o tools/gather_ceiling
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));     \
      exit(1);                                                                       \
    }                                                                                \
  } while (0)

__device__ __forceinline__ uint32_t mix(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}

// slots is a power of two; every lane: iters x U loads, U in flight at once
template <int U>
__global__ void __launch_bounds__(256) gather(const uint4* __restrict__ tab, uint32_t slot_mask, int iters,
                                              uint32_t seed, uint4* __restrict__ sink) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t x = mix(t ^ seed);
  uint4 acc = make_uint4(0, 0, 0, 0);
  for (int it = 0; it < iters; ++it) {
    uint4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      x = x * 0x9E3779B1u + 0x7F4A7C15u;          // (the next slot does not depend on a loaded value)
      v[u] = tab[mix(x) & slot_mask];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      acc.x ^= v[u].x; acc.y ^= v[u].y; acc.z ^= v[u].z; acc.w ^= v[u].w;
    }
  }
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) sink[t & 1023] = acc;   // never (keeps the loads)
}

template <int U>
static void run(const uint4* tab, size_t bytes, uint4* sink, int blocks, int iters) {
  const uint32_t mask = (uint32_t)(bytes / 16 - 1);
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  hipLaunchKernelGGL((gather<U>), dim3(blocks), dim3(256), 0, 0, tab, mask, iters, 1u, sink);   // warm-up
  CK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int r = 0; r < 3; ++r) {
    CK(hipEventRecord(a, 0));
    hipLaunchKernelGGL((gather<U>), dim3(blocks), dim3(256), 0, 0, tab, mask, iters, 2u + r, sink);
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, a, b));
    best = ms < best ? ms : best;
  }
  const double loads = (double)blocks * 256 * iters * U;
  printf("{\"table_bytes\": %zu, \"loads_in_flight_per_lane\": %d, \"loads\": %.0f, \"ms\": %.4f, "
         "\"loads_per_s\": %.4e, \"named_GBps\": %.1f}\n",
         bytes, U, loads, best, loads / (best * 1e-3), loads * 16 / (best * 1e-3) / 1e9);
  fflush(stdout);
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
}

int main() {
  int dev = 0, cus = 0;
  CK(hipGetDevice(&dev));
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  const size_t maxb = (size_t)1 << 30;
  uint4* tab = nullptr;
  uint4* sink = nullptr;
  CK(hipMalloc((void**)&tab, maxb));
  CK(hipMalloc((void**)&sink, 1024 * sizeof(uint4)));
  CK(hipMemset(tab, 0x5A, maxb));
  const int blocks = cus * 8;                      // 32 waves per CU
  const int iters = 64;
  for (size_t bytes : {(size_t)2 << 20, (size_t)32 << 20, (size_t)64 << 20, (size_t)128 << 20, maxb}) {
    run<4>(tab, bytes, sink, blocks, iters);
    run<8>(tab, bytes, sink, blocks, iters);
    run<16>(tab, bytes, sink, blocks, iters);
  }
  CK(hipFree(tab));
  CK(hipFree(sink));
  return 0;
}
