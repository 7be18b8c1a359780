// D2H bandwidth probe: how fast can decode results reach pinned host memory?
//   (a) hipMemcpyAsync device -> pinned host (SDMA unless HSA_ENABLE_SDMA=0)
//   (b) a kernel storing straight into pinned host memory (zero-copy writes)
// Build: hipcc --offload-arch=gfx950 -O3 tools/d2h_probe.hip -o tools/d2h_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

__global__ void store_host(const int4* __restrict__ src, int4* __restrict__ dst, size_t n) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) dst[i] = src[i];
}

int main(int argc, char** argv) {
  const size_t sizes[] = {(size_t)4 << 20, (size_t)8 << 20, (size_t)19 << 20, (size_t)64 << 20};
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (size_t bytes : sizes) {
    void *d, *h, *hc;
    CK(hipMalloc(&d, bytes));
    CK(hipMemset(d, 1, bytes));
    CK(hipHostMalloc(&h, bytes, hipHostMallocDefault));
    CK(hipHostMalloc(&hc, bytes, hipHostMallocCoherent));
    float best_cp = 1e30f, best_k = 1e30f, best_kc = 1e30f;
    for (int it = 0; it < 8; ++it) {
      float ms;
      CK(hipEventRecord(a, st));
      CK(hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, st));
      CK(hipEventRecord(b, st));
      CK(hipEventSynchronize(b));
      CK(hipEventElapsedTime(&ms, a, b));
      if (ms < best_cp) best_cp = ms;
      for (int g = 0; g < 2; ++g) {
        int4* dst = (int4*)(g ? hc : h);
        CK(hipEventRecord(a, st));
        store_host<<<1024, 256, 0, st>>>((const int4*)d, dst, bytes / 16);
        CK(hipEventRecord(b, st));
        CK(hipEventSynchronize(b));
        CK(hipEventElapsedTime(&ms, a, b));
        float& best = g ? best_kc : best_k;
        if (ms < best) best = ms;
      }
    }
    printf("{\"bytes\": %zu, \"memcpy_GBs\": %.2f, \"kernel_store_GBs\": %.2f, \"kernel_store_coherent_GBs\": %.2f}\n",
           bytes, bytes / best_cp / 1e6, bytes / best_k / 1e6, bytes / best_kc / 1e6);
    CK(hipFree(d));
    CK(hipHostFree(h));
    CK(hipHostFree(hc));
  }
  return 0;
}
