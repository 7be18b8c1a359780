// Issue rate of the integer multiplies the probe hash uses (no library, one
// GPU): each kernel runs 8 independent chains of one instruction per lane,
// enough waves to fill every SIMD; prints ns per wave-instruction per SIMD.
//   hipcc --offload-arch=gfx950 -O3 tools/valu_rate.hip -o tools/valu_rate && ./tools/valu_rate
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int ITERS = 4096;

#define CHAIN8(OP)                                                     \
  _Pragma("unroll 8") for (int i = 0; i < ITERS; ++i) {                \
    a0 = OP(a0, k); a1 = OP(a1, k); a2 = OP(a2, k); a3 = OP(a3, k);    \
    a4 = OP(a4, k); a5 = OP(a5, k); a6 = OP(a6, k); a7 = OP(a7, k);    \
  }

__device__ __forceinline__ uint32_t op_mulhi(uint32_t a, uint32_t k) { return __umulhi(a, k) ^ a; }
__device__ __forceinline__ uint32_t op_mullo(uint32_t a, uint32_t k) { return (a * k) ^ 1u; }
__device__ __forceinline__ uint32_t op_mul24(uint32_t a, uint32_t k) { return __umul24(a, k) ^ a; }
__device__ __forceinline__ uint32_t op_xor(uint32_t a, uint32_t k) { return (a ^ k) + 1u; }

#define KERNEL(NAME, OP)                                                                  \
  __global__ void __launch_bounds__(256) NAME(uint32_t* out, uint32_t k) {                \
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4,         \
             a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;                                         \
    CHAIN8(OP)                                                                            \
    out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;             \
  }

KERNEL(k_mulhi, op_mulhi)
KERNEL(k_mullo, op_mullo)
KERNEL(k_mul24, op_mul24)
KERNEL(k_xor, op_xor)

int main() {
  int dev = 0;
  hipDeviceProp_t pr;
  hipGetDeviceProperties(&pr, dev);
  const int blocks = pr.multiProcessorCount * 8;      // 8 x 4 waves per CU: 8 waves per SIMD
  uint32_t* out;
  hipMalloc(&out, (size_t)blocks * 256 * 4);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  struct K { const char* name; void (*fn)(uint32_t*, uint32_t); int ops; };
  const K ks[] = {{"v_mul_hi_u32 (+xor)", k_mulhi, 2}, {"v_mul_lo_u32 (+xor)", k_mullo, 2},
                  {"v_mul_u32_u24 (+xor)", k_mul24, 2}, {"v_xor + v_add", k_xor, 2}};
  for (const K& kk : ks) {
    for (int rep = 0; rep < 2; ++rep) {
      hipEventRecord(a);
      hipLaunchKernelGGL(kk.fn, dim3(blocks), dim3(256), 0, 0, out, 0x9E3779B1u);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms = 0;
      hipEventElapsedTime(&ms, a, b);
      const double wave_insts = (double)blocks * 4 * ITERS * 8 * kk.ops;   // per GPU
      const double simds = pr.multiProcessorCount * 4.0;
      if (rep) printf("%-24s %.3f ms  %.2f ns per wave-instruction pair per SIMD (%.1f cycles at %.0f MHz)\n",
                      kk.name, ms, ms * 1e6 / (wave_insts / kk.ops / simds),
                      ms * 1e-3 * pr.clockRate * 1e3 / (wave_insts / kk.ops / simds), pr.clockRate / 1e3);
    }
  }
  hipFree(out);
  return 0;
}
