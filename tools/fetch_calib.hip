// FETCH_SIZE calibration for the decoder's access patterns (MI355X_MICROARCH.md,
// "HBM": widths other than 16 B/lane streaming reads are uncalibrated).
//
// Kernels, each with a known request count, run once per table size after a
// warm-up so that rocprofv3 --pmc passes can attribute counters per dispatch:
//   calib_stream  : coalesced 16 B/lane reads of `bytes` (the guide's
//                   calibrated case: FETCH_SIZE = bytes / 2)
//   calib_probe2  : the cuckoo probe pattern -- per key two independent 16 B
//                   loads at two hashed slots of a table of 16 B slots
//   calib_probe1  : one 16 B load per key (a bucketed table's single line)
//   calib_rec48   : the node-record pattern: 48 B records, 3 x 16 B loads by
//                   consecutive lanes of a record block
// Output: one JSON line per dispatch with its name, table bytes and the
// requested bytes / loads, in dispatch order (rocprofv3's Dispatch_Id order).
//   hipcc --offload-arch=gfx950 -O3 tools/fetch_calib.hip -o tools/fetch_calib
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

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

__global__ void calib_stream(const int4* __restrict__ a, size_t n16, int4* __restrict__ sink) {
  int4 acc = make_int4(0, 0, 0, 0);
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride) {
    const int4 v = a[i];
    acc.x ^= v.x; acc.y ^= v.y; acc.z ^= v.z; acc.w ^= v.w;
  }
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678) sink[0] = acc;   // never (keeps the loads)
}

// keys [0, n_keys): slot1 = mix(key) % slots, slot2 = mix(key ^ seed) % slots
__global__ void calib_probe2(const int4* __restrict__ tab, uint32_t slots, uint32_t n_keys, int4* __restrict__ sink) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n_keys) return;
  const uint32_t s1 = (uint32_t)(((uint64_t)mix(k) * slots) >> 32);
  const uint32_t s2 = (uint32_t)(((uint64_t)mix(k ^ 0x9e3779b9U) * slots) >> 32);
  const int4 a = tab[s1], b = tab[s2];
  if ((a.x ^ b.y ^ a.z ^ b.w) == 0x12345678) sink[0] = a;
}

__global__ void calib_probe1(const int4* __restrict__ tab, uint32_t slots, uint32_t n_keys, int4* __restrict__ sink) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n_keys) return;
  const uint32_t s1 = (uint32_t)(((uint64_t)mix(k) * slots) >> 32);
  const int4 a = tab[s1];
  if ((a.x ^ a.y ^ a.z ^ a.w) == 0x12345678) sink[0] = a;
}

// records of 48 B: lane t of a wave reads 16 B chunk t of the wave's block of
// 64 chunks (= 21.3 records), blocks at random record offsets
__global__ void calib_rec48(const int4* __restrict__ recs, uint32_t n_recs, uint32_t n_blocks, int4* __restrict__ sink) {
  const uint32_t w = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint32_t lane = threadIdx.x & 63;
  if (w >= n_blocks) return;
  const uint32_t first = (uint32_t)(((uint64_t)mix(w) * (n_recs - 64)) >> 32);
  int4 acc = make_int4(0, 0, 0, 0);
#pragma unroll
  for (int p = 0; p < 3; ++p) {
    const int4 v = recs[(size_t)first * 3 + p * 64 + lane];
    acc.x ^= v.x; acc.y ^= v.w;
  }
  if ((acc.x ^ acc.y) == 0x12345678) sink[0] = acc;
}

int main() {
  const size_t big = (size_t)2 << 30;              // 2 GiB: past the 256 MiB Infinity Cache
  int4* buf = nullptr;
  int4* sink = nullptr;
  CK(hipMalloc(&buf, big));
  CK(hipMalloc(&sink, 64));
  CK(hipMemset(buf, 1, big));
  const size_t tables[] = {(size_t)36 << 20, (size_t)18 << 20, (size_t)1 << 30};
  const uint32_t n_keys = 16u << 20;               // 16M keys per probe dispatch
  // warm-up of each kernel (not reported)
  calib_stream<<<1024, 256>>>(buf, 1 << 20, sink);
  calib_probe2<<<(n_keys + 255) / 256, 256>>>(buf, 1 << 20, n_keys, sink);
  calib_probe1<<<(n_keys + 255) / 256, 256>>>(buf, 1 << 20, n_keys, sink);
  calib_rec48<<<1024, 256>>>(buf, 1 << 20, 4096, sink);
  CK(hipDeviceSynchronize());
  const size_t sbytes = (size_t)1 << 30;
  calib_stream<<<4096, 256>>>(buf, sbytes / 16, sink);
  CK(hipDeviceSynchronize());
  printf("{\"kernel\": \"calib_stream\", \"bytes\": %zu, \"loads16\": %zu}\n", sbytes, sbytes / 16);
  for (size_t tb : tables) {
    const uint32_t slots = (uint32_t)(tb / 16);
    // touch the table once so a resident table starts resident
    calib_stream<<<1024, 256>>>(buf, tb / 16, sink);
    calib_probe2<<<(n_keys + 255) / 256, 256>>>(buf, slots, n_keys, sink);
    CK(hipDeviceSynchronize());
    printf("{\"kernel\": \"calib_probe2\", \"table_bytes\": %zu, \"keys\": %u, \"loads16\": %u}\n", tb, n_keys,
           2 * n_keys);
    calib_probe1<<<(n_keys + 255) / 256, 256>>>(buf, slots, n_keys, sink);
    CK(hipDeviceSynchronize());
    printf("{\"kernel\": \"calib_probe1\", \"table_bytes\": %zu, \"keys\": %u, \"loads16\": %u}\n", tb, n_keys,
           n_keys);
  }
  const uint32_t n_recs = (uint32_t)(big / 48) - 64, n_blocks = 1u << 20;
  calib_rec48<<<(n_blocks * 64 + 255) / 256, 256>>>(buf, n_recs, n_blocks, sink);
  CK(hipDeviceSynchronize());
  printf("{\"kernel\": \"calib_rec48\", \"record_bytes\": %zu, \"blocks\": %u, \"loads16\": %u}\n",
         (size_t)n_recs * 48, n_blocks, n_blocks * 192);
  CK(hipFree(buf));
  CK(hipFree(sink));
  return 0;
}
