// lt_results.hip -- decode results to the host in a compact form.
//
// The decoder writes each mature's path into a fixed slot of n_s codes
// (k * sum(n) int32 per batch, -1 padded; lattice_decode.h "Results"),
// about 2.5x the codes a path actually holds.  Before the results cross
// PCIe (or xGMI, for the multi-GPU gather) they are packed into a *slab*:
//
//   header {n_sent, k, n_codes, bytes}          32 B
//   count  int32[n_sent]                        (16 B aligned sections)
//   length int32[n_sent * k]
//   score  f64  [n_sent * k]
//   codes  int32[n_codes]   mature t of sentence s, t < count[s], in (s, t) order
//
// Three small kernels on the decode stream build the slab on the device
// (per-block length sums, one-block scan of the sums, then a pass that
// copies the entries and gathers the codes with coalesced writes), and a DMA
// (SDMA engine, hipMemcpyAsync) copies the slab's capacity into pinned host
// memory.  Round 6: that copy was a kernel of 64 blocks storing the used
// bytes over PCIe (lt_slab_to_host_k, the size read from the header on the
// device); its blocks sat on CUs for the whole transfer and kept the
// decode's LDS-filling blocks off them -- the k=1 decode of the next step ran
// 0.56 -> 0.94 ms beside it.  The DMA moves the capacity (the worst case,
// about the padded results' bytes), but takes no CU.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lt_internal.h"

using namespace lt;

namespace {

constexpr int PB = 256;          // entries (sentence, rank) per block

__device__ __forceinline__ int64_t entry_len(const ResultsPackParams& p, int64_t e) {
  const int64_t s = e / p.k;
  const int t = (int)(e - s * p.k);
  return t < p.count[s] ? (int64_t)p.len[e] : 0;
}

// Block-wide exclusive scan of one int64 per thread (PB threads = 4 waves).
__device__ __forceinline__ int64_t block_excl_scan(int64_t v, int64_t* sh, int64_t& total) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  int64_t x = v;
  for (int o = 1; o < 64; o <<= 1) {
    const int64_t y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) sh[w] = x;
  __syncthreads();
  int64_t before = 0;
  for (int i = 0; i < w; ++i) before += sh[i];
  total = sh[0] + sh[1] + sh[2] + sh[3];
  __syncthreads();
  return before + x - v;
}

__global__ __launch_bounds__(PB) void lt_pack_sums_k(ResultsPackParams p) {
  __shared__ int64_t sh[PB / 64];
  const int64_t e = (int64_t)blockIdx.x * PB + threadIdx.x;
  const int64_t v = e < p.n_entries ? entry_len(p, e) : 0;
  int64_t total;
  (void)block_excl_scan(v, sh, total);
  if (threadIdx.x == 0) p.block_sum[blockIdx.x] = total;
}

// One block: exclusive scan of the block sums (in place) + the slab header.
__global__ __launch_bounds__(1024) void lt_pack_scan_k(ResultsPackParams p) {
  __shared__ int64_t sh[16];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  int64_t carry = 0;
  for (int64_t base = 0; base < p.n_blocks; base += 1024) {
    const int64_t i = base + tid;
    const int64_t v = i < p.n_blocks ? p.block_sum[i] : 0;
    int64_t x = v;
    for (int o = 1; o < 64; o <<= 1) {
      const int64_t y = __shfl_up(x, o, 64);
      if (lane >= o) x += y;
    }
    if (lane == 63) sh[w] = x;
    __syncthreads();
    int64_t before = carry, total = 0;
    for (int j = 0; j < 16; ++j) {
      if (j < w) before += sh[j];
      total += sh[j];
    }
    if (i < p.n_blocks) p.block_sum[i] = before + x - v;
    carry += total;
    __syncthreads();
  }
  if (tid == 0) {
    SlabHeader* h = reinterpret_cast<SlabHeader*>(p.slab);
    h->n_sent = p.n_sent;
    h->k = p.k;
    h->n_codes = carry;
    h->bytes = (int64_t)slab_used_bytes(p.lay, carry);
    h->reserved = 0;
  }
}

// Entries of block b: count / length / score copied, codes gathered from the
// padded slots into the dense section (thread p of the block's code range
// finds its entry by binary search over the block's offsets in LDS).
__global__ __launch_bounds__(PB) void lt_pack_write_k(ResultsPackParams p) {
  __shared__ int64_t off[PB + 1];
  __shared__ int64_t src[PB];
  __shared__ int64_t sh[PB / 64];
  char* slab = reinterpret_cast<char*>(p.slab);
  int32_t* o_count = reinterpret_cast<int32_t*>(slab + p.lay.count);
  int32_t* o_len = reinterpret_cast<int32_t*>(slab + p.lay.len);
  double* o_score = reinterpret_cast<double*>(slab + p.lay.score);
  int32_t* o_codes = reinterpret_cast<int32_t*>(slab + p.lay.codes);
  const int tid = threadIdx.x;
  const int64_t e = (int64_t)blockIdx.x * PB + tid;
  int64_t v = 0;
  if (e < p.n_entries) {
    const int64_t s = e / p.k;
    const int t = (int)(e - s * p.k);
    const int32_t c = p.count[s];
    v = t < c ? (int64_t)p.len[e] : 0;
    if (t == 0) o_count[s] = c;
    o_len[e] = t < c ? p.len[e] : 0;
    o_score[e] = t < c ? p.score[e] : 0.0;
    src[tid] = (int64_t)p.k * p.cum_n[s] + (int64_t)t * p.sent_n[s];
  }
  int64_t total;
  const int64_t x = block_excl_scan(v, sh, total);
  const int64_t base = p.block_sum[blockIdx.x];
  off[tid] = x;
  if (tid == PB - 1) off[PB] = total;
  __syncthreads();
  const int n_here = (int)min((int64_t)PB, p.n_entries - (int64_t)blockIdx.x * PB);
  for (int64_t q = tid; q < total; q += PB) {
    int lo = 0, hi = n_here - 1;          // last entry with off <= q
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (off[mid] <= q) lo = mid;
      else hi = mid - 1;
    }
    o_codes[base + q] = p.codes[src[lo] + (q - off[lo])];
  }
}

// Used bytes of a device slab (header) -> pinned host memory, 16 B per lane.
__global__ __launch_bounds__(256) void lt_slab_to_host_k(const int4* __restrict__ slab, int4* __restrict__ host,
                                                        int64_t capacity16) {
  const int64_t used = min(capacity16, (reinterpret_cast<const SlabHeader*>(slab)->bytes + 15) / 16);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < used; i += stride) host[i] = slab[i];
}

}  // namespace

namespace lt {

hipError_t launch_pack_results(const ResultsPackParams& p, hipStream_t st) {
  if (p.n_blocks != (p.n_entries + PB - 1) / PB) return hipErrorInvalidValue;
  if (p.n_blocks > 0) {
    hipLaunchKernelGGL(lt_pack_sums_k, dim3((unsigned)p.n_blocks), dim3(PB), 0, st, p);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(lt_pack_scan_k, dim3(1), dim3(1024), 0, st, p);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || p.n_blocks == 0) return e;
  hipLaunchKernelGGL(lt_pack_write_k, dim3((unsigned)p.n_blocks), dim3(PB), 0, st, p);
  return hipGetLastError();
}

int64_t pack_blocks(int64_t n_entries) { return (n_entries + PB - 1) / PB; }

#ifndef LT_SLAB_KERNEL_COPY
#define LT_SLAB_KERNEL_COPY 0           // 1: the round-2..5 copy kernel (A/B builds)
#endif
hipError_t launch_slab_to_host(const void* slab, void* host, size_t capacity, hipStream_t st) {
  if (!LT_SLAB_KERNEL_COPY) return capacity ? hipMemcpyAsync(host, slab, capacity, hipMemcpyDeviceToHost, st) : hipSuccess;
  const int64_t c16 = (int64_t)(capacity / 16);
  if (c16 == 0) return hipSuccess;
  const int64_t want = (c16 + 255) / 256;
  // enough 16 B stores in flight for PCIe (~54 GB/s) from a few blocks
  const unsigned blocks = (unsigned)(want < 64 ? want : 64);
  hipLaunchKernelGGL(lt_slab_to_host_k, dim3(blocks), dim3(256), 0, st, static_cast<const int4*>(slab),
                     static_cast<int4*>(host), c16);
  return hipGetLastError();
}

}  // namespace lt
