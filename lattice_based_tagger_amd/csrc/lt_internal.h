// lt_internal.h -- kernel launch interface between lt_capi.cpp and lt_decode.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "lt_common.h"

namespace lt {

struct DecodeParams {
  // model
  const void* table;            // SlotN[] or SlotW[] (cuckoo, two choices)
  uint32_t slots;
  uint32_t seed;
  NarrowHash hk;                // narrow tables: slot hash constants (from seed)
  const double* d3;             // dense class-3 table (D3_DIM^2) or NULL
  uint32_t d3off;               // the dense class-3 table's bit window (lt_common.h d3_window)
  int32_t narrow;               // 1: SlotN, 0: SlotW
  int32_t has_tri;
  // batch (device pointers)
  int32_t n_sent;
  int32_t max_len;
  int32_t n_post;
  int32_t k;
  int32_t bp_stride;            // backpointer entries per end position (batch max_k)
  int64_t n_nodes;
  const int32_t* order;         // processing order of sentences
  const int32_t* sent_n;
  const int64_t* node_off;
  const int64_t* span_off;
  const int32_t* span_start;
  const NodeRec* nodes;         // AoS node records; mask + span length bits (D_SHIFT)
  const F46* pairs;             // the batch's class-4/6 pair table (NodeRec, PX_SHIFT)
  int32_t n_pairs;
  const F46* esc;               // [n_nodes] pairs of PX_ESC nodes (nullptr: none)
  const double* npost;
  // implicit Unknown candidates (lattice_decode.h n_unk): an in-range span with
  // no node holds one, whose record is unk[d-1] (d = span length) and whose
  // node-local post terms are unk_post[t * n_unk + d - 1]; its local node is
  // UNK_LOCAL.  n_unk = 0: none.
  int32_t n_unk;
  const NodeRec* unk;
  const double* unk_post;
  // edge terms (lt_batch_desc.n_edge; 0 = none): increment = ((pre + t_0) + t_1)...
  int32_t n_edge;
  int32_t n_terms;
  uint64_t term_kinds;          // 2 bits per term: 0 trigram, 1 npost row, 2 edge row
  int64_t n_edges;
  const int64_t* edge_base;     // [n_nodes]: value of predecessor local node j at edge_base[gn] + j
  const double* edge_val;       // [n_edge][n_edges]
  // further trigram terms (lt_batch_desc.n_xtri; general kernel only): scorer
  // t = 1..n_xtri's node mask + flags and class 4/5/6 coefficients at
  // [(t-1) * n_nodes + node], its keys' classes + LT_XTRI_CLASS_STRIDE * t
  int32_t n_xtri;
  const uint32_t* xmask;
  const double* xf4;
  const double* xf5;
  const double* xf6;
  // k=1 lane schedule of the piece (launch_k1_sched): wave w's macro-steps are
  // sched[wave_off[w] * 64 ..] (64 entries each)
  const uint32_t* sched;
  const int64_t* wave_off;
  uint32_t* k1_place;           // [piece chars] placement of (sentence s, end position e) at cum_n[s] + e - 1
                                // (k1_place_word: first macro-step, first lane, dead Unknowns; k1_schedule)
  uint32_t* k1_fill;            // non-NULL: the beam-1 decode fills its waves' rows of sched (== this) first
  // scratch + results
  uint32_t* bp;
  int64_t bp_bytes;             // bytes of bp (< 2^31: 32-bit buffer offsets)
  const int64_t* bp_off;
  const int64_t* cum_n;         // sum_{s2<s} n_s2 (codes of s start at k*cum_n[s])
  int32_t* out_count;
  int32_t* out_len;
  double* out_score;
  int32_t* out_codes;
  unsigned long long* counters; // [3] expansions, feature tuples, probes
  // general kernel (lt_beam_wide: max_len > 8 or k > LT_MAX_BEAM_COMPILED)
  int32_t span_slots;           // span_slots(max_len)
  int32_t wide_threads;         // threads of the launch (each owns a scratch block)
  int64_t wide_block;           // scratch bytes per thread (wide_scratch_bytes)
  char* wide_scratch;           // [wide_threads * wide_block]
};

// Batch evaluate (lt_evaluate): word increments, then per-path sums.
struct EvalParams {
  const void* table;
  uint32_t slots;
  uint32_t seed;
  NarrowHash hk;
  int32_t narrow;
  int32_t has_tri;
  const double* d3;
  uint32_t d3off;               // the dense class-3 table's bit window (lt_common.h d3_window)
  int32_t n_paths;
  int64_t n_words;
  const NodeRec* words;         // AoS word records
  const F46* pairs;             // their class-4/6 pair table (NodeRec, PX_SHIFT)
  const F46* esc;               // [n_words] pairs of PX_ESC words (nullptr: none)
  const int64_t* prev1;
  const int64_t* prev2;
  const int64_t* path_off;
  int32_t n_terms;
  const double* terms;
  int32_t trigram_pos;
  uint32_t coff;                // key class offset of the trigram scorer (LT_XTRI_CLASS_STRIDE * scorer)
  double* inc;                  // [n_words] scratch
  double* out;                  // [n_paths]
};
hipError_t launch_evaluate(const EvalParams& p, hipStream_t st);

// ---- compact results ("slabs", lt_results.hip; lattice_decode.h) ----------
struct SlabHeader {
  int32_t n_sent;
  int32_t k;
  int64_t n_codes;              // path codes in the slab
  int64_t bytes;                // used bytes (header included)
  int64_t reserved;
};
static_assert(sizeof(SlabHeader) == 32, "slab header is 32 B");

__host__ __device__ inline uint64_t al16(uint64_t x) { return (x + 15) & ~(uint64_t)15; }

// Section offsets of a slab of n_sent sentences, beam k, and its capacity
// for `chars` characters (a path of a sentence of n characters has <= n words).
struct SlabLayout {
  uint64_t count, len, score, codes, capacity;
};
__host__ __device__ inline SlabLayout slab_layout(int64_t n_sent, int k, int64_t chars) {
  SlabLayout L;
  L.count = sizeof(SlabHeader);
  L.len = L.count + al16(4 * (uint64_t)n_sent);
  L.score = L.len + al16(4 * (uint64_t)n_sent * k);
  L.codes = L.score + al16(8 * (uint64_t)n_sent * k);
  L.capacity = L.codes + al16(4 * (uint64_t)chars * k);
  return L;
}
__host__ __device__ inline uint64_t slab_used_bytes(const SlabLayout& L, int64_t n_codes) {
  return L.codes + al16(4 * (uint64_t)n_codes);
}

struct ResultsPackParams {
  // the decode's padded results (device)
  const int32_t* count;
  const int32_t* len;
  const double* score;
  const int32_t* codes;
  const int32_t* sent_n;
  const int64_t* cum_n;
  int32_t n_sent;
  int32_t k;
  int64_t n_entries;            // n_sent * k
  int64_t n_blocks;             // pack_blocks(n_entries)
  int64_t* block_sum;           // [n_blocks] scratch
  SlabLayout lay;
  void* slab;                   // device, lay.capacity bytes
};
int64_t pack_blocks(int64_t n_entries);
hipError_t launch_pack_results(const ResultsPackParams& p, hipStream_t st);
// Copies the used bytes of a device slab (its header says how many) into
// pinned host memory of `capacity` bytes.
hipError_t launch_slab_to_host(const void* slab, void* host, size_t capacity, hipStream_t st);

// Trace of a decode (beam_search(debug=True), beam.py:53-57): every expansion
// of every end position in generation order, and each position's beam.  One
// thread per sentence over global memory; the same scoring code as the
// decoders.  Positions of sentence s: pos_off[s] + e (e = 0..n_s).
constexpr int TRACE_ENTRY_BYTES = 64;
struct TraceParams {
  const int64_t* pos_off;       // [n_sent + 1]
  const int64_t* exp_off;       // [positions + 1]: expansion slots of position q: [exp_off[q], exp_off[q+1])
  void* ent;                    // [positions * k] hypothesis entries (scratch)
  int32_t* beam_count;          // [positions]
  uint32_t* beam_gen;           // [positions * k]: generation index of beam[e][r]
  int32_t* exp_count;           // [positions]: expansions enumerated at the position (-1: slots too few)
  double* exp_score;            // [expansion slots]
  uint32_t* exp_node;           // [expansion slots]: bp_pack(node, span, parent rank)
  uint8_t* exp_skip;            // [expansion slots]: 1 = skipped (beam.py:43-45)
  uint64_t* exp_link;           // [expansion slots] or NULL: bpw_pack(node, span, parent rank)
};
hipError_t launch_trace(const DecodeParams& p, const TraceParams& t, hipStream_t st);

// dst = the table src with every slot's overflow flag cleared (the copy the
// beam kernels probe: they load both candidate slots and compare keys plainly)
hipError_t launch_strip_flags(void* dst, const void* src, int64_t bytes, bool narrow, hipStream_t st);

constexpr int LT_MAX_BEAM_COMPILED = 256;
// A decode goes to the general kernel when its max_len or beam is beyond the
// tuned kernels' (backpointers of two words, bpw_pack).
__host__ __device__ inline bool decode_is_wide(int max_len, int k) { return max_len > MAX_SPAN || k > LT_MAX_BEAM_COMPILED; }
// Scratch of one lt_beam_wide thread: the beams of the last S + 1 end
// positions (64 B entries), their sizes, and the selection heap of k items.
constexpr int WIDE_ENTRY_BYTES = 64, WIDE_ITEM_BYTES = 24;
inline int64_t wide_scratch_bytes(int span_slots, int k) {
  const int64_t ring = (int64_t)(span_slots + 1) * k * WIDE_ENTRY_BYTES;
  const int64_t cnt = ((int64_t)(span_slots + 1) * 4 + 15) & ~(int64_t)15;
  const int64_t heap = ((int64_t)k * WIDE_ITEM_BYTES + 15) & ~(int64_t)15;
  return ring + cnt + heap;
}
hipError_t launch_wide(const DecodeParams& p, hipStream_t st, bool count = false, hipEvent_t e0 = nullptr,
                       hipEvent_t e1 = nullptr);
int beam_template_for(int k);
const char* kernel_name_for(int k);
// e0 / e1 (may be NULL): events recorded at the start / end of the kernel.
hipError_t launch_decode(const DecodeParams& p, hipStream_t st, bool count, hipEvent_t e0 = nullptr,
                         hipEvent_t e1 = nullptr);
// k=1 lane schedule of a piece (the kernel's sentence order, K1_W sentences
// per wave): waves = k1_waves(p.n_sent); wave w's macro-steps start at
// wave_off[w] (counted on the host, k1_schedule), the fill kernel writes the
// entries.  A sentence's candidates at end position e are in generation order
// (span slot j = 8 - d ascending, the slot's nodes, or its implicit Unknown)
// on consecutive lanes of one macro-step (of consecutive macro-steps when
// there are more than 64).
#ifndef LT_K1_W
#define LT_K1_W 8
#endif
constexpr int K1_W = LT_K1_W;
static_assert(K1_W <= 8, "the entry's sentence field has 3 bits");
inline int k1_waves(int n_sent) { return (n_sent + K1_W - 1) / K1_W; }
// entry of a lane at a macro-step: bits 0-25 the piece-global node (all ones:
// idle lane) or, with K1_UNK, d - 1 of the lane's implicit Unknown; bits
// 26-28 the lane's sentence in the wave; bit 31 the first macro-step of the
// sentence's next end position (the lane's sentence moves to it)
constexpr uint32_t K1_NODE = 0x03FFFFFFu, K1_IDLE = K1_NODE, K1_UNK = 0x40000000u, K1_FIRST = 0x80000000u;
// a wave's macro-steps stay below 2^K1_TBITS (lt_batch_create checks): the
// fill packs a position's placement into one word -- first macro-step, first
// lane << K1_TBITS, and the position's dead implicit Unknowns (k1_dead_mask)
// << K1_DBITS
constexpr int K1_TBITS = 19, K1_DBITS = 25;
// A statically dead implicit Unknown.  The reference skips an Unknown
// candidate of span (b, e) after a hypothesis whose last word is Unknown
// (num_unk counts the Unknowns at the tail, Sequence.add beam.py:112-113)
// unless b = b_min (beam.py:43-45).  Every hypothesis of beam[b] ends in a
// candidate of end position b; when position b holds no explicit node, all of
// them are implicit Unknowns, so every such hypothesis ends in an Unknown and
// the candidate is skipped after each of them -- it needs no lane.  Position
// b's explicit nodes are span_start[(b-1)*8 .. b*8); `ss` is the sentence's
// span table, d the span length, dmax = min(e, max_len) (d < dmax <=> b >
// b_min).  A conservative rule: an explicit node at b tagged Unknown keeps
// the candidate (the kernel skips it at run time then).
__host__ __device__ inline bool k1_unk_dead(const int32_t* ss, int e, int d, int dmax) {
  const int b = e - d;
  return d < dmax && ss[b * MAX_SPAN] == ss[(b - 1) * MAX_SPAN];
}
// the dead implicit Unknowns of end position e: bit d - 1 for span length d
// (1..7; d = dmax is never dead)
__host__ __device__ inline uint32_t k1_dead_mask(const int32_t* ss, int e, int max_len) {
  const int dmax = e < max_len ? e : max_len;
  uint32_t m = 0;
  for (int d = 1; d < dmax; ++d) {
    const int j = MAX_SPAN - d;
    const bool empty = ss[(e - 1) * MAX_SPAN + j + 1] == ss[(e - 1) * MAX_SPAN + j];
    m |= (empty && k1_unk_dead(ss, e, d, dmax)) ? 1u << (d - 1) : 0u;
  }
  return m;
}
// a placement word (K1_TBITS / K1_DBITS)
__host__ __device__ inline uint32_t k1_place_word(int64_t t, int off, uint32_t dead) {
  return (uint32_t)t | ((uint32_t)off << K1_TBITS) | (dead << K1_DBITS);
}
// k1_candidates and k1_dead_mask of one end position in one pass (the host
// schedule: the count when a sentence reaches the position, the mask kept
// for its placement word)
__host__ __device__ inline int k1_candidates_dead(const int32_t* ss, int e, int max_len, uint32_t* dead) {
  const int dmax = e < max_len ? e : max_len;
  const int32_t* r = ss + (e - 1) * MAX_SPAN;
  int x = 0;
  uint32_t m = 0;
  for (int j = 0; j < MAX_SPAN; ++j) {
    const int c = r[j + 1] - r[j];
    const int d = MAX_SPAN - j;
    if (c != 0) {
      x += c;
    } else if (d <= dmax) {
      if (d < dmax && k1_unk_dead(ss, e, d, dmax)) m |= 1u << (d - 1);
      else x += 1;
    }
  }
  *dead = m;
  return x;
}
// candidates of a sentence at end position e (1 <= e <= n) from its span
// table `ss` (8 slots per position): every slot's nodes, and one implicit
// Unknown for an empty slot within max_len that is not statically dead
__host__ __device__ inline int k1_candidates(const int32_t* ss, int e, int max_len) {
  const int dmax = e < max_len ? e : max_len;
  int x = 0;
  for (int j = 0; j < MAX_SPAN; ++j) {
    const int c = ss[(e - 1) * MAX_SPAN + j + 1] - ss[(e - 1) * MAX_SPAN + j];
    const int d = MAX_SPAN - j;
    x += c != 0 ? c : (d <= dmax && !k1_unk_dead(ss, e, d, dmax)) ? 1 : 0;
  }
  return x;
}

// The macro-steps of one wave.  Its sentences advance through their end
// positions independently: at every macro-step they are taken in priority
// order -- more end positions left first, then the lower index -- while their
// candidates at their next end position fit the lanes left (64 per
// macro-step); a position with more than 64 candidates (dense lattices) takes
// ceil(run / 64) macro-steps alone when its sentence has the priority.  Every
// macro-step takes the first sentence in priority order, so the schedule
// ends.  On the bench lattices W = 8 sentences fill 0.92 of the lanes, against
// 0.82 for the lockstep schedule of W = 6 (every sentence of a wave at the
// same end position; rounds 1-4), 11 % fewer macro-steps.
//   cnt sentences of lengths nw[]; run_at(w, e): candidates of sentence w at
//   end position e; emit(t, w, e, off, run): sentence w's end position e on
//   lanes [off, off + run) of macro-steps t, t + 1, ... laid end to end.
// Returns the wave's macro-steps.  The host count (lt_batch_create), the
// device count (lt_k1_sched_count) and the fill (lt_k1_sched) all run this.
template <class RunAt, class Emit>
__host__ __device__ inline int64_t k1_schedule(int cnt, const int (&nw)[K1_W], RunAt run_at, Emit emit) {
  int rem[K1_W], run[K1_W], pos[K1_W];
  for (int w = 0; w < K1_W; ++w) {
    rem[w] = w < cnt ? nw[w] : 0;
    pos[w] = 1;
    run[w] = rem[w] > 0 ? run_at(w, 1) : 0;
  }
  int64_t t = 0;
  for (;;) {
    int rank[K1_W];
    for (int w = 0; w < K1_W; ++w) {
      int r = 0;
      for (int v = 0; v < K1_W; ++v)
        r += (rem[v] > 0 && (rem[v] > rem[w] || (rem[v] == rem[w] && v < w))) ? 1 : 0;
      rank[w] = r;
    }
    uint32_t take = 0;
    int room = 64, steps = 1;
    for (int r = 0; r < K1_W && room > 0; ++r)
      for (int w = 0; w < K1_W; ++w) {
        if (rem[w] == 0 || rank[w] != r) continue;
        if (run[w] > 64) {
          if (r == 0) {                         // a dense position, alone
            take = 1u << w;
            steps = (run[w] + 63) >> 6;
            emit(t, w, pos[w], 0, run[w]);
            room = 0;
          }
        } else if (run[w] <= room) {
          take |= 1u << w;
          emit(t, w, pos[w], 64 - room, run[w]);
          room -= run[w];
        }
      }
    if (take == 0) return t;
    t += steps;
    for (int w = 0; w < K1_W; ++w)
      if ((take >> w) & 1u) {
        ++pos[w];
        --rem[w];
        run[w] = rem[w] > 0 ? run_at(w, pos[w]) : 0;
      }
  }
}
hipError_t launch_k1_sched_count(const DecodeParams& p, int64_t* steps, hipStream_t st);
hipError_t launch_k1_sched_fill(const DecodeParams& p, const int64_t* wave_off, uint32_t* sched, hipStream_t st,
                                hipEvent_t e0 = nullptr, hipEvent_t e1 = nullptr);

}  // namespace lt
