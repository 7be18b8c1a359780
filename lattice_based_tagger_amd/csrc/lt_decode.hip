// lt_decode.hip -- batched lattice beam decoder for gfx950 (MI355X).
//
// Restates, one sentence per lane group, the reference decoder
//   beam_search            lattice_tagger/beam/beam.py:5-61
//   Beam.append            beam.py:83-86  (stable sort by -score, keep k)
//   Sequence.add           beam.py:112-116
// scored by the lowered composite
//   BeamScoreFunctions     beam/score_funcs.py:50-54 (ordered sum)
//   SimpleTrigramFeatureScore.score  score_funcs.py:137-144
//   trigram_encoder        features/feature.py:76-121
//
// Kernels, chosen per beam size by launch_decode:
//  * lt_viterbi_pk<W>  -- beam_size 1 (default W = 6).  W sentences share a
//    wave in lockstep: the candidates of their current end positions are
//    packed onto the 64 lanes by prefix sums, each lane scores one
//    candidate, a segmented DPP argmax per sentence picks the winner
//    (lowest generation index on ties), and the next position's node records
//    are staged while the current one is probed.
//  * lt_beam_hw<KT,G>  -- beam_size 2..8.  64/G sentences per wave in G-lane
//    groups (G = 16 for k <= 3, 32 above); expansions enumerated in the
//    reference's generation order (begin ascending, hypothesis rank,
//    candidate order), scored one per lane, ranked by counting within the
//    group (Python's stable sort), the top k written to the ring.
//  * lt_beam_pk<KT>    -- beam_size 9..256 (KT = 16 .. 256): one sentence per
//    wave, the same enumeration and rank counting over several scoring
//    rounds (beams above 64: the running list, winners and matures in
//    64-lane chunks).
// All: the frontier (beams of the last 9 end positions) lives in LDS as a
// ring whose entries cache the fields of the hypothesis' last two nodes;
// trigram classes 4/5/6 arrive pre-resolved per node, class 3 (tag, tag)
// comes from a dense LDS table where the kernel stages one, the other
// classes are probed in a two-choice cuckoo table -- all probes of an expansion issued together as buffer loads, an
// unneeded probe gets an out-of-range offset (returns 0, touches no memory)
// instead of a branch.  Present coefficients are summed in numpy's pairwise
// order.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <math.h>
#include "lt_common.h"
#include "lt_internal.h"

using namespace lt;

namespace {

constexpr uint32_t INV = 0xFFFFFFFFu;

// A decode launch: its stream and the events recorded with its dispatch.
struct Launch {
  hipStream_t st;
  hipEvent_t e0, e1;
};
constexpr uint32_t OOB = 0x80000000u;   // >= every buffer's num_records (host-checked)

typedef __amdgpu_buffer_rsrc_t rsrc_t;
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ rsrc_t make_rsrc(const void* ptr, uint64_t bytes) {
  const uint32_t nr = bytes >= 0x80000000ull ? 0x7FFFFFFFu : (uint32_t)bytes;
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(ptr), (short)0, (int)nr, 0x00020000);
}
// make_rsrc for a resource used inside a loop: its base and size pass
// through an empty asm, so the compiler cannot re-derive them from the kernel
// argument.  The argument load is merged with its neighbours (one 16-dword
// s_load of the result pointers).  Under SGPR pressure that tuple is spilled
// and restored whole, 16 v_readlane, at every use.  Opaque, the base and the
// size are three SGPRs of their own.  (lt_beam_hw's backpointer store:
// k=5 4.099 -> 4.057 ms, k=2 2.120 -> 2.091 ms, profiles/r05/ab_bp_opaque/.)
__device__ __forceinline__ rsrc_t make_rsrc_own(const void* ptr, uint64_t bytes) {
  uint64_t base = (uint64_t)(uintptr_t)ptr;
  uint32_t nr = bytes >= 0x80000000ull ? 0x7FFFFFFFu : (uint32_t)bytes;
  asm volatile("" : "+s"(base), "+s"(nr));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(uintptr_t)base, (short)0, (int)nr, 0x00020000);
}
__device__ __forceinline__ u32x4 ld128(rsrc_t r, uint32_t off) {
  return __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
}

struct Bufs {
  rsrc_t node, tab;
  rsrc_t esc;             // class-4/6 pairs of PX_ESC records, by record index
  const F46* pairs;       // class-4/6 pair table of the records (NodeRec)
};

__device__ __forceinline__ Bufs make_bufs(const DecodeParams& p) {
  Bufs B;
  B.node = make_rsrc(p.nodes, (uint64_t)p.n_nodes * sizeof(NodeRec));
  const uint64_t slot_bytes = p.narrow ? sizeof(SlotN) : sizeof(SlotW);
  B.tab = make_rsrc(p.table, (uint64_t)p.slots * slot_bytes);
  B.pairs = p.pairs;
  B.esc = make_rsrc(p.esc, p.esc ? (uint64_t)p.n_nodes * sizeof(F46) : 0u);
  return B;
}

// Candidate node fields (gn = global node index; INV -> zeros, no access).
struct Cand {
  uint32_t word, morph, tag, mask;
  double pre, f4, f5, f6;
};

__device__ __forceinline__ double dbl(uint32_t lo, uint32_t hi) {
  return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}
// The fields of a 32 B record (two 16 B chunks); f4 / f6 -0.0 until
// set_pair.
__device__ __forceinline__ Cand rec_cand(uint4 q0, uint4 q1) {
  Cand c;
  c.word = q0.x; c.morph = q0.y; c.tag = q0.z; c.mask = q0.w;
  c.pre = dbl(q1.x, q1.y); c.f5 = dbl(q1.z, q1.w);
  c.f4 = -0.0; c.f6 = -0.0;
  return c;
}
// The record's class-4/6 pair: entry rec_px(mask) of the table `tab` (the
// batch's pair table, or a block's LDS copy of it), or the escape array's
// entry of record gn.
__device__ __forceinline__ void set_pair(Cand& c, const F46* tab, const Bufs& B, uint32_t gn) {
  const uint32_t px = rec_px(c.mask);
  const F46 f = tab[px == PX_ESC ? 0u : px];
  c.f4 = f.f4; c.f6 = f.f6;
  if (px == PX_ESC && gn != INV) {                 // rare: a batch whose table overflowed
    // (a buffer load: a plain one would be merged with the table read above
    // into one flat load of a selected address)
    const u32x4 e = ld128(B.esc, gn * (uint32_t)sizeof(F46));
    c.f4 = dbl(e.x, e.y); c.f6 = dbl(e.z, e.w);
  }
}
__device__ __forceinline__ Cand load_cand(const Bufs& B, uint32_t gn) {
  const uint32_t o = gn == INV ? OOB : gn * (uint32_t)sizeof(NodeRec);
  const u32x4 a = ld128(B.node, o);
  const u32x4 b = ld128(B.node, o == OOB ? OOB : o + 16u);
  Cand c = rec_cand(make_uint4(a.x, a.y, a.z, a.w), make_uint4(b.x, b.y, b.z, b.w));
  set_pair(c, B.pairs, B, gn);
  return c;
}

// The implicit Unknown of span length d (lattice_decode.h n_unk; beam.py:36-38:
// the synthesised Word of a span with no dictionary candidate).  Its pair is
// always in the table (the library enters the Unknowns' pairs first).
__device__ __forceinline__ Cand unk_cand(const DecodeParams& p, int d) {
  const NodeRec r = p.unk[d - 1];
  const F46 f = p.pairs[rec_px(r.mask)];
  return Cand{r.word, r.morph, r.tag, r.mask, r.pre, f.f4, r.f5, f.f6};
}
// Local node `node` of the sentence whose first node is nbase, or (UNK_LOCAL)
// the implicit Unknown of span length d.
__device__ __forceinline__ Cand cand_at(const Bufs& B, const DecodeParams& p, uint32_t nbase, uint32_t node, int d) {
  return node == UNK_LOCAL ? unk_cand(p, d) : load_cand(B, nbase + node);
}
// The tuned kernels' copy of the 8 implicit-Unknown records in LDS (record
// d - 1 at chunks 2(d - 1), 2(d - 1) + 1, as a staged record; zeros without
// implicit Unknowns).  Every thread of the block calls it before any early
// exit.
__device__ __forceinline__ void stage_unk(const DecodeParams& p, uint4* ul) {
  if (threadIdx.x < REC_CHUNKS * MAX_SPAN)
    ul[threadIdx.x] = p.n_unk ? reinterpret_cast<const uint4*>(p.unk)[threadIdx.x] : make_uint4(0u, 0u, 0u, 0u);
  __syncthreads();
}
// A 32 B record staged in LDS (two chunks at q[0], q[step]) with its pair
__device__ __forceinline__ Cand cand_lds32(const uint4* q, int step, const F46* tab, const Bufs& B, uint32_t gn) {
  Cand c = rec_cand(q[0], q[step]);
  set_pair(c, tab, B, gn);
  return c;
}

typedef __attribute__((address_space(3))) void lds_void;

// Hypothesis fields the scorer needs (from the LDS frontier).
struct Hyp {
  double score, f6;
  uint32_t jword, jmorph, jtag, jmask, iword, imorph, imask, depth;
  uint32_t jnode;                 // local index of wj (edge terms)
  uint32_t inode;                 // local index of wi (further trigram terms; general kernels)
};

template <int G>
__device__ __forceinline__ unsigned long long group_sum(unsigned long long v) {
#pragma unroll
  for (int off = G / 2; off >= 1; off >>= 1) v += __shfl_xor(v, off, G);
  return v;
}

// Sum of the present features in numpy's pairwise order
// (numpy pairwise_sum: n < 8 -> ((0.0 + a0) + a1) + ...;
//  8 <= n < 16 -> r = a[0:8], ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)), then + a8...).
__device__ __forceinline__ double numpy_sum9(const double (&v)[9], const bool (&pr)[9]) {
  int m = 0;
#pragma unroll
  for (int q = 0; q < 9; ++q) m += pr[q] ? 1 : 0;
  if (m < 8) {
    double s = 0.0;
#pragma unroll
    for (int q = 0; q < 9; ++q) s = pr[q] ? s + v[q] : s;
    return s;
  }
  // m is 8 or 9: at most one feature is missing; compact in order.
  int miss = 9;
#pragma unroll
  for (int q = 8; q >= 0; --q) if (!pr[q]) miss = q;
  double r[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) r[q] = (q < miss) ? v[q] : v[q + 1];
  double s = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  if (m == 9) s += v[8];
  return s;
}

// LDS-resident parts of the model a block stages at its start.
struct Aux {
  const double* d3;       // dense class-3 table (D3_DIM^2) or nullptr
  uint32_t d3off;
  NarrowHash hk;          // narrow table slot hash
};

// Slot access per table format.  A slot's key carries the overflow flag of
// the "primary first" cuckoo table (lt_common.h); query keys never do.
template <bool NARROW>
struct Tab;

template <>
struct Tab<true> {
  static constexpr uint32_t SZ = sizeof(SlotN);
  struct S { uint64_t key; double coef; };
  typedef uint64_t Key;
  __device__ static Key key(uint32_t a, uint32_t b, uint32_t c, uint32_t cls) {
    return narrow_key(a, b, c, cls);
  }
  __device__ static bool hit(const S& s, Key k) { return (s.key & ~FLAG_N) == k; }
  __device__ static bool hit_plain(const S& s, Key k) { return s.key == k; }
  __device__ static bool flagged(const S& s) { return (s.key & FLAG_N) != 0; }
  __device__ static uint32_t slot1(const Aux& x, uint32_t a, uint32_t b, uint32_t c, uint32_t cls,
                                   uint32_t, uint32_t slots) {
    return narrow_slot1(x.hk, a, b, c, cls, slots);
  }
  __device__ static uint32_t slot2(const Aux& x, uint32_t a, uint32_t b, uint32_t c, uint32_t cls,
                                   uint32_t, uint32_t slots) {
    return narrow_slot2(x.hk, a, b, c, cls, slots);
  }
  // an arbitrary value (no instruction): lanes that load nothing keep a
  // defined slot, so a check can select on it instead of branching.  An empty
  // asm defines the registers (__builtin_nondeterministic_value is a frozen
  // poison, which the compiler materialised as zeros: two 64-bit moves per
  // probed class and macro-step in the k=1 kernel)
  __device__ static void arbitrary(S& s) {
    asm volatile("" : "=v"(s.key), "=v"(s.coef));
  }
  __device__ static S load(rsrc_t t, uint32_t off) {
    const u32x4 v = ld128(t, off);
    S s;
    s.key = ((uint64_t)v.y << 32) | v.x;
    s.coef = __builtin_bit_cast(double, (u32x2){v.z, v.w});
    return s;
  }
};

template <>
struct Tab<false> {
  static constexpr uint32_t SZ = sizeof(SlotW);
  struct S { uint32_t a, b, c, cls1; double coef; };
  struct Key { uint32_t a, b, c, cls1; };
  __device__ static Key key(uint32_t a, uint32_t b, uint32_t c, uint32_t cls) {
    return Key{a, b, c, cls + 1};
  }
  __device__ static bool hit(const S& s, Key k) {
    return (s.cls1 & ~FLAG_W) == k.cls1 && s.a == k.a && s.b == k.b && s.c == k.c;
  }
  __device__ static bool flagged(const S& s) { return (s.cls1 & FLAG_W) != 0; }
  __device__ static bool hit_plain(const S& s, Key k) {
    return s.cls1 == k.cls1 && s.a == k.a && s.b == k.b && s.c == k.c;
  }
  __device__ static uint32_t slot1(const Aux&, uint32_t a, uint32_t b, uint32_t c, uint32_t cls,
                                   uint32_t seed, uint32_t slots) {
    return wide_slot1(a, b, c, cls, seed, slots);
  }
  __device__ static uint32_t slot2(const Aux&, uint32_t a, uint32_t b, uint32_t c, uint32_t cls,
                                   uint32_t seed, uint32_t slots) {
    return wide_slot2(a, b, c, cls, seed, slots);
  }
  __device__ static void arbitrary(S& s) {
    s.a = __builtin_nondeterministic_value(s.a);
    s.b = __builtin_nondeterministic_value(s.b);
    s.c = __builtin_nondeterministic_value(s.c);
    s.cls1 = __builtin_nondeterministic_value(s.cls1);
    s.coef = __builtin_nondeterministic_value(s.coef);
  }
  __device__ static S load(rsrc_t t, uint32_t off) {
    const u32x4 k = ld128(t, off);
    const u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(t, off == OOB ? OOB : off + 16u, 0, 0);
    S s;
    s.a = k.x; s.b = k.y; s.c = k.z; s.cls1 = k.w;
    s.coef = __builtin_bit_cast(double, v);
    return s;
  }
};

struct Counts {
  unsigned long long exp = 0, tup = 0, probe = 0, load = 0;
};

// Trigram score of appending candidate c after hypothesis h
// (score_funcs.py:137-144 over feature.py:76-121), in two phases so that
// other loads can be issued while the probes are in flight:
//   probe_issue   -- keys, hashes, the primary slot load of each needed probe
//                    (BOTH: the secondary slot too)
//   probe_second  -- primary hit, or a miss at a flagged slot: load the
//                    secondary (nothing to load under BOTH)
//   probe_finish  -- secondary hits, numpy-order sum
// BOTH: load the secondary slot together with the primary (one memory round
// trip, two loads per probe) instead of only at flagged primaries (about 1.2
// loads per probe, a second round trip).  The beam kernels, whose waits are
// ordered around register-prefetched records, take BOTH.
template <bool NARROW, bool BOTH = false>
struct Probe {
  typename Tab<NARROW>::S s1[6];          // the primary slots (valid where needed)
  typename Tab<NARROW>::S s2[6];          // the secondary slots (valid where loaded)
  uint32_t need;                           // bit q: probe q is needed
  uint32_t gneed;                          // bit q: probe q went to the global table
  uint32_t lpres;                          // bit q: resolved from LDS and present (coef in s1)
  uint32_t hit1;                           // bit q: found at the primary slot
  uint32_t need2;                          // bit q: secondary slot loaded
};

// Key components of probe q for (h, c); recomputed where needed instead of
// being kept live across the memory wait.
struct Keys {
  uint32_t a[6], b[6], c[6];
};
__device__ __forceinline__ Keys make_keys(const Hyp& h, const Cand& c, bool use_j8) {
  Keys K;
  // class 0 (wj.word, wk.word, tk) .. class 3 (tj, tk), class 7 (wi, wj, wk)
  K.a[0] = h.jword; K.b[0] = c.word; K.c[0] = c.tag;
  K.a[1] = h.jword; K.b[1] = c.tag;  K.c[1] = 0;
  K.a[2] = h.jtag;  K.b[2] = c.word; K.c[2] = c.tag;
  K.a[3] = h.jtag;  K.b[3] = c.tag;  K.c[3] = 0;
  K.a[4] = h.iword; K.b[4] = h.jword; K.c[4] = c.word;
  // class 8: (wj.morph0 | wi.morph0, wk.morph0) (feature.py:113-119)
  K.a[5] = use_j8 ? h.jmorph : h.imorph; K.b[5] = c.morph; K.c[5] = 0;
  return K;
}

constexpr uint32_t PCLS[6] = {0, 1, 2, 3, 7, 8};

__device__ __forceinline__ bool use_j8_of(const Hyp& h, const Cand& c) {
  return (c.mask & F_CTX) && (h.jmask & F_CTX);
}

// Which of the six probed classes can be present: the candidate's DK bits
// and the hypothesis' bits (exact pre-filter on the component-slot bits, the
// device mask layout of lt_common.h); an absent class issues no load.
__device__ __forceinline__ uint32_t probe_need(const Hyp& h, const Cand& c) {
  return c.mask & hyp_probe_bits(h.jmask, h.imask, (h.imask & F_WI) != 0) & DQ_ALL;
}

// The dense class-3 table in LDS: row d3_index(t_j), column d3_index(t_k)
// XOR the row, so that lanes reading one t_k under different t_j (a common
// tag after several hypotheses' tags) hit different banks (ds_read_b64:
// bank pair = element index mod 32, which unswizzled was the column alone).
#ifndef LT_D3_SWIZZLE
#define LT_D3_SWIZZLE 1                 // 0: the unswizzled layout (A/B builds)
#endif
// (off: the table's bit window, d3_window -- d3_index of its multiplier as
// one bit-field extract)
__device__ __forceinline__ uint32_t d3_lds(uint32_t jtag, uint32_t ktag, uint32_t off) {
  const uint32_t r = __builtin_amdgcn_ubfe(jtag, off, D3_BITS);
  return (r << D3_BITS) | (__builtin_amdgcn_ubfe(ktag, off, D3_BITS) ^ (LT_D3_SWIZZLE ? r : 0u));
}
// copy the host-layout table src (row-major) into the swizzled LDS layout
__device__ __forceinline__ void d3_stage(const double* __restrict__ src, double* dst) {
  for (int i = threadIdx.x; i < D3_DIM * D3_DIM; i += blockDim.x) {
    const int r = i >> D3_BITS, c = i & (D3_DIM - 1);
    dst[(r << D3_BITS) | (c ^ (LT_D3_SWIZZLE ? r : 0))] = src[i];
  }
}

// Stage the LDS parts of the model (all threads of the block, before any
// early exit): the dense class-3 table when the model has one.
template <bool NARROW>
__device__ __forceinline__ Aux stage_aux(const DecodeParams& p, double* d3l) {
  Aux a;
  if (p.d3) d3_stage(p.d3, d3l);
  if (p.d3) __syncthreads();
  a.d3 = p.d3 ? d3l : nullptr;
  a.d3off = p.d3off;
  a.hk = p.hk;
  return a;
}

// coff: the class offset of a further trigram scorer (LT_XTRI_CLASS_STRIDE *
// t, wide tables; 0 otherwise)
template <bool NARROW, bool BOTH>
__device__ __forceinline__ void probe_issue(Probe<NARROW, BOTH>& P, const Bufs& B, uint32_t slots,
                                            uint32_t seed, const Hyp& h, const Cand& c,
                                            uint32_t need, const Aux& aux, uint32_t coff = 0) {
  using T = Tab<NARROW>;
  P.need = need;
  const Keys K = make_keys(h, c, use_j8_of(h, c));
  uint32_t gneed = need, lpres = 0;
  // class 3 from the dense LDS table (the first scorer's class-3 keys only)
  if (aux.d3 && coff == 0 && ((need >> 3) & 1u)) {
    const double v = aux.d3[d3_lds(h.jtag, c.tag, aux.d3off)];
    P.s1[3].coef = v;
    gneed &= ~8u;
    lpres |= (__builtin_bit_cast(uint64_t, v) != D3_ABSENT) ? 8u : 0u;
  }
  P.gneed = gneed;
  P.lpres = lpres;
#pragma unroll
  for (int q = 0; q < 6; ++q) {
    // exec-masked, not out-of-range: an OOB lane still costs the address
    // unit (TA) a slot, an inactive lane does not
    // (slots stay undefined when not needed; probe_finish reads them only
    // under the same predicate)
    if ((gneed >> q) & 1u) {
      P.s1[q] = T::load(B.tab, T::slot1(aux, K.a[q], K.b[q], K.c[q], PCLS[q] + coff, seed, slots) * T::SZ);
      if constexpr (BOTH)
        P.s2[q] = T::load(B.tab, T::slot2(aux, K.a[q], K.b[q], K.c[q], PCLS[q] + coff, seed, slots) * T::SZ);
    }
  }
}

template <bool NARROW, bool BOTH>
__device__ __forceinline__ void probe_second(Probe<NARROW, BOTH>& P, const Bufs& B, uint32_t slots,
                                             uint32_t seed, const Aux& aux, const Hyp& h,
                                             const Cand& c, uint32_t coff = 0) {
  using T = Tab<NARROW>;
  // keys recomputed from (h, c), which stay live anyway
  const Keys K = make_keys(h, c, use_j8_of(h, c));
  uint32_t hit1 = 0, need2 = 0;
  if constexpr (!BOTH) {
#pragma unroll
    for (int q = 0; q < 6; ++q) {
      if ((P.gneed >> q) & 1u) {
        const typename T::Key key = T::key(K.a[q], K.b[q], K.c[q], PCLS[q] + coff);
        if (T::hit(P.s1[q], key)) {
          hit1 |= 1u << q;
        } else if (T::flagged(P.s1[q])) {         // all second loads before any wait
          need2 |= 1u << q;
          P.s2[q] = T::load(B.tab, T::slot2(aux, K.a[q], K.b[q], K.c[q], PCLS[q] + coff, seed, slots) * T::SZ);
        }
      }
    }
  }
  P.hit1 = hit1;
  P.need2 = need2;
}

template <bool NARROW, bool COUNT, bool BOTH>
__device__ __forceinline__ double probe_finish(const Probe<NARROW, BOTH>& P, const Hyp& h,
                                               const Cand& c, Counts& cnt, uint32_t coff = 0) {
  using T = Tab<NARROW>;
  const uint32_t jm = h.jmask, km = c.mask, im = h.imask;
  const uint32_t hit1 = P.hit1, need2 = P.need2;
  const Keys K = make_keys(h, c, use_j8_of(h, c));
  bool pr6[6];
  double cf[6];
#pragma unroll
  for (int q = 0; q < 6; ++q) {
    pr6[q] = false;
    cf[q] = 0.0;
    if constexpr (BOTH) {                       // both slots loaded: branch-free selects
      if ((P.gneed >> q) & 1u) {
        const typename T::Key key = T::key(K.a[q], K.b[q], K.c[q], PCLS[q] + coff);
        // BOTH kernels probe the flag-free copy of the table (lt_model.d_plain)
        const bool m1 = T::hit_plain(P.s1[q], key);
        const bool m2 = T::hit_plain(P.s2[q], key);
        pr6[q] = m1 || m2;
        cf[q] = m1 ? P.s1[q].coef : P.s2[q].coef;
      } else if ((P.lpres >> q) & 1u) {
        pr6[q] = true;
        cf[q] = P.s1[q].coef;
      }
    } else if ((hit1 >> q) & 1u) {
      pr6[q] = true;
      cf[q] = P.s1[q].coef;
    } else if ((need2 >> q) & 1u) {
      const typename T::Key key = T::key(K.a[q], K.b[q], K.c[q], PCLS[q] + coff);
      pr6[q] = T::hit(P.s2[q], key);
      cf[q] = P.s2[q].coef;
    } else if ((P.lpres >> q) & 1u) {          // resolved from LDS
      pr6[q] = true;
      cf[q] = P.s1[q].coef;
    }
  }
  double v[9];
  bool pr[9];
#pragma unroll
  for (int q = 0; q < 4; ++q) { v[q] = cf[q]; pr[q] = pr6[q]; }
  v[4] = c.f4; pr[4] = (km & F_HAS4) != 0;
  v[5] = c.f5; pr[5] = (km & F_HAS5) != 0;
  v[6] = h.f6; pr[6] = (jm & F_HAS6) != 0;
  v[7] = cf[4]; pr[7] = pr6[4];
  v[8] = cf[5]; pr[8] = pr6[5];
  if (COUNT) {
    const bool use_j8 = use_j8_of(h, c);
    const bool has_i = (im & F_WI) != 0;
    const bool use_i8 = (km & F_CTX) && !(jm & F_CTX) && has_i && (im & F_CTX);
    cnt.tup += 6 + ((jm & F_UNK) ? 1 : 0) + (has_i ? 1 : 0) + ((use_j8 || use_i8) ? 1 : 0);
    cnt.probe += __builtin_popcount(P.need);
    cnt.load += BOTH ? 2 * __builtin_popcount(P.gneed) : __builtin_popcount(P.gneed) + __builtin_popcount(need2);
  }
  return numpy_sum9(v, pr);
}

template <bool NARROW, bool COUNT>
__device__ __forceinline__ double trigram(const Bufs& B, uint32_t slots, uint32_t seed,
                                          const Hyp& h, const Cand& c, Counts& cnt,
                                          const Aux& aux, uint32_t coff = 0) {
  Probe<NARROW> P;
  probe_issue<NARROW>(P, B, slots, seed, h, c, probe_need(h, c), aux, coff);
  probe_second<NARROW>(P, B, slots, seed, aux, h, c, coff);
  return probe_finish<NARROW, COUNT, false>(P, h, c, cnt, coff);
}

// Every trigram term of an expansion (general kernels): tris[0] the first
// scorer's (node records), tris[t] scorer t's (lattice_decode.h n_xtri: its
// node masks and class 4/5/6 coefficients from the xtri arrays, its keys'
// classes + LT_XTRI_CLASS_STRIDE * t).  Global node indices: gk of the
// candidate, gj / gi of the hypothesis' last two words (has_i: wi exists).
// Implicit Unknowns never occur with further scorers (lt_batch_create).
template <bool NARROW, bool COUNT>
__device__ __forceinline__ void trigram_terms(const DecodeParams& p, const Bufs& B, const Hyp& h, const Cand& c,
                                              uint32_t gk, uint32_t gj, uint32_t gi, Counts& cnt, const Aux& aux,
                                              double* tris) {
  tris[0] = p.has_tri ? trigram<NARROW, COUNT>(B, p.slots, p.seed, h, c, cnt, aux) : 0.0;
  for (int t = 1; t <= p.n_xtri; ++t) {
    const int64_t o = (int64_t)(t - 1) * p.n_nodes;
    Cand ct = c;
    ct.mask = p.xmask[o + gk];
    ct.f4 = p.xf4[o + gk];
    ct.f5 = p.xf5[o + gk];
    Hyp ht = h;
    ht.jmask = p.xmask[o + gj];
    ht.f6 = p.xf6[o + gj];
    ht.imask = (h.imask & F_WI) ? (p.xmask[o + gi] | F_WI) : 0u;
    tris[t] = trigram<NARROW, COUNT>(B, p.slots, p.seed, ht, ct, cnt, aux, (uint32_t)(XTRI_CLASS_STRIDE * t));
  }
}

// inc = ((0 + pre...) + tri) + post...   (score_funcs.py:50-54).  With edge
// terms (p.n_edge > 0) the terms after `pre` follow the composite's order
// (term_kinds): the trigram, node-local rows, and edge rows -- the value of the
// edge from wj (local node jl) to the candidate gn.  unk_d > 0: the candidate
// is the implicit Unknown of that span length (its post terms from p.unk_post;
// a batch with implicit Unknowns has no edge terms).
// increment() of a composite with several trigram terms (general kernels):
// term kind 0 takes the next of tris[] (constructor order)
__device__ __forceinline__ double increment_x(const DecodeParams& p, const Cand& c, const double* tris,
                                              uint32_t gn, uint32_t jl) {
  double inc = c.pre;
  int nd = 0, ne = 0, nt = 0;
  for (int t = 0; t < p.n_terms; ++t) {
    const uint32_t kind = (uint32_t)(p.term_kinds >> (2 * t)) & 3u;
    double v;
    if (kind == 0) v = tris[nt++];
    else if (kind == 1) v = p.npost[(int64_t)(nd++) * p.n_nodes + gn];
    else v = p.edge_val[(int64_t)(ne++) * p.n_edges + p.edge_base[gn] + jl];
    inc += v;
  }
  return inc;
}

// GEN = false: the composite has no term after the trigram (p.n_post == 0,
// p.n_edge == 0; launch_k picks it), so inc = pre + tri and the kernel keeps
// none of the post / edge arrays or their loops live (round 6: the k=1
// kernel's SGPR spills 43 -> 6, their v_readlane restores out of the loop).
template <bool GEN = true>
__device__ __forceinline__ double increment(const DecodeParams& p, const Cand& c, double tri,
                                            uint32_t gn, uint32_t jl, int unk_d = 0) {
  if constexpr (!GEN) return c.pre + tri;
  if (p.n_edge == 0) {
    double inc = c.pre + tri;
    for (int t = 0; t < p.n_post; ++t)
      inc += unk_d ? p.unk_post[(int64_t)t * p.n_unk + unk_d - 1] : p.npost[(int64_t)t * p.n_nodes + gn];
    return inc;
  }
  double inc = c.pre;
  int nd = 0, ne = 0;
  for (int t = 0; t < p.n_terms; ++t) {
    const uint32_t kind = (uint32_t)(p.term_kinds >> (2 * t)) & 3u;
    double v;
    if (kind == 0) v = tri;
    else if (kind == 1) v = p.npost[(int64_t)(nd++) * p.n_nodes + gn];
    else v = p.edge_val[(int64_t)(ne++) * p.n_edges + p.edge_base[gn] + jl];
    inc += v;
  }
  return inc;
}

// ===========================================================================
// beam_size = 1
// ===========================================================================

// (e - d) mod RING for 1 <= d <= RING - 1 <= e, from em9 = e mod RING: a
// compare and an add instead of a signed division by RING per lane
__device__ __forceinline__ int ring_back(int em9, int d) {
  const int r = em9 - d;
  return r < 0 ? r + RING : r;
}

// Ring entry of the k=1 kernel: the hypothesis (best path ending at one end
// position) reduced to what scoring an expansion of it needs.
struct alignas(16) VEntry {
  double score, f6;             // f6: wj's class-6 coefficient (-0.0 when absent)
  uint32_t jword, jtag, a8, meta;
  uint32_t iword, jmorph, depth, jnode;    // jnode: local index of wj (edge terms)
};
// meta: bits 0-5 the hypothesis' probe bits (hyp_probe_bits), wj's DI_7 /
// DI_8 (bits 13-14, for the next hypothesis), wj's F_UNK / F_CTX / F_HAS6;
// bit 15 (counting builds) wi's F_CTX.  a8: the first component of class 8
// (feature.py:113-119): wj.morph0 when wj's tag is in C, else wi.morph0.
constexpr uint32_t V_META_J = DI_7 | DI_8 | F_UNK | F_CTX | F_HAS6;
constexpr uint32_t V_ICTX = 1u << 15;

// k=1 probe q = 0..5 (classes 0, 1, 2, 3, 7, 8) of appending candidate c to
// the ring entry h: its key components (feature.py:95-119)
struct V1Keys {
  uint32_t a[6], b[6], c[6];
};
__device__ __forceinline__ V1Keys v1_keys(const VEntry& h, const Cand& c) {
  V1Keys K;
  K.a[0] = h.jword; K.b[0] = c.word;  K.c[0] = c.tag;
  K.a[1] = h.jword; K.b[1] = c.tag;   K.c[1] = 0;
  K.a[2] = h.jtag;  K.b[2] = c.word;  K.c[2] = c.tag;
  K.a[3] = h.jtag;  K.b[3] = c.tag;   K.c[3] = 0;
  K.a[4] = h.iword; K.b[4] = h.jword; K.c[4] = c.word;
  K.a[5] = h.a8;    K.b[5] = c.morph; K.c[5] = 0;
  return K;
}

// Exact key match of a slot (the overflow flag ignored), narrow tables as
// two 32-bit halves of c3<<60 | a<<40 | b<<20 | c (v_lshl_or_b32 builds).
template <bool NARROW>
__device__ __forceinline__ bool v1_hit(const typename Tab<NARROW>::S& s, uint32_t a, uint32_t b, uint32_t c,
                                       uint32_t cls) {
  if constexpr (NARROW) {
    const uint32_t lo = (b << 20) | c;
    const uint32_t hi = (cls_code(cls) << 28) | (a << 8) | (b >> 12);
    // (two 32-bit compares: the 64-bit compare of the flag-masked key measured
    // slower here, 0.773 -> 0.781 ms, while it pays in the beams' bm_hit)
    const uint32_t slo = (uint32_t)s.key, shi = (uint32_t)(s.key >> 32) & 0x7FFFFFFFu;
    return (slo == lo) & (shi == hi);
  } else {
    return Tab<false>::hit(s, Tab<false>::key(a, b, c, cls));
  }
}

// One expansion's trigram probes in three phases around the two memory round
// trips: issue the primary slot of every needed probe; check them (hit ->
// coefficient, miss at a flagged slot -> secondary load into the same
// registers); check the secondaries.  cf[q] ends as the coefficient of a
// present feature or -0.0 (the identity of the float64 sum) when absent.
template <bool NARROW>
struct V1Probe {
  typename Tab<NARROW>::S s[6];           // primary slots
  typename Tab<NARROW>::S s2[6];          // secondary slots (where loaded)
  double cf[6];
  uint32_t gneed, need2, pres;
};

// d3tab: the kernel's own LDS copy of the dense class-3 table (used when
// aux.d3 is set) -- passed as the array itself, so that the compiler sees
// that its reads cannot touch the record staging area (an LDS address from
// a register would carry a wait for the record DMA in flight, K1_EARLY_DMA)
template <bool NARROW>
__device__ __forceinline__ void v1_issue(V1Probe<NARROW>& P, const Bufs& B, uint32_t slots, uint32_t seed,
                                         const VEntry& h, const Cand& c, uint32_t need, const Aux& aux,
                                         const double* d3tab) {
  using T = Tab<NARROW>;
  const V1Keys K = v1_keys(h, c);
  uint32_t gneed = need, pres = 0;
  P.cf[3] = -0.0;
  if (aux.d3 && ((need >> 3) & 1u)) {        // class 3 from the dense LDS table
    const double v = d3tab[d3_lds(h.jtag, c.tag, aux.d3off)];
    const bool present = __builtin_bit_cast(uint64_t, v) != D3_ABSENT;
    P.cf[3] = present ? v : -0.0;
    pres = present ? 8u : 0u;
    gneed &= ~8u;
  }
#pragma unroll
  for (int q = 0; q < 6; ++q) {
    T::arbitrary(P.s[q]);
    if ((gneed >> q) & 1u)                    // exec-masked: an idle lane costs the TA nothing
      P.s[q] = T::load(B.tab, T::slot1(aux, K.a[q], K.b[q], K.c[q], PCLS[q], seed, slots) * T::SZ);
  }
  P.gneed = gneed;
  P.pres = pres;
}

template <bool NARROW>
__device__ __forceinline__ void v1_check(V1Probe<NARROW>& P, const Bufs& B, uint32_t slots, uint32_t seed,
                                         const VEntry& h, const Cand& c, const Aux& aux) {
  using T = Tab<NARROW>;
  const V1Keys K = v1_keys(h, c);
  uint32_t need2 = 0, pres = P.pres;
#pragma unroll
  for (int q = 0; q < 6; ++q) {
    if (q == 3 && aux.d3) continue;
    // branch-free: every lane's slot is defined (T::arbitrary)
    const bool n = (P.gneed >> q) & 1u;
    const bool hit = n & v1_hit<NARROW>(P.s[q], K.a[q], K.b[q], K.c[q], PCLS[q]);
    const bool sec = n & !hit & T::flagged(P.s[q]);
    P.cf[q] = hit ? P.s[q].coef : -0.0;
    pres |= hit ? 1u << q : 0u;
    need2 |= sec ? 1u << q : 0u;
  }
  P.need2 = need2;
  P.pres = pres;
}

// The secondary slots of the misses at flagged primaries (fresh registers:
// reusing the primary's would need a copy that waits for the load).
template <bool NARROW>
__device__ __forceinline__ void v1_issue2(V1Probe<NARROW>& P, const Bufs& B, uint32_t slots, uint32_t seed,
                                          const VEntry& h, const Cand& c, const Aux& aux) {
  using T = Tab<NARROW>;
  const V1Keys K = v1_keys(h, c);
#pragma unroll
  for (int q = 0; q < 6; ++q)
    if ((P.need2 >> q) & 1u)
      P.s2[q] = T::load(B.tab, T::slot2(aux, K.a[q], K.b[q], K.c[q], PCLS[q], seed, slots) * T::SZ);
}

template <bool NARROW>
__device__ __forceinline__ void v1_second(V1Probe<NARROW>& P, const VEntry& h, const Cand& c) {
  const V1Keys K = v1_keys(h, c);
#pragma unroll
  for (int q = 0; q < 6; ++q)
    if ((P.need2 >> q) & 1u) {                   // (skipped by the wave when no lane loaded one)
      const bool hit = v1_hit<NARROW>(P.s2[q], K.a[q], K.b[q], K.c[q], PCLS[q]);
      P.cf[q] = hit ? P.s2[q].coef : P.cf[q];
      P.pres |= hit ? 1u << q : 0u;
    }
}

// Trigram score (score_funcs.py:141-144): numpy's pairwise order over the
// present features v = [c0, c1, c2, c3, f4, f5, f6, c7, c8] (H7).  With
// fewer than 8 present it is the left-to-right sum, in which an absent
// feature's -0.0 changes nothing; 8 or 9 present (rare) take numpy_sum9.
__device__ __forceinline__ double v1_sum(const double (&cf)[6], uint32_t pres6, const Cand& c,
                                         const VEntry& h) {
  const uint32_t pres = (pres6 & 0xFu) | ((c.mask >> 14) & 0x30u) | ((h.meta >> 14) & 0x40u) |
                        ((pres6 & 0x30u) << 3);
  const double v[9] = {cf[0], cf[1], cf[2], cf[3], c.f4, c.f5, h.f6, cf[4], cf[5]};
  if (__builtin_popcount(pres) >= 8) {
    // 8 or 9 present: numpy's pairwise block over the first 8 present, then
    // the 9th.  The one absent feature (miss; 9 = none) by a bit scan, the
    // compaction r[q] = v[q + (q >= miss)] by one compare per element.
    const uint32_t miss = (uint32_t)__builtin_ctz(~pres | 0x200u);
    double r[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) r[q] = ((uint32_t)q < miss) ? v[q] : v[q + 1];
    const double s8 = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    return miss == 9u ? s8 + v[8] : s8;
  }
  double t = 0.0;
#pragma unroll
  for (int q = 0; q < 9; ++q) t = t + v[q];
  return t;
}

#ifndef BM_BRANCHY
#define BM_BRANCHY 1                    // per-class checks exec-masked (A/B: 1 is faster at k = 2, 5, 16)
#endif
// The beam kernels' probes: both candidate slots of every needed probe in
// one round trip (the flag-free copy of the table, lt_model.d_plain), checked
// branch-free into cf[q] / pres as v1_check.
template <bool NARROW>
struct BMProbe {
  typename Tab<NARROW>::S s1[6], s2[6];
  double cf3;                              // class 3 from the dense LDS table
  uint32_t gneed, pres3;
};

// INIT: give the slots of lanes that load nothing a (frozen) value -- needed by
// branch-free checks; with exec-masked checks it only shapes register
// allocation: the frozen value is materialised as zeros (two 64-bit moves per
// probed class and round), so only lt_beam_hw with wide keys takes it (it
// spills without it)
template <bool NARROW, bool INIT = !BM_BRANCHY>
__device__ __forceinline__ void bm_issue(BMProbe<NARROW>& P, const Bufs& B, uint32_t slots, uint32_t seed,
                                         const VEntry& h, const Cand& c, uint32_t need, const Aux& aux) {
  using T = Tab<NARROW>;
  const V1Keys K = v1_keys(h, c);
  uint32_t gneed = need;
  P.cf3 = -0.0;
  P.pres3 = 0;
  if (aux.d3 && ((need >> 3) & 1u)) {
    const double v = aux.d3[d3_lds(h.jtag, c.tag, aux.d3off)];
    const bool present = __builtin_bit_cast(uint64_t, v) != D3_ABSENT;
    P.cf3 = present ? v : -0.0;
    P.pres3 = present ? 8u : 0u;
    gneed &= ~8u;
  }
#pragma unroll
  for (int q = 0; q < 6; ++q) {
    if (INIT) {
      T::arbitrary(P.s1[q]);
      T::arbitrary(P.s2[q]);
    }
    if ((gneed >> q) & 1u) {
      P.s1[q] = T::load(B.tab, T::slot1(aux, K.a[q], K.b[q], K.c[q], PCLS[q], seed, slots) * T::SZ);
      P.s2[q] = T::load(B.tab, T::slot2(aux, K.a[q], K.b[q], K.c[q], PCLS[q], seed, slots) * T::SZ);
    }
  }
  P.gneed = gneed;
}

// key match in the flag-free table
template <bool NARROW>
__device__ __forceinline__ bool bm_hit(const typename Tab<NARROW>::S& s, uint32_t a, uint32_t b, uint32_t c,
                                       uint32_t cls) {
  if constexpr (NARROW) {
    const uint32_t lo = (b << 20) | c;
    const uint32_t hi = (cls_code(cls) << 28) | (a << 8) | (b >> 12);
    // one 64-bit compare (was two 32-bit compares and an AND: k=5 4.37 ->
    // 4.28 ms, k=16 12.08 -> 11.98 ms)
    return s.key == (((uint64_t)hi << 32) | lo);
  } else {
    return Tab<false>::hit_plain(s, Tab<false>::key(a, b, c, cls));
  }
}

// The probed classes' coefficients cf[q] (-0.0 when absent) and presence
// bits of one expansion (waits for its slot loads).
template <bool NARROW>
__device__ __forceinline__ void bm_classes(const BMProbe<NARROW>& P, const VEntry& h, const Cand& c, double (&cf)[6],
                                           uint32_t& pres) {
  const V1Keys K = v1_keys(h, c);
  pres = P.pres3;
#pragma unroll
  for (int q = 0; q < 6; ++q) {
    const bool n = (P.gneed >> q) & 1u;
    cf[q] = q == 3 ? P.cf3 : -0.0;
    if (BM_BRANCHY ? n : true) {               // BM_BRANCHY: a class no lane needs is skipped
      const bool m1 = n & bm_hit<NARROW>(P.s1[q], K.a[q], K.b[q], K.c[q], PCLS[q]);
      const bool m2 = n & bm_hit<NARROW>(P.s2[q], K.a[q], K.b[q], K.c[q], PCLS[q]);
      cf[q] = m1 ? P.s1[q].coef : (m2 ? P.s2[q].coef : cf[q]);
      pres |= (m1 | m2) ? 1u << q : 0u;
    }
  }
}

template <bool NARROW>
__device__ __forceinline__ double bm_score(const BMProbe<NARROW>& P, const VEntry& h, const Cand& c) {
  double cf[6];
  uint32_t pres;
  bm_classes<NARROW>(P, h, c, cf, pres);
  return v1_sum(cf, pres, c, h);
}


// Sequence.add into a ring entry (beam.py:112-116): wi = wj, wj = wk
template <bool COUNT>
__device__ __forceinline__ VEntry v_grow(const VEntry& h, const Cand& c, double score, uint32_t cl) {
  VEntry ne;
  ne.score = score; ne.f6 = c.f6;
  ne.jword = c.word; ne.jtag = c.tag; ne.jmorph = c.morph;
  ne.a8 = (c.mask & F_CTX) ? c.morph : h.jmorph;
  ne.meta = hyp_probe_bits(c.mask, h.meta, true) | (c.mask & V_META_J);
  if (COUNT) ne.meta |= (h.meta & F_CTX) ? V_ICTX : 0u;
  ne.iword = h.jword; ne.depth = h.depth + 1; ne.jnode = cl;
  return ne;
}
// beam[0] = [BOS] (beam.py:21-23)
__device__ __forceinline__ VEntry v_bos(const Cand& b0) {
  VEntry e0;
  e0.score = 0.0; e0.f6 = b0.f6;
  e0.jword = b0.word; e0.jtag = b0.tag; e0.jmorph = b0.morph;
  e0.a8 = b0.morph;                          // (used only when BOS's tag is in C)
  e0.meta = hyp_probe_bits(b0.mask, 0u, false) | (b0.mask & V_META_J);
  e0.iword = 0; e0.depth = 0; e0.jnode = 0;
  return e0;
}
// operation counts of one expansion (lt_count_ops)
__device__ __forceinline__ void v_count(Counts& cnt, const VEntry& h, const Cand& c, uint32_t need, uint32_t loads) {
  const bool has_i = h.depth > 0;
  const bool k_ctx = (c.mask & F_CTX) != 0, j_ctx = (h.meta & F_CTX) != 0;
  const bool i_ctx = (h.meta & V_ICTX) != 0;
  ++cnt.exp;
  cnt.tup += 6 + ((h.meta & F_UNK) ? 1 : 0) + (has_i ? 1 : 0) + ((k_ctx && (j_ctx || (has_i && i_ctx))) ? 1 : 0);
  cnt.probe += __builtin_popcount(need);
  cnt.load += loads;
}

// ---------------------------------------------------------------------------
// beam_size = 1, packed lanes.  A wave owns W sentences; the lane schedule
// (k1_schedule) packs the candidates of several sentences' next end positions
// onto the 64 lanes of each macro-step (one contiguous lane segment per
// sentence), the sentences advancing independently, so lanes are not left idle
// by short positions or finished sentences.  Per-sentence argmax: LDS max over
// an order-preserving 64-bit score key, then LDS min over the generation index
// among the lanes holding the maximum -- exactly the reference's (score desc,
// generation asc) order.
// ---------------------------------------------------------------------------
#ifndef PK_WAVES
#define PK_WAVES 4
#endif
#ifndef PK_BPL
// end positions whose backpointer stays in LDS: 96 fills a CU's LDS with two
// 8-wave blocks of W = 8 (81,904 B per block; round 2 at W = 6 and 4-wave
// blocks: window 64: 1.010-1.016 ms, 76: 1.000, 87: 0.987-0.995 ms)
#define PK_BPL 96
#endif
#ifndef PK_WPB
#define PK_WPB 8                        // (one dense class-3 table and pair table per 8 waves)
#endif
#ifndef PK_PAIR_MAX
#define PK_PAIR_MAX 0                   // 1: lane pairs compare in registers before the LDS max (A/B)
#endif
#ifndef PK_DMA_AUX
#define PK_DMA_AUX 2                    // k=1 record DMA nontemporal (streamed once): 0.771 -> 0.766 ms
#endif
#ifndef HW_SPRE
#define HW_SPRE 1
#endif
#ifndef PK_RANK_U
#define PK_RANK_U 1                     // lt_beam_pk single-round ranking by list position (list_rank_u)
#endif
#ifndef HW_D3_MAXKT
#define HW_D3_MAXKT 4                   // lt_beam_hw: the dense class-3 table in LDS up to this KT
#endif
#ifndef HW_RANK_U
#define HW_RANK_U 0                     // lt_beam_hw single-entry ranking by list_rank_u (A/B: k=5 3.75 -> 3.78 ms, k=2 1.87 -> 1.92, k=3 2.53 -> 2.49; off)
#endif
#ifndef HW_LIVE
// lt_beam_hw: 1 = an implicit Unknown slot past b_min expands only the
// hypotheses not ending in Unknown (live-rank lists, cnt_live); 0 = the slot
// expands all of beam[b] unless none survives (cnt_any), the per-expansion
// skip taking the rest.  A/B (profiles/r06/ab_hw_live/): 0 is faster, k=5
// 3.82 -> 3.75 ms, k=2 1.90 -> 1.88, k=8 4.69 -> 4.60
#define HW_LIVE 0
#endif
#ifndef HW_STAGE
#define HW_STAGE 32                     // lt_beam_hw: records staged per wave and position
#endif
#ifndef PK_SPRE
#define PK_SPRE 1
#endif
// waves per block of lt_viterbi_pk: wide keys (more registers, 3 waves per
// SIMD) in 4-wave blocks, three of which fit a CU
template <bool NARROW>
constexpr int k1_wpb() { return NARROW ? PK_WPB : 4; }
// (k=1 lane-schedule entries: K1_* in lt_internal.h)

// Stage the records of the wave's packed candidates (lane l's node gn, INV =
// none) into wave_planes: the 2 x 64 chunks of 16 B form one stream in lane
// order, and DMA instruction pl has lane t fetch chunk 64*pl + t -- part
// (c mod 2) of lane (c / 2)'s record -- so consecutive lanes read consecutive
// bytes of a sentence's node block.  Lane l's record ends up at chunks 2l,
// 2l+1.
__device__ __forceinline__ void dma_packed(const Bufs& B, uint32_t gn, uint4* wave_planes, int lane) {
  static_assert(REC_CHUNKS == 2, "two 16 B chunks per record");
  uint32_t nj[2];
#pragma unroll
  for (int pl = 0; pl < 2; ++pl)                 // both permutes first: one LDS round trip
    nj[pl] = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(((uint32_t)(64 * pl + lane) >> 1) << 2), (int)gn);
#pragma unroll
  for (int pl = 0; pl < 2; ++pl) {
    const uint32_t o = nj[pl] != INV ? nj[pl] * (uint32_t)sizeof(NodeRec) + (uint32_t)(lane & 1) * 16u : OOB;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(B.node, (lds_void*)(wave_planes + pl * 64), 16, o, 0, 0, PK_DMA_AUX);
  }
}

// K1_DMA_DIRECT: DMA instruction pl has lane t fetch part pl of its own
// record (chunks node*32 + 16 pl), so lane t's record lands at chunks t and
// 64 + t: the staged-record reads are 16 B apart per lane (no bank
// conflict) and no permute is needed; each instruction touches twice the
// lines of the packed stream (dma_packed), the pair of them the same lines.
#ifndef K1_DMA_DIRECT
#define K1_DMA_DIRECT 0
#endif
__device__ __forceinline__ void dma_direct(const Bufs& B, uint32_t gn, uint4* wave_planes) {
#pragma unroll
  for (int pl = 0; pl < 2; ++pl) {
    const uint32_t o = gn != INV ? gn * (uint32_t)sizeof(NodeRec) + (uint32_t)pl * 16u : OOB;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(B.node, (lds_void*)(wave_planes + pl * 64), 16, o, 0, 0, PK_DMA_AUX);
  }
}

__device__ __forceinline__ unsigned long long ord_key(double sc) {
  const uint64_t b = __builtin_bit_cast(uint64_t, sc + 0.0);      // -0.0 -> +0.0
  return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}

// Phase stamps of the k=1 macro-step (diagnostic builds with -DPK_PHASES only;
// tools/gpu_phases.sh): s_memtime with its own lgkmcnt(0), fenced by
// scheduling barriers, summed per wave into counters[4..].
#ifdef PK_PHASES
__device__ __forceinline__ unsigned long long pk_stamp() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) :: "memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
#define PK_STAMP(i) do { const unsigned long long t_ = pk_stamp(); ph[i] += t_ - tprev; tprev = t_; } while (0)
#else
#define PK_STAMP(i) do { } while (0)
#endif

// the k=1 kernel's result stores: written once, read by the D2H copy --
// nontemporal with K1_OUT_NT (A/B), so that they do not displace table lines
// cache policy of the decoders' HBM backpointer stores (written once, read
// back once by the backtrace; 2: nontemporal, A/B)
#ifndef BM_BP_AUX
#define BM_BP_AUX 0
#endif
#ifndef K1_OUT_NT
#define K1_OUT_NT 0
#endif
template <typename T>
__device__ __forceinline__ void k1_out(T* a, T v) {
  if constexpr (K1_OUT_NT != 0) __builtin_nontemporal_store(v, a);
  else *a = v;
}

// Non-returning LDS atomics as inline asm.  The compiler puts a vmcnt(0) in
// front of every LDS atomic while a buffer->LDS DMA may be in flight (it does
// not for plain LDS reads and writes of other arrays): at k=1 that made the
// per-sentence argmax wait for the next macro-step's record DMA every step.
// (LDS operations of a wave complete in order, so a later read sees the
// update; the compiler's lgkmcnt waits for its own reads stay correct, since
// they count only operations younger than the read it waits for.)
__device__ __forceinline__ uint32_t lds_addr(const void* a) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)a;
}
__device__ __forceinline__ __attribute__((unused)) void lds_max_u64(unsigned long long* a, unsigned long long v) {
  asm volatile("ds_max_u64 %0, %1" ::"v"(lds_addr(a)), "v"(v) : "memory");
}
__device__ __forceinline__ __attribute__((unused)) void lds_min_u32(uint32_t* a, uint32_t v) {
  asm volatile("ds_min_u32 %0, %1" ::"v"(lds_addr(a)), "v"(v) : "memory");
}
#ifndef K1_ASM_ATOMIC
#define K1_ASM_ATOMIC 1                 // k=1 argmax atomics as inline asm (no DMA wait in front of them)
#endif
#ifndef K1_EARLY_DMA
// k=1: 1 = the next macro-step's records DMA'd right after this step's
// candidate record is read from the staging area (schedule entries loaded two
// steps ahead), in flight with the primary probes.  Measured slower (0.539 vs
// 0.526 ms, profiles/r06/ab_k1_dma/): VMEM completes in order, so the
// primary-slot wait then also waits for the record DMA's longer HBM latency;
// after the hit checks (0), the DMA overlaps the checks, the secondaries, the
// sum and -- with K1_ASM_ATOMIC -- the argmax.
#define K1_EARLY_DMA 0
#endif

// per-sentence static record (LDS)
struct alignas(16) SentRec {
  uint32_t n, bp_lo, bp_hi, nbase;
};

// ---------------------------------------------------------------------------
// The k=1 lane schedule (a static function of the lattice shapes, filled on
// the device once per batch by lt_k1_sched into memory sized by the host,
// lt_batch_create): lt_internal.h k1_schedule -- the sentences of a wave
// advance through their end positions independently, each macro-step packing
// the candidates of the positions it takes.  Entry of lane l: K1_*.
// ---------------------------------------------------------------------------
// The W sentences of wave schedule `wave` (wave-uniform): lengths, first
// nodes, span-table offsets, first placement (cum_n: one per end position).
template <int W>
__device__ __forceinline__ void k1_wave_sents(const DecodeParams& p, int slot0, int (&nS)[W], uint32_t (&nbS)[W],
                                              int64_t (&soS)[W], int64_t (&cnS)[W]) {
#pragma unroll
  for (int w = 0; w < W; ++w) {
    const bool v = slot0 + w < p.n_sent;
    const int sid = v ? p.order[slot0 + w] : 0;
    nS[w] = v ? p.sent_n[sid] : 0;
    nbS[w] = v ? (uint32_t)p.node_off[sid] : 0u;
    soS[w] = v ? p.span_off[sid] : 0;
    cnS[w] = v ? p.cum_n[sid] : 0;
  }
}

#ifndef K1_FILL_AUX
// cache policy of the fill's row stores: nontemporal (the rows are read once,
// by the decode; written through, they displaced table lines the decode right
// after needed -- fresh-batch step 0.752-0.771 -> 0.698-0.736 ms,
// profiles/r06/ab_fill_nt/)
#define K1_FILL_AUX 2
#endif
constexpr int K1_NCAP = 192;                    // end positions per sentence whose counts the schedule kernel keeps in LDS
constexpr int K1_RT = 16;                       // schedule rows per LDS tile of the fill
constexpr int K1_RT_FUSED = 12;                 // ... of the fill inside the beam-1 decode (its ring)

// The schedule of a wave on the device, k1_schedule's rule with a lane per
// sentence (lane w < W: sentence w's positions left, next end position, its
// candidate count): priority ranks by one readlane and compare per sentence,
// the greedy pass over the ranks on wave-uniform values.  The candidate counts
// of end positions e <= K1_NCAP are counted lane-parallel into LDS first,
// those of later positions (long sentences) from the span table when needed.
// Every (sentence, end position) gets its placement -- first macro-step |
// first lane << K1_TBITS -- at p.k1_place[cum_n + e - 1].  Returns the
// macro-steps.  (The host does the same at lt_batch_create, k1_schedule; this
// runs for a batch that gets its schedule at its first beam-1 decode.)
template <int W>
__device__ __forceinline__ int64_t k1_lane_schedule(const DecodeParams& p, const int (&nS)[W], const int64_t (&soS)[W],
                                                    const int64_t (&cnS)[W], uint16_t (*runs)[K1_NCAP]) {
  static_assert(W == K1_W && W <= 8, "one schedule layout, the priority key holds the sentence in 3 bits");
  const int lane = (int)threadIdx.x;
  // the (sentence, position) pairs flattened, four per lane in flight
  int pre[W + 1];
  pre[0] = 0;
#pragma unroll
  for (int w = 0; w < W; ++w) pre[w + 1] = pre[w] + min(nS[w], K1_NCAP);
  constexpr int U = 4;
  for (int i0 = 0; i0 < pre[W]; i0 += 64 * U) {
    int c[U], wu[U], eu[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = i0 + 64 * u + lane;
      int w = 0;
#pragma unroll
      for (int v = 1; v < W; ++v) w += i >= pre[v] ? 1 : 0;
      int64_t so = soS[0];
      int pw = 0;
#pragma unroll
      for (int v = 1; v < W; ++v)
        if (w == v) { so = soS[v]; pw = pre[v]; }
      wu[u] = w;
      eu[u] = i - pw + 1;
      c[u] = i < pre[W] ? k1_candidates(p.span_start + so, eu[u], p.max_len) : 0;
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (i0 + 64 * u + lane < pre[W]) runs[wu[u]][eu[u] - 1] = (uint16_t)min(c[u], 65535);
  }
  __builtin_amdgcn_wave_barrier();               // (one wave: its LDS operations complete in order)
  asm volatile("" ::: "memory");
  // lane w's sentence
  int n = 0;
  int64_t so = 0, cn = 0;
#pragma unroll
  for (int w = 0; w < W; ++w)
    if (lane == w) { n = nS[w]; so = soS[w]; cn = cnS[w]; }
  auto run_at = [&](int e) -> int {              // (e <= n; 65535: a count too large for the LDS copy)
    const int x = e <= K1_NCAP ? (int)runs[lane < W ? lane : 0][e - 1] : 65535;
    return x < 65535 ? x : k1_candidates(p.span_start + so, e, p.max_len);
  };
  int rem = n, pos = 1;
  int run = rem > 0 ? run_at(1) : 0;
  int64_t t = 0;
  for (;;) {
    const int key = rem > 0 ? rem * 8 + (7 - lane) : -1;   // priority: positions left, then the lower index
    int rank = 0;
#pragma unroll
    for (int v = 0; v < W; ++v) rank += __builtin_amdgcn_readlane(key, v) > key ? 1 : 0;
    if (__builtin_amdgcn_ballot_w64(key >= 0) == 0ull) return t;
    uint32_t take = 0;
    int room = 64, steps = 1, off = 0;
#pragma unroll
    for (int r = 0; r < W && room > 0; ++r) {
      const unsigned long long m = __builtin_amdgcn_ballot_w64(key >= 0 && rank == r);
      if (m == 0ull) break;                      // (ranks 0 .. live - 1)
      const int w = __builtin_ctzll(m);
      const int rw = __builtin_amdgcn_readlane(run, w);
      if (rw > 64) {
        if (r == 0) {                            // a dense position, alone
          take = 1u << w;
          steps = (rw + 63) >> 6;
          room = 0;
        }
      } else if (rw <= room) {
        take |= 1u << w;
        off = lane == w ? 64 - room : off;
        room -= rw;
      }
    }
    const bool mine = lane < W && ((take >> lane) & 1u);   // (a shift by 32 or more is not a zero)
    if (mine) p.k1_place[cn + pos - 1] = k1_place_word(t, off, k1_dead_mask(p.span_start + so, pos, p.max_len));
    t += steps;
    if (mine) {
      ++pos;
      --rem;
      run = rem > 0 ? run_at(pos) : 0;
    }
  }
}

// The macro-steps and placements of every wave schedule of a piece, for a
// batch that gets its schedule at its first beam-1 decode (lt_batch_create
// counts and places on the host for a beam-1 batch).
template <int W>
__global__ void __launch_bounds__(64) lt_k1_sched_count(DecodeParams p, int64_t* steps) {
  __shared__ uint16_t runs[W][K1_NCAP];
  const int wave = blockIdx.x;
  const int slot0 = wave * W;
  if (slot0 >= p.n_sent) return;
  int nS[W];
  uint32_t nbS[W];
  int64_t soS[W], cnS[W];
  k1_wave_sents<W>(p, slot0, nS, nbS, soS, cnS);
  const int64_t total = k1_lane_schedule<W>(p, nS, soS, cnS, runs);
  if (threadIdx.x == 0) steps[wave] = total;
}

// The schedule fill: one wave per wave schedule, its rows built K1_RT at a
// time in an LDS tile -- idle entries, then the entries of the positions
// placed in it (lanes over (sentence, position) pairs: the placement and the
// position's span starts loaded together) -- and copied out by coalesced
// 256 B stores.  A sentence's positions are placed in increasing macro-steps,
// so a cursor per sentence (its first position not yet complete) bounds the
// positions a tile can hold: at most one per macro-step, RT.  One wave (lane
// = threadIdx.x & 63) fills wave schedule `wave`; tile: RT x 64 words of LDS,
// curs: W words (the standalone fill lt_k1_sched, or the beam-1 decode of a
// batch without its schedule, p.k1_fill).
template <int W, int RT>
__device__ __forceinline__ void k1_fill_wave(const DecodeParams& p, int wave, const int64_t* wave_off,
                                             uint32_t* sched, uint32_t (*tile)[64], int* curs) {
  const int lane = (int)(threadIdx.x & 63);
  const int slot0 = wave * W;
  int nS[W];
  uint32_t nbS[W];
  int64_t soS[W], cnS[W];
  k1_wave_sents<W>(p, slot0, nS, nbS, soS, cnS);
  if (lane < W) curs[lane] = 1;
  // the wave's rows as a buffer (stores past its rows are dropped)
  const int64_t w0 = wave_off[wave];
  const int nrow = (int)(wave_off[wave + 1] - w0);
  const rsrc_t out = make_rsrc(sched + w0 * 64, (uint64_t)nrow * 256u);
  // lane (sentence g, slot j8) of an 8 x 8 pass over (sentence, position) pairs
  const int g = lane >> 3, j8 = lane & 7;
  int ng = 0;
  uint32_t nbg = 0;
  int64_t sog = 0, cng = 0;
#pragma unroll
  for (int w = 0; w < W; ++w)
    if (g == w) { ng = nS[w]; nbg = nbS[w]; sog = soS[w]; cng = cnS[w]; }
  const uint32_t wb = (uint32_t)g << 26;
  static_assert(RT <= 16, "a tile's positions of a sentence: at most RT, lanes cover 16");
  for (int R0 = 0; R0 < nrow; R0 += RT) {
#pragma unroll
    for (int r = 0; r < RT; ++r) tile[r][lane] = K1_IDLE;
    const int cur = g < W ? curs[g] : 1;
    // positions cur + j8 and cur + 8 + j8: placements and span starts together
    // ss: the position's span starts; dm: its dead implicit Unknowns
    // (k1_dead_mask, from the placement word)
    int ss[2][MAX_SPAN + 1], t0[2], q0[2];
    uint32_t dm[2];
    bool in[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int e = cur + 8 * h + j8;
      in[h] = g < W && e <= ng;
      const uint32_t v = in[h] ? p.k1_place[cng + e - 1] : 0u;
      const int32_t* const src = p.span_start + sog + (int64_t)(max(e, 1) - 1) * MAX_SPAN;
#pragma unroll
      for (int jj = 0; jj <= MAX_SPAN; ++jj) ss[h][jj] = in[h] ? src[jj] : 0;
      t0[h] = (int)(v & ((1u << K1_TBITS) - 1u));
      in[h] = in[h] && t0[h] < R0 + RT;
      q0[h] = (int)((v >> K1_TBITS) & 63u);
      dm[h] = v >> K1_DBITS;
    }
    int done = 0;                                // positions of sentence g completed in this tile
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int e = cur + 8 * h + j8;
      int q = q0[h];
      int last = t0[h];                          // the position's last row
      if (in[h]) {
        const int dmax = min(e, p.max_len);
        int cnt[MAX_SPAN];
        uint32_t e0v[MAX_SPAN];
        int run = 0;
#pragma unroll
        for (int jj = 0; jj < MAX_SPAN; ++jj) {
          const int a = ss[h][jj];
          const int d = MAX_SPAN - jj;
          const bool unk = a == ss[h][jj + 1] && d <= dmax;
          const bool dead = d < MAX_SPAN && ((dm[h] >> (d - 1)) & 1u);   // (k1_unk_dead)
          cnt[jj] = dead ? 0 : unk ? 1 : ss[h][jj + 1] - a;
          // entry i: node nbg + a + i, or the slot's implicit Unknown (d - 1 = 7 - jj)
          e0v[jj] = (unk ? (K1_UNK | (uint32_t)(MAX_SPAN - 1 - jj)) : nbg + (uint32_t)a) | wb;
          run += cnt[jj];
        }
        if (run <= 64) {
          // the usual position: one segment of its first row (t0 is in this tile)
          uint32_t* const rowp = &tile[t0[h] - R0][0];
#pragma unroll
          for (int jj = 0; jj < MAX_SPAN; ++jj) {
#pragma unroll 1
            for (int i = 0; i < cnt[jj]; ++i) rowp[q + i] = (e0v[jj] + (uint32_t)i) | K1_FIRST;
            q += cnt[jj];
          }
        } else {
          // a dense position: rows t0, t0 + 1, ..., of which this tile's
#pragma unroll
          for (int jj = 0; jj < MAX_SPAN; ++jj) {
#pragma unroll 1
            for (int i = 0; i < cnt[jj]; ++i, ++q) {
              const int row = t0[h] + (q >> 6) - R0;
              if (row >= 0 && row < RT) tile[row][q & 63] = (e0v[jj] + (uint32_t)i) | (q < 64 ? K1_FIRST : 0u);
            }
          }
        }
        last = t0[h] + ((q - 1) >> 6);
      }
      const bool complete = in[h] && last < R0 + RT;
      const unsigned long long cm = __builtin_amdgcn_ballot_w64(complete);
      done += __builtin_popcount((uint32_t)(cm >> (g * 8)) & 0xFFu);
    }
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
    if (j8 == 0 && g < W) curs[g] = cur + done;
    const int nr = min(RT, nrow - R0);
#pragma unroll
    for (int r = 0; r < RT; ++r)
      if (r < nr) __builtin_amdgcn_raw_buffer_store_b32(tile[r][lane], out, (uint32_t)lane * 4u, (R0 + r) * 256,
                                                        K1_FILL_AUX);
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
  }
}

template <int W>
__global__ void __launch_bounds__(64) lt_k1_sched(DecodeParams p, const int64_t* wave_off, uint32_t* sched) {
  __shared__ uint32_t tile[K1_RT][64];
  __shared__ int curs[W];
  if ((int)blockIdx.x * W >= p.n_sent) return;
  k1_fill_wave<W, K1_RT>(p, (int)blockIdx.x, wave_off, sched, tile, curs);
}

template <int W, bool NARROW, bool COUNT, bool GEN = true>
__global__ void __launch_bounds__(64 * k1_wpb<NARROW>(), (NARROW && W <= 8) ? PK_WAVES : 3)
lt_viterbi_pk(DecodeParams p) {
  constexpr int BPL = PK_BPL;                   // end positions whose backpointer stays in LDS
  constexpr int P_WPB = k1_wpb<NARROW>();
  __shared__ VEntry ring[P_WPB][W][RING];
  __shared__ uint32_t bpl[P_WPB][W][BPL];
  __shared__ uint4 stg[P_WPB][REC_CHUNKS * 64];
  __shared__ SentRec srec[P_WPB][W];
  __shared__ unsigned long long amax[P_WPB][W];  // the sentence's argmax at its current end position
  __shared__ uint32_t amin[P_WPB][W];
  __shared__ uint32_t sep[P_WPB][W];            // sentence w's current end position e | (e % RING) << 24
  __shared__ double d3l[D3_DIM * D3_DIM];
  __shared__ uint4 ucan[REC_CHUNKS * MAX_SPAN]; // the implicit Unknowns' records (as staged ones)
  __shared__ F46 pxl[MAX_PAIRS];                // the batch's class-4/6 pair table
  // the occupancy the launch bounds ask for must fit a CU's 160 KiB of LDS
  // (4 SIMDs x PK_WAVES waves in blocks of P_WPB waves); the LDS window PK_BPL
  // is sized to the last byte of it
  static_assert(!(NARROW && W <= 8) ||
                    (sizeof(ring) + sizeof(bpl) + sizeof(stg) + sizeof(srec) + sizeof(amax) + sizeof(amin) +
                     sizeof(sep) + sizeof(d3l) + sizeof(ucan) + sizeof(pxl)) * (4 * PK_WAVES / P_WPB) <= 160u * 1024u,
                "lt_viterbi_pk LDS exceeds the CU's share for PK_WAVES waves per SIMD");
  for (int i = (int)threadIdx.x; i < p.n_pairs; i += 64 * P_WPB) pxl[i] = p.pairs[i];
  stage_unk(p, ucan);                           // (its barrier publishes pxl too)
  const Aux aux = stage_aux<NARROW>(p, d3l);

  const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int lane = (int)(threadIdx.x & 63);
  const int wave = blockIdx.x * P_WPB + wv;
  const int slot0 = wave * W;
  if (slot0 >= p.n_sent) return;                // whole wave
  if (p.k1_fill) {
    // a batch's first beam-1 decode (fresh schedule): the wave fills its own
    // rows first (the standalone fill's work, k1_fill_wave), over LDS the
    // decode initialises only after it -- the wave's ring as the row tile,
    // its sep words as the cursors -- so the fill's load latency overlaps the
    // other waves' decoding instead of running as a kernel of its own
    static_assert(sizeof(ring[0]) >= K1_RT_FUSED * 64 * 4, "the fused fill's tile fits the wave's ring");
    k1_fill_wave<W, K1_RT_FUSED>(p, wave, p.wave_off, p.k1_fill, reinterpret_cast<uint32_t (*)[64]>(&ring[wv][0][0]),
                                 reinterpret_cast<int*>(&sep[wv][0]));
    __builtin_amdgcn_s_waitcnt(0);               // the rows are stored before the first schedule load
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
  }
  const Bufs B = make_bufs(p);
  const uint32_t slots = p.slots, seed = p.seed;
  const int has_tri = p.has_tri;
  const int bstride = p.bp_stride;
  // backpointers past the LDS window (long sentences) as a buffer: every
  // macro-step issues exactly one store instruction (non-writer lanes: an
  // out-of-range offset, dropped), so the wait at the top of the next step
  // leaves it in flight
  const rsrc_t bpr = make_rsrc(p.bp, (uint64_t)p.bp_bytes);
  uint4* const wst = stg[wv];
  VEntry (*const R)[RING] = ring[wv];
  Counts cnt;
#ifdef PK_PHASES
  unsigned long long ph[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const unsigned long long tstart = pk_stamp();
  unsigned long long tprev = tstart;
  unsigned long long nsteps_done = 0;
#endif

  // lane w < W owns sentence w of the wave
  const bool own = lane < W && slot0 + lane < p.n_sent;
  const int sid = own ? p.order[slot0 + lane] : 0;
  const int nw = own ? p.sent_n[sid] : 0;
  const uint32_t nbase = own ? (uint32_t)p.node_off[sid] : 0u;
  if (own) {
    const int64_t bo = p.bp_off[sid];
    SentRec r;
    r.n = (uint32_t)nw; r.bp_lo = (uint32_t)bo; r.bp_hi = (uint32_t)(bo >> 32);
    r.nbase = nbase;
    srec[wv][lane] = r;
    R[lane][0] = v_bos(load_cand(B, nbase));  // beam[0] = [BOS] (beam.py:21-23)
  }
  if (lane < W) {
    amax[wv][lane] = 0ull;
    amin[wv][lane] = INV;
    sep[wv][lane] = 0u;
  }
  // this wave's macro-steps in the lane schedule
  const int64_t soff = p.wave_off[wave];
  const int nsteps = (int)(p.wave_off[wave + 1] - soff);
  const uint32_t* const sch = p.sched + soff * 64 + lane;
  // the node whose record a lane stages (INV: idle, or an implicit Unknown)
  auto node_of = [](uint32_t ent) -> uint32_t {
    return ((ent & K1_NODE) == K1_NODE || (ent & K1_UNK)) ? INV : (ent & K1_NODE);
  };
  uint32_t ent = nsteps > 0 ? sch[0] : K1_IDLE;   // (a wave of empty sentences has no step)
#if K1_EARLY_DMA
  uint32_t ent1 = nsteps > 1 ? sch[64] : K1_IDLE;   // the next step's (its records go out early in this one)
#endif
#if K1_DMA_DIRECT
  dma_direct(B, node_of(ent), wst);
#else
  dma_packed(B, node_of(ent), wst, lane);
#endif
  __builtin_amdgcn_raw_buffer_store_b32(0u, bpr, OOB, 0, 0);      // the invariant's first store
  __builtin_amdgcn_wave_barrier();

  for (int t = 0; t < nsteps; ++t) {
    PK_STAMP(0);                                 // [0] loop bookkeeping of the previous step
    // vmcnt(1): staged records, this step's schedule entry (VMEM operations
    // retire in order; the one younger operation is the previous step's
    // backpointer store)
    __builtin_amdgcn_s_waitcnt(0x0F71);
    PK_STAMP(1);                                 // [1] wait for the staged records
#if K1_EARLY_DMA
    // the schedule entry two macro-steps ahead: arrives under this step's probes
    const uint32_t ent2 = t + 2 < nsteps ? sch[(int64_t)(t + 2) * 64] : K1_IDLE;
#else
    // the next macro-step's schedule entry: arrives under this step's probes
    const uint32_t ent1 = t + 1 < nsteps ? sch[(int64_t)(t + 1) * 64] : K1_IDLE;
#endif
    const uint32_t gn0 = node_of(ent);
    const bool imp = (ent & K1_UNK) != 0;        // an implicit Unknown (its record from ucan)
    const bool act = gn0 != INV || imp;
    const int msr = (int)((ent >> 26) & 7u);     // (0 for an idle lane)
    // the lane's sentence's end position: it moves to the next one at the
    // first macro-step of that position (every lane of the segment writes the
    // same value; a wave's LDS operations complete in order), which also
    // clears the sentence's argmax words for it -- long before this step's
    // argmax, and after every LDS access of the previous position's steps
    const bool first = (ent & K1_FIRST) != 0;
    const uint32_t sp0 = sep[wv][msr];
    int e = (int)(sp0 & 0xFFFFFFu), em9 = (int)(sp0 >> 24);
    if (first) {
      ++e;
      em9 = em9 == RING - 1 ? 0 : em9 + 1;
      sep[wv][msr] = (uint32_t)e | ((uint32_t)em9 << 24);
      amax[wv][msr] = 0ull;
      amin[wv][msr] = INV;
    }
    const int dmax = min(e, p.max_len);
    // this lane's candidate: its staged record, or the implicit Unknown's
#if K1_DMA_DIRECT
    const Cand cur = cand_lds32(imp ? ucan + 2u * (ent & 7u) : wst + lane, imp ? 1 : 64, pxl, B, imp ? INV : gn0);
#else
    const Cand cur = cand_lds32(imp ? ucan + 2u * (ent & 7u) : wst + 2 * lane, 1, pxl, B, imp ? INV : gn0);
#endif
#if K1_EARLY_DMA
    // the staging area is read: the next macro-step's records go out now, in
    // flight with this step's ring reads and primary probes (no later LDS
    // access of the step touches the staging area, so the compiler adds no
    // wait for the DMA before them; the argmax atomics are asm, K1_ASM_ATOMIC)
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_waitcnt(0xC07F);         // lgkmcnt(0): cur is out of the staging area
#if K1_DMA_DIRECT
    dma_direct(B, node_of(ent1), wst);
#else
    dma_packed(B, node_of(ent1), wst, lane);
#endif
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("" ::: "memory");
#endif
    const int d0 = (int)((cur.mask & D_MASK) >> D_SHIFT) + 1;
    int bm0 = em9 - d0;
    bm0 += bm0 < 0 ? RING : 0;
    const VEntry h0 = R[msr][act ? bm0 : 0];
    const bool skip0 = !act || ((h0.meta & F_UNK) && (cur.mask & F_UNK) && (d0 < dmax));   // beam.py:43-45

    V1Probe<NARROW> P;
    const uint32_t need = (!skip0 && has_tri) ? (cur.mask & h0.meta & DQ_ALL) : 0u;
    v1_issue<NARROW>(P, B, slots, seed, h0, cur, need, aux, d3l);
#ifdef PK_PHASES
    PK_STAMP(2);                                 // [2] records/ring reads, primary issue
    __builtin_amdgcn_s_waitcnt(0x0F70);
    PK_STAMP(3);                                 // [3] wait for the primary slots
#endif
    // primary slots back: hits; the next macro-step's records DMA'd, then the
    // secondary loads of misses at flagged slots (their wait covers the DMA
    // too: VMEM completes in order).  Issued here, after the primary-slot
    // wait, the DMA's HBM latency overlaps the checks, the secondaries, the
    // sum and the argmax (K1_EARLY_DMA, K1_ASM_ATOMIC).
    const VEntry h1 = R[msr][act ? bm0 : 0];
    v1_check<NARROW>(P, B, slots, seed, h1, cur, aux);
#if !K1_EARLY_DMA
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_waitcnt(0xC07F);         // lgkmcnt(0): cur is out of the staging area
#if K1_DMA_DIRECT
    dma_direct(B, node_of(ent1), wst);
#else
    dma_packed(B, node_of(ent1), wst, lane);
#endif
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("" ::: "memory");
#endif
    v1_issue2<NARROW>(P, B, slots, seed, h1, cur, aux);   // secondaries (K1_EARLY_DMA: the DMA is older)
#ifdef PK_PHASES
    PK_STAMP(4);                                 // [4] hit checks, record DMA issue, secondary issue
    __builtin_amdgcn_s_waitcnt(0x0F70);         // vmcnt(0)
    PK_STAMP(5);                                 // [5] wait for the secondary slots and the DMA
#endif
    double best_s = -INFINITY;
    if (!skip0) {
      v1_second<NARROW>(P, h1, cur);
      const double tri = has_tri ? v1_sum(P.cf, P.pres, cur, h1) : 0.0;
      if (COUNT) v_count(cnt, h1, cur, need, __builtin_popcount(P.gneed) + __builtin_popcount(P.need2));
      best_s = h1.score + increment<GEN>(p, cur, tri, gn0, h1.jnode, imp ? d0 : 0);   // beam.py:115
    }

    // per-sentence argmax over the macro-steps of e (beam.py:112-116): max
    // score key, then the min schedule position among the maxima -- the
    // schedule lists a sentence's candidates of one end position in
    // generation order over consecutive macro-steps, so the smallest position
    // (t * 64 + lane) is the first generated.  A wave's LDS operations
    // complete in order, so each read sees the updates issued before it.  A
    // step that raises a sentence's maximum discards the earlier steps'
    // minimum (it belonged to a smaller key); ties with an earlier step keep
    // it (earlier steps hold smaller positions).
    PK_STAMP(6);                                 // [6] numpy-order sum, increment
    const uint32_t gk = (uint32_t)t * 64u + (uint32_t)lane;
#if PK_PAIR_MAX
    // lanes (l, l ^ 1) of one sentence first compare in registers (a DPP
    // quad permute): only the better of the two -- on a tie the lower lane,
    // whose position is smaller -- takes part in the LDS max / min, which
    // halves the lanes contending for one sentence's LDS word
    unsigned long long key = !skip0 ? ord_key(best_s) : 0ull;
    {
      const uint32_t plo = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)key, 0xB1, 0xF, 0xF, false);
      const uint32_t phi = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)(key >> 32), 0xB1, 0xF, 0xF, false);
      const int pmsr = __builtin_amdgcn_mov_dpp(msr, 0xB1, 0xF, 0xF, false);
      const unsigned long long pk = ((unsigned long long)phi << 32) | plo;
      const bool beaten = pmsr == msr && ((lane & 1) ? pk >= key : pk > key);
      key = beaten ? 0ull : key;
    }
#else
    const unsigned long long key = !skip0 ? ord_key(best_s) : 0ull;
#endif
    const unsigned long long mprev = (key && !first) ? amax[wv][msr] : 0ull;
#if K1_ASM_ATOMIC
    if (key) lds_max_u64(&amax[wv][msr], key);
#else
    if (key) __hip_atomic_fetch_max(&amax[wv][msr], key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
#endif
    const unsigned long long mk = key ? amax[wv][msr] : 0ull;
    const bool top = key && key == mk;
    if (top && mk != mprev) amin[wv][msr] = INV;
#if K1_ASM_ATOMIC
    if (top) lds_min_u32(&amin[wv][msr], gk);
#else
    if (top) __hip_atomic_fetch_min(&amin[wv][msr], gk, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
#endif
    const uint32_t mgw = top ? amin[wv][msr] : INV;
    uint32_t bpv = 0u, bpoff = OOB;
    if (top && mgw == gk) {                      // the (step's) winner writes beam[e]
      const SentRec si = srec[wv][msr];
      const uint32_t local = imp ? UNK_LOCAL : gn0 - si.nbase;
      R[msr][em9] = v_grow<COUNT>(h1, cur, best_s, local);   // Sequence.add (beam.py:112-116)
      bpv = bp_pack(local, (uint32_t)d0, 0u);
      if (e < BPL) bpl[wv][msr][e] = bpv;
      else bpoff = (uint32_t)(((((int64_t)si.bp_hi << 32) | si.bp_lo) + (int64_t)e * bstride) * 4);   // past the window
    }
    __builtin_amdgcn_raw_buffer_store_b32(bpv, bpr, bpoff, 0, BM_BP_AUX);
    __builtin_amdgcn_wave_barrier();
    PK_STAMP(7);                                 // [7] argmax (LDS atomics), ring + backpointer write
#ifdef PK_PHASES
    ++nsteps_done;
#endif
    ent = ent1;
#if K1_EARLY_DMA
    ent1 = ent2;
#endif
  }

  // matures = beam[n] + EOS (beam.py:59-61); backtrace, one owner lane per sentence
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  int pdepth = 0;                                // the owner lane's path length
  const int64_t cumn = own ? p.cum_n[sid] : 0;   // its first path-code slot
  if (own) {
    const VEntry& f = R[lane][nw % RING];
    k1_out(&p.out_count[sid], 1);
    k1_out(&p.out_score[sid], f.score + 0.0);
    // (depth <= n on a consistent beam: the unsigned clamp keeps a corrupted
    // entry from sending the stores below out of the sentence's code rows)
    pdepth = (int)min(f.depth, (uint32_t)nw);
    k1_out(&p.out_len[sid], (int32_t)pdepth);
    int32_t* codes = p.out_codes + cumn;
    const uint32_t* bpg = p.bp + p.bp_off[sid];
    int pos = nw;
    // (pos > 0 and the depth bound hold on a consistent beam; they keep a
    // corrupted one from chasing backpointers out of the sentence's rows).
    // Positions past the LDS window first, from HBM; then the window: a loop
    // of LDS reads only, so its stores are never waited for (one loop reading
    // either memory compiles to a flat load, whose wait covers the stores of
    // the step before -- a store round trip per path word)
    int step = pdepth - 1;
    for (; step >= 0 && pos >= BPL; --step) {
      const uint32_t v = bpg[(int64_t)pos * bstride];
      k1_out(&codes[step], path_code(bp_node(v), pos, (int)bp_d(v), MAX_SPAN));
      pos -= (int)bp_d(v);
    }
    const uint32_t* const bw = bpl[wv][lane];
    for (; step >= 0 && pos > 0; --step) {
      const uint32_t v = bw[pos];
      k1_out(&codes[step], path_code(bp_node(v), pos, (int)bp_d(v), MAX_SPAN));
      pos -= (int)bp_d(v);
    }
  }
  // the padded layout (-1 past each path): every sentence's tail by the whole
  // wave, 64 codes per store (instead of one owner lane storing them in turn)
#pragma unroll 1
  for (int w = 0; w < W; ++w) {
    const int nw_w = __builtin_amdgcn_readlane(nw, w), d_w = __builtin_amdgcn_readlane(pdepth, w);
    if (nw_w <= d_w) continue;                   // (uniform)
    const int64_t cb = ((int64_t)__builtin_amdgcn_readlane((int)(cumn >> 32), w) << 32) |
                       (uint32_t)__builtin_amdgcn_readlane((int)cumn, w);
    for (int j = d_w + lane; j < nw_w; j += 64) k1_out(&p.out_codes[cb + j], -1);
  }

  if (COUNT) {
    const unsigned long long ex = group_sum<64>(cnt.exp), tu = group_sum<64>(cnt.tup),
                             pb = group_sum<64>(cnt.probe), ld = group_sum<64>(cnt.load);
    if (lane == 0) {
      atomicAdd(p.counters + 0, ex);
      atomicAdd(p.counters + 1, tu);
      atomicAdd(p.counters + 2, pb);
      atomicAdd(p.counters + 3, ld);
    }
  }
#ifdef PK_PHASES
  const unsigned long long tend = pk_stamp();
  if (lane == 0) {
    for (int i = 0; i < 8; ++i) atomicAdd(p.counters + 4 + i, ph[i]);
    atomicAdd(p.counters + 12, nsteps_done);
    atomicAdd(p.counters + 13, tend - tstart);
    atomicAdd(p.counters + 14, 1ull);
  }
#endif
}

// The beam kernels' per-position word (their LDS ring cnt9): beam[e]'s size
// in the low 16 bits, the number of its hypotheses whose last word is not
// Unknown in the high 16.  An implicit Unknown of span (b, e) with b > b_min
// is skipped after every hypothesis whose last word is Unknown (num_unk
// counts the Unknowns at the tail: beam.py:43-45, Sequence.add :112-113).
// (A position without explicit nodes has none: the k=1 schedule's static
// rule, lt_internal.h k1_unk_dead.)
constexpr int CNT_BEAM = 0xFFFF;
__device__ __forceinline__ int cnt_entry(int beam, int live) { return beam | (live << 16); }
// HW_LIVE=1 (lt_beam_hw, measured slower): such a slot expands only the
// hypotheses not ending in Unknown, enumerated in rank order through the
// ring's live-rank list (LR[b][q] = the rank of the q-th), which keeps the
// generation order of the expansions scored
__device__ __forceinline__ int cnt_live(int cv, bool empty, int d, int dmax) {
  return (empty && d < dmax) ? (cv >> 16) : (cv & CNT_BEAM);
}
// The shipped rule of both beam kernels: such a slot expands all of
// beam[e - d] unless none of it survives -- the per-expansion skip takes the
// rest (the live-rank lookup in the expansion decode cost more than the
// expansions it saved: lt_beam_pk k=16 10.55 -> 10.99 ms, lt_beam_hw k=5
// 3.75 -> 3.82 ms)
__device__ __forceinline__ int cnt_any(int cv, bool empty, int d, int dmax) {
  return (empty && d < dmax && (cv >> 16) == 0) ? 0 : (cv & CNT_BEAM);
}

// ===========================================================================
// beam_size 2..32
// ===========================================================================
// Hypothesis entry of the untuned kernels (general beam, trace)
struct alignas(16) Entry {
  double score, f6;
  uint32_t jword, jmorph, jtag, jmask;
  uint32_t iword, imorph, imask, depth;
  uint32_t jnode, pad0, pad1, pad2;
};

__device__ __forceinline__ Hyp read_entry(const Entry& e) {
  Hyp h;
  h.score = e.score; h.f6 = e.f6;
  h.jword = e.jword; h.jmorph = e.jmorph; h.jtag = e.jtag; h.jmask = e.jmask;
  h.iword = e.iword; h.imorph = e.imorph; h.imask = e.imask; h.depth = e.depth;
  h.jnode = e.jnode;
  h.inode = e.pad0;
  return h;
}

// k=1 kernel: W = 6 sentences per wave (4 and 5 measured within 5 % at
// 8K-32K sentences, slower at 64K)
constexpr int P_W = K1_W;
static_assert(P_W <= 8, "k=1 schedule entries hold the sentence in 3 bits");

template <int W, bool NARROW, bool COUNT, bool GEN = true>
hipError_t launch_pk(const DecodeParams& p, const Launch& L) {
  constexpr int P_WPB = k1_wpb<NARROW>();
  constexpr int SPB = W * P_WPB;
  const int blocks = (p.n_sent + SPB - 1) / SPB;
  if (blocks == 0) return hipSuccess;
  hipExtLaunchKernelGGL((lt_viterbi_pk<W, NARROW, COUNT, GEN>), dim3(blocks), dim3(64 * P_WPB), 0, L.st, L.e0, L.e1, 0, p);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// beam_size 2..32, one sentence per wave.  The expansions of end position e
// (beam.py:27-58: spans j, hypothesis ranks r, candidates i, in generation
// order g) are scored in rounds of 64 lanes; each lane keeps only the
// expansion's order key and index in LDS.  Top-k (stable sort by score, [:k],
// beam.py:85) is exact rank counting: the rank of an entry is the number of
// entries with a larger key, or an equal key and a smaller index.  A position
// with more expansions than a chunk carries its running top-k into the next
// chunk's ranking.  Only the k winners are materialised into beam[e].
// ---------------------------------------------------------------------------
__device__ __forceinline__ double ord_score(unsigned long long k) {
  const uint64_t b = (k >> 63) ? (k & 0x7FFFFFFFFFFFFFFFull) : ~k;
  return __builtin_bit_cast(double, b);
}

// Rank of key ck at list position ci among the 4-aligned list LK[q0, q1): the
// entries with a larger key and the equal keys earlier in the list (lt_beam_hw;
// no generation indices loaded: 2.43 -> 2.36 ms at k=2, 4.70 -> 4.57 at k=5;
// lt_beam_pk's copy of the loop with the indices measured faster there).
// Every list the beam kernels rank holds equal keys in generation order (the
// running top-k in rank order -- key desc, generation asc -- then the chunk's
// entries in generation order, all younger than the running ones), so the
// list position stands in for the generation index of the tie-break.
__device__ __forceinline__ int list_rank(const unsigned long long* LK, int q0, int q1, unsigned long long ck,
                                         int ci) {
  int rank = 0;
#pragma unroll 2
  for (int q = q0; q < q1; q += 4) {
    const ulonglong2 ka = *reinterpret_cast<const ulonglong2*>(&LK[q]);
    const ulonglong2 kb = *reinterpret_cast<const ulonglong2*>(&LK[q + 2]);
    const unsigned long long kq[4] = {ka.x, ka.y, kb.x, kb.y};
#pragma unroll
    for (int u = 0; u < 4; ++u) rank += (kq[u] > ck || (kq[u] == ck && q + u < ci)) ? 1 : 0;
  }
  return rank;
}

// list_rank over wave-uniform bounds for lanes in groups of G (lt_beam_hw):
// the lane's entry sits at list position base + (lane % G), so entry q ties
// before it iff lane % G > q - base -- a lane mask made in scalar registers
// per entry (inverse ballot) instead of a per-lane compare, and a scalar loop
template <int G>
__device__ __forceinline__ int list_rank_u(const unsigned long long* LK, int q0, int q1, unsigned long long ck,
                                           int base) {
  q0 = __builtin_amdgcn_readfirstlane(q0);
  q1 = __builtin_amdgcn_readfirstlane(q1);
  base = __builtin_amdgcn_readfirstlane(base);
  constexpr unsigned long long REP = G == 64 ? 1ull : G == 32 ? 0x0000000100000001ull : 0x0001000100010001ull;
  static_assert(G == 16 || G == 32 || G == 64, "lane groups of 16, 32 or 64");
  int rank = 0;
  for (int q = q0; q < q1; q += 4) {
    const ulonglong2 ka = *reinterpret_cast<const ulonglong2*>(&LK[q]);
    const ulonglong2 kb = *reinterpret_cast<const ulonglong2*>(&LK[q + 2]);
    const unsigned long long kq[4] = {ka.x, ka.y, kb.x, kb.y};
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int x = q + u - base;                // (uniform)
      const unsigned long long gm = G == 64 ? ~0ull : (1ull << G) - 1ull;
      const unsigned long long m = x < 0 ? gm : x >= G - 1 ? 0ull : ((gm << (x + 1)) & gm);
      const bool before = __builtin_amdgcn_inverse_ballot_w64(m * REP);
      rank += (kq[u] > ck || (kq[u] == ck && before)) ? 1 : 0;
    }
  }
  return rank;
}

// Top-k slots TK/TG [0, k) from the list LK[q0, q1) for the entry (ck, cg)
// at list position ci (ck = 0: none).  (A first pass counting only larger
// keys, with a read-back of the slot to catch ties, measured slower than the
// position compare: k=5 4.81 vs 4.57 ms.)
__device__ __forceinline__ void rank_into(const unsigned long long* LK, int q0, int q1, unsigned long long ck,
                                          uint32_t cg, int ci, int k, unsigned long long* TK, uint32_t* TG) {
  const int r = list_rank(LK, q0, q1, ck, ci);
  if (ck != 0ull && r < k) { TK[r] = ck; TG[r] = cg; }
}

// records lt_beam_pk stages per position (the rest take a global load): the
// dictionary candidates of one end position (implicit Unknowns take none), 2.5
// on average in the bench lattices
#ifndef PK_STAGE
#define PK_STAGE 32
#endif
// occupancy floor of lt_beam_pk per beam template: 4 waves per SIMD for the
// narrow-key k = 9..16 kernel (it fits 128 VGPRs without spilling); the
// wide-key (32 B slot) kernels need more registers than that floor leaves --
// under it they spilled 53 (decode) and 101 (COUNT) VGPRs -- and take none
#ifndef PK_WPE
#define PK_WPE(kt, narrow) ((kt) == 16 && (narrow) ? 4 : 1)
#endif
// The beam kernels' backtraces (beam.py:59-61 matures, Sequence.sequences):
// a sentence's backpointer rows -- (n + 1) x bp_stride words in HBM -- are
// first copied into LDS over its ring (dead once the final entries are read)
// by its NL lanes, all loads in flight at once, when they fit CAP words; the
// chain walks are then LDS reads only.  Walking HBM instead costs one memory
// round trip per path word, the code stores of the word before waited for
// behind it.
// A scoring round's candidate past the staged block (a position with more
// than STAGE candidates): a global load in a wave-uniform branch that waits for
// its own loads.  With the loads' wait inside the branch, no load is in flight
// into a register the common path writes; otherwise the compiler's
// write-after-write wait at the next round (a vmcnt(0), VMEM operations counted
// in order) would also wait for the previous position's backpointer store
// before the round's probes are issued.
__device__ __forceinline__ void beam_far(Cand& c, bool far, const Bufs& B, uint32_t gn) {
  if (__builtin_amdgcn_ballot_w64(far) != 0ull) {
    if (far) c = load_cand(B, gn);
    __builtin_amdgcn_s_waitcnt(0x0F70);          // vmcnt(0)
  }
}
// End of a scoring round: every load of the round has been waited for by its
// use (the probes by the checks of the lanes that issued them, the records and
// pairs by the sum), so this wait costs nothing; it tells the compiler so, and
// the next round's first writes to those registers carry no wait.
__device__ __forceinline__ void round_done() { __builtin_amdgcn_s_waitcnt(0x0F70); }

constexpr int BP_STAGE_PER_LANE = 27;
template <int NL, int CAP>
__device__ __forceinline__ void stage_bp_rows(const uint32_t* __restrict__ bpg, int words, uint32_t* lbp, int li) {
  constexpr int PER = (CAP + NL - 1) / NL;
  uint32_t v[PER];
#pragma unroll
  for (int u = 0; u < PER; ++u) {
    const int q = li + u * NL;
    v[u] = q < words ? bpg[q] : 0u;
  }
#pragma unroll
  for (int u = 0; u < PER; ++u) {
    const int q = li + u * NL;
    if (q < words) lbp[q] = v[u];
  }
}
// Mature rank t's path codes (padded with -1 to n unless the caller has)
// from backpointer rows `bps` (LDS or HBM) of row stride `bstride`.
template <typename P, typename C>
__device__ __forceinline__ void walk_path(P bps, int bstride, int n, int depth, int t, int k, C codes,
                                          bool pad = true) {
  int pos = n, rank = t;
  for (int step = min(depth, n) - 1; step >= 0 && pos > 0; --step) {   // (bounds: lt_viterbi_pk)
    const uint32_t v = bps[pos * bstride + rank];
    codes[step] = path_code(bp_node(v), pos, (int)bp_d(v), MAX_SPAN);
    pos -= (int)bp_d(v);
    rank = min((int)bp_rank(v), k - 1);
  }
  if (pad)
    for (int j = depth; j < n; ++j) codes[j] = -1;                      // padded layout
}
// The sentence's padded codes (k x n words) staged in LDS at lco: filled with
// -1 by the NL lanes before the walks, copied out coalesced after them.
template <int NL>
__device__ __forceinline__ void fill_codes(int32_t* lco, int words, int li) {
#pragma unroll 1
  for (int q = li; q < words; q += NL) lco[q] = -1;
}
template <int NL>
__device__ __forceinline__ void copy_codes(int32_t* __restrict__ out, const int32_t* lco, int words, int li) {
#pragma unroll 1
  for (int q = li; q < words; q += NL) out[q] = lco[q];
}

template <int KT, int WPB, bool NARROW, bool COUNT, bool GEN = true>
__global__ void __launch_bounds__(64 * WPB) __attribute__((amdgpu_waves_per_eu(PK_WPE(KT, NARROW), 8)))
lt_beam_pk(DecodeParams p) {
  constexpr int RPC = KT <= 16 ? 2 : 4;         // scoring rounds per chunk
  // beams above 64 (KT = 128, 256): more than one entry per lane in the
  // running list, the winners and the matures -- loops over 64-lane chunks
  constexpr bool BIG = KT > 64;
  constexpr int KV = BIG ? KT / 64 : 1;
  constexpr int CH = 64 * RPC;                  // expansions per chunk
  constexpr int KTP = KT < 4 ? 4 : KT;          // running-list room (multiple of 4)
  constexpr int LN = KTP + CH;                  // ranked list: running top-k + chunk
  static_assert(KTP % 4 == 0, "list alignment");
  constexpr int STAGE = PK_STAGE;               // candidate records staged per position
  constexpr int PL = (REC_CHUNKS * STAGE + 63) / 64;   // 16 B staging loads per lane
  __shared__ VEntry ring[WPB][RING][KT];
  __shared__ int32_t cntl[WPB][RING];
  __shared__ uint4 stg[WPB][REC_CHUNKS * STAGE];   // records of the current position
  __shared__ __attribute__((aligned(16))) unsigned long long lkey[WPB][LN];
  __shared__ __attribute__((aligned(16))) uint32_t lgen[WPB][LN];
  __shared__ unsigned long long tkey[WPB][KT];
  __shared__ uint32_t tgen[WPB][KT];
  constexpr bool USE_D3 = KT <= 4;              // (its 8 KiB would cost a block per CU above)
  // the position's span starts and expansion prefixes, for the decode of an
  // expansion index (a lane-variable index into wave-uniform values)
  // (sized to the entries read: at KT = 16 every byte counts -- 16 one-wave
  // blocks per CU need at most 10,240 B each)
  __shared__ int sstp[WPB][PK_SPRE ? MAX_SPAN + 1 : 1];
  __shared__ __attribute__((aligned(16))) int sprep[WPB][PK_SPRE ? MAX_SPAN : 4];
  __shared__ uint4 ucan[REC_CHUNKS * MAX_SPAN]; // the implicit Unknowns' records
  stage_unk(p, ucan);
  Aux aux{nullptr, 0u, p.hk};
  if constexpr (USE_D3) {
    // (declared only where used: a 1-element placeholder's 8 B would cost
    // KT = 16 its sixteenth 1-wave block per CU -- 10,248 B > 160 KiB / 16)
    __shared__ double d3l[D3_DIM * D3_DIM];
    aux = stage_aux<NARROW>(p, d3l);
  }

  const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int lane = (int)(threadIdx.x & 63);
  const int slot = blockIdx.x * WPB + wv;
  if (slot >= p.n_sent) return;                 // whole wave
  const Bufs B = make_bufs(p);
  const int s = p.order[slot];
  const int n = p.sent_n[s];
  const uint32_t nbase = (uint32_t)p.node_off[s];
  const int32_t* __restrict__ ssp = p.span_start + p.span_off[s];
  uint32_t* __restrict__ bp = p.bp + p.bp_off[s];
  // the sentence's backpointers as a buffer: every position issues exactly one
  // store instruction (non-writer lanes: out-of-range offset, dropped), so the
  // wait at the top of the next position can leave that store in flight
  const rsrc_t bpr = make_rsrc(bp, (uint64_t)(n + 1) * (uint64_t)p.bp_stride * 4u);
  const int k = p.k;
  const int bstride = p.bp_stride;
  const uint32_t slots = p.slots, seed = p.seed;
  const int has_tri = p.has_tri;
  VEntry (&R)[RING][KT] = ring[wv];
  int32_t* const cnt9 = cntl[wv];
  unsigned long long* const LK = lkey[wv];
  uint32_t* const LG = lgen[wv];
  Counts cnt;

  if (lane == 0) {                              // beam[0] = [BOS] (beam.py:21-23)
    R[0][0] = v_bos(load_cand(B, nbase));
    cnt9[0] = cnt_entry(1, 1);
  }
  // The next position's first 64 records (lane t holds 16 B chunks t,
  // 64 + t, 128 + t of the block: consecutive lanes read consecutive bytes)
  // and span starts (lane j <= 8) are loaded into registers one position
  // ahead and written to LDS at the top of the position: ordinary loads, so
  // the compiler's waits count them exactly (an LDS-DMA in flight would make
  // it drain every memory operation before each LDS access).
  u32x4 pf[PL];
  int pfs = 0;
  auto prefetch = [&](int e1, int first, bool valid) {
    const uint32_t base = (nbase + (uint32_t)first) * (uint32_t)sizeof(NodeRec);
#pragma unroll
    for (int pl = 0; pl < PL; ++pl)
      pf[pl] = ld128(B.node, valid && pl * 64 + lane < REC_CHUNKS * STAGE ? base + (uint32_t)(pl * 64 + lane) * 16u : OOB);
    pfs = (valid && lane <= MAX_SPAN) ? ssp[(e1 - 1) * MAX_SPAN + lane] : 0;
  };
  int ss[MAX_SPAN + 1];
  prefetch(1, n >= 1 ? ssp[0] : 0, n >= 1);
  __builtin_amdgcn_raw_buffer_store_b32(0u, bpr, OOB, 0, 0);      // the invariant's first store
  __builtin_amdgcn_wave_barrier();
#ifdef PK_PHASES
  // diagnostic build: as lt_beam_hw's stamps
  unsigned long long ph[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const unsigned long long tstart = pk_stamp();
  unsigned long long tprev = tstart;
  unsigned long long nsteps_done = 0;
#endif

  for (int e = 1; e <= n; ++e) {
    // vmcnt(1): the prefetched records and span starts landed (VMEM
    // operations retire in order on gfx9; the one younger operation is the
    // previous position's backpointer store).  Big beams store several
    // backpointer chunks per position: vmcnt(0).
    if constexpr (BIG) __builtin_amdgcn_s_waitcnt(0x0F70);
    else __builtin_amdgcn_s_waitcnt(0x0F71);
    uint4* const cst = stg[wv];
#pragma unroll
    for (int pl = 0; pl < PL; ++pl)
      if (pl * 64 + lane < REC_CHUNKS * STAGE) cst[pl * 64 + lane] = make_uint4(pf[pl].x, pf[pl].y, pf[pl].z, pf[pl].w);
#pragma unroll
    for (int j = 0; j <= MAX_SPAN; ++j) ss[j] = __builtin_amdgcn_readlane(pfs, j);
    __builtin_amdgcn_wave_barrier();
    const int dmax = min(e, p.max_len);
    const int em9 = e % RING;
    const int A0 = ss[0];
    int pre[MAX_SPAN + 1];
    pre[0] = 0;
#pragma unroll
    for (int j = 0; j < MAX_SPAN; ++j) {
      const int d = MAX_SPAN - j;
      const int cv = (d <= dmax) ? cnt9[(e - d) % RING] : 0;
      // (an empty in-range slot holds its implicit Unknown, which needs no
      // expansion when every hypothesis of beam[e - d] ends in Unknown:
      // cnt_entry; the others are skipped per expansion)
      const int c = cnt_any(cv, ss[j + 1] == ss[j], d, dmax);
      pre[j + 1] = pre[j] + (int)__umul24((uint32_t)c, (uint32_t)max(ss[j + 1] - ss[j], 1));   // (c <= 256, m < 2^21)
    }
    const int M = pre[MAX_SPAN];
    PK_STAMP(0);
#if PK_SPRE
    if (lane <= MAX_SPAN) sstp[wv][lane] = pfs;
    if (lane == 0) {
      *reinterpret_cast<int4*>(&sprep[wv][0]) = make_int4(pre[0], pre[1], pre[2], pre[3]);
      *reinterpret_cast<int4*>(&sprep[wv][4]) = make_int4(pre[4], pre[5], pre[6], pre[7]);
    }
    __builtin_amdgcn_wave_barrier();
#endif

    // expansion g -> span slot j (d = 8 - j), hypothesis rank r, candidate i
    // (node ss[j] + i, or the slot's implicit Unknown: imp): j is the last
    // slot whose prefix is <= g (pre is nondecreasing), its prefix, size and
    // first node selected by the same compare -- PK_SPRE: j counted, the three
    // values read from LDS
    auto decode = [&](int g, int& j, int& r, int& i, int& sj, bool& imp, int& m) {
#if PK_SPRE
      j = 0;
#pragma unroll
      for (int q = 1; q < MAX_SPAN; ++q) j += g >= pre[q] ? 1 : 0;
      const int pj = sprep[wv][j];
      sj = sstp[wv][j];
      m = sstp[wv][j + 1] - sj;
#else
      j = 0;
      int pj = pre[0];
      m = ss[1] - ss[0];
      sj = ss[0];
#pragma unroll
      for (int q = 1; q < MAX_SPAN; ++q) {
        const bool ge = g >= pre[q];
        j = ge ? q : j;
        pj = ge ? pre[q] : pj;
        m = ge ? ss[q + 1] - ss[q] : m;
        sj = ge ? ss[q] : sj;
      }
#endif
      imp = m == 0;                             // (a slot holding expansion g is in range)
      m = imp ? 1 : m;
      const int local = g - pj;
      // local / m through a float reciprocal (local < 2^24), corrected by one
      r = (int)((float)local * __builtin_amdgcn_rcpf((float)m));
      i = local - r * m;
      if (i < 0) { --r; i += m; }
      else if (i >= m) { ++r; i -= m; }
    };

    int nrun = 0;
    for (int base = 0; base < M; base += CH) {
      unsigned long long myk[RPC];
      uint32_t myg[RPC];
#pragma unroll
      for (int t = 0; t < RPC; ++t) {
        myk[t] = 0ull;
        myg[t] = INV;
        if (base + 64 * t >= M) continue;        // uniform
        const int g = base + 64 * t + lane;
        const bool act = g < M;
        int j = 0, r = 0, i = 0, sj = 0, m = 1;
        bool imp = false;
        if (act) decode(g, j, r, i, sj, imp, m);
        const int d = MAX_SPAN - j;
        const int node = sj + i;
        const int so = node - A0;
        // the staged record (or implicit Unknown) for every lane, then a record
        // past the staged block by a wave-uniform branch that waits for its own
        // loads (beam_far): the common path has no load in flight into a
        // register it writes
        const bool far = act && !imp && so >= STAGE;
        Cand c = cand_lds32(imp ? ucan + 2 * (d - 1) : cst + 2 * min(max(so, 0), STAGE - 1), 1, B.pairs, B,
                            (imp || !act) ? INV : nbase + (uint32_t)node);
        beam_far(c, far, B, nbase + (uint32_t)node);
        const int hb = act ? ring_back(em9, d) : 0;
        const int hr = act ? r : 0;
        const VEntry h0 = R[hb][hr];
        // skip successive unknown words (beam.py:43-45): num_unk > 0 <=> wj is Unk
        const bool skip = !act || ((h0.meta & F_UNK) && (c.mask & F_UNK) && (d < dmax));
        BMProbe<NARROW> P;
        const uint32_t need = (!skip && has_tri) ? (c.mask & h0.meta & DQ_ALL) : 0u;
        bm_issue<NARROW>(P, B, slots, seed, h0, c, need, aux);
        asm volatile("" ::: "memory");
        PK_STAMP(1);
        const VEntry h1 = R[hb][hr];
        double cf[6];
        uint32_t pres = 0;
        if (has_tri) bm_classes<NARROW>(P, h1, c, cf, pres);
        if (!skip) {
          const double tri = has_tri ? v1_sum(cf, pres, c, h1) : 0.0;
          if (COUNT) v_count(cnt, h1, c, need, 2 * __builtin_popcount(P.gneed));
          const double sc = h1.score + increment<GEN>(p, c, tri, nbase + (uint32_t)node, h1.jnode, imp ? d : 0);   // beam.py:115
          myk[t] = ord_key(sc);
          myg[t] = (uint32_t)g;
        }
        LK[KTP + 64 * t + lane] = myk[t];
        LG[KTP + 64 * t + lane] = myg[t];
        round_done();
      }
      PK_STAMP(2);
      // Top-k of this chunk's entries and the running top-k.  The rank of an
      // entry is the number of entries with a larger key, or an equal key and
      // a smaller generation index (0 keys -- skipped / idle -- never win).
      const int R0 = min(RPC, (M - base + 63) >> 6);         // rounds used (uniform)
      unsigned long long rk = lane < nrun ? LK[KTP - nrun + lane] : 0ull;
      uint32_t rg = lane < nrun ? LG[KTP - nrun + lane] : INV;
      unsigned long long rkv[KV];                 // big beams: running entry lane + 64 v
      uint32_t rgv[KV];
      if constexpr (BIG) {
#pragma unroll
        for (int v = 0; v < KV; ++v) {
          const int q = lane + 64 * v;
          rkv[v] = q < nrun ? LK[KTP - nrun + q] : 0ull;
          rgv[v] = q < nrun ? LG[KTP - nrun + q] : INV;
          if (v > 0 && rkv[v] > rk) rk = rkv[v];   // the lane's maximum (pruning below)
        }
      }
      int valid = nrun;
#pragma unroll
      for (int t = 0; t < RPC; ++t)
        if (t < R0) valid += __builtin_popcountll(__ballot(myk[t] != 0ull));
      if (R0 == 1 && nrun == 0) {
        // one entry per lane: rank against the 64 entries of the list
        const int qe = KTP + ((min(64, M - base) + 3) & ~3);   // entries past M are 0
#if PK_RANK_U
        // (the list holds the round's entries in generation order, lane l's at
        // KTP + l: ties broken by list position, masks in scalar registers)
        const int rank = list_rank_u<64>(LK, KTP, qe, myk[0], KTP);
#else
        int rank = 0;
#pragma unroll 2
        for (int q = KTP; q < qe; q += 4) {
          const ulonglong2 ka = *reinterpret_cast<const ulonglong2*>(&LK[q]);
          const ulonglong2 kb = *reinterpret_cast<const ulonglong2*>(&LK[q + 2]);
          const uint4 gg = *reinterpret_cast<const uint4*>(&LG[q]);
          const unsigned long long kq[4] = {ka.x, ka.y, kb.x, kb.y};
          const uint32_t gq[4] = {gg.x, gg.y, gg.z, gg.w};
#pragma unroll
          for (int u = 0; u < 4; ++u) rank += (kq[u] > myk[0] || (kq[u] == myk[0] && gq[u] < myg[0])) ? 1 : 0;
        }
#endif
        if (myk[0] != 0ull && rank < k) { tkey[wv][rank] = myk[0]; tgen[wv][rank] = myg[0]; }
      } else {
        // several entries per lane: prune with tau = the k-th largest of the
        // lanes' maxima -- at least k entries are >= tau, so an entry below it
        // ranks >= k; every entry better than one >= tau is itself >= tau, so
        // ranks taken among the entries >= tau are exact.
        unsigned long long mx = rk;
#pragma unroll
        for (int t = 0; t < RPC; ++t)
          if (t < R0) mx = myk[t] > mx ? myk[t] : mx;
        // tau from the maxima's high 32 bits (a nonzero key's are nonzero):
        // the k-th largest h_k of them, tau = h_k << 32, still has at least k
        // entries >= it.  h_k by a most-significant-bit-first radix select
        // over the wave: the largest v with #{lanes: mh >= v} >= k, one
        // compare (ballot) and a scalar popcount per bit -- no LDS round trip
        // and no 64-lane scan per lane.
        const uint32_t mh = (uint32_t)(mx >> 32);
        const int nz = __builtin_popcountll(__ballot(mx != 0ull));
        uint32_t hk = 0u;
        if (nz >= k) {
#pragma unroll
          for (int b = 31; b >= 0; --b) {
            const uint32_t cand = hk | (1u << b);
            if (__builtin_popcountll(__ballot(mh >= cand)) >= k) hk = cand;
          }
        }
        const unsigned long long tau = nz >= k ? (unsigned long long)hk << 32 : 1ull;
        // compact the entries >= tau to the list head (in lane order per slot)
        int nc = 0;
        auto push = [&](unsigned long long key, uint32_t g) {
          const bool c = key >= tau && key != 0ull;
          const unsigned long long bal = __ballot(c);
          const int at = nc + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32),
                                                            __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
          if (c) { LK[at] = key; LG[at] = g; }
          nc += __builtin_popcountll(bal);
        };
        if constexpr (BIG) {
#pragma unroll
          for (int v = 0; v < KV; ++v)
            if (64 * v < nrun) push(rkv[v], rgv[v]);
        } else {
          if (nrun > 0) push(rk, rg);
        }
#pragma unroll
        for (int t = 0; t < RPC; ++t)
          if (t < R0) push(myk[t], myg[t]);
        const int nc4 = (nc + 3) & ~3;
        if (lane < nc4 - nc) { LK[nc + lane] = 0ull; LG[nc + lane] = INV; }
        // rank candidate c = lane + 64 v among the nc candidates
        for (int c0 = 0; c0 < nc; c0 += 64) {
          const int c = c0 + lane;
          const unsigned long long ck = c < nc ? LK[c] : 0ull;
          const uint32_t cg = c < nc ? LG[c] : INV;
          int rank = 0;
          for (int q = 0; q < nc4; q += 4) {
            const ulonglong2 ka = *reinterpret_cast<const ulonglong2*>(&LK[q]);
            const ulonglong2 kb = *reinterpret_cast<const ulonglong2*>(&LK[q + 2]);
            const uint4 gg = *reinterpret_cast<const uint4*>(&LG[q]);
            const unsigned long long kq[4] = {ka.x, ka.y, kb.x, kb.y};
            const uint32_t gq[4] = {gg.x, gg.y, gg.z, gg.w};
#pragma unroll
            for (int u = 0; u < 4; ++u) rank += (kq[u] > ck || (kq[u] == ck && gq[u] < cg)) ? 1 : 0;
          }
          if (c < nc && rank < k) { tkey[wv][rank] = ck; tgen[wv][rank] = cg; }
        }
      }
      nrun = min(k, valid);
      // running list for the next chunk / beam[e]: at [KTP - nrun, KTP), zero
      // padding below it (in order behind the writes above)
      const int nrp2 = (nrun + 3) & ~3;
      for (int q = lane; q < nrp2; q += 64) {
        const int dst = KTP - nrp2 + q, src = q - (nrp2 - nrun);
        LK[dst] = src >= 0 ? tkey[wv][src] : 0ull;
        LG[dst] = src >= 0 ? tgen[wv][src] : INV;
      }
    }

    // the next position's records and span starts: issued after this
    // position's last load wait (VMEM operations retire in order, so any wait
    // for a younger load would also wait for these)
    PK_STAMP(3);
    prefetch(e + 1, ss[MAX_SPAN], e < n);

    // beam[e] = the running top-k (Sequence.add, beam.py:112-116).  Winners
    // among the staged records read them from LDS; a winner past the staged
    // block (a position with more than STAGE candidates) takes a separate,
    // uniform path with global loads, so the common path has no load to wait
    // for (and does not wait for the prefetch above).
    int nlive = 0;                              // beam[e]'s hypotheses not ending in Unknown
    for (int w0 = 0; w0 < (BIG ? nrun : 1); w0 += 64) {   // one pass unless the beam exceeds 64
    const int wl = w0 + lane;                   // winner (rank) of this lane
    VEntry ne;
    uint32_t bpv = 0;
    const bool writer = wl < nrun;
    int wj = 0, wr = 0, wi = 0, wsj = 0, wm = 1;
    bool wimp = false;
    if (writer) decode((int)LG[KTP - nrun + wl], wj, wr, wi, wsj, wimp, wm);
    const int wd = MAX_SPAN - wj;
    const uint32_t wnode = wimp ? UNK_LOCAL : (uint32_t)(wsj + wi);
    const bool far = writer && !wimp && (int)wnode - A0 >= STAGE;
    auto build = [&](const Cand& c) {
      ne = v_grow<COUNT>(R[ring_back(em9, wd)][wr], c, ord_score(LK[KTP - nrun + wl]), wnode);
      bpv = bp_pack(wnode, (uint32_t)wd, (uint32_t)wr);
    };
    auto near = [&]() {                          // staged record or implicit Unknown
      const int so = min((int)wnode - A0, STAGE - 1);
      return cand_lds32(wimp ? ucan + 2 * (wd - 1) : cst + 2 * so, 1, B.pairs, B, wimp ? INV : nbase + wnode);
    };
    if (__builtin_amdgcn_ballot_w64(far) == 0ull) {
      if (writer) build(near());
    } else if (writer) {
      build(far ? load_cand(B, nbase + wnode) : near());
    }
    __builtin_amdgcn_wave_barrier();
    if (writer) R[em9][wl] = ne;
    nlive += __builtin_popcountll(__builtin_amdgcn_ballot_w64(writer && !(ne.meta & F_UNK)));
    __builtin_amdgcn_raw_buffer_store_b32(bpv, bpr, writer ? (uint32_t)(e * bstride + wl) * 4u : OOB, 0, BM_BP_AUX);
    }
    if (lane == 0) cnt9[em9] = cnt_entry(nrun, nlive);
    __builtin_amdgcn_wave_barrier();
    PK_STAMP(4);
#ifdef PK_PHASES
    ++nsteps_done;
#endif
  }
#ifdef PK_PHASES
  const unsigned long long tloop = pk_stamp();
#endif

  // matures = beam[n] + EOS (beam.py:59-61); backtrace per mature rank
  __builtin_amdgcn_s_waitcnt(0x0F70);           // vmcnt(0): the backpointer stores are done
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  const int nm = cnt9[n % RING] & CNT_BEAM;
  if (lane == 0) p.out_count[s] = nm;
  if constexpr (!BIG) {
    // (one mature per lane) the final entries, then the backpointer rows
    // into LDS over the ring (stage_bp_rows) when they fit
    constexpr int RW = (int)(RING * KT * sizeof(VEntry) / 4);
    constexpr int CAP = RW < BP_STAGE_PER_LANE * 64 ? RW : BP_STAGE_PER_LANE * 64;
    const int t = lane;
    double fs = 0.0;
    int fd = 0;
    if (t < k && t < nm) {
      fs = R[n % RING][t].score;
      fd = (int)R[n % RING][t].depth;
    }
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
    const int words = (n + 1) * bstride, cw = k * n;
    int32_t* const cout = p.out_codes + (int64_t)k * p.cum_n[s];   // the k padded paths
    uint32_t* const lbp = reinterpret_cast<uint32_t*>(&R[0][0]);
    int32_t* const lco = reinterpret_cast<int32_t*>(lbp + words);
    const bool inl = words <= CAP;              // (wave-uniform)
    const bool cinl = words + cw <= CAP;        // the codes staged too
    if (inl) stage_bp_rows<64, CAP>(bp, words, lbp, lane);
    if (cinl) fill_codes<64>(lco, cw, lane);
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
    if (t < k) {
      const int64_t o = (int64_t)s * k + t;
      int32_t* codes = cout + (int64_t)t * n;
      p.out_score[o] = t < nm ? fs + 0.0 : 0.0;
      p.out_len[o] = t < nm ? fd : 0;
      if (t >= nm) {                            // unused mature slots read as empty
        if (!cinl)
          for (int j = 0; j < n; ++j) codes[j] = -1;
      } else if (cinl) {
        walk_path(static_cast<const uint32_t*>(lbp), bstride, n, fd, t, k, lco + t * n, false);
      } else if (inl) {
        walk_path(static_cast<const uint32_t*>(lbp), bstride, n, fd, t, k, codes);
      } else {
        walk_path(static_cast<const uint32_t*>(bp), bstride, n, fd, t, k, codes);
      }
    }
    if (cinl) {
      __builtin_amdgcn_wave_barrier();
      asm volatile("" ::: "memory");
      copy_codes<64>(cout, lco, cw, lane);
    }
  } else {
    for (int t = lane; t < k; t += 64) {        // mature rank t (beams above 64: several passes)
      if (t >= nm) {                            // unused mature slots read as empty
        p.out_score[(int64_t)s * k + t] = 0.0;
        p.out_len[(int64_t)s * k + t] = 0;
        int32_t* codes = p.out_codes + (int64_t)k * p.cum_n[s] + (int64_t)t * n;
        for (int j = 0; j < n; ++j) codes[j] = -1;
        continue;
      }
      const VEntry& f = R[n % RING][t];
      const int64_t o = (int64_t)s * k + t;
      p.out_score[o] = f.score + 0.0;
      p.out_len[o] = (int32_t)f.depth;
      walk_path(static_cast<const uint32_t*>(bp), bstride, n, (int)f.depth, t, k,
                p.out_codes + (int64_t)k * p.cum_n[s] + (int64_t)t * n);
    }
  }
#ifdef PK_PHASES
  {
    const unsigned long long tend = pk_stamp();
    ph[5] += tend - tloop;
    if (lane == 0) {
      for (int i = 0; i < 8; ++i) atomicAdd(p.counters + 4 + i, ph[i]);
      atomicAdd(p.counters + 12, nsteps_done);
      atomicAdd(p.counters + 13, tend - tstart);
      atomicAdd(p.counters + 14, 1ull);
    }
  }
#endif
  if (COUNT) {
    const unsigned long long ex = group_sum<64>(cnt.exp), tu = group_sum<64>(cnt.tup),
                             pb = group_sum<64>(cnt.probe), ld = group_sum<64>(cnt.load);
    if (lane == 0) {
      atomicAdd(p.counters + 0, ex);
      atomicAdd(p.counters + 1, tu);
      atomicAdd(p.counters + 2, pb);
      atomicAdd(p.counters + 3, ld);
    }
  }
}

template <int KT, int WPB, bool NARROW, bool COUNT, bool GEN = true>
hipError_t launch_bp(const DecodeParams& p, const Launch& L) {
  const int blocks = (p.n_sent + WPB - 1) / WPB;
  if (blocks == 0) return hipSuccess;
  hipExtLaunchKernelGGL((lt_beam_pk<KT, WPB, NARROW, COUNT, GEN>), dim3(blocks), dim3(64 * WPB), 0, L.st, L.e0, L.e1, 0, p);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// beam_size 2..8, lane groups: the wave's G-lane groups (G = 32: two
// sentences per wave; G = 16: four, used for k <= 3) decode one sentence each,
// in lockstep over end positions.  lt_beam_pk leaves about half of a wave's
// lanes idle at k = 5 (about 27 expansions per position) and is issue-bound;
// here each group scores its own sentence's expansions in rounds of G lanes,
// so one instruction stream serves 64/G sentences.  Everything per sentence
// (span starts, expansion prefix, counts) lives in VGPRs that are uniform
// within a group; top-k is lt_beam_pk's exact rank counting and threshold
// pruning, per group.
// ---------------------------------------------------------------------------
template <int KT, int G, int WPB, bool NARROW, bool GEN = true>
// (wide keys at KT = 4, G = 32: 3 waves per SIMD would spill 4 VGPRs -- 2)
__global__ void __launch_bounds__(64 * WPB)
__attribute__((amdgpu_waves_per_eu(((G == 16 && KT > 2) || (!NARROW && KT == 4)) ? 2 : 3, 3)))
lt_beam_hw(DecodeParams p) {
  constexpr int S = 64 / G;                     // sentences per wave, one per lane group
  constexpr int RPC = 2;                        // scoring rounds (of G) per chunk
  constexpr int CH = G * RPC;                   // expansions per chunk per group
  constexpr int KTP = KT < 4 ? 4 : KT;
  constexpr int LN = KTP + CH;
  // records staged per group and position (the rest take a global load): a
  // position's dictionary candidates, 2.5 on average in the bench lattices
  constexpr int STAGE = HW_STAGE / S;
  constexpr int CPG = REC_CHUNKS * STAGE;       // staged 16 B chunks per group
  constexpr int PL = (S * CPG + 63) / 64;       // 16 B staging loads per lane
  static_assert(KT <= G && G >= MAX_SPAN + 1, "one writer lane per rank in a group; span starts fit a group");
  __shared__ VEntry ring[WPB][S][RING][KT];
  __shared__ int32_t cntl[WPB][S][RING];
  __shared__ uint8_t lrkl[WPB][S][RING][HW_LIVE ? KT : 1];   // live-rank lists (cnt_entry; HW_LIVE)
  __shared__ uint4 stg[WPB][S * CPG];           // group h's record r: chunks CPG h + 2r, +1
  __shared__ __attribute__((aligned(16))) unsigned long long lkey[WPB][S][LN];
  __shared__ __attribute__((aligned(16))) uint32_t lgen[WPB][S][LN];
  __shared__ unsigned long long tkey[WPB][S][KT];
  __shared__ uint32_t tgen[WPB][S][KT];
  __shared__ __attribute__((aligned(16))) int sst[WPB][S][12];   // each group's span starts of the position
  __shared__ __attribute__((aligned(16))) int spre[WPB][S][HW_SPRE ? 12 : 1];   // and expansion prefixes
  constexpr bool USE_D3 = KT <= HW_D3_MAXKT;
  __shared__ uint4 ucan[REC_CHUNKS * MAX_SPAN]; // the implicit Unknowns' records
  // the batch's class-4/6 pair table (read per expansion: LDS, not the caches)
  __shared__ F46 pxl[MAX_PAIRS];
  for (int i = (int)threadIdx.x; i < p.n_pairs; i += (int)blockDim.x) pxl[i] = p.pairs[i];
  stage_unk(p, ucan);
  Aux aux{nullptr, 0u, p.hk};
  if constexpr (USE_D3) {
    __shared__ double d3l[D3_DIM * D3_DIM];
    aux = stage_aux<NARROW>(p, d3l);
  }

  const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int lane = (int)(threadIdx.x & 63);
  const int hf = lane / G, hl = lane % G;       // lane group (sentence) and lane in the group
  const int slot0 = (blockIdx.x * WPB + wv) * S;
  if (slot0 >= p.n_sent) return;                // whole wave
  const Bufs B = make_bufs(p);
  const int k = p.k;
  const int bstride = p.bp_stride;
  const uint32_t slots = p.slots, seed = p.seed;
  const int has_tri = p.has_tri;
  // this half's sentence (values uniform within the half)
  const bool hv = slot0 + hf < p.n_sent;
  const int s = hv ? p.order[slot0 + hf] : 0;
  const int n = hv ? p.sent_n[s] : 0;
  const uint32_t nbase = hv ? (uint32_t)p.node_off[s] : 0u;
  const int32_t* const ssp = p.span_start + (hv ? p.span_off[s] : 0);
  const int64_t bpo = hv ? p.bp_off[s] : 0;
  // the maximum of a group-uniform value over the groups
  auto gmax = [&](int v) {
    int m = __builtin_amdgcn_readlane(v, 0);
#pragma unroll
    for (int h = 1; h < S; ++h) m = max(m, __builtin_amdgcn_readlane(v, h * G));
    return m;
  };
  const int nmax = gmax(n);
  uint32_t nbS[S];
  int nS[S];
#pragma unroll
  for (int h = 0; h < S; ++h) {
    nbS[h] = (uint32_t)__builtin_amdgcn_readlane((int)nbase, h * G);
    nS[h] = __builtin_amdgcn_readlane(n, h * G);
  }
  const rsrc_t bpr = make_rsrc_own(p.bp, (uint64_t)p.bp_bytes);
  VEntry (*const R)[KT] = ring[wv][hf];
  uint8_t (*const LR)[HW_LIVE ? KT : 1] = lrkl[wv][hf];
  int32_t* const cnt9 = cntl[wv][hf];
  unsigned long long* const LK = lkey[wv][hf];
  uint32_t* const LG = lgen[wv][hf];
  unsigned long long* const TK = tkey[wv][hf];
  uint32_t* const TG = tgen[wv][hf];
  const unsigned long long hmask = (G == 64 ? ~0ull : ((1ull << G) - 1ull)) << (G * hf);
  auto hcount = [&](unsigned long long bal) { return __builtin_popcountll(bal & hmask); };

  if (hv && hl == 0) {                          // beam[0] = [BOS] (beam.py:21-23)
    R[0][0] = v_bos(load_cand(B, nbase));
    if (HW_LIVE) LR[0][0] = 0;
    cnt9[0] = cnt_entry(1, 1);
  }
  if (HW_SPRE && hl == 0) spre[wv][hf][0] = 0;
  // next position's first STAGE records of every group (chunk c = 64 pl +
  // lane of the wave's stream: group c / CPG, chunk c % CPG of that group's
  // block) and span starts (lane G h + j <= 8: span start j of group h), one
  // position ahead, issued after the position's last load wait (lt_beam_pk)
  u32x4 pf[PL];
  int pfs = 0;
  auto prefetch = [&](int e1, int first_own) {
    int fS[S];
#pragma unroll
    for (int h = 0; h < S; ++h) fS[h] = __builtin_amdgcn_readlane(first_own, h * G);
#pragma unroll
    for (int pl = 0; pl < PL; ++pl) {
      const int c = 64 * pl + lane;
      const int hc = c / CPG, cc = c - hc * CPG;
      uint32_t nb = nbS[0], f = (uint32_t)fS[0];
      bool ok = e1 <= nS[0] && c < S * CPG;
#pragma unroll
      for (int h = 1; h < S; ++h)
        if (hc == h) { nb = nbS[h]; f = (uint32_t)fS[h]; ok = e1 <= nS[h]; }
      const uint32_t o = ok ? (nb + f) * (uint32_t)sizeof(NodeRec) + (uint32_t)cc * 16u : OOB;
      pf[pl] = ld128(B.node, o);
    }
    pfs = (e1 <= n && hl <= MAX_SPAN) ? ssp[(e1 - 1) * MAX_SPAN + hl] : 0;
  };
  prefetch(1, n >= 1 ? ssp[0] : 0);
  __builtin_amdgcn_raw_buffer_store_b32(0u, bpr, OOB, 0, 0);
  __builtin_amdgcn_wave_barrier();
#ifdef PK_PHASES
  // diagnostic build: per-wave cycles of [0] position setup, [1] expansion
  // decode + record + probe issue, [2] probe wait + score, [3] top-k, [4]
  // prefetch + beam write (tools/gpu_phases.sh)
  unsigned long long ph[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const unsigned long long tstart = pk_stamp();
  unsigned long long tprev = tstart;
  unsigned long long nsteps_done = 0;
#endif

  for (int e = 1; e <= nmax; ++e) {
    __builtin_amdgcn_s_waitcnt(0x0F71);         // vmcnt(1): the prefetch (older than the store)
    uint4* const cst = stg[wv];
#pragma unroll
    for (int pl = 0; pl < PL; ++pl)
      if (pl * 64 + lane < S * CPG) cst[pl * 64 + lane] = make_uint4(pf[pl].x, pf[pl].y, pf[pl].z, pf[pl].w);
    // the group's span starts through LDS: lanes j <= 8 of each group write
    // theirs, every lane reads its group's nine (three reads instead of a
    // readlane / select per value and group)
    if (hl <= MAX_SPAN) sst[wv][hf][hl] = pfs;
    __builtin_amdgcn_wave_barrier();
    int ss[MAX_SPAN + 1];
    {
      const int4 s0 = *reinterpret_cast<const int4*>(&sst[wv][hf][0]);
      const int4 s1 = *reinterpret_cast<const int4*>(&sst[wv][hf][4]);
      ss[0] = s0.x; ss[1] = s0.y; ss[2] = s0.z; ss[3] = s0.w;
      ss[4] = s1.x; ss[5] = s1.y; ss[6] = s1.z; ss[7] = s1.w;
      ss[8] = sst[wv][hf][8];
    }
    __builtin_amdgcn_wave_barrier();
    const bool live = e <= n;
    const int dmax = min(e, p.max_len);
    const int em9 = e % RING;
    const int A0 = ss[0];
    int pre[MAX_SPAN + 1];
#if HW_SPRE
    // span-slot expansion prefix through LDS: lane j < 8 of a group holds
    // slot j's c_j * m_j, a three-step DPP scan within the group's 16-lane
    // row makes the inclusive prefix, every lane reads the group's nine
    // (instead of an eight-step serial prefix in every lane)
    {
      int term = 0;
      if (hl < MAX_SPAN) {
        const int d = MAX_SPAN - hl;
        const int cv = (live && d <= dmax) ? cnt9[ring_back(em9, d)] : 0;
        const int m = sst[wv][hf][hl + 1] - pfs;
        // (an empty in-range slot holds its implicit Unknown, which needs no
        // expansion when it is statically dead: cnt_dead)
        const int c = HW_LIVE ? cnt_live(cv, m == 0, d, dmax) : cnt_any(cv, m == 0, d, dmax);
        term = (int)__umul24((uint32_t)c, (uint32_t)max(m, 1));   // (c <= 256, m < 2^21)
      }
      term += __builtin_amdgcn_update_dpp(0, term, 0x111, 0xF, 0xF, true);      // row_shr:1
      term += __builtin_amdgcn_update_dpp(0, term, 0x112, 0xF, 0xF, true);      // row_shr:2
      term += __builtin_amdgcn_update_dpp(0, term, 0x114, 0xF, 0xF, true);      // row_shr:4
      if (hl < MAX_SPAN) spre[wv][hf][hl + 1] = term;
      __builtin_amdgcn_wave_barrier();
      const int4 p0 = *reinterpret_cast<const int4*>(&spre[wv][hf][0]);
      const int4 p1 = *reinterpret_cast<const int4*>(&spre[wv][hf][4]);
      pre[0] = p0.x; pre[1] = p0.y; pre[2] = p0.z; pre[3] = p0.w;
      pre[4] = p1.x; pre[5] = p1.y; pre[6] = p1.z; pre[7] = p1.w;
      pre[8] = spre[wv][hf][8];
    }
#else
    pre[0] = 0;
#pragma unroll
    for (int j = 0; j < MAX_SPAN; ++j) {
      const int d = MAX_SPAN - j;
      const int cv = (live && d <= dmax) ? cnt9[(e - d) % RING] : 0;
      const int c = HW_LIVE ? cnt_live(cv, ss[j + 1] == ss[j], d, dmax) : cnt_any(cv, ss[j + 1] == ss[j], d, dmax);
      pre[j + 1] = pre[j] + (int)__umul24((uint32_t)c, (uint32_t)max(ss[j + 1] - ss[j], 1));   // (c <= 256, m < 2^21)
    }
#endif
    const int M = pre[MAX_SPAN];                // this half's expansions
    const int Mmax = gmax(M);
    PK_STAMP(0);

    auto decode = [&](int g, int& j, int& r, int& i, int& sj, bool& imp, int& m) {     // (lt_beam_pk)
#if HW_SPRE
      // pre is nondecreasing: the slot is the number of prefixes <= g; its
      // prefix, first node and size from LDS
      j = 0;
#pragma unroll
      for (int q = 1; q < MAX_SPAN; ++q) j += g >= pre[q] ? 1 : 0;
      const int pj = spre[wv][hf][j];
      sj = sst[wv][hf][j];
      m = sst[wv][hf][j + 1] - sj;
#else
      j = 0;
      int pj = pre[0];
      m = ss[1] - ss[0];
      sj = ss[0];
#pragma unroll
      for (int q = 1; q < MAX_SPAN; ++q) {
        const bool ge = g >= pre[q];
        j = ge ? q : j;
        pj = ge ? pre[q] : pj;
        m = ge ? ss[q + 1] - ss[q] : m;
        sj = ge ? ss[q] : sj;
      }
#endif
      imp = m == 0;                             // (a slot holding expansion g is in range)
      m = imp ? 1 : m;
      const int local = g - pj;
      r = (int)((float)local * __builtin_amdgcn_rcpf((float)m));
      i = local - r * m;
      if (i < 0) { --r; i += m; }
      else if (i >= m) { ++r; i -= m; }
    };

    int nrun = 0;                               // this half's running top-k size
    for (int base = 0; base < Mmax; base += CH) {
      unsigned long long myk[RPC];
      uint32_t myg[RPC];
#pragma unroll
      for (int t = 0; t < RPC; ++t) {
        myk[t] = 0ull;
        myg[t] = INV;
        if (base + G * t >= Mmax) continue;      // uniform
        const int g = base + G * t + hl;
        const bool act = g < M;
        int j = 0, r = 0, i = 0, sj = 0, m = 1;
        bool imp = false;
        if (act) decode(g, j, r, i, sj, imp, m);
        const int d = MAX_SPAN - j;
        const int node = sj + i;
        const int so = node - A0;
        const bool far = act && !imp && so >= STAGE;   // (beam_far, as lt_beam_pk)
        Cand c = cand_lds32(imp ? ucan + 2 * (d - 1) : cst + CPG * hf + 2 * min(max(so, 0), STAGE - 1), 1, pxl, B,
                            (imp || !act) ? INV : nbase + (uint32_t)node);
        beam_far(c, far, B, nbase + (uint32_t)node);
        const int hb = act ? ring_back(em9, d) : 0;
        // (an implicit Unknown past b_min: the r-th hypothesis not ending in Unknown)
        const int hr = !act ? 0 : (HW_LIVE && imp && d < dmax) ? (int)LR[hb][r] : r;
        const VEntry h0 = R[hb][hr];
        const bool skip = !act || ((h0.meta & F_UNK) && (c.mask & F_UNK) && (d < dmax));   // beam.py:43-45
        const uint32_t need = (!skip && has_tri) ? (c.mask & h0.meta & DQ_ALL) : 0u;
        BMProbe<NARROW> P;
        bm_issue<NARROW, !NARROW>(P, B, slots, seed, h0, c, need, aux);   // (INIT: wide keys only)
        asm volatile("" ::: "memory");
        PK_STAMP(1);
        const VEntry h1 = R[hb][hr];
        const double tri = has_tri ? bm_score<NARROW>(P, h1, c) : 0.0;
        if (!skip) {
          const double sc = h1.score + increment<GEN>(p, c, tri, nbase + (uint32_t)node, h1.jnode, imp ? d : 0);   // beam.py:115
          myk[t] = ord_key(sc);
          // the list entry's payload: the expansion as its backpointer word
          // (ranks are by list position, so nothing reads g itself; the
          // writer of beam[e] takes node, span and parent rank from it)
          myg[t] = bp_pack(imp ? UNK_LOCAL : (uint32_t)node, (uint32_t)d, (uint32_t)hr);
        }
        LK[KTP + G * t + hl] = myk[t];
        LG[KTP + G * t + hl] = myg[t];
        round_done();
      }
      PK_STAMP(2);
      // top-k of this half's chunk entries and its running top-k
      const int R0 = max(0, min(RPC, (M - base + G - 1) / G));      // this group's rounds
      const unsigned long long rk = hl < nrun ? LK[KTP - nrun + hl] : 0ull;
      const uint32_t rg = hl < nrun ? LG[KTP - nrun + hl] : INV;
      int valid = nrun;
#pragma unroll
      for (int t = 0; t < RPC; ++t) valid += hcount(__ballot(myk[t] != 0ull));
      const bool single = R0 <= 1 && nrun == 0;
      if (__builtin_amdgcn_ballot_w64(!single) == 0ull) {
        // one entry per lane in both halves: rank against the half's 32 list
        // slots of round 0 (slots past M hold 0 keys)
        const int qe = KTP + ((min(G, max(M - base, 0)) + 3) & ~3);
        const int qmax = gmax(qe);
#if HW_RANK_U
        {
          const int r = list_rank_u<G>(LK, KTP, qmax, myk[0], KTP);
          if (myk[0] != 0ull && r < k) { TK[r] = myk[0]; TG[r] = myg[0]; }
        }
#else
        rank_into(LK, KTP, qmax, myk[0], myg[0], KTP + hl, k, TK, TG);
#endif
      } else {
        // threshold pruning (lt_beam_pk), per half: tau = the k-th largest of
        // the half's lane maxima
        unsigned long long mx = rk;
#pragma unroll
        for (int t = 0; t < RPC; ++t) mx = myk[t] > mx ? myk[t] : mx;
        // (tau from the maxima's high 32 bits, as lt_beam_pk)
        uint32_t* const MX = reinterpret_cast<uint32_t*>(LK + KTP);   // chunk entries are in registers now
        const uint32_t mh = (uint32_t)(mx >> 32);
        MX[hl] = mh;
        if (hl == 0) TK[0] = ~0ull;
        int gtc = 0;
#pragma unroll 4
        for (int q = 0; q < G; q += 4) {
          const uint4 m4 = *reinterpret_cast<const uint4*>(&MX[q]);
          gtc += (m4.x > mh ? 1 : 0) + (m4.y > mh ? 1 : 0) + (m4.z > mh ? 1 : 0) + (m4.w > mh ? 1 : 0);
        }
        const int nz = hcount(__ballot(mx != 0ull));
        if (mx != 0ull && gtc < k)
          __hip_atomic_fetch_min(&TK[0], (unsigned long long)mh << 32, __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_WORKGROUP);
        const unsigned long long tau = nz >= k ? TK[0] : 1ull;
        int nc = 0;
        auto push = [&](unsigned long long key, uint32_t g) {
          const bool c = key >= tau && key != 0ull;
          const uint32_t bh = (uint32_t)((__ballot(c) & hmask) >> (G * hf));
          const int at = nc + __builtin_popcount(bh & ((1u << hl) - 1u));
          if (c) { LK[at] = key; LG[at] = g; }
          nc += __builtin_popcount(bh);
        };
        push(rk, rg);
#pragma unroll
        for (int t = 0; t < RPC; ++t) push(myk[t], myg[t]);
        const int nc4 = (nc + 3) & ~3;
        if (hl < nc4 - nc) { LK[nc + hl] = 0ull; LG[nc + hl] = INV; }
        const int ncmax = gmax(nc);
        if (ncmax <= G) {                         // (the usual case: one candidate per lane)
          const unsigned long long ck = hl < nc ? LK[hl] : 0ull;
          const uint32_t cg = hl < nc ? LG[hl] : INV;
          rank_into(LK, 0, nc4, ck, cg, hl, k, TK, TG);
        } else {
          for (int c0 = 0; c0 < ncmax; c0 += G) {
            const int c = c0 + hl;
            const unsigned long long ck = c < nc ? LK[c] : 0ull;
            const uint32_t cg = c < nc ? LG[c] : INV;
            const int rank = list_rank(LK, 0, nc4, ck, c);
            if (c < nc && rank < k) { TK[rank] = ck; TG[rank] = cg; }
          }
        }
      }
      nrun = min(k, valid);
      const int nrp2 = (nrun + 3) & ~3;
      if (hl < nrp2) {
        const int dst = KTP - nrp2 + hl, src = hl - (nrp2 - nrun);
        LK[dst] = src >= 0 ? TK[src] : 0ull;
        LG[dst] = src >= 0 ? TG[src] : INV;
      }
    }

    PK_STAMP(3);
    prefetch(e + 1, ss[MAX_SPAN]);              // after the position's last load wait

    // beam[e] of each half (Sequence.add, beam.py:112-116)
    VEntry ne;
    const bool writer = live && hl < nrun;
    const uint32_t bpv = writer ? LG[KTP - nrun + hl] : bp_pack(0u, 1u, 0u);   // node, span, parent rank
    const int wd = (int)bp_d(bpv), wr = (int)bp_rank(bpv);
    const uint32_t wnode = bp_node(bpv);
    const bool wimp = wnode == UNK_LOCAL;
    const bool far = writer && !wimp && (int)wnode - A0 >= STAGE;
    auto build = [&](const Cand& c) {
      ne = v_grow<false>(R[ring_back(em9, wd)][wr], c, ord_score(LK[KTP - nrun + hl]), wnode);
    };
    auto near = [&]() {                          // staged record or implicit Unknown
      const int so = min((int)wnode - A0, STAGE - 1);
      return cand_lds32(wimp ? ucan + 2 * (wd - 1) : cst + CPG * hf + 2 * so, 1, pxl, B,
                        wimp ? INV : nbase + wnode);
    };
    if (__builtin_amdgcn_ballot_w64(far) == 0ull) {
      if (writer) build(near());
    } else if (writer) {
      build(far ? load_cand(B, nbase + wnode) : near());
    }
    __builtin_amdgcn_wave_barrier();
    if (writer) R[em9][hl] = ne;
    // the live-rank list of beam[e] (cnt_entry)
    const bool xw = writer && !(ne.meta & F_UNK);
    const uint32_t xb = (uint32_t)((__builtin_amdgcn_ballot_w64(xw) & hmask) >> (G * hf));
    if (HW_LIVE && xw) LR[em9][__builtin_popcount(xb & ((1u << hl) - 1u))] = (uint8_t)hl;
    __builtin_amdgcn_raw_buffer_store_b32(
        bpv, bpr, writer ? (uint32_t)((bpo + (int64_t)e * bstride + hl) * 4) : OOB, 0, BM_BP_AUX);
    if (live && hl == 0) cnt9[em9] = cnt_entry(nrun, __builtin_popcount(xb));
    __builtin_amdgcn_wave_barrier();
    PK_STAMP(4);
#ifdef PK_PHASES
    ++nsteps_done;
#endif
  }

#ifdef PK_PHASES
  const unsigned long long tloop = pk_stamp();
#endif
  // matures = beam[n] + EOS (beam.py:59-61); backtrace per (half, rank)
  __builtin_amdgcn_s_waitcnt(0x0F70);           // vmcnt(0): the backpointer stores are done
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  // the final entries, then each group's backpointer rows into LDS over its
  // ring (stage_bp_rows) when they fit
  constexpr int RW = (int)(RING * KT * sizeof(VEntry) / 4);
  constexpr int CAP = RW < BP_STAGE_PER_LANE * G ? RW : BP_STAGE_PER_LANE * G;
  const int nm = hv ? cnt9[n % RING] & CNT_BEAM : 0;
  double fs = 0.0;
  int fd = 0;
  if (hv && hl < k && hl < nm) {
    fs = R[n % RING][hl].score;
    fd = (int)R[n % RING][hl].depth;
  }
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
  const int words = (n + 1) * bstride, cw = k * n;
  int32_t* const cout = p.out_codes + (hv ? (int64_t)k * p.cum_n[s] : 0);   // the k padded paths
  uint32_t* const lbp = reinterpret_cast<uint32_t*>(&R[0][0]);
  int32_t* const lco = reinterpret_cast<int32_t*>(lbp + words);
  const uint32_t* const bpg = p.bp + bpo;
  const bool inl = hv && words <= CAP;          // (group-uniform)
  const bool cinl = inl && words + cw <= CAP;   // the codes staged too
  if (inl) stage_bp_rows<G, CAP>(bpg, words, lbp, hl);
  if (cinl) fill_codes<G>(lco, cw, hl);
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
  if (hv && hl < k) {
    if (hl == 0) p.out_count[s] = nm;
    const int64_t o = (int64_t)s * k + hl;
    int32_t* codes = cout + (int64_t)hl * n;
    p.out_score[o] = hl < nm ? fs + 0.0 : 0.0;
    p.out_len[o] = hl < nm ? fd : 0;
    if (hl >= nm) {
      if (!cinl)
        for (int j = 0; j < n; ++j) codes[j] = -1;
    } else if (cinl) {
      walk_path(static_cast<const uint32_t*>(lbp), bstride, n, fd, hl, k, lco + hl * n, false);
    } else if (inl) {
      walk_path(static_cast<const uint32_t*>(lbp), bstride, n, fd, hl, k, codes);
    } else {
      walk_path(bpg, bstride, n, fd, hl, k, codes);
    }
  }
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
  if (cinl) copy_codes<G>(cout, lco, cw, hl);
#ifdef PK_PHASES
  {
    // [5] the matures and backtraces
    const unsigned long long tend = pk_stamp();
    ph[5] += tend - tloop;
    if (lane == 0) {
      for (int i = 0; i < 8; ++i) atomicAdd(p.counters + 4 + i, ph[i]);
      atomicAdd(p.counters + 12, nsteps_done);
      atomicAdd(p.counters + 13, tend - tstart);
      atomicAdd(p.counters + 14, 1ull);
    }
  }
#endif
}

template <int KT, int G, int WPB, bool NARROW, bool GEN = true>
hipError_t launch_hw(const DecodeParams& p, const Launch& L) {
  constexpr int SPB = (64 / G) * WPB;
  const int blocks = (p.n_sent + SPB - 1) / SPB;
  if (blocks == 0) return hipSuccess;
  hipExtLaunchKernelGGL((lt_beam_hw<KT, G, WPB, NARROW, GEN>), dim3(blocks), dim3(64 * WPB), 0, L.st, L.e0, L.e1, 0, p);
  return hipGetLastError();
}

// lanes per sentence of lt_beam_hw: 16 (four sentences per wave) where a
// position has few expansions (k <= 3), else 32
static int beam_group_lanes(int k) { return k <= 3 ? 16 : 32; }

// ===========================================================================
// Batch evaluate (BeamScoreFunctions.evaluate, score_funcs.py:44-48)
// ===========================================================================
// One lane per word: the trigram increment of the replayed path
// (score_funcs.py:127-135 -> 137-144) -- the same probe / numpy-order sum code
// as the decoder, with the hypothesis built from the word's replayed
// predecessors.
template <bool NARROW>
__global__ void __launch_bounds__(256) lt_eval_words_k(EvalParams p) {
  __shared__ double d3l[D3_DIM * D3_DIM];
  Aux aux{nullptr, p.d3off, p.hk};
  if (p.d3) {
    d3_stage(p.d3, d3l);
    __syncthreads();
    aux.d3 = d3l;
  }
  const int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= p.n_words) return;
  const int64_t j = p.prev1[w];
  if (j == -2 || !p.has_tri) { p.inc[w] = 0.0; return; }
  Bufs B;
  B.node = make_rsrc(p.words, (uint64_t)p.n_words * sizeof(NodeRec));
  B.tab = make_rsrc(p.table, (uint64_t)p.slots * (NARROW ? sizeof(SlotN) : sizeof(SlotW)));
  B.pairs = p.pairs;
  B.esc = make_rsrc(p.esc, p.esc ? (uint64_t)p.n_words * sizeof(F46) : 0u);
  const Cand c = load_cand(B, (uint32_t)w);
  const Cand cj = load_cand(B, (uint32_t)j);
  const int64_t i = p.prev2[w];
  const Cand ci = load_cand(B, i >= 0 ? (uint32_t)i : INV);
  Hyp h;
  h.score = 0.0; h.f6 = cj.f6;
  h.jword = cj.word; h.jmorph = cj.morph; h.jtag = cj.tag; h.jmask = cj.mask;
  h.iword = ci.word; h.imorph = ci.morph; h.imask = i >= 0 ? (ci.mask | F_WI) : 0u;
  h.depth = 0;
  h.jnode = 0;
  h.inode = 0;
  Counts cnt;
  p.inc[w] = trigram<NARROW, false>(B, p.slots, p.seed, h, c, cnt, aux, p.coff);
}

// One lane per path: the exact-order sums.
__global__ void __launch_bounds__(256) lt_eval_paths_k(EvalParams p) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= p.n_paths) return;
  const int64_t w0 = p.path_off[s], w1 = p.path_off[s + 1];
  double tri = 0.0;
  for (int64_t w = w0; w < w1; ++w)
    if (p.prev1[w] != -2) tri += p.inc[w];
  double total = 0.0;
  int t = 0;
  for (int f = 0; f <= p.n_terms; ++f) {
    if (f == p.trigram_pos) {
      total += tri;
    } else if (t < p.n_terms) {
      const double* v = p.terms + (int64_t)t * p.n_words;
      double e = 0.0;
      for (int64_t w = w0; w < w1; ++w) e += v[w];
      total += e;
      ++t;
    }
  }
  p.out[s] = total;
}

#ifndef HW_WPB
#define HW_WPB 4                        // waves per block of lt_beam_hw, k = 2..4
#endif
#ifndef HW8_WPB
#define HW8_WPB 1                       // waves per block of lt_beam_hw, k = 5..8 (k=5: 4.044 ms at 4)
#endif
#ifndef BP16_WPB
#define BP16_WPB 1                      // waves per block of lt_beam_pk, k = 9..16 (1: 15.9 ms at k=16, 2: 16.7, 4: 16.7)
#endif
#ifndef BP32_WPB
#define BP32_WPB 2                      // waves per block of lt_beam_pk, k = 17..32
#endif

template <bool NARROW, bool COUNT>
hipError_t launch_k(const DecodeParams& p, int kt, const Launch& L) {
  // the composite's usual shape (node-local terms, then the trigram, nothing
  // after it) takes the kernels without the post / edge term code (GEN =
  // false; narrow keys, the tuned beams up to 32)
  if constexpr (NARROW && !COUNT) {
    if (p.n_post == 0 && p.n_edge == 0) switch (kt) {
      case 1: return launch_pk<P_W, NARROW, COUNT, false>(p, L);
      case 2: if (beam_group_lanes(p.k) == 16) return launch_hw<2, 16, HW_WPB, NARROW, false>(p, L); break;
      case 4: return beam_group_lanes(p.k) == 16 ? launch_hw<4, 16, HW_WPB, NARROW, false>(p, L)
                                                  : launch_hw<4, 32, HW_WPB, NARROW, false>(p, L);
      case 8: return launch_hw<8, 32, HW8_WPB, NARROW, false>(p, L);
      case 16: return launch_bp<16, BP16_WPB, NARROW, COUNT, false>(p, L);
      case 32: return launch_bp<32, BP32_WPB, NARROW, COUNT, false>(p, L);
      default: break;
    }
  }
  if (kt == 1) return launch_pk<P_W, NARROW, COUNT>(p, L);
  // k = 2..8: lane groups (16 lanes for k <= 3, 32 above); the operation
  // counts of those beams come from lt_beam_pk's COUNT variant (one sentence
  // per wave, same enumeration), which lt_beam_hw does not have
  if (!COUNT && kt <= 8) {
    if (beam_group_lanes(p.k) == 16) {
      switch (kt) {
        case 2: return launch_hw<2, 16, HW_WPB, NARROW>(p, L);
        case 4: return launch_hw<4, 16, HW_WPB, NARROW>(p, L);
        default: break;
      }
    }
    switch (kt) {
      case 4: return launch_hw<4, 32, HW_WPB, NARROW>(p, L);
      case 8: return launch_hw<8, 32, HW8_WPB, NARROW>(p, L);
      default: return hipErrorInvalidValue;
    }
  }
  if constexpr (COUNT) {                 // (decodes of k <= 8 returned above)
    switch (kt) {
      case 2: return launch_bp<2, 4, NARROW, COUNT>(p, L);
      case 4: return launch_bp<4, 4, NARROW, COUNT>(p, L);
      case 8: return launch_bp<8, 4, NARROW, COUNT>(p, L);
      default: break;
    }
  }
  switch (kt) {
    case 16: return launch_bp<16, BP16_WPB, NARROW, COUNT>(p, L);
    case 32: return launch_bp<32, BP32_WPB, NARROW, COUNT>(p, L);
    // beams above 32: one wave per block (the LDS ring of 9 x KT entries)
    case 64: return launch_bp<64, 1, NARROW, COUNT>(p, L);
    case 128: return launch_bp<128, 1, NARROW, COUNT>(p, L);
    case 256: return launch_bp<256, 1, NARROW, COUNT>(p, L);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace

namespace lt {

hipError_t launch_evaluate(const EvalParams& p, hipStream_t st) {
  if (p.n_words > 0) {
    const int blocks = (int)((p.n_words + 255) / 256);
    if (p.narrow) hipLaunchKernelGGL(lt_eval_words_k<true>, dim3(blocks), dim3(256), 0, st, p);
    else hipLaunchKernelGGL(lt_eval_words_k<false>, dim3(blocks), dim3(256), 0, st, p);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  if (p.n_paths > 0) {
    hipLaunchKernelGGL(lt_eval_paths_k, dim3((p.n_paths + 255) / 256), dim3(256), 0, st, p);
    return hipGetLastError();
  }
  return hipSuccess;
}

const char* kernel_name_for(int k) {
  const int kt = beam_template_for(k);
  if (kt < 0) return nullptr;
  if (kt == 1) return "lt_viterbi_pk";
  return kt <= 8 ? "lt_beam_hw" : "lt_beam_pk";
}

int beam_template_for(int k) {
  if (k <= 1) return 1;
  for (int kt = 2; kt <= LT_MAX_BEAM_COMPILED; kt *= 2)
    if (k <= kt) return kt;
  return -1;
}

hipError_t launch_k1_sched_count(const DecodeParams& p, int64_t* steps, hipStream_t st) {
  const int waves = k1_waves(p.n_sent);
  if (waves == 0) return hipSuccess;
  hipLaunchKernelGGL((lt_k1_sched_count<P_W>), dim3(waves), dim3(64), 0, st, p, steps);
  return hipGetLastError();
}

hipError_t launch_k1_sched_fill(const DecodeParams& p, const int64_t* wave_off, uint32_t* sched, hipStream_t st,
                                hipEvent_t e0, hipEvent_t e1) {
  const int waves = k1_waves(p.n_sent);
  if (waves == 0) {
    hipError_t e = e0 ? hipEventRecord(e0, st) : hipSuccess;
    if (e == hipSuccess && e1) e = hipEventRecord(e1, st);
    return e;
  }
  hipExtLaunchKernelGGL((lt_k1_sched<P_W>), dim3(waves), dim3(64), 0, st, e0, e1, 0, p, wave_off, sched);
  return hipGetLastError();
}

hipError_t launch_decode(const DecodeParams& p, hipStream_t st, bool count, hipEvent_t e0, hipEvent_t e1) {
  const int kt = beam_template_for(p.k);
  if (kt == 1 && (!p.sched || !p.wave_off)) return hipErrorInvalidValue;   // (the library builds it first)
  // the timing events ride on the kernel's dispatch (no extra stream
  // commands between back-to-back decodes); an empty batch launches nothing
  if (p.n_sent == 0) {
    hipError_t e = e0 ? hipEventRecord(e0, st) : hipSuccess;
    if (e == hipSuccess && e1) e = hipEventRecord(e1, st);
    return e;
  }
  const Launch L{st, e0, e1};
  if (p.narrow)
    return count ? launch_k<true, true>(p, kt, L) : launch_k<true, false>(p, kt, L);
  return count ? launch_k<false, true>(p, kt, L) : launch_k<false, false>(p, kt, L);
}

}  // namespace lt

// ===========================================================================
// trace (beam_search debug=True, beam.py:53-57): one thread per sentence walks
// the reference loops literally -- b ascending, each hypothesis of beam[b],
// each candidate of span (b, e) (beam.py:31-48) -- scoring with the decoders'
// own code, records every expansion, and keeps beam[e] as Beam.append does
// (stable by score, beam.py:85) by selection.  Diagnostic path: no tuning.
// ===========================================================================
namespace {
template <bool NARROW>
__global__ void __launch_bounds__(64) lt_trace_k(DecodeParams p, TraceParams t) {
  static_assert(sizeof(Entry) == TRACE_ENTRY_BYTES, "trace entry layout");
  const int s = blockIdx.x * 64 + threadIdx.x;
  if (s >= p.n_sent) return;
  const Bufs B = make_bufs(p);
  const Aux aux{nullptr, 0u, p.hk};             // class 3 from the table itself
  const int k = p.k, S = p.span_slots;
  const bool wide = decode_is_wide(p.max_len, k) || p.n_xtri > 0;
  const int n = p.sent_n[s];
  const uint32_t nbase = (uint32_t)p.node_off[s];
  const int32_t* ssp = p.span_start + p.span_off[s];
  const int64_t po = t.pos_off[s];
  Entry* ent = reinterpret_cast<Entry*>(t.ent) + po * k;
  Counts cnt;
  {
    const Cand b0 = load_cand(B, nbase);        // beam[0] = [BOS] (beam.py:21-23)
    Entry e0;
    e0.score = 0.0; e0.f6 = b0.f6;
    e0.jword = b0.word; e0.jmorph = b0.morph; e0.jtag = b0.tag; e0.jmask = b0.mask;
    e0.iword = 0; e0.imorph = 0; e0.imask = 0; e0.depth = 0;
    e0.jnode = 0; e0.pad0 = e0.pad1 = e0.pad2 = 0;
    ent[0] = e0;
    t.beam_count[po] = 1;
    t.beam_gen[po * k] = 0u;
    t.exp_count[po] = 0;
  }
  for (int e = 1; e <= n; ++e) {
    const int dmax = min(e, p.max_len);
    const int64_t xo = t.exp_off[po + e], xe = t.exp_off[po + e + 1];
    uint32_t g = 0;
    for (int j = S - dmax; j < S; ++j) {        // span j: length d = S - j, begin b = e - d
      const int d = S - j;
      const int b = e - d;
      const int lo = ssp[(int64_t)(e - 1) * S + j], hi = ssp[(int64_t)(e - 1) * S + j + 1];
      const bool imp = lo == hi && p.n_unk;     // the span's implicit Unknown (beam.py:36-38)
      const int hi1 = imp ? lo + 1 : hi;
      const int nb = t.beam_count[po + b];
      for (int r = 0; r < nb; ++r) {
        const Hyp h = read_entry(ent[(int64_t)b * k + r]);
        for (int node = lo; node < hi1; ++node, ++g) {
          if (xo + g >= xe) {                   // the caller's slots are too few: report, stop
            t.exp_count[po + e] = -1;
            return;
          }
          const uint32_t nd = imp ? UNK_LOCAL : (uint32_t)node;
          const Cand c = cand_at(B, p, nbase, nd, d);
          const bool skip = (h.jmask & F_UNK) && (c.mask & F_UNK) && (d < dmax);   // beam.py:43-45
          double sc = 0.0;
          if (!skip && p.n_xtri) {              // several trigram terms (score_funcs.py:50-54)
            double tris[MAX_TRI];
            trigram_terms<NARROW, false>(p, B, h, c, nbase + (uint32_t)node, nbase + h.jnode, nbase + h.inode, cnt,
                                         aux, tris);
            sc = h.score + increment_x(p, c, tris, nbase + (uint32_t)node, h.jnode);   // beam.py:115
          } else if (!skip) {
            const double tri = p.has_tri ? trigram<NARROW, false>(B, p.slots, p.seed, h, c, cnt, aux) : 0.0;
            sc = h.score + increment(p, c, tri, nbase + (uint32_t)node, h.jnode, imp ? d : 0);   // beam.py:115
          }
          t.exp_score[xo + g] = sc;
          t.exp_node[xo + g] = wide ? nd : bp_pack(nd, (uint32_t)d, (uint32_t)r);
          if (t.exp_link) t.exp_link[xo + g] = bpw_pack(nd, (uint32_t)d, (uint32_t)r);
          t.exp_skip[xo + g] = skip ? 1 : 0;
        }
      }
    }
    const uint32_t M = g;
    t.exp_count[po + e] = (int32_t)M;
    // beam[e]: the k first of the stable order (score desc, generation asc)
    int kept = 0;
    unsigned long long pk = ~0ull;
    uint32_t pg = 0;
    bool first = true;
    for (; kept < k; ++kept) {
      unsigned long long bk = 0ull;
      uint32_t bg = INV;
      for (uint32_t q = 0; q < M; ++q) {
        if (t.exp_skip[xo + q]) continue;
        const unsigned long long kk = ord_key(t.exp_score[xo + q]);
        const bool after = first || kk < pk || (kk == pk && q > pg);
        if (after && (bg == INV || kk > bk || (kk == bk && q < bg))) { bk = kk; bg = q; }
      }
      if (bg == INV) break;
      first = false;
      pk = bk; pg = bg;
      const uint64_t v = t.exp_link ? t.exp_link[xo + bg] : 0ull;
      const uint32_t v32 = t.exp_node[xo + bg];
      const int d = t.exp_link ? (int)bpw_d(v) : (int)bp_d(v32);
      const int r = t.exp_link ? (int)bpw_rank(v) : (int)bp_rank(v32);
      const int node = t.exp_link ? (int)bpw_node(v) : (int)bp_node(v32);
      const Entry& h = ent[(int64_t)(e - d) * k + r];
      const Cand c = cand_at(B, p, nbase, (uint32_t)node, d);
      Entry ne;
      ne.score = t.exp_score[xo + bg]; ne.f6 = c.f6;
      ne.jword = c.word; ne.jmorph = c.morph; ne.jtag = c.tag; ne.jmask = c.mask;
      ne.iword = h.jword; ne.imorph = h.jmorph; ne.imask = h.jmask | F_WI;
      ne.depth = h.depth + 1;
      ne.jnode = (uint32_t)node; ne.pad0 = h.jnode; ne.pad1 = ne.pad2 = 0;   // pad0: wi's local node
      ent[(int64_t)e * k + kept] = ne;
      t.beam_gen[(po + e) * k + kept] = bg;
    }
    t.beam_count[po + e] = kept;
  }
}
}  // namespace

namespace lt {
hipError_t launch_trace(const DecodeParams& p, const TraceParams& t, hipStream_t st) {
  const int blocks = (p.n_sent + 63) / 64;
  if (blocks == 0) return hipSuccess;
  if (p.narrow) hipLaunchKernelGGL(lt_trace_k<true>, dim3(blocks), dim3(64), 0, st, p, t);
  else hipLaunchKernelGGL(lt_trace_k<false>, dim3(blocks), dim3(64), 0, st, p, t);
  return hipGetLastError();
}
}  // namespace lt

namespace {
// ===========================================================================
// General kernel (lt_beam_wide): max_len > 8 or beam_size > 256 -- what the
// tuned kernels' layouts (8 span slots, 3-bit span and 8-bit rank fields,
// LDS rings) do not hold.  One thread per sentence, grid-stride over the
// piece; the beams of the last S + 1 end positions and a selection heap of k
// items live in the thread's block of HBM scratch.  The reference loops
// (beam.py:27-48: b ascending, hypothesis rank, candidate) run literally and
// score with the decoders' own code.  Beam.append (beam.py:83-86, stable top
// k by score) is a heap on the order (score desc, generation asc) whose root
// is the worst item kept: expansions arrive in generation order, so a new one
// displaces the root only with a strictly larger score; heap sort then puts
// the k kept best first.  Backpointers are two words (bpw_pack).
// ===========================================================================
struct WItem {
  unsigned long long key;                      // ord_key(score)
  uint32_t g, node, d, r;                      // generation index, local node, span, parent rank
};
static_assert(sizeof(WItem) == WIDE_ITEM_BYTES, "wide heap item");
static_assert(sizeof(Entry) == WIDE_ENTRY_BYTES, "wide beam entry");

// a ranks after b in the stable order of Beam.append
__device__ __forceinline__ bool ranks_after(const WItem& a, const WItem& b) {
  return a.key < b.key || (a.key == b.key && a.g > b.g);
}
__device__ void wheap_down(WItem* H, int n, int i) {
  const WItem x = H[i];
  for (;;) {
    int c = 2 * i + 1;
    if (c >= n) break;
    if (c + 1 < n && ranks_after(H[c + 1], H[c])) ++c;
    if (!ranks_after(H[c], x)) break;
    H[i] = H[c];
    i = c;
  }
  H[i] = x;
}
__device__ void wheap_up(WItem* H, int i) {
  const WItem x = H[i];
  while (i > 0) {
    const int par = (i - 1) >> 1;
    if (!ranks_after(x, H[par])) break;
    H[i] = H[par];
    i = par;
  }
  H[i] = x;
}

template <bool NARROW, bool COUNT>
__global__ void __launch_bounds__(64) lt_beam_wide(DecodeParams p) {
  const int tid = (int)(blockIdx.x * 64 + threadIdx.x);
  if (tid >= p.wide_threads) return;
  const int S = p.span_slots, RW = S + 1, k = p.k;
  const int64_t bstride = p.bp_stride;
  const Bufs B = make_bufs(p);
  const Aux aux{nullptr, 0u, p.hk};             // class 3 from the table itself
  char* const blk = p.wide_scratch + (int64_t)tid * p.wide_block;
  Entry* const R = reinterpret_cast<Entry*>(blk);                     // [RW][k]
  int32_t* const cnt = reinterpret_cast<int32_t*>(blk + (int64_t)RW * k * WIDE_ENTRY_BYTES);
  WItem* const H = reinterpret_cast<WItem*>(reinterpret_cast<char*>(cnt) + (((int64_t)RW * 4 + 15) & ~(int64_t)15));
  Counts cn;
  for (int i = tid; i < p.n_sent; i += p.wide_threads) {
    const int s = p.order[i];
    const int n = p.sent_n[s];
    const uint32_t nbase = (uint32_t)p.node_off[s];
    const int32_t* const ssp = p.span_start + p.span_off[s];
    uint64_t* const bp = reinterpret_cast<uint64_t*>(p.bp + p.bp_off[s]);
    {
      const Cand b0 = load_cand(B, nbase);      // beam[0] = [BOS] (beam.py:21-23)
      Entry e0;
      e0.score = 0.0; e0.f6 = b0.f6;
      e0.jword = b0.word; e0.jmorph = b0.morph; e0.jtag = b0.tag; e0.jmask = b0.mask;
      e0.iword = 0; e0.imorph = 0; e0.imask = 0; e0.depth = 0;
      e0.jnode = 0; e0.pad0 = e0.pad1 = e0.pad2 = 0;
      R[0] = e0;
      cnt[0] = 1;
    }
    for (int e = 1; e <= n; ++e) {
      const int dmax = min(e, p.max_len);
      int hn = 0;
      uint32_t g = 0;
      for (int j = S - dmax; j < S; ++j) {      // span j: d = S - j, b = e - d ascending
        const int d = S - j, b = e - d;
        const int lo = ssp[(int64_t)(e - 1) * S + j], hi = ssp[(int64_t)(e - 1) * S + j + 1];
        const bool imp = lo == hi && p.n_unk;   // the span's implicit Unknown (beam.py:36-38)
        const int hi1 = imp ? lo + 1 : hi;
        const int bs = b % RW;
        const int nb = cnt[bs];
        for (int r = 0; r < nb; ++r) {
          const Hyp h = read_entry(R[(int64_t)bs * k + r]);
          for (int node = lo; node < hi1; ++node, ++g) {
            const uint32_t nd = imp ? UNK_LOCAL : (uint32_t)node;
            const Cand c = cand_at(B, p, nbase, nd, d);
            if ((h.jmask & F_UNK) && (c.mask & F_UNK) && (d < dmax)) continue;    // beam.py:43-45
            if (COUNT) ++cn.exp;
            double sc;
            if (p.n_xtri) {                     // several trigram terms (score_funcs.py:50-54)
              double tris[MAX_TRI];
              trigram_terms<NARROW, COUNT>(p, B, h, c, nbase + (uint32_t)node, nbase + h.jnode, nbase + h.inode, cn,
                                           aux, tris);
              sc = h.score + increment_x(p, c, tris, nbase + (uint32_t)node, h.jnode);   // beam.py:115
            } else {
              const double tri = p.has_tri ? trigram<NARROW, COUNT>(B, p.slots, p.seed, h, c, cn, aux) : 0.0;
              sc = h.score + increment(p, c, tri, nbase + (uint32_t)node, h.jnode, imp ? d : 0);   // beam.py:115
            }
            const WItem it{ord_key(sc), g, nd, (uint32_t)d, (uint32_t)r};
            if (hn < k) {
              H[hn] = it;
              wheap_up(H, hn);
              ++hn;
            } else if (it.key > H[0].key) {
              H[0] = it;
              wheap_down(H, k, 0);
            }
          }
        }
      }
      for (int m = hn - 1; m > 0; --m) {        // heap sort: best first
        const WItem t = H[0];
        H[0] = H[m];
        H[m] = t;
        wheap_down(H, m, 0);
      }
      const int es = e % RW;                    // not the slot of any b in [e - S, e - 1]
      for (int t = 0; t < hn; ++t) {
        const WItem it = H[t];
        const Entry& h = R[(int64_t)((e - (int)it.d) % RW) * k + it.r];
        const Cand c = cand_at(B, p, nbase, it.node, (int)it.d);
        Entry ne;
        ne.score = ord_score(it.key); ne.f6 = c.f6;
        ne.jword = c.word; ne.jmorph = c.morph; ne.jtag = c.tag; ne.jmask = c.mask;
        ne.iword = h.jword; ne.imorph = h.jmorph; ne.imask = h.jmask | F_WI;
        ne.depth = h.depth + 1;
        ne.jnode = it.node; ne.pad0 = h.jnode; ne.pad1 = ne.pad2 = 0;     // pad0: wi's local node
        R[(int64_t)es * k + t] = ne;
        bp[(int64_t)e * bstride + t] = bpw_pack(it.node, it.d, it.r);
      }
      cnt[es] = hn;
    }
    // matures = beam[n] + EOS (beam.py:59-61)
    const int nm = cnt[n % RW];
    p.out_count[s] = nm;
    for (int t = 0; t < k; ++t) {
      const int64_t o = (int64_t)s * k + t;
      int32_t* codes = p.out_codes + (int64_t)k * p.cum_n[s] + (int64_t)t * n;
      if (t >= nm) {                            // unused mature slots read as empty
        p.out_score[o] = 0.0;
        p.out_len[o] = 0;
        for (int j = 0; j < n; ++j) codes[j] = -1;
        continue;
      }
      const Entry& f = R[(int64_t)(n % RW) * k + t];
      p.out_score[o] = f.score + 0.0;
      p.out_len[o] = (int32_t)f.depth;
      int pos = n;
      uint32_t rank = (uint32_t)t;
      for (int step = min((int)f.depth, n) - 1; step >= 0 && pos > 0; --step) {   // (bounds: lt_viterbi_pk)
        const uint64_t v = bp[(int64_t)pos * bstride + rank];
        codes[step] = path_code(bpw_node(v), pos, (int)bpw_d(v), S);
        pos -= (int)bpw_d(v);
        rank = min(bpw_rank(v), (uint32_t)k - 1u);
      }
      for (int j = (int)f.depth; j < n; ++j) codes[j] = -1;      // padded layout
    }
  }
  if (COUNT) {                                  // lt_count_ops: one thread's sentences
    atomicAdd(p.counters + 0, cn.exp);
    atomicAdd(p.counters + 1, cn.tup);
    atomicAdd(p.counters + 2, cn.probe);
    atomicAdd(p.counters + 3, cn.load);
  }
}
}  // namespace

namespace lt {
hipError_t launch_wide(const DecodeParams& p, hipStream_t st, bool count, hipEvent_t e0, hipEvent_t e1) {
  const int blocks = (p.wide_threads + 63) / 64;
  if (p.n_sent == 0 || blocks == 0) {
    hipError_t e = e0 ? hipEventRecord(e0, st) : hipSuccess;
    if (e == hipSuccess && e1) e = hipEventRecord(e1, st);
    return e;
  }
  if (p.narrow) {
    if (count) hipExtLaunchKernelGGL((lt_beam_wide<true, true>), dim3(blocks), dim3(64), 0, st, e0, e1, 0, p);
    else hipExtLaunchKernelGGL((lt_beam_wide<true, false>), dim3(blocks), dim3(64), 0, st, e0, e1, 0, p);
  } else {
    if (count) hipExtLaunchKernelGGL((lt_beam_wide<false, true>), dim3(blocks), dim3(64), 0, st, e0, e1, 0, p);
    else hipExtLaunchKernelGGL((lt_beam_wide<false, false>), dim3(blocks), dim3(64), 0, st, e0, e1, 0, p);
  }
  return hipGetLastError();
}
}  // namespace lt

// ---------------------------------------------------------------------------
// the flag-free copy of a feature table (lt_model.d_plain)
// ---------------------------------------------------------------------------
namespace {
__global__ __launch_bounds__(256) void lt_strip_flags_k(uint4* __restrict__ dst, const uint4* __restrict__ src,
                                                        int64_t n16, uint32_t hi_mask, uint32_t w_mask) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (int64_t)gridDim.x * 256) {
    uint4 v = src[i];
    v.y &= hi_mask;           // narrow slot: key high word (bit 63)
    v.w &= w_mask;            // wide slot, first 16 B: cls1 (bit 31); second 16 B: coef / pad untouched
    dst[i] = v;
  }
}
}  // namespace

namespace lt {
hipError_t launch_strip_flags(void* dst, const void* src, int64_t bytes, bool narrow, hipStream_t st) {
  const int64_t n16 = bytes / 16;
  if (n16 <= 0) return hipSuccess;
  const int blocks = (int)std::min<int64_t>((n16 + 255) / 256, 4096);
  if (narrow) {
    hipLaunchKernelGGL(lt_strip_flags_k, dim3(blocks), dim3(256), 0, st, (uint4*)dst, (const uint4*)src, n16,
                       ~(FLAG_N >> 32) & 0xFFFFFFFFu, 0xFFFFFFFFu);
    return hipGetLastError();
  }
  // wide slots are 32 B: even 16 B chunks hold {a, b, c, cls1}; odd ones coef + pad
  hipLaunchKernelGGL(lt_strip_flags_k, dim3(blocks), dim3(256), 0, st, (uint4*)dst, (const uint4*)src, n16,
                     0xFFFFFFFFu, ~FLAG_W);
  return hipGetLastError();
}
}  // namespace lt
