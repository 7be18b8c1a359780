// lt_common.h -- definitions shared by the HIP kernels and the host library.
//
// Node mask bits must match lattice_based_tagger_amd/lowering.py.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define LT_HD __host__ __device__ __forceinline__
#else
#define LT_HD static inline
#endif

namespace lt {

// -- node pre-filter bits: "component occurs at this key slot" ------------
// as wk (the appended node)
constexpr uint32_t K0B = 1u << 0, K0C = 1u << 1, K1B = 1u << 2, K2B = 1u << 3,
                   K2C = 1u << 4, K3B = 1u << 5, K7C = 1u << 6, K8B = 1u << 7;
// as wj (the hypothesis' last node)
constexpr uint32_t J0A = 1u << 8, J1A = 1u << 9, J2A = 1u << 10, J3A = 1u << 11,
                   J7B = 1u << 12, J8A = 1u << 13;
// as wi (the hypothesis' second-last node)
constexpr uint32_t I7A = 1u << 14, I8A = 1u << 15;
// flags
constexpr uint32_t F_UNK = 1u << 16;   // tag0 == 'Unknown'
constexpr uint32_t F_CTX = 1u << 17;   // tag0 in {Noun, Adverb, Adjective, Verb}
constexpr uint32_t F_HAS4 = 1u << 18;
constexpr uint32_t F_HAS5 = 1u << 19;
constexpr uint32_t F_HAS6 = 1u << 20;
constexpr uint32_t FLAG_BITS = 0x1F0000u;
// set by the library on its device copy of the mask: span length d-1 of the
// node (bits 21-23), the pair index (bits 24-30, PX_SHIFT below); bit 31
// marks "wi exists" in hypothesis entries.
constexpr int D_SHIFT = 21;
constexpr uint32_t D_MASK = 7u << D_SHIFT;
constexpr uint32_t F_WI = 1u << 31;

// -- device node mask (NodeRec.mask) ----------------------------------------
// The library re-encodes the API mask above per role, so that the probes an
// expansion needs are one AND of the candidate's and the hypothesis' bits.
// Probe q = 0..5 is feature class 0, 1, 2, 3, 7, 8 (feature.py:95-119).
//   bits 0-5   DK: probe q can be present with this node as wk
//              (q0 K0B&K0C, q1 K1B, q2 K2B&K2C, q3 K3B, q4 K7C, q5 K8B&ctx)
//   bits 6-11  DJ: ... as wj (q0 J0A, q1 J1A, q2 J2A, q3 J3A, q4 J7B,
//              q5 J8A&ctx -- class 8 from (wj, wk))
//   bit 12     DJ_NCTX: tag0 not in C (class 8 then comes from (wi, wk))
//   bit 13     DI_7: as wi of class 7 (I7A); bit 14 DI_8: as wi of class 8 (I8A&ctx)
//   bits 16-20 the API flags (F_UNK, F_CTX, F_HAS4, F_HAS5, F_HAS6)
//   bits 21-23 span length d-1 (D_SHIFT); bits 24-30 the class-4/6 pair
//   index (PX_SHIFT, NodeRec); bit 31 F_WI (hypothesis entries)
constexpr int DJ_SHIFT = 6;
constexpr uint32_t DQ_ALL = 0x3Fu;
constexpr uint32_t DJ_NCTX = 1u << 12, DI_7 = 1u << 13, DI_8 = 1u << 14;
LT_HD uint32_t device_mask(uint32_t m) {
  const uint32_t ctx = (m & F_CTX) ? 1u : 0u;
  const auto b = [m](uint32_t bit) -> uint32_t { return (m & bit) ? 1u : 0u; };
  uint32_t d = 0;
  d |= (b(K0B) & b(K0C)) << 0 | b(K1B) << 1 | (b(K2B) & b(K2C)) << 2 | b(K3B) << 3 | b(K7C) << 4 |
       (b(K8B) & ctx) << 5;
  d |= (b(J0A) << 0 | b(J1A) << 1 | b(J2A) << 2 | b(J3A) << 3 | b(J7B) << 4 | (b(J8A) & ctx) << 5) << DJ_SHIFT;
  d |= (ctx ^ 1u) << 12 | b(I7A) << 13 | (b(I8A) & ctx) << 14;
  return d | (m & FLAG_BITS);
}
// The hypothesis' half of the probe bits: wj's DJ bits, class 7 only with a
// wi that can take part, class 8 from (wj, wk) or else (wi, wk).  `wi` = the
// device mask of wi (its DI bits used), `has_i` = wi exists.
LT_HD uint32_t hyp_probe_bits(uint32_t wj, uint32_t wi, bool has_i) {
  const uint32_t i7 = has_i ? (wi >> 13) & 1u : 0u, i8 = has_i ? (wi >> 14) & 1u : 0u;
  return ((wj >> DJ_SHIFT) & 0xFu) | ((((wj >> 10) & 1u) & i7) << 4) |
         ((((wj >> 11) & 1u) | (((wj >> 12) & 1u) & i8)) << 5);
}

// several trigram scorers (lattice_decode.h LT_XTRI_CLASS_STRIDE / LT_MAX_TRI):
// scorer t's key classes + XTRI_CLASS_STRIDE * t
constexpr int XTRI_CLASS_STRIDE = 16;
constexpr int MAX_TRI = 8;

constexpr int MAX_SPAN = 8;
constexpr int RING = MAX_SPAN + 1;     // frontier positions e-8 .. e
// span slots per end position of a batch with this max_len: 8 (the tuned
// kernels' layout) up to max_len 8, else max_len (the general kernel)
LT_HD int span_slots(int max_len) { return max_len <= MAX_SPAN ? MAX_SPAN : max_len; }

// -- feature hash table ----------------------------------------------------
// Narrow slot (16 B): exact 64-bit key c3<<60 | a<<40 | b<<20 | c (c3 = the
// class in 3 bits, cls_code), valid when every interned id is < 2^20; bit 63
// is the slot's overflow flag (below).  key 0 = empty (ids are >= 1).
constexpr int NARROW_ID_BITS = 20;
struct alignas(16) SlotN {
  uint64_t key;
  double coef;
};
// Wide slot (32 B): {a, b, c, class+1 | overflow flag in bit 31}; 0 = empty.
struct alignas(32) SlotW {
  uint32_t a, b, c, cls1;
  double coef;
  uint64_t pad;
};

// Overflow flag ("primary first" cuckoo): every key lives in one of its two
// candidate slots i1 (primary) / i2 (secondary), and slot i1 carries the flag
// iff some key whose primary is i1 lives at its secondary.  A lookup loads i1;
// only on a miss at a flagged slot does it load i2 -- about 1.1 loads per
// probe instead of 2 (the probes are bound by random cache-line requests).
constexpr uint64_t FLAG_N = 1ull << 63;
constexpr uint32_t FLAG_W = 1u << 31;
LT_HD uint32_t cls_code(uint32_t cls) { return cls == 8 ? 4u : cls; }   // {0,1,2,3,7,8} -> 3 bits
LT_HD uint64_t narrow_key(uint32_t a, uint32_t b, uint32_t c, uint32_t cls) {
  return ((uint64_t)cls_code(cls) << 60) | ((uint64_t)a << 40) | ((uint64_t)b << 20) | (uint64_t)c;
}

// Cuckoo hashing: every key lives in one of its two candidate slots, so a
// lookup is exactly two independent loads (no probe chains).  Identical on
// host and device.
//
// Two independent key mixes (base1, base2), each avalanched with its own
// seed, give the two candidate slots; a key set can only defeat the build by
// a triple collision of the full 64-bit (base1, base2) pair.  Narrow tables
// (ids < 2^20) mix with full-rate 24-bit multiplies (v_mul_u32_u24); wide
// tables with 32-bit multiplies.
LT_HD uint32_t mul24(uint32_t x, uint32_t k) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __umul24(x, k);                         // v_mul_u32_u24: full rate
#else
  return (x & 0xFFFFFFu) * (k & 0xFFFFFFu);
#endif
}
struct KeyBase {
  uint32_t b1, b2;
};
template <bool NARROW>
LT_HD KeyBase key_base(uint32_t a, uint32_t b, uint32_t c, uint32_t cls) {
  KeyBase k;
  if (NARROW) {
    k.b1 = mul24(a, 0x9E3779u) ^ mul24(b, 0x85EBCBu) ^ mul24(c, 0xC2B2AFu) ^ (cls * 0x27D4EB2Fu);
    k.b2 = mul24(a, 0x7FEB35u) ^ mul24(b, 0x846CA7u) ^ mul24(c, 0xD35A2Du) ^ (cls * 0x165667B1u);
  } else {
    k.b1 = (a * 0x9E3779B1u) ^ (b * 0x85EBCA77u) ^ (c * 0xC2B2AE3Du) ^ (cls * 0x27D4EB2Fu);
    k.b2 = (a * 0x7FEB352Du) ^ (b * 0x846CA68Bu) ^ (c * 0xD35A2D97u) ^ (cls * 0x165667B1u);
  }
  return k;
}
LT_HD uint32_t slot_of(uint32_t h, uint32_t slots) {
  return (uint32_t)(((uint64_t)h * slots) >> 32);
}
LT_HD uint32_t mix1(uint32_t h) {
  h ^= h >> 16;
  h *= 0x85EBCA6Bu;
  h ^= h >> 13;
  return h;
}
LT_HD void cuckoo_slots(KeyBase kb, uint32_t seed, uint32_t slots, uint32_t& i1, uint32_t& i2) {
  i1 = slot_of(mix1(kb.b1 ^ seed), slots);
  i2 = slot_of(mix1(kb.b2 ^ (seed * 0x9E3779B1u + 0x632BE5ABu)), slots);
}

// Narrow tables (ids < 2^20): one key mix, both slots from it.  Every
// integer multiply costs about three simple VALU operations on gfx950
// (tools/valu_rate.hip: v_mul_u32_u24, v_mul_lo_u32 and v_mul_hi_u32 alike),
// and the beam kernels are VALU-bound, so a lookup spends four multiplies:
//   x  = mul24(a,Ka) ^ mul24(b,Kb) ^ mul24(c,Kc) ^ cls*Ks
//   i1 = x >> (32 - log2 slots)
//   i2 = ((x ^ (x >> 16)) * K2) >> (32 - log2 slots)
// on a power-of-two table (load factor 0.225-0.45).  Keys with equal x share
// both slots; a build that meets three of them reseeds, which changes every
// constant.
//
// Line groups (HASH_VERSION 5): a class whose key holds one tag component
// next to its words -- 0 (w_j, w_k, t_k), 1 (w_j, t_k), 2 (t_j, w_k, t_k),
// 3 (t_j, t_k) -- leaves that "sub" component out of x and takes its low
// four bits as the primary slot inside an aligned group of GROUP = 16 slots
// (two 128 B lines):
//   i1 = (x >> s) & ~15 | (sub & 15),   i2 = ((x ^ (x >> 16) ^ sub) * K2) >> s
// so the keys of one word (or word + tag) with different tags share their
// lines, and a popular word's lines stay in L2 (tools/cache_model.py: the
// modelled L2 hit of the k=1 probe stream 0.58 -> 0.65, fewer loads per
// probe).  Classes 7 and 8 (three or two words) have no sub component.
#ifndef LT_LINE_GROUPS
#define LT_LINE_GROUPS 1                 // 0: the version-4 slot hash (A/B builds)
#endif
constexpr uint32_t HASH_VERSION = LT_LINE_GROUPS ? 5 : 4;   // 3: overflow flags, 3-bit class code;
                                                            // 4: one mix, 2^n slots; 5: line groups
constexpr uint32_t GROUP = 16;
LT_HD constexpr int sub_pos(uint32_t cls) {
  return !LT_LINE_GROUPS ? -1 : cls == 0 ? 2 : cls == 1 ? 1 : cls == 2 ? 0 : cls == 3 ? 1 : -1;
}
struct NarrowHash {
  uint32_t k1a, k1b, k1c, k1s, k2a, k2b, k2c, k2s;
};
LT_HD NarrowHash narrow_hash(uint32_t seed) {
  uint32_t x = seed;
  uint32_t v[8];
  for (int i = 0; i < 8; ++i) {
    x = x * 0x9E3779B1u + 0x7F4A7C15u;
    uint32_t y = x ^ (x >> 15);
    y *= 0x2C1B3C6Du;
    y ^= y >> 12;
    y *= 0x297A2D39u;
    y ^= y >> 15;
    v[i] = (i == 3 || i == 7 || i == 4) ? (y | 1u) : ((y & 0xFFFFFFu) | 0x800001u);
  }
  return NarrowHash{v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7]};
}
LT_HD uint32_t slot_shift(uint32_t slots) {            // slots = 2^n, 16 <= slots <= 2^31
#if defined(__HIP_DEVICE_COMPILE__)
  return 32u - (uint32_t)__builtin_ctz(slots);
#else
  uint32_t n = 0;
  while ((1u << n) < slots) ++n;
  return 32u - n;
#endif
}
LT_HD uint32_t narrow_mix(const NarrowHash& h, uint32_t a, uint32_t b, uint32_t c, uint32_t cls) {
  // (the products' high bits carry every bit of the ids below them: slot 1
  // takes the top bits as they are; the sub component stays out)
  const int sp = sub_pos(cls);
  return (sp == 0 ? 0u : mul24(a, h.k1a)) ^ (sp == 1 ? 0u : mul24(b, h.k1b)) ^
         (sp == 2 ? 0u : mul24(c, h.k1c)) ^ (cls * h.k1s);
}
LT_HD uint32_t narrow_sub(uint32_t a, uint32_t b, uint32_t c, uint32_t cls) {
  const int sp = sub_pos(cls);
  return sp == 0 ? a : sp == 1 ? b : sp == 2 ? c : 0u;
}
LT_HD uint32_t narrow_slot1(const NarrowHash& h, uint32_t a, uint32_t b, uint32_t c, uint32_t cls,
                            uint32_t slots) {
  const uint32_t i = narrow_mix(h, a, b, c, cls) >> slot_shift(slots);
  if (sub_pos(cls) < 0) return i;
  return (i & ~(GROUP - 1)) | (narrow_sub(a, b, c, cls) & (GROUP - 1));
}
LT_HD uint32_t narrow_slot2(const NarrowHash& h, uint32_t a, uint32_t b, uint32_t c, uint32_t cls,
                            uint32_t slots) {
  const uint32_t x = narrow_mix(h, a, b, c, cls);
  return ((x ^ (x >> 16) ^ narrow_sub(a, b, c, cls)) * h.k2a) >> slot_shift(slots);
}
LT_HD void narrow_slots(const NarrowHash& h, uint32_t a, uint32_t b, uint32_t c, uint32_t cls,
                        uint32_t slots, uint32_t& i1, uint32_t& i2) {
  i1 = narrow_slot1(h, a, b, c, cls, slots);
  i2 = narrow_slot2(h, a, b, c, cls, slots);
}
// Wide tables: the primary / secondary slot alone (as cuckoo_slots).
LT_HD uint32_t wide_slot1(uint32_t a, uint32_t b, uint32_t c, uint32_t cls, uint32_t seed, uint32_t slots) {
  return slot_of(mix1(((a * 0x9E3779B1u) ^ (b * 0x85EBCA77u) ^ (c * 0xC2B2AE3Du) ^ (cls * 0x27D4EB2Fu)) ^ seed),
                 slots);
}
LT_HD uint32_t wide_slot2(uint32_t a, uint32_t b, uint32_t c, uint32_t cls, uint32_t seed, uint32_t slots) {
  return slot_of(mix1(((a * 0x7FEB352Du) ^ (b * 0x846CA68Bu) ^ (c * 0xD35A2D97u) ^ (cls * 0x165667B1u)) ^
                      (seed * 0x9E3779B1u + 0x632BE5ABu)),
                 slots);
}

// Dense class-3 table: the (t_j, t_k) keys of a model whose class-3 tag values
// are few (<= D3_DIM) live in a D3_DIM x D3_DIM coefficient array, indexed by
// a multiplicative hash the library picks to be injective on those values.
// The node pre-filter bits (J3A / K3B) guarantee both tags of a needed probe
// are among them, so the slot needs no key check; absent pairs hold D3_ABSENT.
constexpr int D3_BITS = 5;
constexpr int D3_DIM = 1 << D3_BITS;
constexpr uint64_t D3_ABSENT = 0x7FF5A5A55A5A0001ull;     // a NaN payload
LT_HD uint32_t d3_index(uint32_t v, uint32_t mul) { return (v * mul) >> (32 - D3_BITS); }
// A multiplier 2^(27 - off) makes d3_index the bit window v[off, off + 5):
// the library tries those first (the interned tags are a short run of ids,
// so a window separates them), and the kernels take the window as one
// bit-field extract instead of a 32-bit multiply.  Its offset, or -1 for any
// other multiplier (the kernels then probe class 3 in the hashed table).
LT_HD int d3_window(uint32_t mul) {
  for (int off = 0; off <= 32 - D3_BITS; ++off)
    if (mul == (1u << (32 - D3_BITS - off))) return off;
  return -1;
}

// Device node record (AoS, 32 B = 2 x 16 B loads), built by the library from
// the SoA arrays of lt_batch_desc.  The node's class-4 and class-6
// coefficients (feature.py:100-104: (4, len) and (6, min(8, len)), functions
// of the length alone, so few distinct values per batch) are a pair in the
// batch's pair table: mask bits 24-30 (PX_SHIFT) hold its index; PX_ESC
// (a batch with more distinct pairs than the table holds) sends the node to
// its own entry of the batch's escape array (piece-global node index).
// Absent coefficients are -0.0 (the identity of a float64 sum).
struct alignas(16) NodeRec {
  uint32_t word, morph, tag, mask;
  double pre, f5;
};
constexpr int REC_CHUNKS = (int)(sizeof(NodeRec) / 16);   // 16 B chunks per record
struct alignas(16) F46 {
  double f4, f6;
};
constexpr int PX_SHIFT = 24;
constexpr uint32_t PX_MASK = 0x7Fu << PX_SHIFT;
constexpr uint32_t PX_ESC = 0x7Fu;                   // the node's pair is in the escape array
constexpr int MAX_PAIRS = (int)PX_ESC;               // table entries 0..126 (0: both absent)
LT_HD uint32_t rec_px(uint32_t mask) { return (mask & PX_MASK) >> PX_SHIFT; }

// Backpointer word: local node index (21 b) | span d-1 (3 b) | parent rank (8 b)
LT_HD uint32_t bp_pack(uint32_t node, uint32_t d, uint32_t r) {
  return (node << 11) | ((d - 1u) << 8) | r;
}
LT_HD uint32_t bp_node(uint32_t v) { return v >> 11; }
LT_HD uint32_t bp_d(uint32_t v) { return ((v >> 8) & 7u) + 1u; }
LT_HD uint32_t bp_rank(uint32_t v) { return v & 255u; }
constexpr int64_t MAX_LOCAL_NODES = (int64_t)1 << 21;     // nodes per sentence
// The node field of a backpointer (and of a decoder's local node) naming the
// implicit Unknown of the span instead of a node (lattice_decode.h n_unk):
// local nodes are < MAX_LOCAL_NODES - 1, so the all-ones value is free.
constexpr uint32_t UNK_LOCAL = (uint32_t)MAX_LOCAL_NODES - 1u;
// Result code of the implicit Unknown of span (e - d, e), S span slots per
// end position: -2 - (its entry in the sentence's span table).
LT_HD int32_t unk_code(int e, int d, int S) { return -2 - ((e - 1) * S + (S - d)); }
LT_HD int32_t path_code(uint32_t node, int e, int d, int S) {
  return node == UNK_LOCAL ? unk_code(e, d, S) : (int32_t)node;
}
// General-kernel backpointer (two words): local node (21 b) | span d-1 (21 b)
// | parent rank (22 b) -- spans and beams above the tuned kernels' 3 / 8 bits
LT_HD uint64_t bpw_pack(uint32_t node, uint32_t d, uint32_t r) {
  return (uint64_t)node | ((uint64_t)(d - 1u) << 21) | ((uint64_t)r << 42);
}
LT_HD uint32_t bpw_node(uint64_t v) { return (uint32_t)(v & 0x1FFFFFu); }
LT_HD uint32_t bpw_d(uint64_t v) { return (uint32_t)((v >> 21) & 0x1FFFFFu) + 1u; }
LT_HD uint32_t bpw_rank(uint64_t v) { return (uint32_t)(v >> 42); }

}  // namespace lt
