// lt_common.h -- definitions shared by the HIP kernels and the host library.
//
// Node mask bits must match lattice_based_tagger_amd/lowering.py.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
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
constexpr uint32_t F_WI = 1u << 31;    // (hypothesis entry only) wi exists
constexpr uint32_t FLAG_BITS = 0x1F0000u;

constexpr int MAX_SPAN = 8;
constexpr int RING = MAX_SPAN + 1;     // frontier positions e-8 .. e
constexpr uint32_t EMPTY = 0u;         // slot.cls1 of an empty slot

// One hash-table slot: key {a, b, c, class+1} + coefficient.  32 B, so a
// slot never straddles a 64 B line.
struct alignas(32) Slot {
  uint32_t a, b, c, cls1;
  double coef;
  uint64_t pad;
};

// 32-bit mix of the interned key.  Identical on host (table build) and
// device (probe).
LT_HD uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
LT_HD uint32_t key_hash(uint32_t a, uint32_t b, uint32_t c, uint32_t cls) {
  uint32_t h = cls * 0x27D4EB2Fu + 0x165667B1u;
  h ^= a * 0x9E3779B1u;
  h = rotl32(h, 13) * 0x85EBCA77u;
  h ^= b * 0xC2B2AE3Du;
  h = rotl32(h, 17) * 0x9E3779B1u;
  h ^= c * 0x85EBCA77u;
  // fmix32
  h ^= h >> 16; h *= 0x85EBCA6Bu;
  h ^= h >> 13; h *= 0xC2B2AE35u;
  h ^= h >> 16;
  return h;
}

// Backpointer word: local node index (24 b) | span d-1 (3 b) | parent rank (5 b)
LT_HD uint32_t bp_pack(uint32_t node, uint32_t d, uint32_t r) {
  return (node << 8) | ((d - 1u) << 5) | r;
}
LT_HD uint32_t bp_node(uint32_t v) { return v >> 8; }
LT_HD uint32_t bp_d(uint32_t v) { return ((v >> 5) & 7u) + 1u; }
LT_HD uint32_t bp_rank(uint32_t v) { return v & 31u; }
constexpr int64_t MAX_LOCAL_NODES = (int64_t)1 << 24;

}  // namespace lt
