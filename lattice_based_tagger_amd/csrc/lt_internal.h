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
  const SlotN* hot;             // HOT_SLOTS-slot LDS hot table (narrow only) or NULL
  const double* d3;             // dense class-3 table (D3_DIM^2) or NULL
  uint32_t d3mul;
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
  const double* npost;
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
  uint32_t d3mul;
  int32_t n_paths;
  int64_t n_words;
  const NodeRec* words;         // AoS word records
  const int64_t* prev1;
  const int64_t* prev2;
  const int64_t* path_off;
  int32_t n_terms;
  const double* terms;
  int32_t trigram_pos;
  double* inc;                  // [n_words] scratch
  double* out;                  // [n_paths]
};
hipError_t launch_evaluate(const EvalParams& p, hipStream_t st);

int beam_template_for(int k);
const char* kernel_name_for(int k);
hipError_t launch_decode(const DecodeParams& p, hipStream_t st, bool count);

}  // namespace lt
