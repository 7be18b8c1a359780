// lt_handles.h -- definitions of the opaque C-ABI handles shared by the
// host-side translation units of liblt.so (lt_capi.cpp, lt_comm.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <mutex>
#include <vector>

#include "lt_common.h"

// One batch's device buffers (one hipMalloc) and pinned result buffers (one
// hipHostMalloc), carved into the lt_batch pointers.  lt_batch_destroy hands
// a small arena back to its context (lt_ctx::spare) for the next batch that
// fits: a sentence-at-a-time caller (Tagger.tag) then allocates and frees
// nothing per call (each hipFree / hipHostFree synchronises the device).
struct lt_arena {
  char* d = nullptr;
  size_t d_bytes = 0;
  char* h = nullptr;
  size_t h_bytes = 0;
};

struct lt_ctx {
  int device = 0;
  hipStream_t stream = nullptr;    // decodes, result copies, gathers
  hipStream_t ustream = nullptr;   // lt_batch_create's uploads (a pipeline's upload
                                   // thread does not queue behind the decodes)
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  unsigned long long* d_counters = nullptr;
  std::mutex mu;                   // spare (batches are created and destroyed on several threads)
  std::vector<lt_arena> spare;     // arenas of destroyed batches, kept for reuse
};

struct lt_batch {
  lt_ctx* ctx = nullptr;
  int32_t n_sent = 0, max_len = 8, n_post = 0, has_tri = 0, max_k = 1;
  int64_t n_nodes = 0, n_span = 0, total_chars = 0, bp_entries = 0;
  int last_k = 0;
  // device inputs
  int32_t *d_order = nullptr, *d_sent_n = nullptr, *d_span_start = nullptr;
  int64_t *d_node_off = nullptr, *d_span_off = nullptr, *d_bp_off = nullptr, *d_cum_n = nullptr;
  lt::NodeRec* d_nodes = nullptr;
  double* d_post = nullptr;
  // scratch + device results (sized for max_k)
  uint32_t* d_bp = nullptr;
  int32_t *d_count = nullptr, *d_len = nullptr, *d_codes = nullptr;
  double* d_score = nullptr;
  // pinned host results
  int32_t *h_count = nullptr, *h_len = nullptr, *h_codes = nullptr;
  double* h_score = nullptr;
  // component frequencies of the batch's nodes (ids < 2^20) and the hot table
  // built for the last model decoded with this batch
  std::vector<uint32_t> f_word, f_tag, f_morph;
  uint64_t hot_uid = 0;      // lt_model::uid the hot table was built for (0: none)
  lt::SlotN* d_hot = nullptr;
  lt_arena arena;
};
