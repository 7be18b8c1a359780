// lt_handles.h -- definitions of the opaque C-ABI handles shared by the
// host-side translation units of liblt.so (lt_capi.cpp, lt_comm.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <mutex>
#include <vector>

#include "lt_common.h"
#include "lt_internal.h"

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
  hipStream_t stream = nullptr;    // decodes, gather staging copies
  hipStream_t ustream = nullptr;   // lt_batch_create's uploads (a pipeline's upload
                                   // thread does not queue behind the decodes)
  hipStream_t cstream = nullptr;   // result copies to the host: the D2H of decode i
                                   // runs under decode i+1 (lt_result_fetch)
  // start / end events of the last KRING decode launches (lt_kernel_ms_recent)
  static constexpr int KRING = 64;
  hipEvent_t kev0[KRING] = {}, kev1[KRING] = {};
  int64_t n_launch = 0;            // timed decode launches (KRING index)
  int64_t n_serial = 0;            // every decode-kernel launch (result slot freshness)
  unsigned long long* d_counters = nullptr;
  char* d_wide = nullptr;          // lt_beam_wide scratch (grown on demand, decode stream only)
  size_t wide_bytes = 0;
  std::mutex mu;                   // spare (batches are created and destroyed on several threads)
  std::vector<lt_arena> spare;     // arenas of destroyed batches, kept for reuse
};

// One launch piece of a batch: sentences [s0, s0 + n_sent), its inputs with
// offsets rebased to the piece, its backpointers.
struct lt_piece {
  int32_t s0 = 0, n_sent = 0;
  int64_t node0 = 0, span0 = 0, chars0 = 0;      // first node / span entry / character
  int64_t n_nodes = 0, n_span = 0, bp_entries = 0;
  int32_t *d_order = nullptr, *d_sent_n = nullptr, *d_span_start = nullptr;
  int64_t *d_node_off = nullptr, *d_span_off = nullptr, *d_bp_off = nullptr, *d_cum_n = nullptr;
  lt::NodeRec* d_nodes = nullptr;
  double* d_post = nullptr;
  uint32_t* d_bp = nullptr;
  int64_t edge0 = 0, n_edges = 0;                // the piece's edge values (edge terms)
  // the k=1 lane schedule (arena memory sized at lt_batch_create; built on the
  // device by the fill kernel, lt_batch_create or the first beam-1 decode)
  uint32_t* d_sched = nullptr;                   // [sched_steps * 64]
  int64_t* d_wave_off = nullptr;                 // [waves + 1]
  uint32_t* d_place = nullptr;                   // [piece chars] k=1 placements (DecodeParams.k1_place)
  int64_t sched_steps = 0;
  int64_t* d_edge_base = nullptr;                // [n_nodes], rebased to the piece
  double* d_edge_val = nullptr;                  // [n_edge][n_edges]
  lt::F46* d_esc = nullptr;                      // [n_nodes] class-4/6 pairs of PX_ESC nodes (or none)
  // further trigram scorers (lt_batch_desc.n_xtri): [n_xtri][n_nodes], rebased to the piece
  uint32_t* d_xmask = nullptr;
  double *d_xf4 = nullptr, *d_xf5 = nullptr, *d_xf6 = nullptr;
};

struct lt_batch {
  lt_ctx* ctx = nullptr;
  int32_t n_sent = 0, max_len = 8, n_post = 0, has_tri = 0, max_k = 1;
  int32_t n_edge = 0, n_terms = 0;    // edge terms (lt_batch_desc.n_edge)
  int32_t n_xtri = 0;                  // further trigram terms (lt_batch_desc.n_xtri): general kernel
  uint64_t term_kinds = 0;
  int64_t n_nodes = 0, n_span = 0, total_chars = 0, bp_entries = 0;
  int inf_signs = 0;                  // +inf (1) / -inf (2) among the node score terms
  int last_k = 0;
  // implicit Unknown records (lt_batch_desc.n_unk): device AoS [n_unk] with
  // the span-length bits, post terms [n_post][n_unk]; shared by the pieces
  int32_t n_unk = 0;
  lt::NodeRec* d_unk = nullptr;
  double* d_unk_post = nullptr;
  // the class-4/6 pair table of the records (NodeRec, PX_SHIFT): [n_pairs]
  int32_t n_pairs = 0;
  lt::F46* d_pairs = nullptr;
  // device preparation (the k=1 lane schedules of the pieces): has_sched = the
  // batch has them (max_len <= 8; at create for max_k = 1, else at the first
  // beam-1 decode -- lazy_sched: then in buffers of their own, not the
  // arena); prep_done = the fill kernels are queued
  // prep_fused = the last fill ran inside the beam-1 decode (p.k1_fill; no
  // prep events of its own)
  bool has_sched = false, prep_done = false, lazy_sched = false, prep_fused = false;
  double host_sched_ms = 0.0;          // lt_batch_create's host schedule pass (wall time)
  hipEvent_t prep_ev0 = nullptr, prep_ev1 = nullptr;   // around the last fill
  // device inputs, per launch piece (lt_batch_create: node records and
  // backpointers of a piece stay below 2^31 B)
  std::vector<lt_piece> pieces;
  int32_t* d_sent_n = nullptr;        // whole batch (result packing)
  int64_t* d_cum_n = nullptr;
  // device results (sized for max_k)
  // two result slots: decodes alternate between them, so the D2H of one
  // decode's results (lt_result_fetch, copy stream) overlaps the next decode
  struct Slot {
    int32_t *count = nullptr, *len = nullptr, *codes = nullptr;
    double* score = nullptr;
    void* slab = nullptr;             // the slot's results packed (lt_results.hip)
    int64_t packed_launch = -1;       // launch_serial of the decode the slab holds
  } res[2];
  int64_t launch_serial = -1;         // lt_ctx::n_serial of the last decode
  uint64_t slab_cap = 0;              // slab capacity at max_k (+ pack scratch behind it)
  char* h_slab = nullptr;             // pinned: the last lt_result_fetch_packed
  int cur = 1;                        // slot of the last decode (the first decode takes slot 0)
  hipEvent_t last_end = nullptr;      // end event of the last decode (a lt_ctx::kev1), or NULL
  // readers of result slot i on other streams (RD_COPY: the ctx copy stream,
  // RD_GATHER: a communicator's stream); a decode reusing slot i waits for them
  static constexpr int RD_COPY = 0, RD_GATHER = 1;
  hipEvent_t ev_rd[2][2] = {{nullptr, nullptr}, {nullptr, nullptr}};
  bool rd_pending[2][2] = {{false, false}, {false, false}};
  // the last decode's slot (what lt_gather_launch and lt_result_fetch read)
  int32_t *d_count = nullptr, *d_len = nullptr, *d_codes = nullptr;
  double* d_score = nullptr;
  // pinned host results
  int32_t *h_count = nullptr, *h_len = nullptr, *h_codes = nullptr;
  double* h_score = nullptr;
  lt_arena arena;
};

namespace lt {
// Bytes of a slab buffer for n_sent sentences, beam k, `chars` characters:
// the slab's capacity plus the packing scratch behind it.
uint64_t slab_alloc_bytes(int64_t n_sent, int k, int64_t chars);
// Stream `st` (another stream of b's ctx) waits until the last decode of b
// is complete, and starts reading its result slot: packs it into `slab`
// (slab_alloc_bytes(b->n_sent, b->last_k, b->total_chars) bytes) and records
// that `reader` (lt_batch::RD_*) is done with the slot at that point of st.
hipError_t pack_last_results_on(lt_batch* b, int reader, void* slab, hipStream_t st);
}  // namespace lt
