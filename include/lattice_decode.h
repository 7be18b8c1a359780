/*
 * lattice_decode.h -- C-ABI of the MI355X lattice decoder (liblt.so).
 *
 * The reference decoder is the pure-Python `beam_search(bindex, chars,
 * score_functions, beam_size=5, max_len=8)` (lattice_tagger/beam/beam.py:5-61)
 * driven by `Tagger.tag` (lattice_tagger/tagger/tagger.py:68-78) and scored by
 * the plugin composite `BeamScoreFunctions` (lattice_tagger/beam/score_funcs.py:18-54)
 * over the trigram schema of lattice_tagger/features/feature.py:76-121.
 * The reference has no FFI; this header is the boundary a ctypes binding of
 * that Python API binds to.  Every entry point below
 * cites the reference interface it replaces.
 *
 * Conventions: plain pointers + sizes, no C++ or torch types.  All host
 * buffers passed in are owned by the caller and only read (inputs) or written
 * (outputs) during the call; the library never frees them.  Device memory is
 * owned by the handles.  Functions return lt_status (0 = OK, < 0 = error);
 * lt_last_error() returns a thread-local message for the last failure.
 * A handle is not re-entrant: one thread at a time per lt_ctx, except that
 * lt_batch_create / lt_batch_destroy may run on another thread while that
 * ctx decodes (uploads go to the ctx's own upload stream; the cache of
 * recycled batch buffers is locked) -- a pipeline uploads batch i+1 while
 * batch i decodes.
 */
#ifndef LATTICE_DECODE_H
#define LATTICE_DECODE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LT_ABI_VERSION 6   /* 2: compact results (slabs), gathers of slabs;
                              3: any max_len / beam (general kernel), lt_trace.exp_link;
                              4: edge terms (lt_batch_desc.n_edge ...);
                              5: implicit Unknown candidates (lt_batch_desc.n_unk ...),
                                 negative path codes, lt_batch_reset_prep, lt_batch_prep_ms;
                              6: several trigram terms (lt_batch_desc.n_xtri ..., key
                                 classes + LT_XTRI_CLASS_STRIDE * t), lt_batch_prepare_k1,
                                 lt_batch_host_sched_ms */
/* Several trigram scorers in one composite (score_funcs.py:50-54 sums any
 * BeamScoreFunctions): scorer t's keys carry class + LT_XTRI_CLASS_STRIDE * t
 * in the one model; at most LT_MAX_TRI scorers. */
#define LT_XTRI_CLASS_STRIDE 16
#define LT_MAX_TRI 8
#define LT_MAX_SPAN 8      /* span slots per end position (reference max_len default, beam.py:5) */
#define LT_MAX_BEAM 256    /* largest beam_size of the tuned kernels */
/* Any other configuration -- max_len > 8 (span slots = max_len) or a beam
 * above LT_MAX_BEAM -- decodes on the general kernel (lt_beam_wide): beams up
 * to LT_MAX_BEAM_ANY, span lengths up to LT_MAX_LEN_ANY. */
#define LT_MAX_BEAM_ANY (1 << 20)
#define LT_MAX_LEN_ANY (1 << 20)

typedef int32_t lt_status;
enum {
  LT_OK = 0,
  LT_EINVAL = -1,        /* bad argument / malformed batch                  */
  LT_EHIP = -2,          /* HIP runtime error                               */
  LT_ENOMEM = -3,        /* host or device allocation failed                */
  LT_EUNSUPPORTED = -4,  /* configuration not compiled in (k, max_len)      */
  LT_ERCCL = -5          /* RCCL error                                      */
};

typedef struct lt_ctx lt_ctx;
typedef struct lt_model lt_model;
typedef struct lt_batch lt_batch;

/* ---- library ------------------------------------------------------------ */
int lt_abi_version(void);
/* The slot hash of this library's model tables (lt_model_image.hash_version
 * of the images it builds; an image of another version is refused). */
uint32_t lt_hash_version(void);
const char* lt_last_error(void);
/* Number of visible HIP devices (0 when no GPU). */
int lt_device_count(void);

/* ---- context: one device, a decode stream, a copy stream ---------------- */
lt_status lt_ctx_create(int device, lt_ctx** out);
lt_status lt_ctx_destroy(lt_ctx* ctx);
/* Waits for everything queued on the ctx (decodes and result copies). */
lt_status lt_sync(lt_ctx* ctx);

/* ---- model: the lowered scorer composite ---------------------------------
 * Replaces the per-expansion call `score_functions(immature, expand)`
 * (beam.py:47 -> score_funcs.py:50-54).  Holds the probed trigram feature
 * classes 0,1,2,3,7,8 (score_funcs.py:137-144, feature.py:95-119) as an
 * open-addressing hash table keyed by interned component ids.
 * keys[4*i .. 4*i+3] = {a, b, c, class}; ids are >= 1, unused components 0.
 */
typedef struct {
  int64_t n_keys;
  const uint32_t* keys;   /* [n_keys][4] */
  const double* coefs;    /* [n_keys]  coefficient of each key (float64) */
} lt_model_desc;

lt_status lt_model_create(lt_ctx* ctx, const lt_model_desc* desc, lt_model** out);

/* ---- model images (SURVEY §8(f) model pack format) -------------------------
 * The host-side part of lt_model_create -- validated keys, built cuckoo table,
 * dense class-3 table -- as a self-contained image that can be written to a
 * file once (after scan_features, features/utils.py:50-55) and uploaded on
 * later runs without rebuilding (replaces the per-run set_encoder work,
 * beam/score_funcs.py:106-125).  lt_image_build needs no GPU. */
typedef struct lt_image lt_image;
typedef struct {
  uint32_t hash_version; /* slot hash of the library that built the image */
  int32_t narrow;        /* 1: 16 B slots {key64, coef}; 0: 32 B slots */
  uint32_t seed;         /* cuckoo hash seed */
  int64_t slots;         /* table slots */
  const void* table;     /* slots * (narrow ? 16 : 32) bytes */
  int64_t table_bytes;
  uint32_t d3mul;        /* dense class-3 index multiplier; 0 = none */
  const double* d3;      /* 32 x 32 float64, or NULL */
} lt_model_image;
lt_status lt_image_build(const lt_model_desc* desc, lt_image** out);
/* Pointers into the image (valid until lt_image_destroy). */
lt_status lt_image_view(const lt_image* image, lt_model_image* view);
lt_status lt_image_destroy(lt_image* image);
/* Upload an image (e.g. memory-mapped from a model file); no table build. */
lt_status lt_model_create_from_image(lt_ctx* ctx, const lt_model_image* image, lt_model** out);
lt_status lt_model_destroy(lt_model* model);
/* Hash-table slots allocated on the device (32 B each). */
int64_t lt_model_slots(const lt_model* model);

/* ---- batch: packed lattices ----------------------------------------------
 * Replaces the `bindex` / `chars` arguments of beam_search (beam.py:5,
 * consumed at beam.py:25-38).  Layout: DESIGN.md "Data layout in HBM".
 *   sentence s owns local nodes [sent_node_off[s], sent_node_off[s+1]) (node 0 = BOS)
 *   and span entries [sent_span_off[s], sent_span_off[s+1]) (= S*n_s + 1 entries,
 *   S = 8 for max_len <= 8, else S = max_len);
 *   span_start[sent_span_off[s] + (e-1)*S + (S-d)] = local index of the first
 *   candidate of span (e-d, e).
 */
typedef struct {
  int32_t n_sent;
  int32_t max_len;        /* 1..LT_MAX_LEN_ANY (beam_search max_len, beam.py:5,30) */
  int32_t n_post;         /* node-local terms that follow the trigram term */
  int32_t has_trigram;
  int64_t n_nodes;
  int64_t n_span;         /* = sent_span_off[n_sent] */
  const int32_t* sent_n;          /* [n_sent] characters per sentence */
  const int64_t* sent_node_off;   /* [n_sent+1] */
  const int64_t* sent_span_off;   /* [n_sent+1] */
  const int32_t* span_start;      /* [n_span] */
  const int32_t* node_word;       /* [n_nodes] interned ids (0 = in no key) */
  const int32_t* node_morph0;
  const int32_t* node_tag;
  const uint32_t* node_mask;      /* pre-filter bits 0-15, flags 16-20 */
  const double* node_pre;         /* node-local terms before the trigram, summed */
  const double* node_f4;          /* coef of (4, len)                 if flag */
  const double* node_f5;          /* coef of (5, word, tag0, is_l)    if flag */
  const double* node_f6;          /* coef of (6, min(8, len))         if flag */
  const double* node_post;        /* [n_post][n_nodes] or NULL */
  /* Edge terms: scorers of (wj, wk) -- BeamScoreFunction plugins that read
   * only seq.sequences[-1] and word_k (score_funcs.py:7-15, 50-54), one value
   * per lattice edge.  n_edge = 0: none (the fields below are ignored and the
   * increment is node_pre + trigram + node_post..., as before).  Otherwise
   * the increment (score_funcs.py:50-54) is ((node_pre + t_0) + t_1) + ...
   * over the n_terms terms that follow the leading node-local ones, in
   * constructor order; term_kinds holds 2 bits per term: 0 the trigram,
   * 1 the next node_post row, 2 the next edge_val row.  The predecessors
   * of a node of span (b, e) are the local nodes of end position b (BOS for
   * b = 0): the value of predecessor local node j is
   * edge_val[t * n_edges + node_edge_base[node] + j], inside its sentence's
   * block [sent_edge_off[s], sent_edge_off[s+1]). */
  int32_t n_edge;
  int32_t n_terms;                /* <= 32 */
  uint64_t term_kinds;
  int64_t n_edges;
  const int64_t* sent_edge_off;   /* [n_sent+1] */
  const int64_t* node_edge_base;  /* [n_nodes] */
  const double* edge_val;         /* [n_edge][n_edges] */
  /* Implicit Unknown candidates (ABI 5).  beam_search synthesises one
   * Unknown word Word(chars[b:e], chars[b:e], None, 'Unknown', None, e-b, b, e,
   * False) for every span (b, e) inside the sentence and within max_len that
   * has no dictionary candidate (beam.py:33-38).  Most lattice spans are such
   * spans, and the record of a synthesised word whose surface occurs in no
   * key of the model depends on its length d = e-b alone.  With n_unk = S
   * (the span slots per end position) an in-range span may hold no node: it
   * then holds that implicit Unknown, whose record is entry d-1 of the unk_*
   * arrays (same meaning as the node_* arrays).  n_unk = 0: every in-range
   * span holds at least one node (the ABI 4 layout).  Not combinable with edge
   * terms (n_edge > 0).  An implicit Unknown on a decoded path is reported by
   * the negative code -2 - ((e-1)*S + (S-d)): its span entry in the
   * sentence's span table (lt_result.codes). */
  int32_t n_unk;
  const int32_t* unk_word;        /* [n_unk], entry d-1: span length d */
  const int32_t* unk_morph0;
  const int32_t* unk_tag;
  const uint32_t* unk_mask;
  const double* unk_pre;
  const double* unk_f4;
  const double* unk_f5;
  const double* unk_f6;
  const double* unk_post;         /* [n_post][n_unk] or NULL */
  /* Further trigram terms (ABI 6): the composite's trigram scorers 1..n_xtri
   * (the first is the has_trigram term above).  Each is a term of its own,
   * summed in numpy's order over its own features (score_funcs.py:137-144),
   * placed by term_kinds: the i-th trigram term (kind 0) is scorer i, so
   * n_terms / term_kinds are read whenever n_xtri > 0 (as with edge terms).
   * Per scorer t = 1..n_xtri and node: the pre-filter bits + flags (as
   * node_mask, under scorer t's features) and its class 4 / 5 / 6
   * coefficients, at [(t-1) * n_nodes + node].  The model's keys of scorer t
   * carry class + LT_XTRI_CLASS_STRIDE * t (a wide-slot model).  Such a batch
   * decodes on the general kernel; not combinable with implicit Unknowns
   * (n_unk > 0).  n_xtri = 0: one trigram term at most (ABI 5). */
  int32_t n_xtri;
  const uint32_t* xtri_mask;      /* [n_xtri][n_nodes] */
  const double* xtri_f4;          /* [n_xtri][n_nodes] */
  const double* xtri_f5;
  const double* xtri_f6;
} lt_batch_desc;

/* Copies the batch to the device (H2D) and allocates result buffers for
 * beams up to max_k.  Blocking.  The batch's device buffers are one
 * allocation and its pinned result buffers another; lt_batch_destroy keeps
 * up to two such pairs (each up to 1 GiB) in the ctx for later batches that
 * fit, so per-call decoding frees and allocates nothing.
 * Device preparation: the beam-1 decoder reads a lane schedule (which
 * candidate each lane scores at each step), a function of the lattice shapes
 * alone.  A batch created with max_k = 1 (and max_len <= LT_MAX_SPAN) gets
 * one: the schedule's steps and every (sentence, end position)'s placement
 * are computed here on the host (4 bytes per character, uploaded with the
 * batch), its memory is part of the batch's allocation, and its rows are
 * built on the device by a kernel on the upload stream (after
 * lt_batch_reset_prep: by the next beam-1 decode kernel itself, each of its
 * waves filling its own rows before decoding; environment LT_K1_FUSED_FILL=0:
 * by the fill kernel queued in front of it).  Neither blocks nor allocates.
 * A batch created for larger beams gets none here (no host work, no arena
 * bytes); its first beam-1 decode builds one: steps and placements computed
 * on the device, one host synchronisation, buffers of its own (freed with
 * the batch), the rows filled by that decode.  Candidates that the reference
 * skips for sure take no lane: the implicit Unknown of a span (b, e) past
 * b_min when end position b holds no explicit node (beam.py:43-45). */
lt_status lt_batch_create(lt_ctx* ctx, const lt_batch_desc* desc, int max_k, lt_batch** out);
lt_status lt_batch_destroy(lt_batch* batch);
/* Benchmark hook: forget the device preparation, so that the next beam-1
 * decode rebuilds it on the decode stream (a "fresh batch" step). */
lt_status lt_batch_reset_prep(lt_batch* batch);
/* Device time (ms, HIP events) of the last device preparation of the batch;
 * valid once that work is complete (after lt_sync).  0 when none ran as a
 * kernel of its own (also when the decode filled the schedule). */
lt_status lt_batch_prep_ms(lt_batch* batch, float* ms);
/* Bytes of the batch's device preparation (the lane schedules and their wave
 * offsets) -- what a beam-1 decode reads of them.  Not counted: the
 * per-character placements the fill reads (4 bytes per character), which are
 * uploaded with the batch (or, for a lazily prepared batch, live in a buffer
 * of their own). */
int64_t lt_batch_prep_bytes(const lt_batch* batch);
/* Wall time (ms) lt_batch_create spent computing the beam-1 schedule's steps
 * and placements on the host threads (0 for a batch created for larger
 * beams, whose schedule is computed on the device). */
double lt_batch_host_sched_ms(const lt_batch* batch);
/* Build the beam-1 device preparation of a batch created for larger beams
 * now, instead of at its first beam-1 decode: allocates, synchronises the
 * context stream once, and queues the schedule fill on it.  A pipeline calls
 * this off its launch path, so that no lt_decode_launch blocks.  No-op for a
 * batch that has one (or for max_len > LT_MAX_SPAN, decoded without).  Here
 * the rows are filled by the standalone kernel. */
lt_status lt_batch_prepare_k1(lt_batch* batch);
/* Total path-code slots of the results for beam k: k * sum_s n_s. */
int64_t lt_batch_code_slots(const lt_batch* batch, int k);
/* Kernel launches per decode of the batch: a batch of any size is decoded in
 * consecutive sentence pieces whose node records and backpointers each stay
 * below 2^31 B (32-bit buffer offsets in the kernels); all pieces write the
 * one result array. */
int32_t lt_batch_pieces(const lt_batch* batch);
/* Test hook: launch pieces of batches created afterwards hold at most
 * `bytes` of node records / backpointers (bytes < 1: the 2^31 - 1 default);
 * returns the previous limit.  Process-wide. */
int64_t lt_set_piece_bytes(int64_t bytes);

/* ---- decode ---------------------------------------------------------------
 * Replaces beam_search(bindex, chars, score_functions, beam_size=k, max_len)
 * (beam.py:5-61) for every sentence of the batch.  Asynchronous on the ctx
 * stream; results stay on the device until lt_result_fetch.
 */
lt_status lt_decode_launch(lt_ctx* ctx, const lt_model* model, lt_batch* batch, int k);
/* Device time of the last decode kernel (HIP events on the ctx stream), ms.
 * Valid after lt_sync. */
lt_status lt_last_kernel_ms(lt_ctx* ctx, float* ms);
/* Device times of the ctx's last min(n, 64) decode kernels, oldest first;
 * *got receives how many were written.  Valid after lt_sync. */
lt_status lt_kernel_ms_recent(lt_ctx* ctx, int n, float* ms, int* got);
/* Name of the HIP kernel lt_decode_launch runs for beam k (profiling:
 * matches the rocprofv3 kernel name prefix); NULL for an unsupported k. */
const char* lt_kernel_name(int k);

/* Results of beam_search's `matures` (beam.py:59-61), per sentence s:
 *   count[s]               number of matures (<= k)
 *   length[s*k + t]        words in mature t, excluding BOS/EOS
 *   score[s*k + t]         float64 path score (after the EOS `+ 0`)
 *   codes[k*off_s + t*n_s + j]  local node index of word j of mature t, or
 *                          -2 - x for the implicit Unknown of span entry x
 *                          (lt_batch_desc.n_unk; x = (e-1)*S + (S-d))
 *                          (off_s = sum_{s'<s} n_{s'}); slots j >= length are -1
 * Matures are ordered best first, ties by expansion order (beam.py:85). */
typedef struct {
  int32_t* count;    /* [n_sent] */
  int32_t* length;   /* [n_sent * k] */
  double* score;     /* [n_sent * k] */
  int32_t* codes;    /* [lt_batch_code_slots(batch, k)] */
} lt_result;

/* D2H of the last decode's results into library-owned pinned buffers.
 * Asynchronous: the copies run on the ctx's copy stream once the decode
 * stream has produced the results, so they overlap the next decode (a batch
 * keeps two device result slots and decodes alternate between them; a
 * decode reusing a slot whose copy is still queued waits for it on the
 * device).  Complete after lt_sync; the pinned buffers are overwritten by
 * the next fetch of the batch. */
lt_status lt_result_fetch(lt_ctx* ctx, lt_batch* batch);
/* Pointers to the pinned result buffers (valid until the next decode). */
lt_status lt_result_view(lt_batch* batch, lt_result* view);
/* ---- compact results ------------------------------------------------------
 * A path holds about 1/2.5 of its sentence's code slots, so results cross
 * PCIe (and xGMI, lt_gather_*) as a *slab*: a 32 B header {int32 n_sent,
 * int32 k, int64 n_codes, int64 bytes, int64 0}, then 16 B aligned sections
 * count int32[n_sent], length int32[n_sent*k], score f64[n_sent*k] (entries
 * t >= count[s] are 0) and codes int32[n_codes] -- the length[s*k+t] codes of
 * every mature t < count[s], sentence-major, best mature first.  The slab is
 * built by kernels on the device and only its used bytes are copied (the
 * size is read on the device; the host never waits for it). */
typedef struct {
  int32_t n_sent;
  int32_t k;
  int64_t n_codes;
  const int32_t* count;    /* [n_sent] */
  const int32_t* length;   /* [n_sent * k] */
  const double* score;     /* [n_sent * k] */
  const int32_t* codes;    /* [n_codes] */
} lt_packed_view;
/* As lt_result_fetch, for the slab: the packing kernels and the copy of the
 * used bytes into the batch's pinned slab both run on the ctx's copy stream
 * (after the decode, under the next one).  Complete after lt_sync;
 * overwritten by the next fetch. */
lt_status lt_result_fetch_packed(lt_ctx* ctx, lt_batch* batch);
/* View of the batch's pinned slab (after lt_result_fetch_packed + lt_sync). */
lt_status lt_result_view_packed(lt_batch* batch, lt_packed_view* view);
/* View of any slab in host memory of `bytes` bytes (checks the header). */
lt_status lt_slab_parse(const void* slab, uint64_t bytes, lt_packed_view* view);

/* Blocking convenience: launch + fetch + sync + copy into caller buffers. */
lt_status lt_decode(lt_ctx* ctx, const lt_model* model, lt_batch* batch, int k, lt_result* out);

/* Reference-algorithm operation counts of the batch for beam k (a separate
 * counting launch, not timed): expansions scored (beam.py:47) and candidate
 * feature tuples generated by trigram_encoder (feature.py:76-121); and the
 * kernel's own work: feature probes past the node pre-filter (LDS + table)
 * and the table slot loads they issued (primary, plus secondary at flagged
 * slots).  Every kernel has a counting variant, the general one included.
 * Any output pointer may be NULL. */
lt_status lt_count_ops(lt_ctx* ctx, const lt_model* model, lt_batch* batch, int k,
                       int64_t* expansions, int64_t* feature_tuples, int64_t* probes,
                       int64_t* table_loads);

/* Trace of a decode for beam_search(debug=True) (beam.py:53-57: the growns
 * of every end position, in generation order, and each position's beam):
 * a separate, untuned launch with the decoders' scoring code.  Positions of
 * sentence s are pos_off[s] + e, e = 0..n_s; the caller sizes every array:
 * position q's expansion slots are [exp_off[q], exp_off[q + 1]) (a position
 * has at most k x (its candidates) expansions; too few slots -> LT_EINVAL).
 * The batch must be one launch piece. */
typedef struct {
  const int64_t* pos_off;   /* [n_sent + 1] */
  const int64_t* exp_off;   /* [pos_off[n_sent] + 1], exp_off[pos_off[n_sent]] == n_exp */
  int64_t n_exp;            /* expansion slots */
  int32_t* beam_count;      /* [pos_off[n_sent]]: |beam[e]| */
  uint32_t* beam_gen;       /* [pos_off[n_sent] * k]: expansion index of beam[e][r] */
  int32_t* exp_count;       /* [pos_off[n_sent]]: expansions enumerated at e */
  double* exp_score;        /* [n_exp]: score of the grown sequence (0 if skipped) */
  uint32_t* exp_node;       /* [n_exp]: local node << 11 | (span - 1) << 8 | parent rank */
  uint8_t* exp_skip;        /* [n_exp]: 1 = skipped (unknown after unknown, beam.py:43-45) */
  uint64_t* exp_link;       /* [n_exp] or NULL: local node | (span - 1) << 21 | parent rank << 42
                               -- required past max_len 8 / beam 256, where exp_node holds the
                               local node only */
} lt_trace;
lt_status lt_decode_trace(lt_ctx* ctx, const lt_model* model, lt_batch* batch, int k, lt_trace* trace);

/* ---- multi-GPU result gather --------------------------------
 * One process per GPU decodes its own shard of sentences: sentences are
 * independent (beam_search keeps no cross-sentence state, beam.py:5-61, and
 * Tagger.tag is per sentence, tagger.py:68-78), so the only exchange is one
 * RCCL gather of every rank's decode results to a root rank over xGMI.
 * RCCL is loaded on first use (dlopen of ROCm's librccl); the root's unique
 * id travels between the processes through the caller (e.g. a gloo
 * broadcast).  lt_comm_create, lt_gather_prepare and lt_gather_launch are
 * collective: every rank of the communicator calls them in the same
 * order. */
#define LT_COMM_ID_BYTES 128
typedef struct lt_comm lt_comm;
/* Path of the RCCL library in use (the one next to the HIP runtime this
 * library is bound to), loading it if needed; NULL if none loads. */
const char* lt_comm_library(void);
/* Fresh communicator id (call on one rank, share with the others). */
lt_status lt_comm_unique_id(uint8_t id[LT_COMM_ID_BYTES]);
lt_status lt_comm_create(lt_ctx* ctx, int nranks, int rank, const uint8_t id[LT_COMM_ID_BYTES],
                         lt_comm** out);
lt_status lt_comm_destroy(lt_comm* comm);
/* Agree on every rank's result sizes for beam k (<= the batch's max_k) and
 * allocate two send slots (and, on the root, two receive slots of nranks
 * slabs and one pinned mirror).  Blocking. */
lt_status lt_gather_prepare(lt_comm* comm, lt_batch* batch, int k, int root);
/* Gather the last decode's results (beam k of the prepare) to the root: the
 * results are packed into the next send slot (a slab, see "compact
 * results") and one ncclGather of the slabs runs, both on the communicator's
 * own stream -- so the next decode on the ctx stream overlaps this gather.
 * Complete after lt_gather_sync (lt_sync does not cover it);
 * lt_batch_destroy waits for the pack's reads of the batch. */
lt_status lt_gather_launch(lt_comm* comm, lt_batch* batch);
/* Wait for this rank's outstanding gathers (local, not collective). */
lt_status lt_gather_sync(lt_comm* comm);
/* Root only: copy the used bytes of every rank's slab of the last gather
 * into pinned host memory (on the ctx's copy stream, after the gather;
 * complete after lt_sync). */
lt_status lt_gather_fetch(lt_comm* comm);
/* Root only: rank r's results (host pointers valid until the next fetch). */
lt_status lt_gather_view(lt_comm* comm, int r, lt_packed_view* view);
/* Device time of the last lt_gather_launch (HIP events around the RCCL
 * group on the communicator stream), ms.  Valid after lt_gather_sync. */
lt_status lt_last_gather_ms(lt_comm* comm, float* ms);

/* ---- evaluate -------------------------------------------
 * Batch form of BeamScoreFunctions.evaluate(seq) (score_funcs.py:44-48) for
 * given paths (e.g. gold sequences):
 *   total = ((0 + E_0) + E_1) + ...   over the scorers in constructor order,
 *   node-local scorer t (score_funcs.py:62-63, 81-82, 96-97):
 *       E_t = ((0 + v_t(w_0)) + v_t(w_1)) + ...  over every word of the path
 *   trigram scorer (score_funcs.py:127-135): the Sequence.add replay
 *       E = ((0 + inc_a) + inc_b) + ...  over the words not tagged BOS/EOS,
 *       inc = the trigram score of (prev2, prev1, w) in the replayed path.
 * Word records are lattice-node records as in lt_batch_desc; prev1/prev2 are
 * the replayed predecessors of each word (global word index, -1 = None);
 * prev1 = -2 marks a word the replay skips. */
typedef struct {
  int32_t n_paths;
  int64_t n_words;
  const int64_t* path_off;      /* [n_paths + 1] */
  const int32_t* word;          /* [n_words] interned ids (0 = in no key) */
  const int32_t* morph0;
  const int32_t* tag;
  const uint32_t* mask;         /* pre-filter bits + flags, as lt_batch_desc.node_mask */
  const double* f4;
  const double* f5;
  const double* f6;
  const int64_t* prev1;         /* [n_words] */
  const int64_t* prev2;         /* [n_words] */
  int32_t n_terms;              /* node-local scorers */
  const double* terms;          /* [n_terms * n_words], scorer-major */
  int32_t trigram_pos;          /* position of the trigram scorer among the n_terms + 1; -1 = none */
  int32_t trigram_scorer;       /* ABI 6: which of the composite's trigram scorers the trigram term is
                                   (its keys' classes + LT_XTRI_CLASS_STRIDE * trigram_scorer; the
                                   word records then hold that scorer's masks and class 4-6
                                   coefficients); 0 = the first */
} lt_paths_desc;
/* Blocking: scores[n_paths] (host buffer) receives the totals. */
lt_status lt_evaluate(lt_ctx* ctx, const lt_model* model, const lt_paths_desc* paths, double* scores);

#ifdef __cplusplus
}
#endif
#endif /* LATTICE_DECODE_H */
