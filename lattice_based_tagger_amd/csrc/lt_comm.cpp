// lt_comm.cpp -- multi-GPU result gather of liblt.so (include/lattice_decode.h,
// "multi-GPU result gather").
//
// Sentences shard across GPUs with no data-path exchange;
// the only collective is one RCCL gather of the per-rank result blocks to a
// root rank over xGMI.  Each rank's results travel as a slab (packed
// results, lt_results.hip); gathers need equal counts on every rank, so
// lt_gather_prepare agrees on the largest slab capacity (one small
// ncclAllGather) and sizes two send slots (and, on the root, two receive
// slots of nranks slabs) once.  Each gather packs the decode's results into
// the next send slot and runs one ncclGather, both on the communicator's own
// stream, so gather i overlaps decode i+1; a decode reuses a result slot
// only after the packing has read it, the root reuses a receive slot only
// after its host copy (event waits).  The root copies the used bytes of every rank's slab to pinned host
// memory on the context's copy stream.
//
// RCCL is dlopen'ed on first use so that single-GPU users of the library
// never load it; its ABI comes from ROCm's rccl.h (types only).
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <new>
#include <string>
#include <vector>

#include "../../include/lattice_decode.h"
#include "lt_error.h"
#include "lt_handles.h"
#include "lt_internal.h"

namespace {

struct Rccl {
  bool ok = false;
  std::string why, path;
  ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
  ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
  ncclResult_t (*all_gather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*gather)(const void*, void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*group_start)() = nullptr;
  ncclResult_t (*group_end)() = nullptr;
  const char* (*error_string)(ncclResult_t) = nullptr;
};

const Rccl& rccl() {
  static Rccl r;
  static std::once_flag once;
  std::call_once(once, [] {
    // RCCL must run on the HIP runtime this library is bound to: a process
    // that imported PyTorch-ROCm first has bound liblt to torch's bundled
    // libamdhip64 (same soname), so take the librccl next to whichever
    // libamdhip64 provides the HIP API (an already-loaded one is reused), then
    // ROCm's.  RTLD_DEEPBIND keeps a freshly loaded RCCL on its own symbols
    // when another RCCL is already in the process.
    std::vector<std::string> names;
    Dl_info info;
    if (dladdr(reinterpret_cast<void*>(&hipGetDeviceCount), &info) && info.dli_fname) {
      std::string dir(info.dli_fname);
      const size_t slash = dir.rfind('/');
      if (slash != std::string::npos) {
        dir.resize(slash);
        names.push_back(dir + "/librccl.so.1");
        names.push_back(dir + "/librccl.so");
      }
    }
    if (const char* p = std::getenv("ROCM_PATH")) names.push_back(std::string(p) + "/lib/librccl.so.1");
    names.push_back("/opt/rocm/lib/librccl.so.1");
    void* h = nullptr;
    for (const std::string& n : names) {
      if ((h = dlopen(n.c_str(), RTLD_NOW | RTLD_NOLOAD))) break;             // already in the process
      if ((h = dlopen(n.c_str(), RTLD_NOW | RTLD_LOCAL | RTLD_DEEPBIND))) break;
    }
    if (!h) {
      const char* e = dlerror();
      r.why = std::string("cannot load librccl: ") + (e ? e : "?");
      return;
    }
    {
      Dl_info li;
      void* f = dlsym(h, "ncclGetUniqueId");
      r.path = (f && dladdr(f, &li) && li.dli_fname) ? li.dli_fname : "?";
    }
    bool all = true;
    auto sym = [&](auto& fn, const char* name) {
      fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(h, name));
      if (!fn) {
        all = false;
        r.why = std::string("librccl lacks ") + name;
      }
    };
    sym(r.get_unique_id, "ncclGetUniqueId");
    sym(r.comm_init_rank, "ncclCommInitRank");
    sym(r.comm_destroy, "ncclCommDestroy");
    sym(r.all_gather, "ncclAllGather");
    sym(r.gather, "ncclGather");
    sym(r.group_start, "ncclGroupStart");
    sym(r.group_end, "ncclGroupEnd");
    sym(r.error_string, "ncclGetErrorString");
    r.ok = all;
  });
  return r;
}

#define HIP_TRY(expr)                                                                     \
  do {                                                                                    \
    hipError_t _e = (expr);                                                               \
    if (_e != hipSuccess)                                                                 \
      return lt::set_error(LT_EHIP, "%s failed: %s", #expr, hipGetErrorString(_e));      \
  } while (0)

#define NCCL_TRY(expr)                                                                    \
  do {                                                                                    \
    ncclResult_t _r = (expr);                                                             \
    if (_r != ncclSuccess)                                                                \
      return lt::set_error(LT_ERCCL, "%s failed: %s", #expr, rccl().error_string(_r));   \
  } while (0)

void dfree(void* p) {
  if (p) (void)hipFree(p);
}

void hfree(void* p) {
  if (p) (void)hipHostFree(p);
}

}  // namespace

struct lt_comm {
  lt_ctx* ctx = nullptr;
  ncclComm_t comm = nullptr;
  hipStream_t stream = nullptr;          // RCCL stream: gathers overlap the next decode
  int nranks = 0, rank = 0, root = -1, k = 0;
  const lt_batch* batch = nullptr;       // prepared batch
  uint64_t cap = 0;                      // slab bytes per rank (max over ranks)
  std::vector<int64_t> rank_s, rank_c;   // every rank's sentences / characters
  // two slots (ping-pong): this rank's packed results (send) and, on the
  // root, every rank's slab at stride cap (receive)
  char* send[2] = {nullptr, nullptr};
  char* recv[2] = {nullptr, nullptr};
  bool used[2] = {false, false};
  int next = 0, last = -1;
  hipEvent_t done[2] = {nullptr, nullptr};
  hipEvent_t g0[2] = {nullptr, nullptr}, g1[2] = {nullptr, nullptr};
  hipEvent_t fetched[2] = {nullptr, nullptr};   // root: copy of receive slot i to the host queued
  hipEvent_t packed[2] = {nullptr, nullptr};    // send slot i packed (on the decode stream)
  bool fetch_pending[2] = {false, false};
  // root: pinned mirror of one receive block (nranks slabs at stride cap)
  char* h_slabs = nullptr;
};

namespace {

void free_slots(lt_comm* c) {
  for (int i = 0; i < 2; ++i) {
    dfree(c->send[i]);
    dfree(c->recv[i]);
    c->send[i] = c->recv[i] = nullptr;
    c->used[i] = false;
  }
  hfree(c->h_slabs);
  c->h_slabs = nullptr;
  c->next = 0;
  c->last = -1;
}

}  // namespace

extern "C" {

lt_status lt_comm_unique_id(uint8_t id[LT_COMM_ID_BYTES]) {
  if (!id) return lt::set_error(LT_EINVAL, "lt_comm_unique_id: id is NULL");
  const Rccl& r = rccl();
  if (!r.ok) return lt::set_error(LT_ERCCL, "lt_comm_unique_id: %s", r.why.c_str());
  static_assert(sizeof(ncclUniqueId) == LT_COMM_ID_BYTES, "ncclUniqueId size");
  ncclUniqueId u;
  NCCL_TRY(r.get_unique_id(&u));
  memcpy(id, &u, sizeof u);
  return LT_OK;
}

const char* lt_comm_library(void) {
  const Rccl& r = rccl();
  return r.ok ? r.path.c_str() : nullptr;
}

lt_status lt_comm_create(lt_ctx* ctx, int nranks, int rank, const uint8_t id[LT_COMM_ID_BYTES],
                         lt_comm** out) {
  if (!ctx || !id || !out) return lt::set_error(LT_EINVAL, "lt_comm_create: NULL argument");
  *out = nullptr;
  if (nranks < 1 || rank < 0 || rank >= nranks)
    return lt::set_error(LT_EINVAL, "lt_comm_create: rank %d of %d", rank, nranks);
  const Rccl& r = rccl();
  if (!r.ok) return lt::set_error(LT_ERCCL, "lt_comm_create: %s", r.why.c_str());
  HIP_TRY(hipSetDevice(ctx->device));
  ncclUniqueId u;
  memcpy(&u, id, sizeof u);
  ncclComm_t nc = nullptr;
  NCCL_TRY(r.comm_init_rank(&nc, nranks, u, rank));
  lt_comm* c = new (std::nothrow) lt_comm;
  if (!c) {
    r.comm_destroy(nc);
    return lt::set_error(LT_ENOMEM, "lt_comm_create: out of host memory");
  }
  c->ctx = ctx;
  c->comm = nc;
  c->nranks = nranks;
  c->rank = rank;
  // high priority: its packing kernels must find CUs while a decode runs
  int lo = 0, hi = 0;
  hipError_t e = hipDeviceGetStreamPriorityRange(&lo, &hi);
  if (e == hipSuccess) e = hipStreamCreateWithPriority(&c->stream, hipStreamNonBlocking, hi);
  for (int i = 0; i < 2 && e == hipSuccess; ++i) {
    e = hipEventCreateWithFlags(&c->done[i], hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreate(&c->g0[i]);
    if (e == hipSuccess) e = hipEventCreate(&c->g1[i]);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->packed[i], hipEventDisableTiming);
  }
  for (int i = 0; i < 2 && e == hipSuccess; ++i) e = hipEventCreateWithFlags(&c->fetched[i], hipEventDisableTiming);
  if (e != hipSuccess) {
    lt_comm_destroy(c);
    return lt::set_error(LT_EHIP, "lt_comm_create: %s", hipGetErrorString(e));
  }
  *out = c;
  return LT_OK;
}

lt_status lt_comm_destroy(lt_comm* c) {
  if (!c) return LT_OK;
  (void)hipSetDevice(c->ctx->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  (void)hipStreamSynchronize(c->ctx->stream);
  (void)hipStreamSynchronize(c->ctx->cstream);
  free_slots(c);
  for (hipEvent_t ev : c->fetched)
    if (ev) (void)hipEventDestroy(ev);
  for (int i = 0; i < 2; ++i) {
    hipEvent_t evs[] = {c->done[i], c->g0[i], c->g1[i], c->packed[i]};
    for (hipEvent_t ev : evs)
      if (ev) (void)hipEventDestroy(ev);
  }
  if (c->comm) rccl().comm_destroy(c->comm);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
  return LT_OK;
}

lt_status lt_gather_prepare(lt_comm* c, lt_batch* b, int k, int root) {
  if (!c || !b) return lt::set_error(LT_EINVAL, "lt_gather_prepare: NULL argument");
  if (b->ctx != c->ctx) return lt::set_error(LT_EINVAL, "lt_gather_prepare: batch of another context");
  if (k < 1 || k > b->max_k)
    return lt::set_error(LT_EINVAL, "lt_gather_prepare: beam %d not in 1..%d", k, b->max_k);
  if (root < 0 || root >= c->nranks) return lt::set_error(LT_EINVAL, "lt_gather_prepare: root %d", root);
  const Rccl& r = rccl();
  lt_ctx* x = c->ctx;
  HIP_TRY(hipSetDevice(x->device));
  HIP_TRY(hipStreamSynchronize(c->stream));
  HIP_TRY(hipStreamSynchronize(x->stream));
  // every rank's (sentences, characters, slab capacity)
  const int R = c->nranks;
  int64_t mine[3] = {b->n_sent, b->total_chars, (int64_t)lt::slab_layout(b->n_sent, k, b->total_chars).capacity};
  int64_t *d_mine = nullptr, *d_all = nullptr;
  std::vector<int64_t> all(3 * (size_t)R);
  hipError_t e = hipMalloc((void**)&d_mine, sizeof mine);
  if (e == hipSuccess) e = hipMalloc((void**)&d_all, all.size() * sizeof(int64_t));
  if (e == hipSuccess) e = hipMemcpy(d_mine, mine, sizeof mine, hipMemcpyHostToDevice);
  ncclResult_t nr = ncclSuccess;
  if (e == hipSuccess) nr = r.all_gather(d_mine, d_all, 3, ncclInt64, c->comm, c->stream);
  if (e == hipSuccess && nr == ncclSuccess) e = hipStreamSynchronize(c->stream);
  if (e == hipSuccess && nr == ncclSuccess)
    e = hipMemcpy(all.data(), d_all, all.size() * sizeof(int64_t), hipMemcpyDeviceToHost);
  dfree(d_mine);
  dfree(d_all);
  if (nr != ncclSuccess)
    return lt::set_error(LT_ERCCL, "lt_gather_prepare: ncclAllGather: %s", r.error_string(nr));
  if (e != hipSuccess) return lt::set_error(LT_EHIP, "lt_gather_prepare: %s", hipGetErrorString(e));
  c->rank_s.assign(R, 0);
  c->rank_c.assign(R, 0);
  uint64_t cap = 0;
  for (int q = 0; q < R; ++q) {
    c->rank_s[q] = all[3 * q];
    c->rank_c[q] = all[3 * q + 1];
    cap = std::max<uint64_t>(cap, (uint64_t)all[3 * q + 2]);
  }
  // send slots and, on the root, receive slots + one pinned mirror
  free_slots(c);
  const uint64_t scratch = lt::slab_alloc_bytes(b->n_sent, k, b->total_chars) -
                           lt::slab_layout(b->n_sent, k, b->total_chars).capacity;
  for (int i = 0; i < 2 && e == hipSuccess; ++i) {
    e = hipMalloc((void**)&c->send[i], cap + scratch);
    if (e == hipSuccess && c->rank == root) e = hipMalloc((void**)&c->recv[i], cap * R);
  }
  if (e == hipSuccess && c->rank == root) e = hipHostMalloc((void**)&c->h_slabs, cap * R, hipHostMallocDefault);
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (e != hipSuccess) {
    free_slots(c);
    return lt::set_error(e == hipErrorOutOfMemory ? LT_ENOMEM : LT_EHIP, "lt_gather_prepare: %s",
                         hipGetErrorString(e));
  }
  c->root = root;
  c->k = k;
  c->batch = b;
  c->cap = cap;
  return LT_OK;
}

lt_status lt_gather_launch(lt_comm* c, lt_batch* b) {
  if (!c || !b) return lt::set_error(LT_EINVAL, "lt_gather_launch: NULL argument");
  if (c->batch != b || c->root < 0) return lt::set_error(LT_EINVAL, "lt_gather_launch: batch not prepared");
  if (b->last_k != c->k)
    return lt::set_error(LT_EINVAL, "lt_gather_launch: last decode was beam %d, prepared for %d", b->last_k, c->k);
  const Rccl& r = rccl();
  lt_ctx* x = c->ctx;
  const int i = c->next;
  const bool at_root = c->rank == c->root;
  HIP_TRY(hipSetDevice(x->device));
  // the decode's results are packed into send slot i on the decode stream,
  // right behind the decode (round 6: packed on the communicator stream, the
  // pack kernels' blocks took CUs beside the next decode, whose LDS-filling
  // blocks then waited -- a k=1 decode 0.56 -> 0.72 ms with the packed-result
  // copy on one GPU); slot i's previous gather must be done with it.  The
  // gather itself runs on the communicator stream (the decode stream goes on
  // with the next decode); on the root, the host copy of receive slot i must
  // be done with it first
  if (c->used[i]) HIP_TRY(hipStreamWaitEvent(x->stream, c->done[i], 0));
  HIP_TRY(lt::pack_last_results_on(b, lt_batch::RD_GATHER, c->send[i], x->stream));
  HIP_TRY(hipEventRecord(c->packed[i], x->stream));
  if (at_root && c->fetch_pending[i]) {
    HIP_TRY(hipStreamWaitEvent(c->stream, c->fetched[i], 0));
    c->fetch_pending[i] = false;
  }
  HIP_TRY(hipStreamWaitEvent(c->stream, c->packed[i], 0));
  HIP_TRY(hipEventRecord(c->g0[i], c->stream));
  // one gather of the padded slabs (the used part of each is what the root
  // copies to the host)
  NCCL_TRY(r.gather(c->send[i], at_root ? c->recv[i] : nullptr, c->cap, ncclUint8, c->root, c->comm,
                    c->stream));
  HIP_TRY(hipEventRecord(c->g1[i], c->stream));
  HIP_TRY(hipEventRecord(c->done[i], c->stream));
  c->used[i] = true;
  c->last = i;
  c->next = i ^ 1;
  return LT_OK;
}

lt_status lt_gather_sync(lt_comm* c) {
  if (!c) return lt::set_error(LT_EINVAL, "lt_gather_sync: NULL argument");
  HIP_TRY(hipSetDevice(c->ctx->device));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return LT_OK;
}

lt_status lt_gather_fetch(lt_comm* c) {
  if (!c) return lt::set_error(LT_EINVAL, "lt_gather_fetch: NULL argument");
  if (c->root < 0 || c->rank != c->root) return lt::set_error(LT_EINVAL, "lt_gather_fetch: not the root");
  if (c->last < 0) return lt::set_error(LT_EINVAL, "lt_gather_fetch: nothing gathered");
  lt_ctx* x = c->ctx;
  HIP_TRY(hipSetDevice(x->device));
  // on the ctx's copy stream once the gather is done: each rank's used bytes
  HIP_TRY(hipStreamWaitEvent(x->cstream, c->done[c->last], 0));
  // (the receive slot holds the ranks' slabs back to back: one DMA)
  HIP_TRY(lt::launch_slab_to_host(c->recv[c->last], c->h_slabs, (size_t)c->nranks * c->cap, x->cstream));
  HIP_TRY(hipEventRecord(c->fetched[c->last], x->cstream));
  c->fetch_pending[c->last] = true;
  return LT_OK;
}

lt_status lt_gather_view(lt_comm* c, int q, lt_packed_view* v) {
  if (!c || !v) return lt::set_error(LT_EINVAL, "lt_gather_view: NULL argument");
  if (c->root < 0 || c->rank != c->root) return lt::set_error(LT_EINVAL, "lt_gather_view: not the root");
  if (q < 0 || q >= c->nranks) return lt::set_error(LT_EINVAL, "lt_gather_view: rank %d", q);
  return lt_slab_parse(c->h_slabs + (size_t)q * c->cap, c->cap, v);
}

lt_status lt_last_gather_ms(lt_comm* c, float* ms) {
  if (!c || !ms) return lt::set_error(LT_EINVAL, "lt_last_gather_ms: NULL argument");
  if (c->last < 0) return lt::set_error(LT_EINVAL, "lt_last_gather_ms: nothing gathered");
  HIP_TRY(hipEventElapsedTime(ms, c->g0[c->last], c->g1[c->last]));
  return LT_OK;
}

}  // extern "C"
