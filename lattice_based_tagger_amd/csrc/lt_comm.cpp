// lt_comm.cpp -- multi-GPU result gather of liblt.so (include/lattice_decode.h,
// "multi-GPU result gather").
//
// Sentences shard across GPUs with no data-path exchange;
// the only collective is one RCCL gather of the per-rank result blocks to a
// root rank over xGMI.  Gathers need equal counts on every rank, so
// lt_gather_prepare agrees on the largest per-rank sentence count and code
// slot count (one small ncclAllGather) and sizes two padded send slots (and,
// on the root, two receive slots) once.  Each gather snapshots the decode's
// results into the next send slot with a device copy on the decoder stream
// (a few microseconds at HBM speed) and runs the RCCL group on the
// communicator's own stream, so gather i overlaps decode i+1; a slot is
// reused only after its previous gather has completed (event wait).
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

template <class T>
hipError_t dalloc_fill(T** p, size_t n, int byte) {
  *p = nullptr;
  if (n == 0) return hipSuccess;
  hipError_t e = hipMalloc((void**)p, n * sizeof(T));
  if (e == hipSuccess) e = hipMemset(*p, byte, n * sizeof(T));
  return e;
}

void dfree(void* p) {
  if (p) (void)hipFree(p);
}

void hfree(void* p) {
  if (p) (void)hipHostFree(p);
}

}  // namespace

// One result block (count, length, score, codes) at the padded per-rank size,
// or world x that on the root.
struct Block {
  int32_t *count = nullptr, *len = nullptr, *codes = nullptr;
  double* score = nullptr;
};

struct lt_comm {
  lt_ctx* ctx = nullptr;
  ncclComm_t comm = nullptr;
  hipStream_t stream = nullptr;          // RCCL stream: gathers overlap the next decode
  int nranks = 0, rank = 0, root = -1, k = 0;
  const lt_batch* batch = nullptr;       // prepared batch
  int64_t s_pad = 0, c_pad = 0;          // per-rank padded sentences / characters
  std::vector<int64_t> rank_s, rank_c;   // every rank's sentences / characters
  // two slots (ping-pong): the send copy of a decode's results and, on the
  // root, the receive block
  Block send[2], recv[2];
  bool used[2] = {false, false};
  int next = 0, last = -1;
  hipEvent_t ready[2] = {nullptr, nullptr}, done[2] = {nullptr, nullptr};
  hipEvent_t g0[2] = {nullptr, nullptr}, g1[2] = {nullptr, nullptr};
  // root: pinned mirror of one receive block
  int32_t *h_count = nullptr, *h_len = nullptr, *h_codes = nullptr;
  double* h_score = nullptr;
};

namespace {

void free_block(Block& b) {
  dfree(b.count);
  dfree(b.len);
  dfree(b.score);
  dfree(b.codes);
  b = Block{};
}

hipError_t alloc_block(Block& b, size_t n_count, size_t n_res, size_t n_codes) {
  hipError_t e = dalloc_fill(&b.count, n_count, 0);
  if (e == hipSuccess) e = dalloc_fill(&b.len, n_res, 0);
  if (e == hipSuccess) e = dalloc_fill(&b.score, n_res, 0);
  if (e == hipSuccess) e = dalloc_fill(&b.codes, n_codes, 0xFF);
  return e;
}

void free_slots(lt_comm* c) {
  for (int i = 0; i < 2; ++i) {
    free_block(c->send[i]);
    free_block(c->recv[i]);
    c->used[i] = false;
  }
  hfree(c->h_count);
  hfree(c->h_len);
  hfree(c->h_score);
  hfree(c->h_codes);
  c->h_count = c->h_len = c->h_codes = nullptr;
  c->h_score = nullptr;
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
  hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
  for (int i = 0; i < 2 && e == hipSuccess; ++i) {
    e = hipEventCreateWithFlags(&c->ready[i], hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->done[i], hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreate(&c->g0[i]);
    if (e == hipSuccess) e = hipEventCreate(&c->g1[i]);
  }
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
  free_slots(c);
  for (int i = 0; i < 2; ++i) {
    hipEvent_t evs[] = {c->ready[i], c->done[i], c->g0[i], c->g1[i]};
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
  // every rank's (sentences, characters)
  const int R = c->nranks;
  int64_t mine[2] = {b->n_sent, b->total_chars};
  int64_t *d_mine = nullptr, *d_all = nullptr;
  std::vector<int64_t> all(2 * (size_t)R);
  hipError_t e = hipMalloc((void**)&d_mine, sizeof mine);
  if (e == hipSuccess) e = hipMalloc((void**)&d_all, all.size() * sizeof(int64_t));
  if (e == hipSuccess) e = hipMemcpy(d_mine, mine, sizeof mine, hipMemcpyHostToDevice);
  ncclResult_t nr = ncclSuccess;
  if (e == hipSuccess) nr = r.all_gather(d_mine, d_all, 2, ncclInt64, c->comm, c->stream);
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
  int64_t s_pad = 0, c_pad = 0;
  for (int q = 0; q < R; ++q) {
    c->rank_s[q] = all[2 * q];
    c->rank_c[q] = all[2 * q + 1];
    s_pad = std::max(s_pad, c->rank_s[q]);
    c_pad = std::max(c_pad, c->rank_c[q]);
  }
  s_pad = std::max<int64_t>(s_pad, 1);
  c_pad = std::max<int64_t>(c_pad, 1);
  // send slots (padding past this rank's results stays 0 / -1) and, on the
  // root, receive slots + one pinned mirror
  free_slots(c);
  const size_t sp = (size_t)s_pad, cp = (size_t)c_pad;
  for (int i = 0; i < 2 && e == hipSuccess; ++i) {
    e = alloc_block(c->send[i], sp, sp * k, cp * k);
    if (e == hipSuccess && c->rank == root) e = alloc_block(c->recv[i], R * sp, R * sp * k, R * cp * k);
  }
  if (c->rank == root) {
    const size_t rc = (size_t)R * sp, rr = rc * k, rcd = (size_t)R * cp * k;
    if (e == hipSuccess) e = hipHostMalloc((void**)&c->h_count, rc * 4, hipHostMallocDefault);
    if (e == hipSuccess) e = hipHostMalloc((void**)&c->h_len, rr * 4, hipHostMallocDefault);
    if (e == hipSuccess) e = hipHostMalloc((void**)&c->h_score, rr * 8, hipHostMallocDefault);
    if (e == hipSuccess) e = hipHostMalloc((void**)&c->h_codes, rcd * 4, hipHostMallocDefault);
  }
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (e != hipSuccess) {
    free_slots(c);
    return lt::set_error(e == hipErrorOutOfMemory ? LT_ENOMEM : LT_EHIP, "lt_gather_prepare: %s",
                         hipGetErrorString(e));
  }
  c->root = root;
  c->k = k;
  c->batch = b;
  c->s_pad = s_pad;
  c->c_pad = c_pad;
  return LT_OK;
}

lt_status lt_gather_launch(lt_comm* c, lt_batch* b) {
  if (!c || !b) return lt::set_error(LT_EINVAL, "lt_gather_launch: NULL argument");
  if (c->batch != b || c->root < 0) return lt::set_error(LT_EINVAL, "lt_gather_launch: batch not prepared");
  if (b->last_k != c->k)
    return lt::set_error(LT_EINVAL, "lt_gather_launch: last decode was beam %d, prepared for %d", b->last_k, c->k);
  const Rccl& r = rccl();
  lt_ctx* x = c->ctx;
  const int k = c->k, i = c->next;
  const size_t sp = (size_t)c->s_pad, cp = (size_t)c->c_pad, S = (size_t)b->n_sent;
  const size_t nc = (size_t)b->total_chars * k;
  const bool at_root = c->rank == c->root;
  Block& snd = c->send[i];
  Block& rcv = c->recv[i];
  HIP_TRY(hipSetDevice(x->device));
  // the slot's previous gather (two launches ago) must be done with it
  if (c->used[i]) HIP_TRY(hipStreamWaitEvent(x->stream, c->done[i], 0));
  // snapshot the decode's results into the send slot (decoder stream), so the
  // next decode may overwrite the batch's buffers while this gather runs
  if (S) {
    HIP_TRY(hipMemcpyAsync(snd.count, b->d_count, S * 4, hipMemcpyDeviceToDevice, x->stream));
    HIP_TRY(hipMemcpyAsync(snd.len, b->d_len, S * k * 4, hipMemcpyDeviceToDevice, x->stream));
    HIP_TRY(hipMemcpyAsync(snd.score, b->d_score, S * k * 8, hipMemcpyDeviceToDevice, x->stream));
  }
  if (nc) HIP_TRY(hipMemcpyAsync(snd.codes, b->d_codes, nc * 4, hipMemcpyDeviceToDevice, x->stream));
  HIP_TRY(hipEventRecord(c->ready[i], x->stream));
  HIP_TRY(hipStreamWaitEvent(c->stream, c->ready[i], 0));
  HIP_TRY(hipEventRecord(c->g0[i], c->stream));
  NCCL_TRY(r.group_start());
  ncclResult_t nr = r.gather(snd.count, at_root ? rcv.count : nullptr, sp, ncclInt32, c->root, c->comm,
                             c->stream);
  if (nr == ncclSuccess)
    nr = r.gather(snd.len, at_root ? rcv.len : nullptr, sp * k, ncclInt32, c->root, c->comm, c->stream);
  if (nr == ncclSuccess)
    nr = r.gather(snd.score, at_root ? rcv.score : nullptr, sp * k, ncclFloat64, c->root, c->comm, c->stream);
  if (nr == ncclSuccess)
    nr = r.gather(snd.codes, at_root ? rcv.codes : nullptr, cp * k, ncclInt32, c->root, c->comm, c->stream);
  ncclResult_t ne = r.group_end();
  if (nr != ncclSuccess) return lt::set_error(LT_ERCCL, "lt_gather_launch: ncclGather: %s", r.error_string(nr));
  if (ne != ncclSuccess) return lt::set_error(LT_ERCCL, "lt_gather_launch: ncclGroupEnd: %s", r.error_string(ne));
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
  const Block& rcv = c->recv[c->last];
  const size_t rc = (size_t)c->nranks * c->s_pad, rr = rc * c->k, rcd = (size_t)c->nranks * c->c_pad * c->k;
  HIP_TRY(hipSetDevice(x->device));
  HIP_TRY(hipStreamWaitEvent(x->stream, c->done[c->last], 0));
  HIP_TRY(hipMemcpyAsync(c->h_count, rcv.count, rc * 4, hipMemcpyDeviceToHost, x->stream));
  HIP_TRY(hipMemcpyAsync(c->h_len, rcv.len, rr * 4, hipMemcpyDeviceToHost, x->stream));
  HIP_TRY(hipMemcpyAsync(c->h_score, rcv.score, rr * 8, hipMemcpyDeviceToHost, x->stream));
  HIP_TRY(hipMemcpyAsync(c->h_codes, rcv.codes, rcd * 4, hipMemcpyDeviceToHost, x->stream));
  return LT_OK;
}

lt_status lt_gather_view(lt_comm* c, int q, lt_result* v, int32_t* n_sent, int64_t* code_slots) {
  if (!c || !v) return lt::set_error(LT_EINVAL, "lt_gather_view: NULL argument");
  if (c->root < 0 || c->rank != c->root) return lt::set_error(LT_EINVAL, "lt_gather_view: not the root");
  if (q < 0 || q >= c->nranks) return lt::set_error(LT_EINVAL, "lt_gather_view: rank %d", q);
  const size_t sp = (size_t)c->s_pad, cp = (size_t)c->c_pad, k = (size_t)c->k;
  v->count = c->h_count + q * sp;
  v->length = c->h_len + q * sp * k;
  v->score = c->h_score + q * sp * k;
  v->codes = c->h_codes + q * cp * k;
  if (n_sent) *n_sent = (int32_t)c->rank_s[q];
  if (code_slots) *code_slots = c->rank_c[q] * (int64_t)k;
  return LT_OK;
}

lt_status lt_last_gather_ms(lt_comm* c, float* ms) {
  if (!c || !ms) return lt::set_error(LT_EINVAL, "lt_last_gather_ms: NULL argument");
  if (c->last < 0) return lt::set_error(LT_EINVAL, "lt_last_gather_ms: nothing gathered");
  HIP_TRY(hipEventElapsedTime(ms, c->g0[c->last], c->g1[c->last]));
  return LT_OK;
}

}  // extern "C"
