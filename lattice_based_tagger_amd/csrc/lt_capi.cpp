// lt_capi.cpp -- host side of liblt.so: the C-ABI declared in
// include/lattice_decode.h (contexts, the model hash table, batch upload and
// validation, decode launch, result download).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdarg>
#include <cstddef>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "../../include/lattice_decode.h"
#include "lt_common.h"
#include "lt_internal.h"
#include "lt_error.h"
#include "lt_handles.h"
#include "lt_host.h"

using namespace lt;

namespace {

thread_local std::string g_err;

lt_status fail(lt_status st, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return st;
}

}  // namespace

int lt::host_threads() {
  static const int n = [] {
    if (const char* e = std::getenv("OMP_NUM_THREADS")) {
      const int v = std::atoi(e);
      if (v > 0) return v;
    }
    return (int)std::max(1u, std::thread::hardware_concurrency());
  }();
  return n;
}

lt_status lt::set_error(lt_status st, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return st;
}

namespace {

#define HIP_TRY(expr)                                                          \
  do {                                                                         \
    hipError_t _e = (expr);                                                    \
    if (_e != hipSuccess)                                                      \
      return fail(LT_EHIP, "%s failed: %s", #expr, hipGetErrorString(_e));   \
  } while (0)

template <class T>
hipError_t dalloc_copy(T** dst, const T* src, size_t count, hipStream_t st) {
  *dst = nullptr;
  if (count == 0) return hipSuccess;
  hipError_t e = hipMalloc((void**)dst, count * sizeof(T));
  if (e != hipSuccess) return e;
  if (src) return hipMemcpyAsync(*dst, src, count * sizeof(T), hipMemcpyHostToDevice, st);
  return hipSuccess;
}

void dfree(void* p) {
  if (p) (void)hipFree(p);
}

}  // namespace


namespace {

struct KeyRec {
  uint32_t a, b, c, cls;
  double coef;
};

// The class-4/6 pair table of a set of records (NodeRec): distinct (f4, f6)
// bit patterns -> index, at most MAX_PAIRS entries (entry 0 = both absent);
// a record whose pair does not fit takes PX_ESC and the escape array.
struct PairTable {
  static constexpr int CAP = 256;                  // open addressing, > 2 x MAX_PAIRS
  std::vector<F46> vals;
  uint64_t ka[CAP], kb[CAP];
  int16_t idx[CAP];
  bool full = false;                               // some pair did not fit
  PairTable() { std::fill(idx, idx + CAP, (int16_t)-1); }
  static uint64_t bits(double v) {
    uint64_t u;
    std::memcpy(&u, &v, 8);
    return u;
  }
  static uint32_t home(uint64_t a, uint64_t b) {
    return (uint32_t)(((a * 0x9E3779B97F4A7C15ull) ^ (b * 0xC2B2AE3D27D4EB4Full)) >> 56);
  }
  int find(double f4, double f6) const {
    const uint64_t a = bits(f4), b = bits(f6);
    for (uint32_t i = home(a, b);; i = (i + 1) & (CAP - 1)) {
      if (idx[i] < 0) return -1;
      if (ka[i] == a && kb[i] == b) return idx[i];
    }
  }
  int add(double f4, double f6) {
    const uint64_t a = bits(f4), b = bits(f6);
    uint32_t i = home(a, b);
    for (;; i = (i + 1) & (CAP - 1)) {
      if (idx[i] < 0) break;
      if (ka[i] == a && kb[i] == b) return idx[i];
    }
    if ((int)vals.size() >= MAX_PAIRS) {
      full = true;
      return -1;
    }
    ka[i] = a; kb[i] = b;
    idx[i] = (int16_t)vals.size();
    vals.push_back(F46{f4, f6});
    return idx[i];
  }
};
// The pair of a record from the API columns (absent: -0.0)
static inline F46 api_pair(uint32_t am, const double* f4, const double* f6, int64_t i) {
  return F46{(am & F_HAS4) ? f4[i] : -0.0, (am & F_HAS6) ? f6[i] : -0.0};
}
// The table of records [0, n) (masks / f4 / f6 columns), the `first` pairs
// entered before them: per thread, then merged in thread order.
static PairTable pair_table(int64_t n, const uint32_t* mask, const double* f4, const double* f6,
                            const std::vector<F46>& first) {
  PairTable tab;
  tab.add(-0.0, -0.0);
  for (const F46& f : first) tab.add(f.f4, f.f6);
  std::vector<PairTable> local(32);
  parallel_ranges(n, [&](int t, int64_t lo, int64_t hi) {
    PairTable& lt = local[(size_t)t];
    F46 last{-0.0, -0.0};
    for (int64_t i = lo; i < hi && !lt.full; ++i) {
      const F46 f = api_pair(mask[i], f4, f6, i);
      if (std::memcmp(&f, &last, sizeof f) == 0) continue;
      last = f;
      lt.add(f.f4, f.f6);
    }
  }, 1 << 16);
  for (const PairTable& lt : local) {
    for (const F46& f : lt.vals) tab.add(f.f4, f.f6);
    tab.full |= lt.full;
  }
  return tab;
}

}  // namespace

// Infinite score terms: +inf and -inf may each occur, but not both in one
// decode -- their sum is a NaN, and the reference ranks by Python's sort,
// whose order over NaN (every comparison false) is not reproduced.  Bit 0:
// some +inf, bit 1: some -inf.
static inline int inf_sign_bits(double v) { return std::isinf(v) ? (v > 0 ? 1 : 2) : 0; }

struct lt_model {
  lt_ctx* ctx = nullptr;
  int inf_signs = 0;            // inf_sign_bits of the coefficients
  void* d_table = nullptr;      // with overflow flags (beam 1: primary first)
  void* d_plain = nullptr;      // the same slots, flags cleared (beams > 1 load both slots)
  int64_t slots = 0;
  uint32_t seed = 0;
  int narrow = 0;          // 16 B SlotN (all ids < 2^20) or 32 B SlotW
  double* d_d3 = nullptr;    // dense class-3 table or NULL
  uint32_t d3mul = 0;
  uint32_t d3off = 0;        // its bit window (d3_window; set when d_d3 is)
};

namespace {

// The two candidate slots of a key, as the kernels compute them.
template <typename SlotT>
void table_slots(const KeyRec& k, uint32_t seed, const NarrowHash& hk, uint32_t slots, uint32_t& i1,
                 uint32_t& i2) {
  if constexpr (sizeof(SlotT) == sizeof(SlotN))
    narrow_slots(hk, k.a, k.b, k.c, k.cls, slots, i1, i2);
  else
    cuckoo_slots(key_base<false>(k.a, k.b, k.c, k.cls), seed, slots, i1, i2);
}

// Cuckoo table build (two choices, one slot per bucket).  Returns false when
// the random walk fails; the caller reseeds / grows and retries.
template <class SlotT>
bool cuckoo_build(const std::vector<KeyRec>& keys, uint32_t slots, uint32_t seed,
                  std::vector<SlotT>& tab, int64_t* dup) {
  tab.assign(slots, SlotT{});
  const NarrowHash hk = narrow_hash(seed);
  std::vector<int32_t> who(slots, -1);          // key index held by each slot
  uint64_t rng = 0x9E3779B97F4A7C15ull ^ seed;
  const int max_kicks = 2000;
  // Phase 1: every key whose primary slot is still free takes it (the fewest
  // keys end up at a secondary: only those whose primary another key took).
  // Phase 2: the rest by cuckoo insertion.
  std::vector<uint32_t> prim(keys.size()), sec(keys.size());
  std::vector<int32_t> rest;
  for (size_t i = 0; i < keys.size(); ++i) {
    table_slots<SlotT>(keys[i], seed, hk, slots, prim[i], sec[i]);
    if (who[prim[i]] < 0) who[prim[i]] = (int32_t)i;
    else rest.push_back((int32_t)i);
  }
  auto same = [&](int32_t w, const KeyRec& k) {
    return w >= 0 && keys[(size_t)w].a == k.a && keys[(size_t)w].b == k.b && keys[(size_t)w].c == k.c &&
           keys[(size_t)w].cls == k.cls;
  };
  for (int32_t i : rest) {
    // a key equal to this one (placed earlier) sits at one of its two slots
    const KeyRec& ki = keys[(size_t)i];
    if (same(who[prim[(size_t)i]], ki) || same(who[sec[(size_t)i]], ki)) {
      *dup = i;
      return false;
    }
    int32_t cur = i;
    uint32_t i1, i2;
    uint32_t pos = 0;
    bool placed = false;
    for (int kick = 0; kick < max_kicks; ++kick) {
      const KeyRec& k = keys[(size_t)cur];
      table_slots<SlotT>(k, seed, hk, slots, i1, i2);
      uint32_t target;
      if (who[i1] < 0) target = i1;
      else if (who[i2] < 0) target = i2;
      else {
        rng ^= rng << 13; rng ^= rng >> 7; rng ^= rng << 17;
        target = (kick == 0) ? ((rng & 1) ? i1 : i2) : (pos == i1 ? i2 : i1);
        if (i1 == i2) target = i1;
      }
      const int32_t evicted = who[target];
      who[target] = cur;
      if (evicted < 0) { placed = true; break; }
      cur = evicted;
      pos = target;                              // the evicted key must leave this slot
    }
    if (!placed) return false;
  }
  // Primary first: move keys that sit at their secondary slot back to their
  // primary when it is free, or when its holder sits at its own secondary and
  // can go back to a free primary.  Fewer secondaries = fewer flagged slots =
  // fewer second loads per lookup (lt_common.h).
  for (int pass = 0; pass < 4; ++pass) {
    int64_t moved = 0;
    for (uint32_t x = 0; x < slots; ++x) {
      const int32_t kx = who[x];
      if (kx < 0 || prim[(size_t)kx] == x) continue;
      const uint32_t p = prim[(size_t)kx];
      const int32_t y = who[p];
      if (y < 0) {
        who[p] = kx; who[x] = -1; ++moved;
      } else if (prim[(size_t)y] != p && who[prim[(size_t)y]] < 0) {
        who[prim[(size_t)y]] = y; who[p] = kx; who[x] = -1; ++moved;
      }
    }
    if (!moved) break;
  }
  for (uint32_t x = 0; x < slots; ++x) {
    if (who[x] < 0) continue;
    const KeyRec& k = keys[(size_t)who[x]];
    SlotT& sl = tab[x];
    if constexpr (sizeof(SlotT) == sizeof(SlotN)) {
      sl.key |= narrow_key(k.a, k.b, k.c, k.cls);
      sl.coef = k.coef;
    } else {
      sl.a = k.a; sl.b = k.b; sl.c = k.c; sl.cls1 |= k.cls + 1; sl.coef = k.coef;
    }
    const uint32_t p = prim[(size_t)who[x]];
    if (p != x) {                                // at its secondary: flag the primary
      if constexpr (sizeof(SlotT) == sizeof(SlotN)) tab[p].key |= FLAG_N;
      else tab[p].cls1 |= FLAG_W;
    }
  }
  return true;
}

}  // namespace


extern "C" {

int lt_abi_version(void) { return LT_ABI_VERSION; }
static_assert(LT_XTRI_CLASS_STRIDE == XTRI_CLASS_STRIDE && LT_MAX_TRI == MAX_TRI, "lt_common.h vs lattice_decode.h");
uint32_t lt_hash_version(void) { return HASH_VERSION; }

const char* lt_last_error(void) { return g_err.c_str(); }

int lt_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

lt_status lt_ctx_create(int device, lt_ctx** out) {
  if (!out) return fail(LT_EINVAL, "lt_ctx_create: out is NULL");
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0)
    return fail(LT_EHIP, "lt_ctx_create: no HIP device visible");
  if (device < 0 || device >= n) return fail(LT_EINVAL, "lt_ctx_create: device %d of %d", device, n);
  HIP_TRY(hipSetDevice(device));
  lt_ctx* c = new (std::nothrow) lt_ctx;
  if (!c) return fail(LT_ENOMEM, "lt_ctx_create: out of host memory");
  c->device = device;
  hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->ustream, hipStreamNonBlocking);
  if (e == hipSuccess) {
    // the copy stream's kernels (slab -> host) must get CUs while a decode
    // occupies them all: highest stream priority
    int lo = 0, hi = 0;
    e = hipDeviceGetStreamPriorityRange(&lo, &hi);
    if (e == hipSuccess) e = hipStreamCreateWithPriority(&c->cstream, hipStreamNonBlocking, hi);
  }
  for (int i = 0; i < lt_ctx::KRING && e == hipSuccess; ++i) {
    e = hipEventCreate(&c->kev0[i]);
    if (e == hipSuccess) e = hipEventCreate(&c->kev1[i]);
  }
  if (e == hipSuccess) e = hipMalloc((void**)&c->d_counters, 16 * sizeof(unsigned long long));
  if (e != hipSuccess) {
    lt_ctx_destroy(c);
    return fail(LT_EHIP, "lt_ctx_create: %s", hipGetErrorString(e));
  }
  *out = c;
  return LT_OK;
}

lt_status lt_ctx_destroy(lt_ctx* c) {
  if (!c) return LT_OK;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  if (c->cstream) (void)hipStreamSynchronize(c->cstream);
  dfree(c->d_counters);
  dfree(c->d_wide);
  for (lt_arena& a : c->spare) {
    dfree(a.d);
    if (a.h) (void)hipHostFree(a.h);
  }
  for (int i = 0; i < lt_ctx::KRING; ++i) {
    if (c->kev0[i]) (void)hipEventDestroy(c->kev0[i]);
    if (c->kev1[i]) (void)hipEventDestroy(c->kev1[i]);
  }
  if (c->stream) (void)hipStreamDestroy(c->stream);
  if (c->ustream) (void)hipStreamDestroy(c->ustream);
  if (c->cstream) (void)hipStreamDestroy(c->cstream);
  delete c;
  return LT_OK;
}

lt_status lt_sync(lt_ctx* c) {
  if (!c) return fail(LT_EINVAL, "lt_sync: ctx is NULL");
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(hipStreamSynchronize(c->stream));
  HIP_TRY(hipStreamSynchronize(c->cstream));
  return LT_OK;
}

// ---------------------------------------------------------------- model --
// Dense class-3 table (see lt_common.h): the tag values of the class-3 keys,
// a multiplier whose d3_index is injective on them, and the coefficient
// array.  Left disabled (mul 0) when there are more than D3_DIM values, no
// multiplier is found, or a coefficient collides with the absent marker.
static void build_dense3(const std::vector<KeyRec>& keys, uint32_t& mul, std::vector<double>& tab) {
  mul = 0;
  std::vector<uint32_t> vals;
  for (const KeyRec& k : keys)
    if (k.cls == 3) {
      vals.push_back(k.a);
      vals.push_back(k.b);
      uint64_t bits;
      std::memcpy(&bits, &k.coef, 8);
      if (bits == D3_ABSENT) return;
    }
  if (vals.empty()) return;
  std::sort(vals.begin(), vals.end());
  vals.erase(std::unique(vals.begin(), vals.end()), vals.end());
  if (vals.size() > (size_t)D3_DIM) return;
  // bit windows first (d3_window), then odd multipliers
  for (int off = 0; off <= 32 - D3_BITS && !mul; ++off) {
    const uint32_t cand = 1u << (32 - D3_BITS - off);
    uint64_t used = 0;
    bool inj = true;
    for (uint32_t v : vals) {
      const uint64_t bit = 1ull << d3_index(v, cand);
      if (used & bit) { inj = false; break; }
      used |= bit;
    }
    if (inj) mul = cand;
  }
  uint32_t m = 0x9E3779B1u;
  for (int trial = 0; trial < 20000 && !mul; ++trial, m = m * 0x2C1B3C6Du + 0x297A2D39u) {
    const uint32_t cand = m | 1u;
    uint64_t used = 0;
    bool inj = true;
    for (uint32_t v : vals) {
      const uint64_t bit = 1ull << d3_index(v, cand);
      if (used & bit) { inj = false; break; }
      used |= bit;
    }
    if (inj) mul = cand;
  }
  if (!mul) return;
  double absent;
  std::memcpy(&absent, &D3_ABSENT, 8);
  tab.assign((size_t)D3_DIM * D3_DIM, absent);
  for (const KeyRec& k : keys)
    if (k.cls == 3) tab[(size_t)d3_index(k.a, mul) * D3_DIM + d3_index(k.b, mul)] = k.coef;
}

// Host-side model image: validated keys, the built cuckoo table and the
// dense class-3 table.  Built without a GPU (lt_image_build), uploaded by
// lt_model_create_from_image; lt_model_create does both.
struct lt_image {
  int narrow = 0;
  uint32_t seed = 0;
  int64_t slots = 0;
  std::vector<SlotN> tn;
  std::vector<SlotW> tw;
  uint32_t d3mul = 0;
  std::vector<double> d3;
  std::vector<KeyRec> keys;   // validated keys (freed once the tables are built)
};

lt_status lt_image_build(const lt_model_desc* d, lt_image** out) {
  if (!d || !out) return fail(LT_EINVAL, "lt_image_build: NULL argument");
  *out = nullptr;
  if (d->n_keys < 0 || (d->n_keys > 0 && (!d->keys || !d->coefs)))
    return fail(LT_EINVAL, "lt_model_create: bad key arrays");
  if (d->n_keys > ((int64_t)1 << 29)) return fail(LT_EUNSUPPORTED, "lt_model_create: too many keys");
  std::unique_ptr<lt_image> img(new (std::nothrow) lt_image);
  if (!img) return fail(LT_ENOMEM, "lt_model_create: out of host memory");
  std::vector<KeyRec>& keys = img->keys;
  uint32_t max_id = 0;
  bool any_x = false;                         // keys of a further trigram scorer: wide slots
  try {
    keys.resize((size_t)d->n_keys);
  } catch (...) {
    return fail(LT_ENOMEM, "lt_model_create: out of host memory");
  }
  for (int64_t i = 0; i < d->n_keys; ++i) {
    const uint32_t a = d->keys[4 * i], b = d->keys[4 * i + 1], cc = d->keys[4 * i + 2],
                   cls = d->keys[4 * i + 3];
    // class + LT_XTRI_CLASS_STRIDE * t: trigram scorer t of the composite
    const uint32_t base = cls % LT_XTRI_CLASS_STRIDE, scorer = cls / LT_XTRI_CLASS_STRIDE;
    if (!(base <= 3 || base == 7 || base == 8) || scorer >= LT_MAX_TRI)
      return fail(LT_EINVAL, "lt_model_create: key %lld has class %u (only 0,1,2,3,7,8 are probed, "
                             "+ %d per further trigram scorer, at most %d scorers)",
                  (long long)i, cls, LT_XTRI_CLASS_STRIDE, LT_MAX_TRI);
    if (scorer > 0) any_x = true;
    const bool two = (base == 1 || base == 3 || base == 8);
    if (a == 0 || b == 0 || (two ? cc != 0 : cc == 0))
      return fail(LT_EINVAL, "lt_model_create: key %lld has a bad component id", (long long)i);
    if (std::isnan(d->coefs[i]))
      return fail(LT_EUNSUPPORTED, "lt_model_create: NaN coefficient at key %lld", (long long)i);
    keys[(size_t)i] = KeyRec{a, b, cc, cls, d->coefs[i]};
    max_id = std::max(max_id, std::max(a, std::max(b, cc)));
  }
  // (the narrow key holds a 3-bit class code: a further scorer's classes
  // need the wide slot)
  const bool narrow = max_id < (1u << NARROW_ID_BITS) && !any_x;
  const int64_t slot_bytes = narrow ? (int64_t)sizeof(SlotN) : (int64_t)sizeof(SlotW);
  // load factor <= 0.45 (LT_TABLE_LOAD: a lower bound for table-size
  // experiments -- fewer keys displaced to their secondary slot, so fewer
  // flagged primaries, against a larger footprint in the caches)
  double max_load = 0.45;
  if (const char* env = std::getenv("LT_TABLE_LOAD")) {
    const double v = std::atof(env);
    if (v > 0.0 && v < max_load) max_load = v;
  }
  int64_t slots = std::max<int64_t>(64, (int64_t)(d->n_keys / max_load) + 1);
  if (narrow) {                                 // narrow slot hash: a power of two (lt_common.h)
    int64_t p2 = 64;
    while (p2 < slots) p2 <<= 1;
    slots = p2;
  }
  uint32_t seed = 0x2545F491u;
  bool ok = false;
  for (int attempt = 0; attempt < 24 && !ok; ++attempt) {
    if (slots * slot_bytes >= ((int64_t)1 << 31))
      return fail(LT_EUNSUPPORTED, "lt_model_create: table of %lld slots exceeds 2 GiB",
                  (long long)slots);
    int64_t dup = -1;
    try {
      ok = narrow ? cuckoo_build(keys, (uint32_t)slots, seed, img->tn, &dup)
                  : cuckoo_build(keys, (uint32_t)slots, seed, img->tw, &dup);
    } catch (...) {
      return fail(LT_ENOMEM, "lt_model_create: cannot allocate %lld slots", (long long)slots);
    }
    if (dup >= 0) return fail(LT_EINVAL, "lt_model_create: duplicate key %lld", (long long)dup);
    if (!ok) {
      seed = seed * 0x9E3779B1u + 0x7F4A7C15u;
      if (attempt % 3 == 2) slots = narrow ? slots * 2 : slots + slots / 8;
    }
  }
  if (!ok) return fail(LT_EINVAL, "lt_model_create: cuckoo table build failed");
  build_dense3(keys, img->d3mul, img->d3);
  img->narrow = narrow ? 1 : 0;
  img->seed = seed;
  img->slots = slots;
  std::vector<KeyRec>().swap(keys);
  *out = img.release();
  return LT_OK;
}

lt_status lt_image_view(const lt_image* img, lt_model_image* v) {
  if (!img || !v) return fail(LT_EINVAL, "lt_image_view: NULL argument");
  v->hash_version = HASH_VERSION;
  v->narrow = img->narrow;
  v->seed = img->seed;
  v->slots = img->slots;
  v->table = img->narrow ? (const void*)img->tn.data() : (const void*)img->tw.data();
  v->table_bytes = img->slots * (img->narrow ? (int64_t)sizeof(SlotN) : (int64_t)sizeof(SlotW));
  v->d3mul = img->d3mul;
  v->d3 = img->d3mul ? img->d3.data() : nullptr;
  return LT_OK;
}

lt_status lt_image_destroy(lt_image* img) {
  delete img;
  return LT_OK;
}

static lt_status model_upload(lt_ctx* c, const lt_model_image* v, lt_model** out) {
  HIP_TRY(hipSetDevice(c->device));
  lt_model* m = new (std::nothrow) lt_model;
  if (!m) return fail(LT_ENOMEM, "lt_model_create: out of host memory");
  m->ctx = c;
  m->slots = v->slots;
  m->seed = v->seed;
  m->narrow = v->narrow ? 1 : 0;
  {
    const int64_t sb = m->narrow ? (int64_t)sizeof(SlotN) : (int64_t)sizeof(SlotW);
    const char* t = static_cast<const char*>(v->table);
    for (int64_t i = 0; i < v->slots && m->inf_signs != 3; ++i) {
      double cf;
      std::memcpy(&cf, t + i * sb + (m->narrow ? offsetof(SlotN, coef) : offsetof(SlotW, coef)), 8);
      m->inf_signs |= inf_sign_bits(cf);
    }
    if (v->d3mul && v->d3)
      for (int i = 0; i < D3_DIM * D3_DIM; ++i) m->inf_signs |= inf_sign_bits(v->d3[i]);
  }
  hipError_t e = hipMalloc(&m->d_table, (size_t)v->table_bytes);
  if (e == hipSuccess)
    e = hipMemcpyAsync(m->d_table, v->table, (size_t)v->table_bytes, hipMemcpyHostToDevice, c->stream);
  if (e == hipSuccess) e = hipMalloc(&m->d_plain, (size_t)v->table_bytes);
  if (e == hipSuccess) e = launch_strip_flags(m->d_plain, m->d_table, v->table_bytes, m->narrow != 0, c->stream);
  // (an image whose multiplier is not a bit window -- a pack from an older
  // build -- decodes without the dense table: class 3 from the hashed table)
  if (e == hipSuccess && v->d3mul && d3_window(v->d3mul) >= 0) {
    m->d3mul = v->d3mul;
    m->d3off = (uint32_t)d3_window(v->d3mul);
    e = dalloc_copy(&m->d_d3, v->d3, (size_t)D3_DIM * D3_DIM, c->stream);
  }
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  if (e != hipSuccess) {
    dfree(m->d_table);
    dfree(m->d_plain);
    dfree(m->d_d3);
    delete m;
    return fail(LT_EHIP, "lt_model_create: %s", hipGetErrorString(e));
  }
  *out = m;
  return LT_OK;
}

lt_status lt_model_create_from_image(lt_ctx* c, const lt_model_image* v, lt_model** out) {
  if (!c || !v || !out) return fail(LT_EINVAL, "lt_model_create_from_image: NULL argument");
  *out = nullptr;
  if (v->hash_version != HASH_VERSION)
    return fail(LT_EUNSUPPORTED, "model image: hash version %u, this library uses %u (rebuild the image)",
                v->hash_version, HASH_VERSION);
  if (v->narrow != 0 && v->narrow != 1) return fail(LT_EINVAL, "model image: bad narrow flag");
  if (v->slots < 64 || !v->table) return fail(LT_EINVAL, "model image: empty table");
  if (v->narrow && (v->slots & (v->slots - 1)) != 0)
    return fail(LT_EINVAL, "model image: a narrow table has a power-of-two slot count");
  const int64_t sb = v->narrow ? (int64_t)sizeof(SlotN) : (int64_t)sizeof(SlotW);
  if (v->slots > (((int64_t)1 << 31) - 1) / sb || v->table_bytes != v->slots * sb)
    return fail(LT_EINVAL, "model image: table size %lld does not match %lld slots",
                (long long)v->table_bytes, (long long)v->slots);
  if (v->d3mul && !v->d3) return fail(LT_EINVAL, "model image: dense table missing");
  return model_upload(c, v, out);
}

lt_status lt_model_create(lt_ctx* c, const lt_model_desc* d, lt_model** out) {
  if (!c || !d || !out) return fail(LT_EINVAL, "lt_model_create: NULL argument");
  *out = nullptr;
  lt_image* img = nullptr;
  lt_status st = lt_image_build(d, &img);
  if (st != LT_OK) return st;
  lt_model_image v;
  lt_image_view(img, &v);
  st = model_upload(c, &v, out);
  lt_image_destroy(img);
  return st;
}

lt_status lt_model_destroy(lt_model* m) {
  if (!m) return LT_OK;
  (void)hipSetDevice(m->ctx->device);
  dfree(m->d_table);
  dfree(m->d_plain);
  dfree(m->d_d3);
  delete m;
  return LT_OK;
}

int64_t lt_model_slots(const lt_model* m) { return m ? m->slots : 0; }

// ---------------------------------------------------------------- batch --
static lt_status validate(const lt_batch_desc* d, int* inf_signs) {
  if (d->n_sent < 0 || d->n_nodes < 0 || d->n_span < 0 || d->n_post < 0)
    return fail(LT_EINVAL, "batch: negative size");
  if (d->max_len < 1 || d->max_len > LT_MAX_LEN_ANY)
    return fail(LT_EUNSUPPORTED, "batch: max_len %d not in 1..%d", d->max_len, LT_MAX_LEN_ANY);
  const int SS = span_slots(d->max_len);
  if (!d->sent_n || !d->sent_node_off || !d->sent_span_off)
    return fail(LT_EINVAL, "batch: NULL sentence arrays");
  if (d->n_nodes > 0 && (!d->node_word || !d->node_morph0 || !d->node_tag || !d->node_mask ||
                         !d->node_pre || !d->node_f4 || !d->node_f5 || !d->node_f6))
    return fail(LT_EINVAL, "batch: NULL node arrays");
  if (d->n_post > 0 && !d->node_post) return fail(LT_EINVAL, "batch: NULL node_post");
  if (d->n_edge < 0) return fail(LT_EINVAL, "batch: negative n_edge");
  if (d->n_xtri < 0 || d->n_xtri >= LT_MAX_TRI)
    return fail(LT_EUNSUPPORTED, "batch: n_xtri %d not in 0..%d", d->n_xtri, LT_MAX_TRI - 1);
  if (d->n_xtri > 0) {
    if (!d->has_trigram) return fail(LT_EINVAL, "batch: n_xtri > 0 without the first trigram term");
    if (d->n_unk != 0) return fail(LT_EUNSUPPORTED, "batch: implicit Unknowns (n_unk) with several trigram terms");
    if (d->n_nodes > 0 && (!d->xtri_mask || !d->xtri_f4 || !d->xtri_f5 || !d->xtri_f6))
      return fail(LT_EINVAL, "batch: NULL xtri arrays");
  }
  if (d->n_edge > 0 || d->n_xtri > 0) {
    // the term plan: every node_post row, every edge row and every trigram
    // term (when the batch has them) exactly once
    if (d->n_terms < 1 || d->n_terms > 32) return fail(LT_EINVAL, "batch: n_terms %d not in 1..32", d->n_terms);
    if (d->n_terms < 32 && (d->term_kinds >> (2 * d->n_terms)) != 0)
      return fail(LT_EINVAL, "batch: term_kinds has bits past n_terms");
    int kinds[4] = {0, 0, 0, 0};
    for (int t = 0; t < d->n_terms; ++t) ++kinds[(d->term_kinds >> (2 * t)) & 3u];
    if (kinds[3] || kinds[1] != d->n_post || kinds[2] != d->n_edge ||
        kinds[0] != (d->has_trigram ? 1 + d->n_xtri : 0))
      return fail(LT_EINVAL, "batch: term_kinds does not list the %d trigram terms, the %d node_post rows and the %d "
                             "edge rows once each", d->has_trigram ? 1 + d->n_xtri : 0, d->n_post, d->n_edge);
  }
  if (d->n_edge > 0) {
    if (!d->sent_edge_off || (d->n_nodes > 0 && !d->node_edge_base) || (d->n_edges > 0 && !d->edge_val))
      return fail(LT_EINVAL, "batch: NULL edge arrays");
    if (d->sent_edge_off[0] != 0 || d->sent_edge_off[d->n_sent] != d->n_edges || d->n_edges < 0)
      return fail(LT_EINVAL, "batch: sent_edge_off must run from 0 to n_edges");
    for (int32_t s = 0; s < d->n_sent; ++s)
      if (d->sent_edge_off[s + 1] < d->sent_edge_off[s]) return fail(LT_EINVAL, "batch: sent_edge_off not monotone");
  }
  if (d->n_unk != 0) {
    // implicit Unknowns: one canonical record per span length d = 1..S
    if (d->n_unk != SS) return fail(LT_EINVAL, "batch: n_unk %d is neither 0 nor the %d span slots", d->n_unk, SS);
    if (d->n_edge > 0) return fail(LT_EUNSUPPORTED, "batch: implicit Unknowns (n_unk) with edge terms");
    if (!d->unk_word || !d->unk_morph0 || !d->unk_tag || !d->unk_mask || !d->unk_pre || !d->unk_f4 ||
        !d->unk_f5 || !d->unk_f6 || (d->n_post > 0 && !d->unk_post))
      return fail(LT_EINVAL, "batch: NULL implicit-Unknown arrays");
  }
  if (d->n_span > 0 && !d->span_start) return fail(LT_EINVAL, "batch: NULL span_start");
  if (d->sent_node_off[0] != 0 || d->sent_span_off[0] != 0)
    return fail(LT_EINVAL, "batch: offsets must start at 0");
  if (d->sent_node_off[d->n_sent] != d->n_nodes || d->sent_span_off[d->n_sent] != d->n_span)
    return fail(LT_EINVAL, "batch: offsets do not end at n_nodes / n_span");
  // per-sentence and per-node checks on threads; the first failure (lowest
  // index) is reported
  struct Bad {
    int64_t at = -1;
    lt_status st = LT_OK;
    std::string msg;
  };
  auto first_bad = [](std::vector<Bad>& bad) -> const Bad* {
    for (const Bad& x : bad)
      if (x.at >= 0) return &x;
    return nullptr;
  };
  std::vector<Bad> bad(32);
  std::vector<int> sgn(32, 0);            // inf_sign_bits of the node terms, per worker
  auto note = [](Bad& b, int64_t at, lt_status st, const char* fmt, long long a, long long c, long long e) {
    char buf[256];
    snprintf(buf, sizeof buf, fmt, a, c, e);
    b.at = at;
    b.st = st;
    b.msg = buf;
  };
  // sentence ranges: a sentence is hundreds of nodes, so split at 256 sentences
  parallel_ranges(d->n_sent, [&](int t, int64_t lo, int64_t hi) {
    for (int64_t s = lo; s < hi; ++s) {
      const int64_t n = d->sent_n[s];
      const int64_t nodes = d->sent_node_off[s + 1] - d->sent_node_off[s];
      const int64_t spans = d->sent_span_off[s + 1] - d->sent_span_off[s];
      if (n < 0 || spans != SS * n + 1)
        return note(bad[t], s, LT_EINVAL, "batch: sentence %lld has %lld span entries for %lld chars", s, spans, n);
      if (nodes < 1 || nodes >= MAX_LOCAL_NODES)
        return note(bad[t], s, LT_EINVAL, "batch: sentence %lld has %lld nodes%.0lld", s, nodes, 0);
      const int32_t* ss = d->span_start + d->sent_span_off[s];
      if (ss[0] != 1 || ss[spans - 1] != nodes)
        return note(bad[t], s, LT_EINVAL, "batch: sentence %lld span table does not cover its nodes%.0lld%.0lld", s, 0, 0);
      for (int64_t e = 1; e <= n; ++e) {
        const int64_t dmax = std::min<int64_t>(e, d->max_len);
        for (int j = 0; j < SS; ++j) {
          const int64_t idx = (e - 1) * SS + j;
          const int32_t cnt = ss[idx + 1] - ss[idx];
          const int dd = SS - j;
          if (cnt < 0)
            return note(bad[t], s, LT_EINVAL, "batch: sentence %lld span table not monotone%.0lld%.0lld", s, 0, 0);
          if (dd <= dmax && cnt == 0 && d->n_unk == 0)
            return note(bad[t], s, LT_EINVAL, "batch: sentence %lld span (e=%lld,d=%lld) has no candidate", s, e, dd);
          if (dd > dmax && cnt != 0)
            return note(bad[t], s, LT_EINVAL, "batch: sentence %lld span (e=%lld,d=%lld) is out of range", s, e, dd);
          if (d->n_edge > 0 && cnt > 0) {
            // the candidates' predecessors: the nodes of end position b (BOS
            // for b = 0); their values must lie in the sentence's edge block
            const int64_t b = e - dd;
            const int64_t plo = b == 0 ? 0 : ss[(b - 1) * SS], phi = b == 0 ? 1 : ss[b * SS];
            for (int32_t v = ss[idx]; v < ss[idx + 1]; ++v) {
              const int64_t base = d->node_edge_base[d->sent_node_off[s] + v];
              if (base + plo < d->sent_edge_off[s] || base + phi > d->sent_edge_off[s + 1])
                return note(bad[t], s, LT_EINVAL, "batch: sentence %lld node %lld edge values outside the "
                                                  "sentence's block%.0lld", s, v, 0);
            }
          }
        }
      }
    }
  }, 256);
  if (const Bad* x = first_bad(bad)) return fail(x->st, "%s", x->msg.c_str());
  parallel_ranges(d->n_nodes, [&](int t, int64_t lo, int64_t hi) {
    for (int64_t i = lo; i < hi; ++i) {
      if (d->node_word[i] < 0 || d->node_morph0[i] < 0 || d->node_tag[i] < 0)
        return note(bad[t], i, LT_EINVAL, "batch: node %lld has a negative id%.0lld%.0lld", i, 0, 0);
      if (std::isnan(d->node_pre[i]) || std::isnan(d->node_f4[i]) || std::isnan(d->node_f5[i]) ||
          std::isnan(d->node_f6[i]))
        return note(bad[t], i, LT_EUNSUPPORTED, "batch: node %lld has a NaN score term%.0lld%.0lld", i, 0, 0);
      sgn[t] |= inf_sign_bits(d->node_pre[i]) | inf_sign_bits(d->node_f4[i]) | inf_sign_bits(d->node_f5[i]) |
                inf_sign_bits(d->node_f6[i]);
    }
  });
  if (const Bad* x = first_bad(bad)) return fail(x->st, "%s", x->msg.c_str());
  int signs = 0;
  for (int v : sgn) signs |= v;
  for (int64_t i = 0; i < (int64_t)d->n_post * d->n_nodes; ++i) {
    if (std::isnan(d->node_post[i])) return fail(LT_EUNSUPPORTED, "batch: NaN post term %lld", (long long)i);
    signs |= inf_sign_bits(d->node_post[i]);
  }
  for (int32_t i = 0; i < d->n_unk; ++i) {
    if (d->unk_word[i] < 0 || d->unk_morph0[i] < 0 || d->unk_tag[i] < 0)
      return fail(LT_EINVAL, "batch: implicit Unknown %d has a negative id", i);
    const double v[4] = {d->unk_pre[i], d->unk_f4[i], d->unk_f5[i], d->unk_f6[i]};
    for (double x : v) {
      if (std::isnan(x)) return fail(LT_EUNSUPPORTED, "batch: implicit Unknown %d has a NaN score term", i);
      signs |= inf_sign_bits(x);
    }
    for (int32_t t = 0; t < d->n_post; ++t) {
      const double x = d->unk_post[(int64_t)t * d->n_unk + i];
      if (std::isnan(x)) return fail(LT_EUNSUPPORTED, "batch: implicit Unknown %d has a NaN post term", i);
      signs |= inf_sign_bits(x);
    }
  }
  for (int64_t i = 0; d->n_edge > 0 && i < (int64_t)d->n_edge * d->n_edges; ++i) {
    if (std::isnan(d->edge_val[i])) return fail(LT_EUNSUPPORTED, "batch: NaN edge term %lld", (long long)i);
    signs |= inf_sign_bits(d->edge_val[i]);
  }
  for (int64_t i = 0; i < (int64_t)d->n_xtri * d->n_nodes; ++i) {
    const double v[3] = {d->xtri_f4[i], d->xtri_f5[i], d->xtri_f6[i]};
    for (double x : v) {
      if (std::isnan(x)) return fail(LT_EUNSUPPORTED, "batch: NaN trigram coefficient of node entry %lld", (long long)i);
      signs |= inf_sign_bits(x);
    }
  }
  if (signs == 3)
    return fail(LT_EUNSUPPORTED, "batch: both +inf and -inf among the node score terms (their sum is a NaN, "
                                 "whose place in Python's sort is not reproduced)");
  *inf_signs = signs;
  return LT_OK;
}

static void arena_free(lt_arena& a) {
  dfree(a.d);
  if (a.h) (void)hipHostFree(a.h);
  a = lt_arena{};
}

// Arenas up to this size are kept for reuse, at most SPARE_N per context
// (Tagger.tag_batch keeps up to four chunk batches in flight, one more is
// queued)
// and at most SPARE_BYTES (device + pinned host) in all: the largest batches
// seen do not pin gigabytes for the context's lifetime.
constexpr size_t SPARE_MAX = (size_t)1 << 30;
constexpr size_t SPARE_N = 6;
constexpr size_t SPARE_BYTES = (size_t)3 << 30;

static size_t arena_bytes(const lt_arena& a) { return a.d_bytes + a.h_bytes; }

// New arenas are sized with headroom and rounded up to one of eight size
// classes per power of two, so that a recycled arena fits the next batches
// of similar size (chunks of one pipeline differ by a few per cent) instead
// of each slightly larger batch paying a device and a pinned host allocation.
static size_t arena_class(size_t n) {
  if (n == 0) return 0;
  n += n / 16;
  size_t g = 256;
  while ((g << 4) <= n) g <<= 1;                 // granule: 1/8 .. 1/16 of n
  return (n + g - 1) / g * g;
}

// An arena with at least (dn, hn) bytes: the smallest fitting spare, else a
// new allocation (a spare that does not fit stays for a later batch).  When
// the allocation fails, the spares (none of which fit) are freed and it is
// tried once more, so idle pooled memory never causes LT_ENOMEM.
static hipError_t arena_take(lt_ctx* c, size_t dn, size_t hn, lt_arena& out) {
  {
    std::lock_guard<std::mutex> g(c->mu);
    int best = -1;
    for (int i = 0; i < (int)c->spare.size(); ++i)
      if (c->spare[i].d_bytes >= dn && c->spare[i].h_bytes >= hn &&
          (best < 0 || c->spare[i].d_bytes < c->spare[best].d_bytes))
        best = i;
    if (best >= 0) {
      out = c->spare[best];
      c->spare.erase(c->spare.begin() + best);
      return hipSuccess;
    }
  }
  dn = arena_class(dn);
  hn = arena_class(hn);
  hipError_t e = hipSuccess;
  for (int attempt = 0; attempt < 2; ++attempt) {
    out = lt_arena{};
    e = hipSuccess;
    if (dn) e = hipMalloc((void**)&out.d, dn);
    if (e == hipSuccess) out.d_bytes = dn;
    if (e == hipSuccess && hn) e = hipHostMalloc((void**)&out.h, hn, hipHostMallocDefault);
    if (e == hipSuccess) out.h_bytes = hn;
    if (e == hipSuccess) return e;
    arena_free(out);
    std::vector<lt_arena> drop;
    {
      std::lock_guard<std::mutex> g(c->mu);
      drop.swap(c->spare);
    }
    if (drop.empty()) break;                    // nothing pooled to give back
    (void)hipGetLastError();                    // (clear the failed allocation's error)
    for (lt_arena& a : drop) arena_free(a);
  }
  return e;
}

// Back to the spares; with SPARE_N kept, the smallest of them and this one
// is freed.
static void arena_give(lt_ctx* c, lt_arena& a) {
  if (!a.d && !a.h) return;
  if (a.d_bytes <= SPARE_MAX) {
    std::lock_guard<std::mutex> g(c->mu);
    size_t held = 0;
    for (const lt_arena& x : c->spare) held += arena_bytes(x);
    if (c->spare.size() < SPARE_N && held + arena_bytes(a) <= SPARE_BYTES) {
      c->spare.push_back(a);
      a = lt_arena{};
      return;
    }
    // full: the smallest of the spares and this one is freed, as long as the
    // swap keeps the pool within SPARE_BYTES
    int small = 0;
    for (int i = 1; i < (int)c->spare.size(); ++i)
      if (arena_bytes(c->spare[i]) < arena_bytes(c->spare[small])) small = i;
    if (!c->spare.empty() && arena_bytes(c->spare[small]) < arena_bytes(a) &&
        held - arena_bytes(c->spare[small]) + arena_bytes(a) <= SPARE_BYTES)
      std::swap(c->spare[small], a);
  }
  arena_free(a);
}

static void batch_free(lt_batch* b) {
  if (!b) return;
  for (auto& evs : b->ev_rd)
    for (hipEvent_t ev : evs)
      if (ev) (void)hipEventDestroy(ev);
  if (b->prep_ev0) (void)hipEventDestroy(b->prep_ev0);
  if (b->prep_ev1) (void)hipEventDestroy(b->prep_ev1);
  if (b->lazy_sched)
    for (lt_piece& pc : b->pieces) {
      dfree(pc.d_sched);
      dfree(pc.d_wave_off);
      dfree(pc.d_place);
    }
  arena_give(b->ctx, b->arena);
  delete b;
}

// Point the batch's current-result pointers at result slot i.
static void use_slot(lt_batch* b, int i) {
  b->cur = i;
  b->d_count = b->res[i].count;
  b->d_len = b->res[i].len;
  b->d_score = b->res[i].score;
  b->d_codes = b->res[i].codes;
}

// Sub-buffers of an arena: 256 B aligned, nullptr for empty ones.
struct Carve {
  size_t d = 0, h = 0;
  static size_t al(size_t x) { return (x + 255) & ~(size_t)255; }
  size_t dev(size_t bytes) {
    const size_t o = d;
    d += al(bytes);
    return bytes ? o : SIZE_MAX;
  }
  size_t host(size_t bytes) {
    const size_t o = h;
    h += al(bytes);
    return bytes ? o : SIZE_MAX;
  }
};
extern "C++" {
template <class T>
static T* at(char* base, size_t off) {
  return off == SIZE_MAX ? nullptr : reinterpret_cast<T*>(base + off);
}
}  // extern "C++"

// Launch pieces: consecutive sentence ranges whose node records and
// backpointers each stay below 2^31 B (the kernels address them with 32-bit
// buffer offsets).  A batch of any size is decoded as one launch per piece,
// all writing one result array.
static std::atomic<int64_t> g_piece_bytes{((int64_t)1 << 31) - 1};

// Backpointer words per (position, rank): two for the general kernel.
static int bp_words(int max_len, int max_k, int n_xtri = 0) {
  return (decode_is_wide(max_len, max_k) || n_xtri > 0) ? 2 : 1;
}
// the general kernel decodes every beam of a batch with further trigram terms
static bool batch_wide(const lt_batch* b, int k) { return decode_is_wide(b->max_len, k) || b->n_xtri > 0; }

static std::vector<std::pair<int32_t, int32_t>> piece_ranges(const lt_batch_desc* d, int max_k) {
  const int64_t lim = g_piece_bytes.load();
  std::vector<std::pair<int32_t, int32_t>> out;
  int32_t s0 = 0;
  int64_t nodes = 0, bp = 0;
  for (int32_t s = 0; s < d->n_sent; ++s) {
    const int64_t sn = (d->sent_node_off[s + 1] - d->sent_node_off[s]) * (int64_t)sizeof(NodeRec);
    const int64_t sb = ((int64_t)d->sent_n[s] + 1) * max_k * 4 * bp_words(d->max_len, max_k, d->n_xtri);
    if (s > s0 && (nodes + sn > lim || bp + sb > lim)) {
      out.emplace_back(s0, s);
      s0 = s;
      nodes = bp = 0;
    }
    nodes += sn;
    bp += sb;
  }
  if (d->n_sent > s0 || out.empty()) out.emplace_back(s0, d->n_sent);
  return out;
}

static void piece_params(const lt_batch* b, size_t q, int k, DecodeParams& p);

// The batch's device preparation, queued on `st` unless done: the k=1 lane
// schedule of every piece (lt_k1_sched), between the batch's prep events.  No
// allocation (arena memory) and no wait.
// characters (end positions) of piece q
static int64_t piece_chars(const lt_batch* b, size_t q) {
  return (q + 1 < b->pieces.size() ? b->pieces[q + 1].chars0 : b->total_chars) - b->pieces[q].chars0;
}

static hipError_t prep_fill(lt_batch* b, hipStream_t st) {
  if (!b->has_sched || b->prep_done) return hipSuccess;
  hipError_t e = hipSuccess;
  if (!b->prep_ev0) e = hipEventCreate(&b->prep_ev0);
  if (e == hipSuccess && !b->prep_ev1) e = hipEventCreate(&b->prep_ev1);
  const size_t P = b->pieces.size();
  for (size_t q = 0; e == hipSuccess && q < P; ++q) {
    DecodeParams p{};
    piece_params(b, q, 1, p);
    p.max_len = b->max_len;
    p.n_unk = b->n_unk;
    e = launch_k1_sched_fill(p, b->pieces[q].d_wave_off, b->pieces[q].d_sched, st, q == 0 ? b->prep_ev0 : nullptr,
                             q + 1 == P ? b->prep_ev1 : nullptr);
  }
  if (e == hipSuccess) {
    b->prep_done = true;
    b->prep_fused = false;
  }
  return e;
}

// LT_K1_FUSED_FILL (default 1): a fresh beam-1 schedule filled inside the decode
static bool fused_fill_on() {
  static const bool on = [] {
    const char* v = std::getenv("LT_K1_FUSED_FILL");
    return !(v && v[0] == '0');
  }();
  return on;
}

// The k=1 lane schedule of a batch created for larger beams, at its first
// beam-1 decode: each wave's macro-steps counted on the device
// (lt_k1_sched_count), the offsets summed on the host (one synchronisation),
// the schedule in buffers of its own; prep_fill then fills it as for a beam-1
// batch.
static lt_status lazy_sched(lt_ctx* c, lt_batch* b) {
  if (b->has_sched || b->max_len > MAX_SPAN || b->n_xtri > 0) return LT_OK;
  // every buffer in locals first, published to the pieces only once all of
  // them exist (a failure frees what it allocated: a later decode retries
  // from scratch, nothing leaks)
  const size_t P = b->pieces.size();
  std::vector<int64_t*> d_off(P, nullptr);
  std::vector<uint32_t*> d_place(P, nullptr), d_sched(P, nullptr);
  std::vector<int64_t> steps(P, 0);
  auto undo = [&]() {
    (void)hipStreamSynchronize(c->stream);
    for (size_t q = 0; q < P; ++q) {
      dfree(d_off[q]);
      dfree(d_place[q]);
      dfree(d_sched[q]);
    }
  };
  std::vector<std::vector<int64_t>> offs(P);
  for (size_t q = 0; q < P; ++q) {
    const lt_piece& pc = b->pieces[q];
    if (pc.n_nodes >= (int64_t)K1_NODE) {
      undo();
      return fail(LT_EUNSUPPORTED, "decode: %lld nodes in one launch piece for the beam-1 schedule",
                  (long long)pc.n_nodes);
    }
    const int waves = k1_waves(pc.n_sent);
    hipError_t e = hipMalloc((void**)&d_off[q], ((size_t)waves + 1) * 8);
    if (e == hipSuccess) e = hipMalloc((void**)&d_place[q], (size_t)std::max<int64_t>(piece_chars(b, q), 1) * 4);
    DecodeParams p{};
    if (e == hipSuccess) {
      piece_params(b, q, 1, p);
      p.max_len = b->max_len;
      p.k1_place = d_place[q];
      e = launch_k1_sched_count(p, d_off[q], c->stream);
    }
    offs[q].assign((size_t)waves + 1, 0);
    if (e == hipSuccess)
      e = hipMemcpyAsync(offs[q].data(), d_off[q], (size_t)waves * 8, hipMemcpyDeviceToHost, c->stream);
    if (e != hipSuccess) {
      undo();
      return fail(e == hipErrorOutOfMemory ? LT_ENOMEM : LT_EHIP, "decode: beam-1 schedule: %s", hipGetErrorString(e));
    }
  }
  hipError_t e = hipStreamSynchronize(c->stream);
  for (size_t q = 0; e == hipSuccess && q < P; ++q) {
    std::vector<int64_t>& wo = offs[q];
    int64_t run = 0;
    for (size_t w = 0; w + 1 < wo.size(); ++w) {   // exclusive prefix sum
      const int64_t x = wo[w];
      if (x >= ((int64_t)1 << K1_TBITS)) {
        undo();
        return fail(LT_EUNSUPPORTED, "decode: %lld macro-steps in one beam-1 wave schedule", (long long)x);
      }
      wo[w] = run;
      run += x;
    }
    wo.back() = run;
    steps[q] = run;
    e = hipMalloc((void**)&d_sched[q], (size_t)std::max<int64_t>(run, 1) * 64 * 4);
    if (e == hipSuccess) e = hipMemcpyAsync(d_off[q], wo.data(), wo.size() * 8, hipMemcpyHostToDevice, c->stream);
  }
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);        // (the host offsets go out of scope)
  if (e != hipSuccess) {
    undo();
    return fail(e == hipErrorOutOfMemory ? LT_ENOMEM : LT_EHIP, "decode: beam-1 schedule: %s", hipGetErrorString(e));
  }
  for (size_t q = 0; q < P; ++q) {
    lt_piece& pc = b->pieces[q];
    pc.d_wave_off = d_off[q];
    pc.d_place = d_place[q];
    pc.d_sched = d_sched[q];
    pc.sched_steps = steps[q];
  }
  b->lazy_sched = true;
  b->has_sched = true;
  b->prep_done = false;
  return LT_OK;
}

// LT_TIMING=1: per-phase wall times of lt_batch_create on stderr (diagnostic)
static bool timing_on() {
  static const bool on = [] {
    const char* v = std::getenv("LT_TIMING");
    return v && *v && *v != '0';
  }();
  return on;
}
static double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

lt_status lt_batch_create(lt_ctx* c, const lt_batch_desc* d, int max_k, lt_batch** out) {
  if (!c || !d || !out) return fail(LT_EINVAL, "lt_batch_create: NULL argument");
  *out = nullptr;
  const double t_start = timing_on() ? now_s() : 0.0;
  double t_valid = 0, t_arena = 0, t_recs = 0;
  if (max_k < 1 || max_k > LT_MAX_BEAM_ANY)
    return fail(LT_EUNSUPPORTED, "lt_batch_create: max_k %d not in 1..%d", max_k, LT_MAX_BEAM_ANY);
  int inf_signs = 0;
  lt_status st = validate(d, &inf_signs);
  if (st != LT_OK) return st;
  if (timing_on()) t_valid = now_s();
  HIP_TRY(hipSetDevice(c->device));
  lt_batch* b = new (std::nothrow) lt_batch;
  if (!b) return fail(LT_ENOMEM, "lt_batch_create: out of host memory");
  b->ctx = c;
  b->inf_signs = inf_signs;
  b->n_sent = d->n_sent;
  b->max_len = d->max_len;
  b->n_post = d->n_post;
  b->has_tri = d->has_trigram ? 1 : 0;
  b->n_edge = d->n_edge;
  b->n_xtri = d->n_xtri;
  b->n_terms = (d->n_edge || d->n_xtri) ? d->n_terms : 0;
  b->term_kinds = (d->n_edge || d->n_xtri) ? d->term_kinds : 0;
  b->max_k = max_k;
  b->n_nodes = d->n_nodes;
  b->n_span = d->n_span;

  const int32_t S = d->n_sent;
  std::vector<int64_t> cum_n(S + 1);
  cum_n[0] = 0;
  for (int32_t s = 0; s < S; ++s) cum_n[s + 1] = cum_n[s] + d->sent_n[s];
  b->total_chars = cum_n[S];
  const auto ranges = piece_ranges(d, max_k);
  const size_t P = ranges.size();
  b->pieces.resize(P);
  // per piece: local sentence order (longest first: the grid drains
  // evenly), offsets rebased to the piece
  std::vector<std::vector<int32_t>> order(P);
  std::vector<std::vector<int64_t>> node_off(P), span_off(P), bp_off(P), pcum(P);
  for (size_t q = 0; q < P; ++q) {
    lt_piece& pc = b->pieces[q];
    const int32_t s0 = ranges[q].first, s1 = ranges[q].second, n = s1 - s0;
    pc.s0 = s0;
    pc.n_sent = n;
    pc.node0 = d->sent_node_off[s0];
    pc.span0 = d->sent_span_off[s0];
    pc.n_nodes = d->sent_node_off[s1] - pc.node0;
    pc.n_span = d->sent_span_off[s1] - pc.span0;
    pc.chars0 = cum_n[s0];
    if (d->n_edge > 0) {
      pc.edge0 = d->sent_edge_off[s0];
      pc.n_edges = d->sent_edge_off[s1] - pc.edge0;
    }
    order[q].resize(n);
    node_off[q].resize(n + 1);
    span_off[q].resize(n + 1);
    bp_off[q].resize(n + 1);
    pcum[q].resize(n + 1);
    for (int32_t s = 0; s < n; ++s) order[q][s] = s;
    std::stable_sort(order[q].begin(), order[q].end(),
                     [&](int32_t x, int32_t y) { return d->sent_n[s0 + x] > d->sent_n[s0 + y]; });
    bp_off[q][0] = 0;
    for (int32_t s = 0; s <= n; ++s) {
      node_off[q][s] = d->sent_node_off[s0 + s] - pc.node0;
      span_off[q][s] = d->sent_span_off[s0 + s] - pc.span0;
      pcum[q][s] = cum_n[s0 + s] - pc.chars0;
      if (s < n) bp_off[q][s + 1] = bp_off[q][s] + (int64_t)(d->sent_n[s0 + s] + 1) * max_k * bp_words(d->max_len, max_k, d->n_xtri);
    }
    pc.bp_entries = bp_off[q][n];
    b->bp_entries += pc.bp_entries;
  }
  // the k=1 lane schedule of every piece of a beam-1 batch (the tuned
  // kernels' layout, max_len <= 8): each wave's macro-steps counted here from
  // the span tables (threads over waves), so that the schedule is part of the
  // arena; its entries are filled on the device (prep_fill).  A batch created
  // for larger beams carries none (no host counting, no arena bytes); a k=1
  // decode of it runs on the lane-group beam kernel (launch_decode)
  b->has_sched = d->max_len <= MAX_SPAN && max_k == 1 && d->n_xtri == 0;
  b->n_unk = d->n_unk;
  std::vector<std::vector<int64_t>> wave_off(P);
  std::vector<std::vector<uint32_t>> place(P);   // k=1 placements, uploaded with the batch
  const double t_sched0 = b->has_sched ? now_s() : 0.0;
  if (b->has_sched) {
    for (size_t q = 0; q < P; ++q) {
      lt_piece& pc = b->pieces[q];
      if (pc.n_nodes >= (int64_t)K1_NODE) {
        delete b;
        return fail(LT_EUNSUPPORTED, "lt_batch_create: %lld nodes in one launch piece", (long long)pc.n_nodes);
      }
      const int waves = k1_waves(pc.n_sent);
      std::vector<int64_t>& wo = wave_off[q];
      wo.assign((size_t)waves + 1, 0);
      place[q].assign((size_t)pcum[q][(size_t)pc.n_sent], 0u);
      std::atomic<int64_t> longest{0};
      parallel_ranges(waves, [&](int, int64_t lo, int64_t hi) {
        for (int64_t w = lo; w < hi; ++w) {
          const int32_t* ssw[K1_W] = {};
          int nw[K1_W] = {}, cnt = 0;
          uint32_t* plw[K1_W] = {};
          for (int i = 0; i < K1_W && w * K1_W + i < pc.n_sent; ++i, ++cnt) {
            const int32_t sl = order[q][(size_t)(w * K1_W + i)];
            const int32_t s = pc.s0 + sl;
            ssw[cnt] = d->span_start + d->sent_span_off[s];
            nw[cnt] = d->sent_n[s];
            plw[cnt] = place[q].data() + pcum[q][(size_t)sl];
          }
          // run_at reaches every (sentence, position) once, before its
          // placement: it leaves the position's dead mask in the placement
          // word, which emit completes
          const int64_t steps = k1_schedule(
              cnt, nw,
              [&](int i, int e) {
                uint32_t dead = 0;
                const int x = k1_candidates_dead(ssw[i], e, d->max_len, &dead);
                plw[i][e - 1] = k1_place_word(0, 0, dead);
                return x;
              },
              [&](int64_t t, int i, int e, int off, int) {
                plw[i][e - 1] |= k1_place_word(t, off, 0u);   // (t < 2^K1_TBITS: checked below)
              });
          wo[(size_t)w + 1] = steps;
          int64_t m = longest.load();
          while (steps > m && !longest.compare_exchange_weak(m, steps)) {
          }
        }
      }, 64);
      if (longest.load() >= ((int64_t)1 << K1_TBITS)) {
        delete b;
        return fail(LT_EUNSUPPORTED, "lt_batch_create: %lld macro-steps in one beam-1 wave schedule",
                    (long long)longest.load());
      }
      for (int w = 0; w < waves; ++w) wo[(size_t)w + 1] += wo[(size_t)w];
      pc.sched_steps = wo[(size_t)waves];
    }
    b->host_sched_ms = (now_s() - t_sched0) * 1e3;
  }

  // the class-4/6 pair table of the records (NodeRec): the implicit
  // Unknowns' pairs first (their records are read without an escape)
  std::vector<F46> unk_pairs;
  for (int32_t i = 0; i < d->n_unk; ++i) unk_pairs.push_back(api_pair(d->unk_mask[i], d->unk_f4, d->unk_f6, i));
  const PairTable ptab = pair_table(d->n_nodes, d->node_mask, d->node_f4, d->node_f6, unk_pairs);
  for (const F46& f : unk_pairs)
    if (ptab.find(f.f4, f.f6) < 0) {
      delete b;
      return fail(LT_EUNSUPPORTED, "lt_batch_create: more than %d distinct class-4/6 coefficient pairs among "
                                   "the implicit Unknowns", MAX_PAIRS - 1);
    }
  const bool has_esc = ptab.full && d->n_nodes > 0;
  b->n_pairs = (int32_t)ptab.vals.size();

  hipStream_t stm = c->ustream;     // complete when this returns (synchronised below)
  const size_t nres = (size_t)S * max_k;
  const size_t ncodes = (size_t)b->total_chars * max_k;
  // the batch's buffers as offsets into one arena
  Carve cv;
  struct PieceOff {
    size_t order, sent_n, node_off, span_off, bp_off, cum_n, span_start, nodes, post, bp, edge_base, edge_val,
        sched, wave_off, place, xmask, xf4, xf5, xf6;
  };
  std::vector<PieceOff> po(P);
  for (size_t q = 0; q < P; ++q) {
    const lt_piece& pc = b->pieces[q];
    const size_t n = (size_t)pc.n_sent;
    const bool ed = d->n_edge > 0;
    po[q] = PieceOff{cv.dev(n * 4), cv.dev(n * 4), cv.dev((n + 1) * 8), cv.dev((n + 1) * 8),
                     cv.dev((n + 1) * 8), cv.dev((n + 1) * 8), cv.dev((size_t)pc.n_span * 4),
                     cv.dev((size_t)pc.n_nodes * sizeof(NodeRec)),
                     cv.dev((size_t)d->n_post * (size_t)pc.n_nodes * 8), cv.dev((size_t)pc.bp_entries * 4),
                     cv.dev(ed ? (size_t)pc.n_nodes * 8 : 0),
                     cv.dev(ed ? (size_t)d->n_edge * (size_t)pc.n_edges * 8 : 0),
                     cv.dev(b->has_sched ? (size_t)std::max<int64_t>(pc.sched_steps, 1) * 64 * 4 : 0),
                     cv.dev(b->has_sched ? wave_off[q].size() * 8 : 0), cv.dev(place[q].size() * 4),
                     cv.dev((size_t)d->n_xtri * (size_t)pc.n_nodes * 4), cv.dev((size_t)d->n_xtri * (size_t)pc.n_nodes * 8),
                     cv.dev((size_t)d->n_xtri * (size_t)pc.n_nodes * 8), cv.dev((size_t)d->n_xtri * (size_t)pc.n_nodes * 8)};
  }
  const size_t o_sent_n = cv.dev((size_t)S * 4), o_cum_n = cv.dev(((size_t)S + 1) * 8);
  const size_t o_unk = cv.dev((size_t)d->n_unk * sizeof(NodeRec)),
               o_unk_post = cv.dev((size_t)d->n_post * (size_t)d->n_unk * 8);
  const size_t o_pairs = cv.dev(ptab.vals.size() * sizeof(F46)),
               o_esc = cv.dev(has_esc ? (size_t)d->n_nodes * sizeof(F46) : 0);
  b->slab_cap = slab_layout(S, max_k, b->total_chars).capacity;
  const uint64_t slab_alloc = slab_alloc_bytes(S, max_k, b->total_chars);
  size_t o_count[2], o_len[2], o_score[2], o_codes[2], o_slab[2];
  for (int i = 0; i < 2; ++i) {
    o_count[i] = cv.dev((size_t)S * 4);
    o_len[i] = cv.dev(nres * 4);
    o_score[i] = cv.dev(nres * 8);
    o_codes[i] = cv.dev(ncodes * 4);
    o_slab[i] = cv.dev(slab_alloc);
  }
  const size_t h_slab = cv.host(b->slab_cap);
  const size_t h_count = cv.host((size_t)S * 4), h_len = cv.host(nres * 4), h_score = cv.host(nres * 8),
               h_codes = cv.host(ncodes * 4);
  // node records staged in the arena's pinned memory when the arena is kept
  // for reuse (a pipeline's chunks): the upload is then a DMA from pinned
  // memory, no runtime staging copy on the host, and no fresh pages to fault
  // in per batch.  A larger batch stages them in pageable memory (pinning
  // gigabytes once costs more than the copy).
  const bool pin_recs = cv.d <= SPARE_MAX && d->n_nodes > 0;
  const size_t h_recs = pin_recs ? cv.host((size_t)d->n_nodes * sizeof(NodeRec)) : SIZE_MAX;
  hipError_t e = arena_take(c, cv.d, cv.h, b->arena);
  if (e != hipSuccess) {
    delete b;
    return fail(e == hipErrorOutOfMemory ? LT_ENOMEM : LT_EHIP, "lt_batch_create: %s", hipGetErrorString(e));
  }
  if (timing_on()) t_arena = now_s();
  char* D = b->arena.d;
  char* H = b->arena.h;
  for (size_t q = 0; q < P; ++q) {
    lt_piece& pc = b->pieces[q];
    pc.d_order = at<int32_t>(D, po[q].order);
    pc.d_sent_n = at<int32_t>(D, po[q].sent_n);
    pc.d_node_off = at<int64_t>(D, po[q].node_off);
    pc.d_span_off = at<int64_t>(D, po[q].span_off);
    pc.d_bp_off = at<int64_t>(D, po[q].bp_off);
    pc.d_cum_n = at<int64_t>(D, po[q].cum_n);
    pc.d_span_start = at<int32_t>(D, po[q].span_start);
    pc.d_nodes = at<NodeRec>(D, po[q].nodes);
    pc.d_post = at<double>(D, po[q].post);
    pc.d_bp = at<uint32_t>(D, po[q].bp);
    pc.d_edge_base = d->n_edge > 0 ? at<int64_t>(D, po[q].edge_base) : nullptr;
    pc.d_edge_val = d->n_edge > 0 ? at<double>(D, po[q].edge_val) : nullptr;
    pc.d_sched = at<uint32_t>(D, po[q].sched);
    pc.d_wave_off = at<int64_t>(D, po[q].wave_off);
    pc.d_place = at<uint32_t>(D, po[q].place);
    pc.d_xmask = at<uint32_t>(D, po[q].xmask);
    pc.d_xf4 = at<double>(D, po[q].xf4);
    pc.d_xf5 = at<double>(D, po[q].xf5);
    pc.d_xf6 = at<double>(D, po[q].xf6);
  }
  b->d_sent_n = at<int32_t>(D, o_sent_n);
  b->d_cum_n = at<int64_t>(D, o_cum_n);
  b->d_unk = at<NodeRec>(D, o_unk);
  b->d_unk_post = at<double>(D, o_unk_post);
  b->d_pairs = at<F46>(D, o_pairs);
  for (size_t q = 0; q < P; ++q)
    b->pieces[q].d_esc = has_esc ? at<F46>(D, o_esc) + b->pieces[q].node0 : nullptr;
  for (int i = 0; i < 2; ++i) {
    b->res[i].count = at<int32_t>(D, o_count[i]);
    b->res[i].len = at<int32_t>(D, o_len[i]);
    b->res[i].score = at<double>(D, o_score[i]);
    b->res[i].codes = at<int32_t>(D, o_codes[i]);
    b->res[i].slab = at<char>(D, o_slab[i]);
  }
  b->h_slab = at<char>(H, h_slab);
  use_slot(b, 0);
  b->h_count = at<int32_t>(H, h_count);
  b->h_len = at<int32_t>(H, h_len);
  b->h_score = at<double>(H, h_score);
  b->h_codes = at<int32_t>(H, h_codes);
  auto up = [&](auto* dst, const auto* src, size_t count) {
    if (e == hipSuccess && count)
      e = hipMemcpyAsync(dst, src, count * sizeof(*src), hipMemcpyHostToDevice, stm);
  };
  up(b->d_sent_n, d->sent_n, (size_t)S);
  up(b->d_cum_n, cum_n.data(), (size_t)S + 1);
  // device node records: AoS, mask + each node's span length d-1 (bits 24-26)
  std::unique_ptr<NodeRec[]> heap_recs(pin_recs ? nullptr
                                               : new (std::nothrow) NodeRec[(size_t)std::max<int64_t>(d->n_nodes, 1)]);
  NodeRec* const recs = pin_recs ? at<NodeRec>(H, h_recs) : heap_recs.get();
  if (!recs) {
    batch_free(b);
    return fail(LT_ENOMEM, "lt_batch_create: out of host memory");
  }
  // the escape array of nodes whose pair is not in the table (host copy)
  std::unique_ptr<F46[]> esc_h(has_esc ? new (std::nothrow) F46[(size_t)d->n_nodes] : nullptr);
  if (has_esc && !esc_h) {
    batch_free(b);
    return fail(LT_ENOMEM, "lt_batch_create: out of host memory");
  }
  // sentence by sentence on threads: the records, then each node's span
  // length d-1 (bits 21-23) from the span table
  parallel_ranges(S, [&](int, int64_t lo, int64_t hi) {
    for (int64_t s = lo; s < hi; ++s) {
      const int64_t base = d->sent_node_off[s];
      F46 last{-0.0, -0.0};
      uint32_t last_px = 0;
      for (int64_t i = base; i < d->sent_node_off[s + 1]; ++i) {
        NodeRec& r = recs[(size_t)i];
        r.word = (uint32_t)d->node_word[i];
        r.morph = (uint32_t)d->node_morph0[i];
        r.tag = (uint32_t)d->node_tag[i];
        // device mask layout (lt_common.h device_mask); an absent class 4/5/6
        // coefficient is stored as -0.0, the identity of a float64 sum, so a
        // decoder may add it unconditionally; classes 4 / 6 as the index of
        // their pair
        const uint32_t am = d->node_mask[i];
        const F46 f = api_pair(am, d->node_f4, d->node_f6, i);
        if (std::memcmp(&f, &last, sizeof f) != 0) {
          const int x = ptab.find(f.f4, f.f6);
          last = f;
          last_px = x < 0 ? PX_ESC : (uint32_t)x;
        }
        if (last_px == PX_ESC) esc_h[(size_t)i] = f;
        r.mask = device_mask(am) | (last_px << PX_SHIFT);
        r.pre = d->node_pre[i];
        r.f5 = (am & F_HAS5) ? d->node_f5[i] : -0.0;
      }
      // (the general kernel of max_len > 8 takes the span from the table)
      const int32_t* ss = d->span_start + d->sent_span_off[s];
      const int SS = span_slots(d->max_len);
      for (int64_t x = 0; x < (int64_t)SS * d->sent_n[s]; ++x) {
        const uint32_t dd = (uint32_t)std::min<int64_t>(MAX_SPAN, SS - (x % SS));
        for (int32_t v = ss[x]; v < ss[x + 1]; ++v) recs[(size_t)(base + v)].mask |= (dd - 1u) << D_SHIFT;
      }
    }
  }, 256);
  if (timing_on()) t_recs = now_s();
  // the implicit Unknowns' records, one per span length d (device layout as
  // the nodes', span-length bits d - 1 up to 8)
  std::vector<NodeRec> unk_recs((size_t)d->n_unk);
  for (int32_t i = 0; i < d->n_unk; ++i) {
    NodeRec& r = unk_recs[(size_t)i];
    const uint32_t am = d->unk_mask[i];
    r.word = (uint32_t)d->unk_word[i];
    r.morph = (uint32_t)d->unk_morph0[i];
    r.tag = (uint32_t)d->unk_tag[i];
    const F46 f = unk_pairs[(size_t)i];
    r.mask = device_mask(am) | ((uint32_t)(std::min(MAX_SPAN, i + 1) - 1) << D_SHIFT) |
             ((uint32_t)ptab.find(f.f4, f.f6) << PX_SHIFT);
    r.pre = d->unk_pre[i];
    r.f5 = (am & F_HAS5) ? d->unk_f5[i] : -0.0;
  }
  up(b->d_unk, unk_recs.data(), unk_recs.size());
  up(b->d_pairs, ptab.vals.data(), ptab.vals.size());
  if (has_esc) up(at<F46>(D, o_esc), esc_h.get(), (size_t)d->n_nodes);
  if (d->n_post > 0) up(b->d_unk_post, d->unk_post, (size_t)d->n_post * (size_t)d->n_unk);
  std::vector<std::vector<int64_t>> edge_base_tmp(P);
  // the further trigram scorers' node masks in the device layout (as the
  // records' masks: lt_common.h device_mask)
  std::vector<uint32_t> xdm((size_t)d->n_xtri * (size_t)d->n_nodes);
  parallel_ranges((int64_t)xdm.size(), [&](int, int64_t lo, int64_t hi) {
    for (int64_t i = lo; i < hi; ++i) xdm[(size_t)i] = device_mask(d->xtri_mask[i]);
  });
  for (size_t q = 0; q < P; ++q) {
    const lt_piece& pc = b->pieces[q];
    const size_t n = (size_t)pc.n_sent;
    up(pc.d_order, order[q].data(), n);
    up(pc.d_sent_n, d->sent_n + pc.s0, n);
    up(pc.d_node_off, node_off[q].data(), n + 1);
    up(pc.d_span_off, span_off[q].data(), n + 1);
    up(pc.d_bp_off, bp_off[q].data(), n + 1);
    up(pc.d_cum_n, pcum[q].data(), n + 1);
    up(pc.d_span_start, d->span_start + pc.span0, (size_t)pc.n_span);
    up(pc.d_nodes, recs + pc.node0, (size_t)pc.n_nodes);
    for (int32_t t = 0; t < d->n_post; ++t)
      up(pc.d_post + (size_t)t * pc.n_nodes, d->node_post + (size_t)t * d->n_nodes + pc.node0, (size_t)pc.n_nodes);
    if (d->n_edge > 0) {
      // bases rebased to the piece's edge block (host copy kept alive past the
      // upload: the stream is synchronised below)
      edge_base_tmp[q].resize((size_t)pc.n_nodes);
      for (int64_t i = 0; i < pc.n_nodes; ++i) edge_base_tmp[q][(size_t)i] = d->node_edge_base[pc.node0 + i] - pc.edge0;
      up(pc.d_edge_base, edge_base_tmp[q].data(), (size_t)pc.n_nodes);
      for (int32_t t = 0; t < d->n_edge; ++t)
        up(pc.d_edge_val + (size_t)t * pc.n_edges, d->edge_val + (size_t)t * d->n_edges + pc.edge0, (size_t)pc.n_edges);
    }
    for (int32_t t = 0; t < d->n_xtri; ++t) {       // scorer t+1's rows, rebased to the piece
      const size_t src = (size_t)t * (size_t)d->n_nodes + (size_t)pc.node0, dst = (size_t)t * (size_t)pc.n_nodes;
      up(pc.d_xmask + dst, xdm.data() + src, (size_t)pc.n_nodes);
      up(pc.d_xf4 + dst, d->xtri_f4 + src, (size_t)pc.n_nodes);
      up(pc.d_xf5 + dst, d->xtri_f5 + src, (size_t)pc.n_nodes);
      up(pc.d_xf6 + dst, d->xtri_f6 + src, (size_t)pc.n_nodes);
    }
    if (b->has_sched) {
      up(pc.d_wave_off, wave_off[q].data(), wave_off[q].size());
      up(pc.d_place, place[q].data(), place[q].size());
    }
  }
  // a beam-1 batch gets its lane schedule now, behind its uploads (a
  // pipeline's upload thread prepares chunk i+1 while chunk i decodes)
  if (e == hipSuccess && max_k == 1) e = prep_fill(b, stm);
  if (e == hipSuccess) e = hipStreamSynchronize(stm);
  if (e != hipSuccess) {
    batch_free(b);
    return fail(e == hipErrorOutOfMemory ? LT_ENOMEM : LT_EHIP, "lt_batch_create: %s",
                hipGetErrorString(e));
  }
  if (timing_on())
    fprintf(stderr, "LT_TIMING batch_create nodes=%lld validate=%.4f arena=%.4f records=%.4f upload=%.4f s\n",
            (long long)d->n_nodes, t_valid - t_start, t_arena - t_valid, t_recs - t_arena, now_s() - t_recs);
  *out = b;
  return LT_OK;
}

int32_t lt_batch_pieces(const lt_batch* b) { return b ? (int32_t)b->pieces.size() : 0; }

lt_status lt_batch_reset_prep(lt_batch* b) {
  if (!b) return fail(LT_EINVAL, "lt_batch_reset_prep: NULL batch");
  b->prep_done = false;
  return LT_OK;
}

int64_t lt_batch_prep_bytes(const lt_batch* b) {
  if (!b || !b->has_sched) return 0;
  int64_t bytes = 0;
  for (const lt_piece& pc : b->pieces) bytes += pc.sched_steps * 64 * 4 + ((int64_t)k1_waves(pc.n_sent) + 1) * 8;
  return bytes;
}

double lt_batch_host_sched_ms(const lt_batch* b) { return b ? b->host_sched_ms : 0.0; }

lt_status lt_batch_prepare_k1(lt_batch* b) {
  if (!b) return fail(LT_EINVAL, "lt_batch_prepare_k1: NULL batch");
  lt_ctx* c = b->ctx;
  HIP_TRY(hipSetDevice(c->device));
  lt_status st = lazy_sched(c, b);
  if (st != LT_OK) return st;
  HIP_TRY(prep_fill(b, c->stream));
  return LT_OK;
}

lt_status lt_batch_prep_ms(lt_batch* b, float* ms) {
  if (!b || !ms) return fail(LT_EINVAL, "lt_batch_prep_ms: NULL argument");
  *ms = 0.0f;
  if (!b->prep_ev0 || !b->prep_ev1 || b->prep_fused) return LT_OK;
  HIP_TRY(hipEventElapsedTime(ms, b->prep_ev0, b->prep_ev1));
  return LT_OK;
}

int64_t lt_set_piece_bytes(int64_t bytes) {
  const int64_t full = ((int64_t)1 << 31) - 1;
  return g_piece_bytes.exchange(bytes < 1 || bytes > full ? full : bytes);
}

lt_status lt_batch_destroy(lt_batch* b) {
  if (!b) return LT_OK;
  (void)hipSetDevice(b->ctx->device);
  (void)hipStreamSynchronize(b->ctx->stream);
  (void)hipStreamSynchronize(b->ctx->cstream);
  // readers of the result slots on other streams (a gather's pack on its
  // communicator stream, lt_gather_launch): the arena may be recycled by the
  // next lt_batch_create, so they must be done with it first
  for (int i = 0; i < 2; ++i)
    for (int r = 0; r < 2; ++r)
      if (b->rd_pending[i][r] && b->ev_rd[i][r]) {
        (void)hipEventSynchronize(b->ev_rd[i][r]);
        b->rd_pending[i][r] = false;
      }
  batch_free(b);
  return LT_OK;
}

int64_t lt_batch_code_slots(const lt_batch* b, int k) { return b ? b->total_chars * (int64_t)k : 0; }

// --------------------------------------------------------------- decode --
// Parameters of the model / batch / beam; the per-piece fields are set by
// piece_params.
static lt_status fill_params(lt_ctx* c, const lt_model* m, lt_batch* b, int k, DecodeParams& p) {
  if (!c || !m || !b) return fail(LT_EINVAL, "decode: NULL argument");
  if (m->ctx != c || b->ctx != c) return fail(LT_EINVAL, "decode: handles from another context");
  if (k < 1 || k > b->max_k)
    return fail(LT_EUNSUPPORTED, "decode: beam %d not in 1..%d (batch max_k)", k, b->max_k);
  if (!batch_wide(b, k) && beam_template_for(k) < 0)
    return fail(LT_EUNSUPPORTED, "decode: beam %d not compiled", k);
  if ((m->inf_signs | b->inf_signs) == 3)
    return fail(LT_EUNSUPPORTED, "decode: both +inf and -inf among the model's and the batch's score terms "
                                 "(their sum is a NaN, whose place in Python's sort is not reproduced)");
  p = DecodeParams{};
  // beam 1 and the general kernel probe primary first (flags); the tuned beam
  // kernels load both slots of the flag-free copy
  p.table = (k == 1 || batch_wide(b, k)) ? m->d_table : m->d_plain;
  if (b->n_xtri > 0 && m->narrow)
    return fail(LT_EINVAL, "decode: a batch with several trigram terms needs a model with their keys "
                           "(classes + %d per further scorer)", LT_XTRI_CLASS_STRIDE);
  p.slots = (uint32_t)m->slots;
  p.seed = m->seed;
  p.hk = narrow_hash(m->seed);
  p.d3 = m->d_d3;
  p.d3off = m->d3off;
  p.narrow = m->narrow;
  p.has_tri = b->has_tri;
  p.max_len = b->max_len;
  p.n_post = b->n_post;
  p.n_edge = b->n_edge;
  p.n_xtri = b->n_xtri;
  p.n_terms = b->n_terms;
  p.term_kinds = b->term_kinds;
  p.k = k;
  p.bp_stride = b->max_k;
  p.counters = c->d_counters;
  p.span_slots = span_slots(b->max_len);
  p.n_unk = b->n_unk;
  p.unk = b->d_unk;
  p.unk_post = b->d_unk_post;
  p.pairs = b->d_pairs;
  p.n_pairs = b->n_pairs;
  return LT_OK;
}

// Piece q of b, writing the current result slot: its sentences' results
// land at their places in the batch's result arrays.
static void piece_params(const lt_batch* b, size_t q, int k, DecodeParams& p) {
  const lt_piece& pc = b->pieces[q];
  p.n_sent = pc.n_sent;
  p.n_nodes = pc.n_nodes;
  p.order = pc.d_order;
  p.sent_n = pc.d_sent_n;
  p.node_off = pc.d_node_off;
  p.span_off = pc.d_span_off;
  p.span_start = pc.d_span_start;
  p.nodes = pc.d_nodes;
  p.esc = pc.d_esc;
  p.npost = pc.d_post;
  p.sched = b->has_sched ? pc.d_sched : nullptr;
  p.wave_off = b->has_sched ? pc.d_wave_off : nullptr;
  p.k1_place = b->has_sched ? pc.d_place : nullptr;
  p.k1_fill = nullptr;                // (lt_decode_launch: a fresh schedule filled by the decode)
  p.n_edges = pc.n_edges;
  p.edge_base = pc.d_edge_base;
  p.edge_val = pc.d_edge_val;
  p.xmask = pc.d_xmask;
  p.xf4 = pc.d_xf4;
  p.xf5 = pc.d_xf5;
  p.xf6 = pc.d_xf6;
  p.bp = pc.d_bp;
  p.bp_bytes = pc.bp_entries * 4;
  p.bp_off = pc.d_bp_off;
  p.cum_n = pc.d_cum_n;
  p.out_count = b->d_count + pc.s0;
  p.out_len = b->d_len + (int64_t)pc.s0 * k;
  p.out_score = b->d_score + (int64_t)pc.s0 * k;
  p.out_codes = b->d_codes + (int64_t)k * pc.chars0;
}

// The next decode writes the result slot the previous one did not: the D2H
// of the previous results (copy stream) can run meanwhile.  A copy still
// queued on the slot being reused is waited for on the decode stream.
static lt_status next_slot(lt_ctx* c, lt_batch* b) {
  const int i = b->cur ^ 1;
  for (int r = 0; r < 2; ++r)
    if (b->rd_pending[i][r]) {
      // a reader that is already done costs the decode stream nothing
      if (hipEventQuery(b->ev_rd[i][r]) != hipSuccess) HIP_TRY(hipStreamWaitEvent(c->stream, b->ev_rd[i][r], 0));
      b->rd_pending[i][r] = false;
    }
  use_slot(b, i);
  return LT_OK;
}

// Scratch of the general kernel for beam k over b's pieces: one block per
// thread, threads = the largest piece's sentences, fewer when the blocks of
// that many would pass WIDE_BUDGET (each thread then walks several
// sentences).  Grown on demand; decodes on the ctx stream share it in order.
constexpr size_t WIDE_BUDGET = (size_t)1 << 30;
static lt_status wide_scratch(lt_ctx* c, const lt_batch* b, int k, DecodeParams& p) {
  int32_t most = 0;
  for (const lt_piece& pc : b->pieces) most = std::max(most, pc.n_sent);
  const int64_t blk = wide_scratch_bytes(span_slots(b->max_len), k);
  const int64_t fit = std::max<int64_t>(1, (int64_t)WIDE_BUDGET / blk);
  const int32_t threads = (int32_t)std::max<int64_t>(1, std::min<int64_t>(most, fit));
  const size_t need = (size_t)threads * (size_t)blk;
  if (need > c->wide_bytes) {
    if (c->d_wide) {
      HIP_TRY(hipStreamSynchronize(c->stream));
      dfree(c->d_wide);
      c->d_wide = nullptr;
      c->wide_bytes = 0;
    }
    hipError_t e = hipMalloc((void**)&c->d_wide, need);
    if (e != hipSuccess) {
      c->d_wide = nullptr;
      return fail(e == hipErrorOutOfMemory ? LT_ENOMEM : LT_EHIP, "decode: general-kernel scratch of %zu B: %s",
                  need, hipGetErrorString(e));
    }
    c->wide_bytes = need;
  }
  p.wide_threads = threads;
  p.wide_block = blk;
  p.wide_scratch = c->d_wide;
  return LT_OK;
}

lt_status lt_decode_launch(lt_ctx* c, const lt_model* m, lt_batch* b, int k) {
  DecodeParams p;
  lt_status st = fill_params(c, m, b, k, p);
  if (st != LT_OK) return st;
  HIP_TRY(hipSetDevice(c->device));
  const bool wide = batch_wide(b, k);
  if (wide && (st = wide_scratch(c, b, k, p)) != LT_OK) return st;
  // the k=1 lane schedule, if the batch has not got it yet: queued in front
  // of the decode on its stream (lt_batch_create builds it for max_k = 1; a
  // batch for larger beams gets it here, at its first beam-1 decode)
  bool fuse = false;
  if (!wide && beam_template_for(k) == 1) {
    if ((st = lazy_sched(c, b)) != LT_OK) return st;
    // a schedule not filled yet is filled by the decode itself (p.k1_fill);
    // LT_K1_FUSED_FILL=0: by the standalone fill kernel in front of it
    fuse = b->has_sched && !b->prep_done && fused_fill_on();
    if (!fuse) HIP_TRY(prep_fill(b, c->stream));
  }
  if ((st = next_slot(c, b)) != LT_OK) return st;
  const int r = (int)(c->n_launch % lt_ctx::KRING);
  const size_t P = b->pieces.size();
  const int32_t wide_threads = p.wide_threads;
  for (size_t q = 0; q < P; ++q) {           // timing: start of the first piece .. end of the last
    piece_params(b, q, k, p);
    p.k1_fill = fuse ? b->pieces[q].d_sched : nullptr;
    hipEvent_t e0 = q == 0 ? c->kev0[r] : nullptr, e1 = q + 1 == P ? c->kev1[r] : nullptr;
    if (wide) {
      p.wide_threads = std::max(1, std::min(wide_threads, p.n_sent));
      HIP_TRY(launch_wide(p, c->stream, false, e0, e1));
    } else {
      HIP_TRY(launch_decode(p, c->stream, false, e0, e1));
    }
  }
  if (fuse) {
    b->prep_done = true;
    b->prep_fused = true;
  }
  b->last_end = c->kev1[r];          // other streams wait for this decode here
  b->launch_serial = c->n_serial++;
  ++c->n_launch;
  b->last_k = k;
  return LT_OK;
}

const char* lt_kernel_name(int k) { return k > LT_MAX_BEAM_COMPILED ? "lt_beam_wide" : kernel_name_for(k); }

// ------------------------------------------------------------- evaluate --
lt_status lt_evaluate(lt_ctx* c, const lt_model* m, const lt_paths_desc* d, double* scores) {
  if (!c || !m || !d || (!scores && d->n_paths > 0)) return fail(LT_EINVAL, "lt_evaluate: NULL argument");
  if (m->ctx != c) return fail(LT_EINVAL, "lt_evaluate: model from another context");
  if (d->n_paths < 0 || d->n_words < 0 || d->n_terms < 0)
    return fail(LT_EINVAL, "lt_evaluate: negative size");
  if (d->n_words * (int64_t)sizeof(NodeRec) >= ((int64_t)1 << 31))
    return fail(LT_EUNSUPPORTED, "lt_evaluate: %lld words exceed one launch", (long long)d->n_words);
  if (d->trigram_pos < -1 || d->trigram_pos > d->n_terms)
    return fail(LT_EINVAL, "lt_evaluate: trigram_pos %d out of range", d->trigram_pos);
  if (d->trigram_scorer < 0 || d->trigram_scorer >= LT_MAX_TRI)
    return fail(LT_EINVAL, "lt_evaluate: trigram_scorer %d not in 0..%d", d->trigram_scorer, LT_MAX_TRI - 1);
  if (d->trigram_scorer > 0 && m->narrow)
    return fail(LT_EINVAL, "lt_evaluate: the model holds no keys of trigram scorer %d", d->trigram_scorer);
  if (!d->path_off || (d->n_words > 0 && (!d->word || !d->morph0 || !d->tag || !d->mask || !d->f4 ||
                                          !d->f5 || !d->f6 || !d->prev1 || !d->prev2)) ||
      (d->n_terms > 0 && d->n_words > 0 && !d->terms))
    return fail(LT_EINVAL, "lt_evaluate: NULL arrays");
  if (d->path_off[0] != 0 || d->path_off[d->n_paths] != d->n_words)
    return fail(LT_EINVAL, "lt_evaluate: path offsets do not cover the words");
  for (int32_t s = 0; s < d->n_paths; ++s)
    if (d->path_off[s + 1] < d->path_off[s]) return fail(LT_EINVAL, "lt_evaluate: path offsets decrease");
  for (int64_t w = 0; w < d->n_words; ++w) {
    const int64_t j = d->prev1[w], i = d->prev2[w];
    if (j == -2) continue;
    if (j < 0 || j >= d->n_words || i < -1 || i >= d->n_words)
      return fail(LT_EINVAL, "lt_evaluate: word %lld has a bad predecessor", (long long)w);
  }
  for (int64_t x = 0; x < (int64_t)d->n_terms * d->n_words; ++x)
    if (std::isnan(d->terms[x])) return fail(LT_EUNSUPPORTED, "lt_evaluate: NaN term");
  HIP_TRY(hipSetDevice(c->device));
  std::vector<NodeRec> recs((size_t)d->n_words);
  std::vector<F46> esc((size_t)d->n_words);
  for (int64_t w = 0; w < d->n_words; ++w) {
    NodeRec& r = recs[(size_t)w];
    r.word = (uint32_t)d->word[w];
    r.morph = (uint32_t)d->morph0[w];
    r.tag = (uint32_t)d->tag[w];
    // lt_common.h device layout; every word's class-4/6 pair from the escape
    // array (evaluate is no hot path)
    r.mask = device_mask((uint32_t)d->mask[w]) | (PX_ESC << PX_SHIFT);
    r.pre = 0.0;
    r.f5 = d->f5[w];
    esc[(size_t)w] = F46{d->f4[w], d->f6[w]};
  }
  const F46 absent{-0.0, -0.0};
  hipStream_t st = c->stream;
  hipError_t e = hipSuccess;
  NodeRec* d_words = nullptr;
  F46 *d_pairs = nullptr, *d_esc = nullptr;
  int64_t *d_p1 = nullptr, *d_p2 = nullptr, *d_off = nullptr;
  double *d_terms = nullptr, *d_inc = nullptr, *d_out = nullptr;
  const size_t nw = (size_t)d->n_words, np = (size_t)d->n_paths;
  e = dalloc_copy(&d_words, recs.data(), nw, st);
  if (e == hipSuccess) e = dalloc_copy(&d_pairs, &absent, 1, st);
  if (e == hipSuccess) e = dalloc_copy(&d_esc, esc.data(), nw, st);
  if (e == hipSuccess) e = dalloc_copy(&d_p1, d->prev1, nw, st);
  if (e == hipSuccess) e = dalloc_copy(&d_p2, d->prev2, nw, st);
  if (e == hipSuccess) e = dalloc_copy(&d_off, d->path_off, np + 1, st);
  if (e == hipSuccess) e = dalloc_copy(&d_terms, d->terms, (size_t)d->n_terms * nw, st);
  if (e == hipSuccess) e = dalloc_copy(&d_inc, (const double*)nullptr, nw, st);
  if (e == hipSuccess) e = dalloc_copy(&d_out, (const double*)nullptr, np, st);
  if (e == hipSuccess) {
    EvalParams p{};
    p.table = m->d_table;
    p.slots = (uint32_t)m->slots;
    p.seed = m->seed;
    p.hk = narrow_hash(m->seed);
    p.narrow = m->narrow;
    p.has_tri = d->trigram_pos >= 0 ? 1 : 0;
    p.d3 = m->d_d3;
    p.d3off = m->d3off;
    p.n_paths = d->n_paths;
    p.n_words = d->n_words;
    p.words = d_words;
    p.pairs = d_pairs;
    p.esc = d_esc;
    p.prev1 = d_p1;
    p.prev2 = d_p2;
    p.path_off = d_off;
    p.n_terms = d->n_terms;
    p.terms = d_terms;
    p.trigram_pos = d->trigram_pos;
    p.coff = (uint32_t)(LT_XTRI_CLASS_STRIDE * d->trigram_scorer);
    p.inc = d_inc;
    p.out = d_out;
    e = launch_evaluate(p, st);
  }
  if (e == hipSuccess && np) e = hipMemcpyAsync(scores, d_out, np * sizeof(double), hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  void* bufs[] = {d_words, d_pairs, d_esc, d_p1, d_p2, d_off, d_terms, d_inc, d_out};
  for (void* b : bufs) dfree(b);
  if (e != hipSuccess) return fail(LT_EHIP, "lt_evaluate: %s", hipGetErrorString(e));
  return LT_OK;
}

lt_status lt_last_kernel_ms(lt_ctx* c, float* ms) {
  if (!c || !ms) return fail(LT_EINVAL, "lt_last_kernel_ms: NULL argument");
  if (c->n_launch < 1) return fail(LT_EINVAL, "lt_last_kernel_ms: no decode launched");
  const int r = (int)((c->n_launch - 1) % lt_ctx::KRING);
  HIP_TRY(hipEventElapsedTime(ms, c->kev0[r], c->kev1[r]));
  return LT_OK;
}

lt_status lt_kernel_ms_recent(lt_ctx* c, int n, float* ms, int* got) {
  if (!c || (!ms && n > 0) || !got) return fail(LT_EINVAL, "lt_kernel_ms_recent: NULL argument");
  const int64_t have = std::min<int64_t>(c->n_launch, lt_ctx::KRING);
  const int m = (int)std::min<int64_t>(std::max(n, 0), have);
  for (int j = 0; j < m; ++j) {   // oldest first
    const int r = (int)((c->n_launch - m + j) % lt_ctx::KRING);
    HIP_TRY(hipEventElapsedTime(&ms[j], c->kev0[r], c->kev1[r]));
  }
  *got = m;
  return LT_OK;
}

// Stream `st` waits for the last decode of b (the decode stream's current end).
// The decode's own end event (lt_ctx::kev1 of its launch; re-recorded at most
// by a later launch of the same stream, which only waits longer) -- no extra
// command on the decode stream.
static hipError_t after_decode(lt_batch* b, hipStream_t st) {
  if (!b->last_end) return hipSuccess;     // the last launch completed synchronously
  return hipStreamWaitEvent(st, b->last_end, 0);
}

// Reader `r` is done with the current result slot at this point of `st`.
static hipError_t slot_read(lt_batch* b, int r, hipStream_t st) {
  const int i = b->cur;
  hipError_t e = hipSuccess;
  if (!b->ev_rd[i][r]) e = hipEventCreateWithFlags(&b->ev_rd[i][r], hipEventDisableTiming);
  if (e == hipSuccess) e = hipEventRecord(b->ev_rd[i][r], st);
  if (e == hipSuccess) b->rd_pending[i][r] = true;
  return e;
}

lt_status lt_result_fetch(lt_ctx* c, lt_batch* b) {
  if (!c || !b) return fail(LT_EINVAL, "lt_result_fetch: NULL argument");
  if (b->ctx != c) return fail(LT_EINVAL, "lt_result_fetch: batch of another context");
  if (b->last_k < 1) return fail(LT_EINVAL, "lt_result_fetch: no decode launched");
  const int k = b->last_k;
  const size_t S = (size_t)b->n_sent;
  HIP_TRY(hipSetDevice(c->device));
  hipStream_t cs = c->cstream;
  // DMA copies on the copy stream once the decode is done -- under the next decode
  HIP_TRY(after_decode(b, cs));
  if (S) {
    HIP_TRY(hipMemcpyAsync(b->h_count, b->d_count, S * 4, hipMemcpyDeviceToHost, cs));
    HIP_TRY(hipMemcpyAsync(b->h_len, b->d_len, S * k * 4, hipMemcpyDeviceToHost, cs));
    HIP_TRY(hipMemcpyAsync(b->h_score, b->d_score, S * k * 8, hipMemcpyDeviceToHost, cs));
  }
  const size_t nc = (size_t)b->total_chars * k;
  if (nc) HIP_TRY(hipMemcpyAsync(b->h_codes, b->d_codes, nc * 4, hipMemcpyDeviceToHost, cs));
  HIP_TRY(slot_read(b, lt_batch::RD_COPY, cs));
  return LT_OK;
}

}  // extern "C"

uint64_t lt::slab_alloc_bytes(int64_t n_sent, int k, int64_t chars) {
  return slab_layout(n_sent, k, chars).capacity + al16(8 * (uint64_t)(pack_blocks(n_sent * k) + 1));
}

hipError_t lt::pack_last_results_on(lt_batch* b, int reader, void* slab, hipStream_t st) {
  hipError_t e = after_decode(b, st);
  if (e != hipSuccess) return e;
  ResultsPackParams p{};
  p.count = b->d_count;
  p.len = b->d_len;
  p.score = b->d_score;
  p.codes = b->d_codes;
  p.sent_n = b->d_sent_n;
  p.cum_n = b->d_cum_n;
  p.n_sent = b->n_sent;
  p.k = b->last_k;
  p.n_entries = (int64_t)b->n_sent * b->last_k;
  p.n_blocks = pack_blocks(p.n_entries);
  p.lay = slab_layout(b->n_sent, b->last_k, b->total_chars);
  p.block_sum = reinterpret_cast<int64_t*>(static_cast<char*>(slab) + p.lay.capacity);
  p.slab = slab;
  e = launch_pack_results(p, st);
  if (e == hipSuccess) e = slot_read(b, reader, st);
  return e;
}

extern "C" {

lt_status lt_result_fetch_packed(lt_ctx* c, lt_batch* b) {
  if (!c || !b) return fail(LT_EINVAL, "lt_result_fetch_packed: NULL argument");
  if (b->ctx != c) return fail(LT_EINVAL, "lt_result_fetch_packed: batch of another context");
  if (b->last_k < 1) return fail(LT_EINVAL, "lt_result_fetch_packed: no decode launched");
  HIP_TRY(hipSetDevice(c->device));
  const int i = b->cur;
  // the pack (once per decode) on the decode stream, right behind the
  // decode: its kernels take the CUs briefly between two decodes (round 6:
  // on the copy stream, beside the next decode, they kept its LDS-filling
  // blocks waiting -- k=1 0.56 -> 0.72 ms); the DMA of the slab on the copy
  // stream, under the next decode; the slot's reader event after the DMA
  if (b->res[i].packed_launch != b->launch_serial) {
    HIP_TRY(pack_last_results_on(b, lt_batch::RD_COPY, b->res[i].slab, c->stream));
    b->res[i].packed_launch = b->launch_serial;
  }
  HIP_TRY(hipStreamWaitEvent(c->cstream, b->ev_rd[i][lt_batch::RD_COPY], 0));
  HIP_TRY(launch_slab_to_host(b->res[i].slab, b->h_slab, b->slab_cap, c->cstream));
  HIP_TRY(slot_read(b, lt_batch::RD_COPY, c->cstream));
  return LT_OK;
}

lt_status lt_slab_parse(const void* slab, uint64_t bytes, lt_packed_view* v) {
  if (!slab || !v) return fail(LT_EINVAL, "lt_slab_parse: NULL argument");
  if (bytes < sizeof(SlabHeader)) return fail(LT_EINVAL, "lt_slab_parse: %llu bytes", (unsigned long long)bytes);
  const SlabHeader* h = static_cast<const SlabHeader*>(slab);
  if (h->n_sent < 0 || h->k < 1 || h->n_codes < 0)
    return fail(LT_EINVAL, "lt_slab_parse: bad header");
  const SlabLayout L = slab_layout(h->n_sent, h->k, 0);
  if ((uint64_t)h->bytes != slab_used_bytes(L, h->n_codes) || (uint64_t)h->bytes > bytes)
    return fail(LT_EINVAL, "lt_slab_parse: slab of %lld bytes in a buffer of %llu", (long long)h->bytes,
                (unsigned long long)bytes);
  const char* base = static_cast<const char*>(slab);
  v->n_sent = h->n_sent;
  v->k = h->k;
  v->n_codes = h->n_codes;
  v->count = reinterpret_cast<const int32_t*>(base + L.count);
  v->length = reinterpret_cast<const int32_t*>(base + L.len);
  v->score = reinterpret_cast<const double*>(base + L.score);
  v->codes = reinterpret_cast<const int32_t*>(base + L.codes);
  return LT_OK;
}

lt_status lt_result_view_packed(lt_batch* b, lt_packed_view* v) {
  if (!b || !v) return fail(LT_EINVAL, "lt_result_view_packed: NULL argument");
  return lt_slab_parse(b->h_slab, b->slab_cap, v);
}

lt_status lt_result_view(lt_batch* b, lt_result* v) {
  if (!b || !v) return fail(LT_EINVAL, "lt_result_view: NULL argument");
  v->count = b->h_count;
  v->length = b->h_len;
  v->score = b->h_score;
  v->codes = b->h_codes;
  return LT_OK;
}

lt_status lt_decode(lt_ctx* c, const lt_model* m, lt_batch* b, int k, lt_result* out) {
  if (!out) return fail(LT_EINVAL, "lt_decode: out is NULL");
  lt_status st = lt_decode_launch(c, m, b, k);
  if (st != LT_OK) return st;
  if ((st = lt_result_fetch(c, b)) != LT_OK) return st;
  if ((st = lt_sync(c)) != LT_OK) return st;
  const size_t S = (size_t)b->n_sent;
  if (S) {
    if (out->count) memcpy(out->count, b->h_count, S * 4);
    if (out->length) memcpy(out->length, b->h_len, S * k * 4);
    if (out->score) memcpy(out->score, b->h_score, S * k * 8);
  }
  const size_t nc = (size_t)b->total_chars * k;
  if (nc && out->codes) memcpy(out->codes, b->h_codes, nc * 4);
  return LT_OK;
}

lt_status lt_decode_trace(lt_ctx* c, const lt_model* m, lt_batch* b, int k, lt_trace* t) {
  DecodeParams p;
  lt_status st = fill_params(c, m, b, k, p);
  if (st != LT_OK) return st;
  if (!t || !t->pos_off || !t->exp_off || !t->beam_count || !t->beam_gen || !t->exp_count ||
      (t->n_exp > 0 && (!t->exp_score || !t->exp_node || !t->exp_skip)) || t->n_exp < 0)
    return fail(LT_EINVAL, "lt_decode_trace: bad trace arrays");
  if (b->pieces.size() != 1) return fail(LT_EUNSUPPORTED, "lt_decode_trace: batch of several launch pieces");
  if (batch_wide(b, k) && t->n_exp > 0 && !t->exp_link)
    return fail(LT_EINVAL, "lt_decode_trace: exp_link is required past max_len %d / beam %d", MAX_SPAN,
                LT_MAX_BEAM_COMPILED);
  const int64_t S = b->n_sent;
  if (t->pos_off[0] != 0) return fail(LT_EINVAL, "lt_decode_trace: pos_off[0] != 0");
  const int64_t P = t->pos_off[S];
  // (a position whose expansions exceed its slots stops its sentence on the
  // device and is reported below)
  for (int64_t s = 0; s < S; ++s)
    if (t->pos_off[s + 1] <= t->pos_off[s]) return fail(LT_EINVAL, "lt_decode_trace: pos_off not increasing");
  for (int64_t q = 1; q <= P; ++q)
    if (t->exp_off[q] < t->exp_off[q - 1]) return fail(LT_EINVAL, "lt_decode_trace: exp_off not increasing");
  if (t->exp_off[0] < 0 || t->exp_off[P] != t->n_exp)
    return fail(LT_EINVAL, "lt_decode_trace: exp_off[0] < 0 or exp_off[positions] != n_exp");
  HIP_TRY(hipSetDevice(c->device));
  piece_params(b, 0, k, p);
  p.table = m->d_table;                  // the trace probes primary first (flags)
  TraceParams tp{};
  int64_t *d_pos = nullptr, *d_exp = nullptr;
  void* d_ent = nullptr;
  int32_t *d_bc = nullptr, *d_ec = nullptr;
  uint32_t *d_bg = nullptr, *d_node = nullptr;
  double* d_score = nullptr;
  uint8_t* d_skip = nullptr;
  uint64_t* d_link = nullptr;
  const size_t ne = (size_t)std::max<int64_t>(t->n_exp, 1);
  hipError_t e = dalloc_copy(&d_pos, t->pos_off, (size_t)S + 1, c->stream);
  if (e == hipSuccess) e = dalloc_copy(&d_exp, t->exp_off, (size_t)P + 1, c->stream);
  if (e == hipSuccess) e = hipMalloc(&d_ent, (size_t)P * k * TRACE_ENTRY_BYTES);
  if (e == hipSuccess) e = hipMalloc((void**)&d_bc, (size_t)P * 4);
  if (e == hipSuccess) e = hipMalloc((void**)&d_ec, (size_t)P * 4);
  if (e == hipSuccess) e = hipMalloc((void**)&d_bg, (size_t)P * k * 4);
  if (e == hipSuccess) e = hipMalloc((void**)&d_node, ne * 4);
  if (e == hipSuccess) e = hipMalloc((void**)&d_score, ne * 8);
  if (e == hipSuccess) e = hipMalloc((void**)&d_skip, ne);
  if (e == hipSuccess && t->exp_link) e = hipMalloc((void**)&d_link, ne * 8);
  if (e == hipSuccess) {
    tp.pos_off = d_pos; tp.exp_off = d_exp; tp.ent = d_ent;
    tp.beam_count = d_bc; tp.beam_gen = d_bg; tp.exp_count = d_ec;
    tp.exp_score = d_score; tp.exp_node = d_node; tp.exp_skip = d_skip; tp.exp_link = d_link;
    e = launch_trace(p, tp, c->stream);
  }
  if (e == hipSuccess) e = hipMemcpyAsync(t->beam_count, d_bc, (size_t)P * 4, hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(t->exp_count, d_ec, (size_t)P * 4, hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(t->beam_gen, d_bg, (size_t)P * k * 4, hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess && t->n_exp > 0) {
    e = hipMemcpyAsync(t->exp_score, d_score, (size_t)t->n_exp * 8, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(t->exp_node, d_node, (size_t)t->n_exp * 4, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(t->exp_skip, d_skip, (size_t)t->n_exp, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess && d_link)
      e = hipMemcpyAsync(t->exp_link, d_link, (size_t)t->n_exp * 8, hipMemcpyDeviceToHost, c->stream);
  }
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  dfree(d_pos); dfree(d_exp); dfree(d_ent); dfree(d_bc); dfree(d_ec); dfree(d_bg);
  dfree(d_node); dfree(d_score); dfree(d_skip); dfree(d_link);
  if (e != hipSuccess) return fail(LT_EHIP, "lt_decode_trace: %s", hipGetErrorString(e));
  for (int64_t q = 0; q < P; ++q)
    if (t->exp_count[q] < 0) return fail(LT_EINVAL, "lt_decode_trace: position %lld has more expansions than slots",
                                         (long long)q);
  return LT_OK;
}

lt_status lt_count_ops(lt_ctx* c, const lt_model* m, lt_batch* b, int k, int64_t* expansions,
                       int64_t* feature_tuples, int64_t* probes, int64_t* table_loads) {
  DecodeParams p;
  lt_status st = fill_params(c, m, b, k, p);
  if (st != LT_OK) return st;
  const bool wide = batch_wide(b, k);
  HIP_TRY(hipSetDevice(c->device));
  if (wide && (st = wide_scratch(c, b, k, p)) != LT_OK) return st;
  if (!wide && beam_template_for(k) == 1) {
    if ((st = lazy_sched(c, b)) != LT_OK) return st;
    HIP_TRY(prep_fill(b, c->stream));
  }
  if ((st = next_slot(c, b)) != LT_OK) return st;
  HIP_TRY(hipMemsetAsync(c->d_counters, 0, 16 * sizeof(unsigned long long), c->stream));
#ifdef PK_PHASES
  // diagnostic build: the shipping (non-counting) kernel, its phase stamps
  for (size_t q = 0; q < (wide ? 0 : b->pieces.size()); ++q) {
    piece_params(b, q, k, p);
    HIP_TRY(launch_decode(p, c->stream, false));
  }
  {
    unsigned long long ph[16];
    HIP_TRY(hipMemcpyAsync(ph, c->d_counters, sizeof ph, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    fprintf(stderr, "PK_PHASES k=%d waves=%llu steps=%llu lifetime=%llu phases=", k, ph[14], ph[12], ph[13]);
    for (int i = 0; i < 8; ++i) fprintf(stderr, "%s%llu", i ? "," : "", ph[4 + i]);
    fprintf(stderr, "\n");
  }
  HIP_TRY(hipMemsetAsync(c->d_counters, 0, 16 * sizeof(unsigned long long), c->stream));
#endif
  const int32_t wide_threads = p.wide_threads;
  for (size_t q = 0; q < b->pieces.size(); ++q) {
    piece_params(b, q, k, p);
    if (wide) {
      p.wide_threads = std::max(1, std::min(wide_threads, p.n_sent));
      HIP_TRY(launch_wide(p, c->stream, true));
    } else {
      HIP_TRY(launch_decode(p, c->stream, true));
    }
  }
  b->launch_serial = c->n_serial++;
  b->last_end = nullptr;             // complete below
  unsigned long long h[4] = {0, 0, 0, 0};
  HIP_TRY(hipMemcpyAsync(h, c->d_counters, sizeof h, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  b->last_k = k;
  if (expansions) *expansions = (int64_t)h[0];
  if (feature_tuples) *feature_tuples = (int64_t)h[1];
  if (probes) *probes = (int64_t)h[2];
  if (table_loads) *table_loads = (int64_t)h[3];
  return LT_OK;
}

}  // extern "C"
