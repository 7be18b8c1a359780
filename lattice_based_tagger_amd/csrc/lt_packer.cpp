// lt_packer.cpp -- native lattice packer (include/lattice_pack.h).
//
// Restates lattice_based_tagger_amd/packer.py (itself following
// lattice_tagger/beam/beam.py:25-38 and the node-local scorers of
// beam/score_funcs.py:50-54, 65-73, 84-88, 99-100) over columnar lattices, so
// that whole corpora pack without one Python call per node.  Every value is
// computed with the same float64 operations in the same order as the Python
// packer; tests/test_native_packer.py checks the arrays bit for bit.
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <new>
#include <string>
#include <string_view>
#include <thread>
#include <unordered_map>
#include <algorithm>
#include <vector>

#include "../../include/lattice_pack.h"
#include "lt_common.h"
#include "lt_error.h"
#include "lt_host.h"
#include "lt_lattice_store.h"

using namespace lt;

namespace {

std::string_view str_at(const lt_strings& t, int64_t i) {
  return std::string_view(t.data + t.off[i], (size_t)(t.off[i + 1] - t.off[i]));
}
bool is_null(const lt_strings& t, int64_t i) { return t.null && t.null[i]; }

// key-slot bits of the vocabulary mask (lowering.py SLOT_BITS)
constexpr int S00 = 0, S01 = 1, S02 = 2, S10 = 3, S11 = 4, S20 = 5, S21 = 6, S22 = 7, S30 = 8,
              S31 = 9, S70 = 10, S71 = 11, S72 = 12, S80 = 13, S81 = 14;
inline uint32_t bit(uint32_t vm, int s) { return (vm >> s) & 1u; }
// lowering.node_mask_from_vocab
uint32_t node_mask(uint32_t vw, uint32_t vmo, uint32_t vt) {
  return bit(vw, S01) * K0B | bit(vt, S02) * K0C | bit(vt, S11) * K1B | bit(vw, S21) * K2B |
         bit(vt, S22) * K2C | bit(vt, S31) * K3B | bit(vw, S72) * K7C | bit(vmo, S81) * K8B |
         bit(vw, S00) * J0A | bit(vw, S10) * J1A | bit(vt, S20) * J2A | bit(vt, S30) * J3A |
         bit(vw, S71) * J7B | bit(vmo, S80) * J8A | bit(vw, S70) * I7A | bit(vmo, S80) * I8A;
}

// Key of a (string, string) tuple written into a reused buffer: a, b, then
// a's length (strings with any byte, NUL included, split unambiguously).
std::string_view tuple_key(std::string& buf, std::string_view a, std::string_view b) {
  buf.clear();
  buf.append(a);
  buf.append(b);
  const uint32_t la = (uint32_t)a.size();
  buf.append(reinterpret_cast<const char*>(&la), sizeof la);
  return buf;
}

// string_view-keyed map over strings the packer owns: open addressing over
// (hash, pointer, length, value) records, so a lookup is one probe sequence
// in one array (no allocation, no node chasing) -- the packer does several
// per lattice node.
template <typename V>
struct ViewMap {
  struct E {
    uint64_t h;                                  // 0: empty
    const char* s;
    uint64_t n;
    V v;
  };
  std::vector<std::unique_ptr<std::string>> store;
  std::vector<E> tab = std::vector<E>(16, E{0, nullptr, 0, V()});
  uint64_t mask = 15, count = 0;

  static uint64_t hash(std::string_view k) {
    uint64_t h = 0x9E3779B97F4A7C15ull ^ (uint64_t)k.size();
    const char* s = k.data();
    size_t n = k.size();
    auto mix = [&](uint64_t x) {
      h = (h ^ x) * 0xBF58476D1CE4E5B9ull;
      h ^= h >> 31;
    };
    for (; n >= 8; n -= 8, s += 8) {
      uint64_t x;
      std::memcpy(&x, s, 8);
      mix(x);
    }
    if (n) {
      uint64_t x = 0;
      std::memcpy(&x, s, n);
      mix(x);
    }
    h ^= h >> 29;
    h *= 0x94D049BB133111EBull;
    h ^= h >> 32;
    return h ? h : 1;
  }
  const E* find(std::string_view k, uint64_t h) const {
    for (uint64_t i = h & mask;; i = (i + 1) & mask) {
      const E& e = tab[i];
      if (e.h == 0) return nullptr;
      if (e.h == h && e.n == k.size() && std::memcmp(e.s, k.data(), k.size()) == 0) return &e;
    }
  }
  void insert(const E& x) {
    uint64_t i = x.h & mask;
    while (tab[i].h) i = (i + 1) & mask;
    tab[i] = x;
  }
  void put(std::string_view k, V v) {
    const uint64_t h = hash(k);
    if (find(k, h)) return;                      // first entry wins (Python dict semantics)
    if (2 * (count + 1) > tab.size()) {
      std::vector<E> old(tab.size() * 2, E{0, nullptr, 0, V()});
      old.swap(tab);
      mask = tab.size() - 1;
      for (const E& e : old)
        if (e.h) insert(e);
    }
    store.emplace_back(new std::string(k));
    insert(E{h, store.back()->data(), (uint64_t)k.size(), v});
    ++count;
  }
  const V* get(std::string_view k) const {
    const E* e = find(k, hash(k));
    return e ? &e->v : nullptr;
  }
  V* get_mut(std::string_view k) { return const_cast<V*>(get(k)); }
};

// A vocabulary string's id (0: absent) and its class-5 coefficients
// (word, tag0, is_l) -> coef as entries [c5_lo, c5_lo + c5_n) of
// lt_packer::c5e: one probe answers both per node (the tables are far larger
// than the caches, so each probe is a memory round trip).
struct WordInfo {
  int32_t id = 0, c5_lo = 0, c5_n = 0;
};
struct C5Entry {
  std::string tag;
  int64_t is_l;
  double coef;
};

const std::string_view kUnk = "Unknown", kNoun = "Noun", kBOS = "BOS";
bool contextual(std::string_view t) {        // CONTEXTUAL_TAGS (feature.py:92)
  return t == "Noun" || t == "Adverb" || t == "Adjective" || t == "Verb";
}

void utf8_append(std::string& out, uint32_t cp) {
  if (cp < 0x80) {
    out.push_back((char)cp);
  } else if (cp < 0x800) {
    out.push_back((char)(0xC0 | (cp >> 6)));
    out.push_back((char)(0x80 | (cp & 0x3F)));
  } else if (cp < 0x10000) {
    out.push_back((char)(0xE0 | (cp >> 12)));
    out.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
    out.push_back((char)(0x80 | (cp & 0x3F)));
  } else {
    out.push_back((char)(0xF0 | (cp >> 18)));
    out.push_back((char)(0x80 | ((cp >> 12) & 0x3F)));
    out.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
    out.push_back((char)(0x80 | (cp & 0x3F)));
  }
}

// Strict UTF-8 -> code points (false on malformed input).
bool utf8_cps(std::string_view s, std::vector<uint32_t>& out) {
  out.clear();
  for (size_t i = 0; i < s.size();) {
    const unsigned char c = (unsigned char)s[i];
    uint32_t cp;
    size_t n;
    if (c < 0x80) { cp = c; n = 1; }
    else if ((c >> 5) == 6) { cp = c & 0x1F; n = 2; }
    else if ((c >> 4) == 14) { cp = c & 0x0F; n = 3; }
    else if ((c >> 3) == 30) { cp = c & 0x07; n = 4; }
    else return false;
    if (i + n > s.size()) return false;
    for (size_t k = 1; k < n; ++k) {
      const unsigned char d = (unsigned char)s[i + k];
      if ((d >> 6) != 2) return false;
      cp = (cp << 6) | (d & 0x3F);
    }
    static const uint32_t lo[5] = {0, 0, 0x80, 0x800, 0x10000};
    if (cp < lo[n] || cp > 0x10FFFF || (cp >= 0xD800 && cp <= 0xDFFF)) return false;
    out.push_back(cp);
    i += n;
  }
  return true;
}

// The vocabulary keyed by code points, for the synthesised Unknown nodes
// (beam.py:36-38): their word is chars[b:e] of the sentence, so the packer
// hashes the characters it already has -- every suffix ending at e in one
// pass, last character first -- instead of encoding each span to UTF-8 and
// hashing that.  A string's UTF-8 form and its code points are equal iff the
// strings are (malformed vocabulary strings cannot equal a decoded sentence
// and are left out).
struct CpVocab {
  struct E {
    uint64_t h;                                  // 0: empty
    uint32_t off, n;
    const WordInfo* wi;
  };
  std::vector<uint32_t> pool;
  std::vector<E> tab;
  uint64_t mask = 0;
  static constexpr uint64_t SEED = 0x2545F4914F6CDD1Dull;
  static uint64_t step(uint64_t h, uint32_t cp) {
    h = (h ^ cp) * 0x9E3779B97F4A7C15ull;
    return h ^ (h >> 29);
  }
  static uint64_t fin(uint64_t h, uint32_t n) {
    h ^= (uint64_t)n * 0xC2B2AE3D27D4EB4Full;
    h *= 0xBF58476D1CE4E5B9ull;
    h ^= h >> 32;
    return h | 1ull;
  }
  static uint64_t hash(const uint32_t* s, uint32_t n) {     // last code point first
    uint64_t h = SEED;
    for (uint32_t i = n; i-- > 0;) h = step(h, s[i]);
    return fin(h, n);
  }
  void build(const std::vector<std::pair<std::string_view, const WordInfo*>>& words) {
    size_t cap = 16;
    while (cap < 2 * words.size() + 16) cap <<= 1;
    tab.assign(cap, E{0, 0, 0, nullptr});
    mask = cap - 1;
    std::vector<uint32_t> cps;
    for (const auto& w : words) {
      if (!utf8_cps(w.first, cps)) continue;
      const uint64_t h = hash(cps.data(), (uint32_t)cps.size());
      uint64_t i = h & mask;
      while (tab[i].h) i = (i + 1) & mask;
      tab[i] = E{h, (uint32_t)pool.size(), (uint32_t)cps.size(), w.second};
      pool.insert(pool.end(), cps.begin(), cps.end());
    }
  }
  const WordInfo* find(const uint32_t* s, uint32_t n, uint64_t h) const {
    for (uint64_t i = h & mask;; i = (i + 1) & mask) {
      const E& e = tab[i];
      if (e.h == 0) return nullptr;
      if (e.h == h && e.n == n && std::equal(s, s + n, pool.data() + e.off)) return e.wi;
    }
  }
};

// coefficient by a small non-negative integer (class 4 / 6 lengths): a flat
// array below SMALL, the map above
struct LenCoef {
  static constexpr int64_t SMALL = 64;
  double v[SMALL];
  bool has[SMALL] = {};
  std::unordered_map<int64_t, double> big;
  void put(int64_t k, double c) {                // first entry wins (emplace)
    if (k >= 0 && k < SMALL) {
      if (!has[k]) { has[k] = true; v[k] = c; }
    } else {
      big.emplace(k, c);
    }
  }
  const double* get(int64_t k) const {
    if (k >= 0 && k < SMALL) return has[k] ? &v[k] : nullptr;
    auto it = big.find(k);
    return it == big.end() ? nullptr : &it->second;
  }
};

}  // namespace

// One pack's output arrays, handed to the caller through lt_packed.owner
// (uninitialised: every element is written by the thread that packs its
// sentence, which also first-touches the pages).  A released block goes back
// to its packer's pool (at most two, up to 2 GiB each), so a pipeline of packs
// reuses mapped memory instead of faulting in fresh pages every call.
struct PackPool;
struct PackOut {
  Arr<int32_t> sent_n, span_start, node_word, node_morph0, node_tag;
  Arr<int64_t> sent_node_off, sent_span_off, node_src;
  Arr<uint32_t> node_mask;
  Arr<double> node_pre, node_f4, node_f5, node_f6, node_post;
  // the implicit Unknowns' canonical records (lattice_decode.h n_unk) and the
  // pass-1 verdict per span entry: 1 = its Unknown is a node
  Arr<int32_t> unk_word, unk_morph0, unk_tag;
  Arr<uint32_t> unk_mask;
  Arr<double> unk_pre, unk_f4, unk_f5, unk_f6, unk_post;
  Arr<uint8_t> unk_node;
  std::shared_ptr<PackPool> pool;             // while handed out
  size_t bytes() const {
    return sent_n.bytes() + span_start.bytes() + node_word.bytes() + node_morph0.bytes() +
           node_tag.bytes() + sent_node_off.bytes() + sent_span_off.bytes() + node_src.bytes() +
           node_mask.bytes() + node_pre.bytes() + node_f4.bytes() + node_f5.bytes() + node_f6.bytes() +
           node_post.bytes() + unk_node.bytes();
  }
};
struct PackPool {
  std::mutex mu;
  std::vector<std::unique_ptr<PackOut>> free;
  std::unique_ptr<PackOut> take() {
    std::lock_guard<std::mutex> g(mu);
    if (free.empty()) return std::unique_ptr<PackOut>(new (std::nothrow) PackOut);
    std::unique_ptr<PackOut> o = std::move(free.back());
    free.pop_back();
    return o;
  }
};
static void release_block(PackOut* o) {
  std::shared_ptr<PackPool> pool = std::move(o->pool);
  if (pool && o->bytes() <= ((size_t)2 << 30)) {
    std::lock_guard<std::mutex> g(pool->mu);
    if (pool->free.size() < 2) {
      pool->free.emplace_back(o);
      return;
    }
  }
  delete o;
}

struct lt_packer {
  std::shared_ptr<PackPool> pool = std::make_shared<PackPool>();
  ViewMap<WordInfo> vocab;                          // vocabulary strings and class-5 words
  std::vector<uint32_t> vmask;
  LenCoef c4, c6;
  std::vector<C5Entry> c5e;                         // grouped by word (WordInfo::c5_lo)
  int32_t n_local = 0, n_pre = 0;
  std::vector<int32_t> kind;
  std::vector<double> reg;                          // 3 per scorer
  std::vector<ViewMap<double>> pref;                // per scorer: (tag, key) -> value
  std::string kb;                                   // key buffer
  CpVocab cpv;                                      // vocab by code points (Unknown nodes)
  bool pref_unk = false;                            // a preference entry for tag 'Unknown'
  bool has_pref = false;                            // any preference entry
  bool implicit = false;                            // implicit Unknowns (lt_packer_desc.implicit_unk)

  int32_t id_of(std::string_view s) const {
    const WordInfo* v = vocab.get(s);
    return v ? v->id : 0;
  }
  uint32_t vm(int32_t id) const { return id >= 0 && (size_t)id < vmask.size() ? vmask[(size_t)id] : 0u; }
};

lt_status lt_packer_create(const lt_packer_desc* d, lt_packer** out) {
  if (!d || !out) return set_error(LT_EINVAL, "lt_packer_create: NULL argument");
  *out = nullptr;
  if (d->n_local < 0 || d->n_pre < 0 || d->n_pre > d->n_local)
    return set_error(LT_EINVAL, "lt_packer_create: bad scorer counts");
  lt_packer* p = new (std::nothrow) lt_packer;
  if (!p) return set_error(LT_ENOMEM, "lt_packer_create: out of memory");
  try {
    for (int64_t i = 0; i < d->vocab.n; ++i)
      if (!is_null(d->vocab, i)) p->vocab.put(str_at(d->vocab, i), WordInfo{d->vocab_id[i], 0, 0});
    p->vmask.assign(d->vmask, d->vmask + d->n_vmask);
    for (int64_t i = 0; i < d->n4; ++i) p->c4.put(d->c4_len[i], d->c4_coef[i]);
    for (int64_t i = 0; i < d->n6; ++i) p->c6.put(d->c6_len[i], d->c6_coef[i]);
    // class-5 entries grouped by word, in input order within a word (the
    // first of equal keys wins, as the Python dict the entries come from)
    std::vector<int64_t> c5_order((size_t)d->c5_word.n);
    for (int64_t i = 0; i < d->c5_word.n; ++i) c5_order[(size_t)i] = i;
    std::stable_sort(c5_order.begin(), c5_order.end(), [&](int64_t x, int64_t y) {
      return str_at(d->c5_word, x) < str_at(d->c5_word, y);
    });
    for (size_t j = 0; j < c5_order.size();) {
      const std::string_view w = str_at(d->c5_word, c5_order[j]);
      if (!p->vocab.get(w)) p->vocab.put(w, WordInfo{0, 0, 0});
      WordInfo* wi = p->vocab.get_mut(w);
      wi->c5_lo = (int32_t)p->c5e.size();
      for (; j < c5_order.size() && str_at(d->c5_word, c5_order[j]) == w; ++j) {
        const int64_t i = c5_order[j];
        p->c5e.push_back(C5Entry{std::string(str_at(d->c5_tag, i)), d->c5_isl[i], d->c5_coef[i]});
      }
      wi->c5_n = (int32_t)p->c5e.size() - wi->c5_lo;
    }
    p->n_local = d->n_local;
    p->n_pre = d->n_pre;
    p->implicit = d->implicit_unk != 0;
    p->kind.assign(d->local_kind, d->local_kind + d->n_local);
    p->reg.assign(d->reg_params, d->reg_params + 3 * (size_t)d->n_local);
    p->pref.resize((size_t)d->n_local);
    for (int64_t i = 0; i < d->pref_tag.n; ++i) {
      const int32_t s = d->pref_scorer[i];
      if (s < 0 || s >= d->n_local) {
        delete p;
        return set_error(LT_EINVAL, "lt_packer_create: preference entry %lld names scorer %d",
                         (long long)i, s);
      }
      p->pref[(size_t)s].put(tuple_key(p->kb, str_at(d->pref_tag, i), str_at(d->pref_key, i)),
                             d->pref_value[i]);
      if (str_at(d->pref_tag, i) == kUnk) p->pref_unk = true;
      p->has_pref = true;
    }
    std::vector<std::pair<std::string_view, const WordInfo*>> words;
    for (const auto& e : p->vocab.tab)
      if (e.h) words.emplace_back(std::string_view(e.s, (size_t)e.n), &e.v);
    p->cpv.build(words);
  } catch (...) {
    delete p;
    return set_error(LT_ENOMEM, "lt_packer_create: out of memory");
  }
  *out = p;
  return LT_OK;
}

lt_status lt_packer_destroy(lt_packer* p) {
  delete p;
  return LT_OK;
}

namespace {

// One lattice node's fields, as lattice_based_tagger_amd.word.Word.
struct NodeView {
  std::string_view word, morph0, tag0, morph1, tag1;
  bool has_morph1, has_tag1;
  int64_t len, is_l;
};

// score_funcs.py:65-73 (value = 0; value += ...; value += ...)
double regularization(const double* prm, const NodeView& w) {
  double v = 0.0;
  if (w.tag0 == kUnk) v = v + prm[0] * ((double)w.len + 0.1);
  else v = v + prm[1] * (double)w.len;
  if (w.len == 1 && w.tag0 == kNoun) v = v + prm[2];
  return v;
}

double lookup(std::string& kb, const ViewMap<double>& m, std::string_view t, std::string_view k) {
  const double* v = m.get(tuple_key(kb, t, k));
  return v ? *v : 0.0;
}

// A node's packed record (packer.py _record: node_record + node_terms).
struct Rec {
  int32_t wid, mid, tid;
  uint32_t m;
  double pre, f4, f5, f6;
};

// The record of node w: its word's vocabulary entry wi (null: none), morph0 id
// mid and tag0 id tid; post[t]: the node-local terms after the trigram.
// nostr: w's strings equal no preference-table key (the canonical Unknown's
// surface, packer.py _NOSTR).
void node_rec(const lt_packer* p, std::string& kb, const NodeView& w, const WordInfo* wi, int32_t mid,
              int32_t tid, Rec& r, double* post, bool nostr = false) {
  const int32_t wid = wi ? wi->id : 0;
  uint32_t m = node_mask(p->vm(wid), p->vm(mid), p->vm(tid));
  const bool unk_node = w.tag0 == kUnk;
  if (unk_node) m |= F_UNK;
  if (contextual(w.tag0)) m |= F_CTX;
  double f4 = 0.0, f5 = 0.0, f6 = 0.0;
  if (const double* c = p->c4.get(w.len)) { m |= F_HAS4; f4 = *c; }
  if (wi) {                                          // (word, tag0, is_l) -> coef
    for (int32_t j = wi->c5_lo; j < wi->c5_lo + wi->c5_n; ++j) {
      const C5Entry& c = p->c5e[(size_t)j];
      if (c.is_l == w.is_l && c.tag == w.tag0) {
        m |= F_HAS5;
        f5 = c.coef;
        break;
      }
    }
  }
  if (unk_node) {
    if (const double* c = p->c6.get(w.len < 8 ? w.len : 8)) { m |= F_HAS6; f6 = *c; }
  }
  // node-local scorers in constructor order (lowering.node_terms)
  double pre = 0.0;
  for (int t = 0; t < p->n_local; ++t) {
    double v;
    switch (p->kind[(size_t)t]) {
      case LT_SCORER_REGULARIZATION: v = regularization(&p->reg[3 * (size_t)t], w); break;
      case LT_SCORER_MORPH_PREF:                   // score_funcs.py:84-88
        v = nostr ? 0.0 : lookup(kb, p->pref[(size_t)t], w.tag0, w.morph0);
        if (w.has_tag1) v = v + (w.has_morph1 ? lookup(kb, p->pref[(size_t)t], w.tag1, w.morph1) : 0.0);
        break;
      default:                                     // WordPreference, score_funcs.py:99-100
        v = nostr ? 0.0 : lookup(kb, p->pref[(size_t)t], w.tag0, w.word);
    }
    if (t < p->n_pre) pre = pre + v;
    else post[t - p->n_pre] = v;
  }
  r = Rec{wid, mid, tid, m, pre, f4, f5, f6};
}

// bit-identical records (floats compared as bit patterns: -0.0 kept)
bool same_rec(const Rec& a, const double* pa, const Rec& b, const double* pb, int n_post) {
  return a.wid == b.wid && a.mid == b.mid && a.tid == b.tid && a.m == b.m &&
         std::memcmp(&a.pre, &b.pre, 4 * sizeof(double)) == 0 &&
         (n_post == 0 || std::memcmp(pa, pb, (size_t)n_post * sizeof(double)) == 0);
}

}  // namespace

namespace {

// Node sources of the packer: the generic columnar lattices (UTF-8 strings,
// lt_lattice_desc) and the native builder's compact lattices (strings as code
// point references, lt_lattice_store.h).  node() gives a dictionary node's
// fields, its vocabulary entry and its morph0 id.
struct DescSrc {
  const lt_lattice_desc* L;
  const lt_packer* p;
  int32_t n_sent() const { return L->n_sent; }
  int64_t n_words() const { return L->n_words; }
  const uint32_t* chars() const { return L->chars; }
  const int64_t* char_off() const { return L->char_off; }
  const int64_t* slot_off() const { return L->slot_off; }
  int64_t e(int64_t i) const { return L->e[i]; }
  struct Buf {};
  void node(int64_t i, Buf&, NodeView& v, const WordInfo*& wi, int32_t& mid) const {
    v.word = str_at(L->word, i);
    v.morph0 = str_at(L->morph0, i);
    v.tag0 = str_at(L->tag0, i);
    v.has_morph1 = !is_null(L->morph1, i);
    v.has_tag1 = !is_null(L->tag1, i);
    v.morph1 = v.has_morph1 ? str_at(L->morph1, i) : std::string_view();
    v.tag1 = v.has_tag1 ? str_at(L->tag1, i) : std::string_view();
    v.len = L->len[i];
    v.is_l = L->is_l[i];
    wi = p->vocab.get(v.word);
    const int32_t wid = wi ? wi->id : 0;
    mid = v.morph0.data() == v.word.data() && v.morph0.size() == v.word.size() ? wid : p->id_of(v.morph0);
  }
};

struct LatSrc {
  const lt_lattices* L;
  const lt_packer* p;
  bool strings;                                  // preference scorers read the node strings
  int32_t n_sent() const { return (int32_t)L->n_sent; }
  int64_t n_words() const { return L->n_words; }
  const uint32_t* chars() const { return L->chars.data(); }
  const int64_t* char_off() const { return L->char_off.data(); }
  const int64_t* slot_off() const { return L->slot_off.data(); }
  int64_t e(int64_t i) const { return L->e[i]; }
  struct Buf {
    std::string w, m0, m1;
  };
  void node(int64_t i, Buf& buf, NodeView& v, const WordInfo*& wi, int32_t& mid) const {
    const uint32_t* wc = L->text.data() + L->w_off[i];
    const uint32_t wn = L->w_len[i];
    wi = p->cpv.find(wc, wn, CpVocab::hash(wc, wn));
    const int32_t wid = wi ? wi->id : 0;
    const bool own0 = L->m0_off[i] != LT_NOREF;
    if (own0) {
      const uint32_t* mc = L->pool.data() + L->m0_off[i];
      const WordInfo* mi = p->cpv.find(mc, L->m0_len[i], CpVocab::hash(mc, L->m0_len[i]));
      mid = mi ? mi->id : 0;
    } else {
      mid = wid;
    }
    v.tag0 = L->names[(size_t)L->tag0[i]];
    v.has_tag1 = L->tag1[i] >= 0;
    v.tag1 = v.has_tag1 ? std::string_view(L->names[(size_t)L->tag1[i]]) : std::string_view();
    v.has_morph1 = L->m1_off[i] != LT_NOREF;
    v.len = L->len[i];
    v.is_l = L->is_l[i];
    if (strings) {
      buf.w.clear();
      for (uint32_t k = 0; k < wn; ++k) utf8_append(buf.w, wc[k]);
      v.word = buf.w;
      if (own0) {
        buf.m0.clear();
        for (uint32_t k = 0; k < L->m0_len[i]; ++k) utf8_append(buf.m0, L->pool[L->m0_off[i] + k]);
        v.morph0 = buf.m0;
      } else {
        v.morph0 = v.word;
      }
      buf.m1.clear();
      if (v.has_morph1)
        for (uint32_t k = 0; k < L->m1_len[i]; ++k) utf8_append(buf.m1, L->pool[L->m1_off[i] + k]);
      v.morph1 = v.has_morph1 ? std::string_view(buf.m1) : std::string_view();
    } else {
      v.word = v.morph0 = v.morph1 = std::string_view();
    }
  }
};

template <class Src>
lt_status pack_impl(lt_packer* p, const Src& L, int max_len, lt_packed* out) {
  if (max_len < 1) return set_error(LT_EUNSUPPORTED, "lt_packer_pack: max_len %d < 1", max_len);
  if (L.n_sent() < 0 || L.n_words() < 0) return set_error(LT_EINVAL, "lt_packer_pack: negative size");
  const int32_t S = L.n_sent();
  const int64_t* const char_off = L.char_off();
  const int64_t* const slot_off = L.slot_off();
  const uint32_t* const chars = L.chars();
  const int64_t T = S ? char_off[S] : 0;
  int64_t longest = 0;
  for (int32_t s = 0; s < S; ++s) {
    if (char_off[s + 1] < char_off[s]) return set_error(LT_EINVAL, "lt_packer_pack: char offsets decrease");
    longest = std::max<int64_t>(longest, char_off[s + 1] - char_off[s]);
  }
  // a span never exceeds its sentence: max_len beyond max(8, longest) decodes
  // as that (beam.py:29-30), which keeps the span table small
  max_len = (int)std::min<int64_t>(max_len, std::max<int64_t>(MAX_SPAN, longest));
  if (max_len > LT_MAX_LEN_ANY)
    return set_error(LT_EUNSUPPORTED, "lt_packer_pack: max_len %d > %d", max_len, LT_MAX_LEN_ANY);
  const int SS = span_slots(max_len);           // span slots per end position
  for (int64_t g = 0; g < T; ++g)
    if (slot_off[g + 1] < slot_off[g] || slot_off[g + 1] > L.n_words())
      return set_error(LT_EINVAL, "lt_packer_pack: bad begin-slot offsets");
  const int n_post = p->n_local - p->n_pre;

  // dictionary candidates of span (b, e) in begin slot g: words with w.e == e (beam.py:33)
  auto span_count = [&](int64_t g, int32_t e) {
    int64_t c = 0;
    for (int64_t i = slot_off[g]; i < slot_off[g + 1]; ++i) c += L.e(i) == e;
    return c;
  };
  std::unique_ptr<PackOut> o = p->pool->take();
  if (!o) return set_error(LT_ENOMEM, "lt_packer_pack: out of memory");
  o->pool = p->pool;
  if (!o->sent_n.alloc(S) || !o->sent_node_off.alloc((int64_t)S + 1) || !o->sent_span_off.alloc((int64_t)S + 1))
    return set_error(LT_ENOMEM, "lt_packer_pack: out of memory");
  // span entries: SS n + 1 per sentence
  o->sent_span_off[0] = 0;
  for (int32_t s = 0; s < S; ++s) o->sent_span_off[s + 1] = o->sent_span_off[s] + SS * (char_off[s + 1] - char_off[s]) + 1;
  const int64_t NSP = o->sent_span_off[S];
  // implicit Unknowns: the canonical record of every span length (an Unknown
  // whose surface is in no vocabulary entry: packer.py unknown_records)
  const bool implicit = p->implicit;
  const int32_t unk_tid = p->id_of(kUnk);
  std::vector<Rec> canon;
  std::vector<double> canon_post;
  if (implicit) {
    if (!o->unk_word.alloc(SS) || !o->unk_morph0.alloc(SS) || !o->unk_tag.alloc(SS) || !o->unk_mask.alloc(SS) ||
        !o->unk_pre.alloc(SS) || !o->unk_f4.alloc(SS) || !o->unk_f5.alloc(SS) || !o->unk_f6.alloc(SS) ||
        !o->unk_post.alloc((int64_t)n_post * SS))
      return set_error(LT_ENOMEM, "lt_packer_pack: out of memory");
    canon.resize((size_t)SS);
    canon_post.assign((size_t)SS * (size_t)n_post, 0.0);
    std::string kb;
    static constexpr std::string_view none;
    for (int d = 1; d <= SS; ++d) {
      const NodeView u{none, none, kUnk, {}, {}, false, false, (int64_t)d, 0};
      Rec& r = canon[(size_t)d - 1];
      node_rec(p, kb, u, nullptr, 0, unk_tid, r, canon_post.data() + (size_t)(d - 1) * n_post, true);
      o->unk_word[d - 1] = r.wid;
      o->unk_morph0[d - 1] = r.mid;
      o->unk_tag[d - 1] = r.tid;
      o->unk_mask[d - 1] = r.m;
      o->unk_pre[d - 1] = r.pre;
      o->unk_f4[d - 1] = r.f4;
      o->unk_f5[d - 1] = r.f5;
      o->unk_f6[d - 1] = r.f6;
      for (int t = 0; t < n_post; ++t) o->unk_post[(int64_t)t * SS + d - 1] = canon_post[(size_t)(d - 1) * n_post + t];
    }
    if (!o->unk_node.alloc(NSP)) return set_error(LT_ENOMEM, "lt_packer_pack: out of memory");
  }
  // words per span (b, d) of a sentence from one pass over its words (a
  // begin slot's words are otherwise rescanned for every end position); too
  // large a table (long sentences at a large max_len): scan as before
  auto span_table = [&](int64_t c0, int32_t n, std::vector<uint16_t>& tab) {
    if ((int64_t)n * max_len > (1 << 20)) return false;
    tab.assign((size_t)n * (size_t)max_len, 0);
    for (int32_t b = 0; b < n; ++b)
      for (int64_t i = slot_off[c0 + b]; i < slot_off[c0 + b + 1]; ++i) {
        const int64_t d = L.e(i) - b;
        if (d >= 1 && d <= max_len) {
          uint16_t& t = tab[(size_t)b * (size_t)max_len + (size_t)(d - 1)];
          if (t == 0xFFFF) return false;                  // (counts past 16 bits: scan)
          ++t;
        }
      }
    return true;
  };
  // Unknown nodes by code points (CpVocab) unless a preference scorer has an
  // entry for the tag 'Unknown' (its value would depend on the string)
  const bool fast_unk = !p->pref_unk;
  constexpr int HMAX = 16;
  // The Unknown of span (b, e) of the sentence at c0 (beam.py:36-38): its
  // vocabulary entry (null: none), found by the code points of chars[b:e]
  // (hs: CpVocab hashes of the suffixes ending at e, computed on first use),
  // or by its UTF-8 string `unk` (built when the fast path cannot answer).
  struct UnkProbe {
    uint64_t hs[HMAX + 1];
    bool hashed = false;
    bool have_str = false;
    std::string unk;
  };
  auto unk_entry = [&](UnkProbe& u, int64_t c0, int32_t e, int d, const WordInfo*& wi) {
    const uint32_t* cs = chars + c0;
    const int32_t b = e - d;
    if (fast_unk && d <= HMAX) {
      if (!u.hashed) {
        uint64_t h = CpVocab::SEED;
        for (int k = 1; k <= HMAX && k <= e; ++k) {
          h = CpVocab::step(h, cs[e - k]);
          u.hs[k] = CpVocab::fin(h, (uint32_t)k);
        }
        u.hashed = true;
      }
      wi = p->cpv.find(cs + b, (uint32_t)d, u.hs[d]);
      if (!wi) return;                                  // not a vocabulary string: no string needed
    }
    u.unk.clear();
    for (int32_t x = b; x < e; ++x) utf8_append(u.unk, cs[x]);
    u.have_str = true;
    wi = p->vocab.get(u.unk);
  };
  // pass 1: nodes per sentence (threads over sentences) -> offsets; with
  // implicit Unknowns, the verdict on every empty span's Unknown (unk_node)
  parallel_ranges(S, [&](int, int64_t lo, int64_t hi) {
    std::vector<uint16_t> tab;
    std::string kb;
    std::vector<double> post((size_t)std::max(n_post, 1));
    for (int64_t s = lo; s < hi; ++s) {
      const int64_t c0 = char_off[s];
      const int32_t n = (int32_t)(char_off[s + 1] - c0);
      int64_t cnt = 1;                                    // BOS
      const bool tabbed = span_table(c0, n, tab);
      uint8_t* const un = implicit ? o->unk_node.data() + o->sent_span_off[s] : nullptr;
      for (int32_t e = 1; e <= n; ++e) {
        UnkProbe u;
        for (int d = std::min<int>(max_len, e); d >= 1; --d) {
          const int64_t c = tabbed ? tab[(size_t)(e - d) * (size_t)max_len + (size_t)(d - 1)]
                                   : span_count(c0 + e - d, e);
          if (c) {
            cnt += c;
            continue;
          }
          if (!implicit) {
            ++cnt;
            continue;
          }
          // the Unknown is implicit iff its record is the canonical one of d
          const WordInfo* wi = nullptr;
          u.have_str = false;
          unk_entry(u, c0, e, d, wi);
          bool node = false;
          if (wi || u.have_str) {
            const std::string_view sv = u.have_str ? std::string_view(u.unk) : std::string_view();
            const NodeView v{sv, sv, kUnk, {}, {}, false, false, (int64_t)d, 0};
            Rec r;
            node_rec(p, kb, v, wi, wi ? wi->id : 0, unk_tid, r, post.data());
            node = !same_rec(r, post.data(), canon[(size_t)d - 1], canon_post.data() + (size_t)(d - 1) * n_post,
                             n_post);
          }
          un[(e - 1) * SS + (SS - d)] = node ? 1 : 0;
          cnt += node ? 1 : 0;
        }
      }
      o->sent_n[s] = n;
      o->sent_node_off[s + 1] = cnt;
    }
  }, 256);
  o->sent_node_off[0] = 0;
  for (int32_t s = 0; s < S; ++s) o->sent_node_off[s + 1] += o->sent_node_off[s];
  const int64_t N = o->sent_node_off[S];
  if (!o->span_start.alloc(NSP) || !o->node_word.alloc(N) || !o->node_morph0.alloc(N) ||
      !o->node_tag.alloc(N) || !o->node_mask.alloc(N) || !o->node_pre.alloc(N) || !o->node_f4.alloc(N) ||
      !o->node_f5.alloc(N) || !o->node_f6.alloc(N) || !o->node_src.alloc(N) ||
      !o->node_post.alloc((int64_t)n_post * N))
    return set_error(LT_ENOMEM, "lt_packer_pack: out of memory");

  // pass 2: fill, sentences split over threads (the tables are read-only)
  PackOut& q = *o;

  auto fill = [&](int, int64_t s_lo, int64_t s_hi) {
    std::string kb;
    typename Src::Buf nbuf;
    std::vector<uint16_t> tab;
    std::vector<double> post((size_t)std::max(n_post, 1));
    // tags are few: remember the last distinct ones (their strings live in
    // the lattice blobs for the whole call)
    std::string_view memo_s[16];
    int32_t memo_id[16];
    int n_memo = 0;
    auto tag_id = [&](std::string_view t) {
      for (int i = 0; i < n_memo; ++i)
        if (memo_s[i] == t) return memo_id[i];
      const int32_t id = p->id_of(t);
      if (n_memo < 16) {
        memo_s[n_memo] = t;
        memo_id[n_memo++] = id;
      }
      return id;
    };
    auto put = [&](int64_t x, const Rec& r, int64_t src) {
      for (int t = 0; t < n_post; ++t) q.node_post[(int64_t)t * N + x] = post[(size_t)t];
      q.node_word[x] = r.wid;
      q.node_mask[x] = r.m;
      q.node_morph0[x] = r.mid;
      q.node_tag[x] = r.tid;
      q.node_pre[x] = r.pre;
      q.node_f4[x] = r.f4;
      q.node_f5[x] = r.f5;
      q.node_f6[x] = r.f6;
      q.node_src[x] = src;
    };
    auto add_node_wi = [&](int64_t x, const NodeView& w, const WordInfo* wi, int32_t mid, int64_t src) {
      Rec r;
      node_rec(p, kb, w, wi, mid, tag_id(w.tag0), r, post.data());
      put(x, r, src);
    };
    for (int64_t s = s_lo; s < s_hi; ++s) {
      const int64_t c0 = char_off[s];
      const int32_t n = q.sent_n[s];
      const int64_t base = q.sent_node_off[s];
      int32_t* ss = q.span_start.data() + q.sent_span_off[s];
      const uint8_t* const un = implicit ? q.unk_node.data() + q.sent_span_off[s] : nullptr;
      NodeView bos{kBOS, kBOS, kBOS, {}, {}, false, false, 0, 0};
      {
        const WordInfo* wi = p->vocab.get(bos.word);
        add_node_wi(base, bos, wi, wi ? wi->id : 0, -1);
      }
      int32_t local = 1;
      const bool tabbed = span_table(c0, n, tab);
      for (int32_t e = 1; e <= n; ++e) {
        UnkProbe u;
        for (int d = SS; d >= 1; --d) {
          *ss++ = local;
          const int32_t b = e - d;
          if (d > max_len || b < 0) continue;
          const int64_t g = c0 + b;
          bool any = false;
          const bool empty = tabbed && tab[(size_t)b * (size_t)max_len + (size_t)(d - 1)] == 0;
          for (int64_t i = empty ? slot_off[g + 1] : slot_off[g]; i < slot_off[g + 1]; ++i) {
            if (L.e(i) != e) continue;                  // beam.py:33 (w.e == e)
            NodeView v;
            const WordInfo* wi;
            int32_t mid;
            L.node(i, nbuf, v, wi, mid);
            add_node_wi(base + local, v, wi, mid, i);
            ++local;
            any = true;
          }
          if (any) continue;
          // beam.py:36-38: Unknown chars[b:e] -- implicit (no node) unless the
          // pass-1 verdict made it one
          if (implicit && !un[(e - 1) * SS + (SS - d)]) continue;
          const int64_t src = -2 - (((int64_t)b << 32) | (int64_t)(d - 1));
          const WordInfo* wi = nullptr;
          u.have_str = false;
          unk_entry(u, c0, e, d, wi);
          const std::string_view sv = u.have_str ? std::string_view(u.unk) : std::string_view();
          const NodeView w{sv, sv, kUnk, {}, {}, false, false, (int64_t)d, 0};
          add_node_wi(base + local, w, wi, wi ? wi->id : 0, src);
          ++local;
        }
      }
      *ss = local;
    }
  };
  int64_t per = 256;                                   // sentences per thread range, at least
  if (const char* env = std::getenv("LT_PACK_THREADS"))
    per = std::max<int64_t>(1, ((int64_t)S + std::max(1, std::atoi(env)) - 1) / std::max(1, std::atoi(env)));
  try {
    parallel_ranges(S, fill, per);
  } catch (...) {
    return set_error(LT_ENOMEM, "lt_packer_pack: out of memory");
  }

  lt_batch_desc& b = out->batch;
  std::memset(out, 0, sizeof *out);
  b.n_sent = S;
  b.max_len = max_len;
  b.n_post = n_post;
  b.has_trigram = 0;            // set by the caller (the trigram is not the packer's concern)
  b.n_nodes = N;
  b.n_span = o->sent_span_off[S];
  b.sent_n = o->sent_n.data();
  b.sent_node_off = o->sent_node_off.data();
  b.sent_span_off = o->sent_span_off.data();
  b.span_start = o->span_start.data();
  b.node_word = o->node_word.data();
  b.node_morph0 = o->node_morph0.data();
  b.node_tag = o->node_tag.data();
  b.node_mask = o->node_mask.data();
  b.node_pre = o->node_pre.data();
  b.node_f4 = o->node_f4.data();
  b.node_f5 = o->node_f5.data();
  b.node_f6 = o->node_f6.data();
  b.node_post = n_post ? o->node_post.data() : nullptr;
  if (implicit) {
    b.n_unk = SS;
    b.unk_word = o->unk_word.data();
    b.unk_morph0 = o->unk_morph0.data();
    b.unk_tag = o->unk_tag.data();
    b.unk_mask = o->unk_mask.data();
    b.unk_pre = o->unk_pre.data();
    b.unk_f4 = o->unk_f4.data();
    b.unk_f5 = o->unk_f5.data();
    b.unk_f6 = o->unk_f6.data();
    b.unk_post = n_post ? o->unk_post.data() : nullptr;
  }
  out->node_src = o->node_src.data();
  out->owner = o.release();
  return LT_OK;
}

}  // namespace

lt_status lt_packer_pack(lt_packer* p, const lt_lattice_desc* L, int max_len, lt_packed* out) {
  if (!p || !L || !out) return set_error(LT_EINVAL, "lt_packer_pack: NULL argument");
  return pack_impl(p, DescSrc{L, p}, max_len, out);
}

lt_status lt_packer_pack_lattices(lt_packer* p, const lt_lattices* L, int max_len, lt_packed* out) {
  if (!p || !L || !out) return set_error(LT_EINVAL, "lt_packer_pack_lattices: NULL argument");
  return pack_impl(p, LatSrc{L, p, p->has_pref}, max_len, out);
}

lt_status lt_packed_release(lt_packed* out) {
  if (!out) return LT_OK;
  if (out->owner) release_block(static_cast<PackOut*>(out->owner));
  std::memset(out, 0, sizeof *out);
  return LT_OK;
}
