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

// Key of a (string, string[, int]) tuple written into a reused buffer: a, b,
// then a's length (strings with any byte, NUL included, split unambiguously),
// then the optional integer.
std::string_view tuple_key(std::string& buf, std::string_view a, std::string_view b) {
  buf.clear();
  buf.append(a);
  buf.append(b);
  const uint32_t la = (uint32_t)a.size();
  buf.append(reinterpret_cast<const char*>(&la), sizeof la);
  return buf;
}
std::string_view tuple_key(std::string& buf, std::string_view a, std::string_view b, int64_t x) {
  tuple_key(buf, a, b);
  buf.append(reinterpret_cast<const char*>(&x), sizeof x);
  return buf;
}

// string_view-keyed map over strings the packer owns (no allocation per lookup)
template <typename V>
struct ViewMap {
  std::vector<std::unique_ptr<std::string>> store;
  std::unordered_map<std::string_view, V> map;
  void put(std::string_view k, V v) {
    if (map.count(k)) return;                    // first entry wins (Python dict semantics)
    store.emplace_back(new std::string(k));
    map.emplace(std::string_view(*store.back()), v);
  }
  const V* get(std::string_view k) const {
    auto it = map.find(k);
    return it == map.end() ? nullptr : &it->second;
  }
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

}  // namespace

struct lt_packer {
  ViewMap<int32_t> vocab;
  std::vector<uint32_t> vmask;
  std::unordered_map<int64_t, double> c4, c6;
  ViewMap<double> c5;                               // (word, tag0, is_l)
  int32_t n_local = 0, n_pre = 0;
  std::vector<int32_t> kind;
  std::vector<double> reg;                          // 3 per scorer
  std::vector<ViewMap<double>> pref;                // per scorer: (tag, key) -> value
  std::string kb;                                   // key buffer
  // output buffers
  std::vector<int32_t> sent_n, span_start, node_word, node_morph0, node_tag;
  std::vector<int64_t> sent_node_off, sent_span_off, node_src;
  std::vector<uint32_t> node_mask;
  std::vector<double> node_pre, node_f4, node_f5, node_f6, node_post;

  int32_t id_of(std::string_view s) const {
    const int32_t* v = vocab.get(s);
    return v ? *v : 0;
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
      if (!is_null(d->vocab, i)) p->vocab.put(str_at(d->vocab, i), d->vocab_id[i]);
    p->vmask.assign(d->vmask, d->vmask + d->n_vmask);
    for (int64_t i = 0; i < d->n4; ++i) p->c4.emplace(d->c4_len[i], d->c4_coef[i]);
    for (int64_t i = 0; i < d->n6; ++i) p->c6.emplace(d->c6_len[i], d->c6_coef[i]);
    for (int64_t i = 0; i < d->c5_word.n; ++i)
      p->c5.put(tuple_key(p->kb, str_at(d->c5_word, i), str_at(d->c5_tag, i), d->c5_isl[i]), d->c5_coef[i]);
    p->n_local = d->n_local;
    p->n_pre = d->n_pre;
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
    }
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

}  // namespace

lt_status lt_packer_pack(lt_packer* p, const lt_lattice_desc* L, int max_len, lt_packed* out) {
  if (!p || !L || !out) return set_error(LT_EINVAL, "lt_packer_pack: NULL argument");
  if (max_len < 1 || max_len > LT_MAX_SPAN)
    return set_error(LT_EUNSUPPORTED, "lt_packer_pack: max_len %d not in 1..%d", max_len, LT_MAX_SPAN);
  if (L->n_sent < 0 || L->n_words < 0) return set_error(LT_EINVAL, "lt_packer_pack: negative size");
  const int32_t S = L->n_sent;
  const int64_t T = S ? L->char_off[S] : 0;
  for (int32_t s = 0; s < S; ++s)
    if (L->char_off[s + 1] < L->char_off[s]) return set_error(LT_EINVAL, "lt_packer_pack: char offsets decrease");
  for (int64_t g = 0; g < T; ++g)
    if (L->slot_off[g + 1] < L->slot_off[g] || L->slot_off[g + 1] > L->n_words)
      return set_error(LT_EINVAL, "lt_packer_pack: bad begin-slot offsets");
  const int n_post = p->n_local - p->n_pre;

  // candidates of span (b, e) in begin slot g: words with w.e == e (beam.py:33),
  // or one synthesised Unknown node (beam.py:36-38)
  auto span_count = [&](int64_t g, int32_t e) {
    int64_t c = 0;
    for (int64_t i = L->slot_off[g]; i < L->slot_off[g + 1]; ++i) c += L->e[i] == e;
    return c ? c : 1;
  };
  try {
    // pass 1: nodes per sentence -> offsets (span entries: 8 n + 1 per sentence)
    p->sent_n.resize((size_t)S);
    p->sent_node_off.assign((size_t)S + 1, 0);
    p->sent_span_off.assign((size_t)S + 1, 0);
    for (int32_t s = 0; s < S; ++s) {
      const int64_t c0 = L->char_off[s];
      const int32_t n = (int32_t)(L->char_off[s + 1] - c0);
      int64_t cnt = 1;                                    // BOS
      for (int32_t e = 1; e <= n; ++e)
        for (int d = 1; d <= max_len && d <= e; ++d) cnt += span_count(c0 + e - d, e);
      p->sent_n[(size_t)s] = n;
      p->sent_node_off[(size_t)s + 1] = p->sent_node_off[(size_t)s] + cnt;
      p->sent_span_off[(size_t)s + 1] = p->sent_span_off[(size_t)s] + 8 * (int64_t)n + 1;
    }
    const size_t N = (size_t)p->sent_node_off[(size_t)S];
    p->span_start.resize((size_t)p->sent_span_off[(size_t)S]);
    p->node_word.resize(N); p->node_morph0.resize(N); p->node_tag.resize(N);
    p->node_mask.resize(N); p->node_pre.resize(N); p->node_f4.resize(N); p->node_f5.resize(N);
    p->node_f6.resize(N); p->node_src.resize(N);
    p->node_post.assign((size_t)n_post * N, 0.0);

    // pass 2: fill, sentences split over threads (the tables are read-only)
    auto fill = [&](int32_t s_lo, int32_t s_hi) {
      std::string kb, unk;
      auto add_node = [&](size_t x, const NodeView& w, int64_t src) {
        const int32_t wid = p->id_of(w.word), tid = p->id_of(w.tag0);
        const int32_t mid = w.morph0.data() == w.word.data() && w.morph0.size() == w.word.size()
                                ? wid : p->id_of(w.morph0);
        uint32_t m = node_mask(p->vm(wid), p->vm(mid), p->vm(tid));
        const bool unk_node = w.tag0 == kUnk;
        if (unk_node) m |= F_UNK;
        if (contextual(w.tag0)) m |= F_CTX;
        double f4 = 0.0, f5 = 0.0, f6 = 0.0;
        if (auto it = p->c4.find(w.len); it != p->c4.end()) { m |= F_HAS4; f4 = it->second; }
        if (const double* v = p->c5.get(tuple_key(kb, w.word, w.tag0, w.is_l))) { m |= F_HAS5; f5 = *v; }
        if (unk_node) {
          if (auto it = p->c6.find(w.len < 8 ? w.len : 8); it != p->c6.end()) { m |= F_HAS6; f6 = it->second; }
        }
        // node-local scorers in constructor order (lowering.node_terms)
        double pre = 0.0;
        for (int t = 0; t < p->n_local; ++t) {
          double v;
          switch (p->kind[(size_t)t]) {
            case LT_SCORER_REGULARIZATION: v = regularization(&p->reg[3 * (size_t)t], w); break;
            case LT_SCORER_MORPH_PREF:                   // score_funcs.py:84-88
              v = lookup(kb, p->pref[(size_t)t], w.tag0, w.morph0);
              if (w.has_tag1) v = v + (w.has_morph1 ? lookup(kb, p->pref[(size_t)t], w.tag1, w.morph1) : 0.0);
              break;
            default:                                     // WordPreference, score_funcs.py:99-100
              v = lookup(kb, p->pref[(size_t)t], w.tag0, w.word);
          }
          if (t < p->n_pre) pre = pre + v;
          else p->node_post[(size_t)(t - p->n_pre) * N + x] = v;
        }
        p->node_word[x] = wid;
        p->node_morph0[x] = mid;
        p->node_tag[x] = tid;
        p->node_mask[x] = m;
        p->node_pre[x] = pre;
        p->node_f4[x] = f4;
        p->node_f5[x] = f5;
        p->node_f6[x] = f6;
        p->node_src[x] = src;
      };
      for (int32_t s = s_lo; s < s_hi; ++s) {
        const int64_t c0 = L->char_off[s];
        const int32_t n = p->sent_n[(size_t)s];
        const size_t base = (size_t)p->sent_node_off[(size_t)s];
        int32_t* ss = p->span_start.data() + p->sent_span_off[(size_t)s];
        NodeView bos{kBOS, kBOS, kBOS, {}, {}, false, false, 0, 0};
        add_node(base, bos, -1);
        int32_t local = 1;
        for (int32_t e = 1; e <= n; ++e) {
          for (int d = LT_MAX_SPAN; d >= 1; --d) {
            *ss++ = local;
            const int32_t b = e - d;
            if (d > max_len || b < 0) continue;
            const int64_t g = c0 + b;
            bool any = false;
            for (int64_t i = L->slot_off[g]; i < L->slot_off[g + 1]; ++i) {
              if (L->e[i] != e) continue;                 // beam.py:33 (w.e == e)
              NodeView v;
              v.word = str_at(L->word, i);
              v.morph0 = str_at(L->morph0, i);
              v.tag0 = str_at(L->tag0, i);
              v.has_morph1 = !is_null(L->morph1, i);
              v.has_tag1 = !is_null(L->tag1, i);
              v.morph1 = v.has_morph1 ? str_at(L->morph1, i) : std::string_view();
              v.tag1 = v.has_tag1 ? str_at(L->tag1, i) : std::string_view();
              v.len = L->len[i];
              v.is_l = L->is_l[i];
              add_node(base + (size_t)local, v, i);
              ++local;
              any = true;
            }
            if (!any) {                                   // beam.py:36-38: Unknown chars[b:e]
              unk.clear();
              for (int32_t x = b; x < e; ++x) utf8_append(unk, L->chars[c0 + x]);
              NodeView u{unk, unk, kUnk, {}, {}, false, false, (int64_t)d, 0};
              add_node(base + (size_t)local, u, -2 - (8 * (int64_t)b + d - 1));
              ++local;
            }
          }
        }
        *ss = local;
      }
    };
    const int64_t work = (int64_t)N;
    int nt = std::min(lt::host_threads(), 16);
    if (work < 200000) nt = 1;
    if (const char* env = std::getenv("LT_PACK_THREADS")) nt = std::max(1, std::atoi(env));
    nt = std::min<int>(nt, std::max<int32_t>(S, 1));
    if (nt <= 1) {
      fill(0, S);
    } else {
      std::vector<std::thread> th;
      for (int t = 0; t < nt; ++t) {
        const int32_t lo = (int32_t)((int64_t)S * t / nt), hi = (int32_t)((int64_t)S * (t + 1) / nt);
        th.emplace_back(fill, lo, hi);
      }
      for (auto& x : th) x.join();
    }
  } catch (...) {
    return set_error(LT_ENOMEM, "lt_packer_pack: out of memory");
  }

  lt_batch_desc& b = out->batch;
  std::memset(&b, 0, sizeof b);
  b.n_sent = S;
  b.max_len = max_len;
  b.n_post = n_post;
  b.has_trigram = 0;            // set by the caller (the trigram is not the packer's concern)
  b.n_nodes = (int64_t)p->node_word.size();
  b.n_span = (int64_t)p->span_start.size();
  b.sent_n = p->sent_n.data();
  b.sent_node_off = p->sent_node_off.data();
  b.sent_span_off = p->sent_span_off.data();
  b.span_start = p->span_start.data();
  b.node_word = p->node_word.data();
  b.node_morph0 = p->node_morph0.data();
  b.node_tag = p->node_tag.data();
  b.node_mask = p->node_mask.data();
  b.node_pre = p->node_pre.data();
  b.node_f4 = p->node_f4.data();
  b.node_f5 = p->node_f5.data();
  b.node_f6 = p->node_f6.data();
  b.node_post = n_post ? p->node_post.data() : nullptr;
  out->node_src = p->node_src.data();
  return LT_OK;
}
