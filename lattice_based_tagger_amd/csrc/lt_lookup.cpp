// lt_lookup.cpp -- native lattice builder (include/lattice_lookup.h).
//
// Restates, over UTF-32 code points and for whole corpora at once, the
// reference's lattice construction that Tagger.tag runs before beam_search
// (lattice_tagger/tagger/tagger.py:72-74):
//   sentence_lookup_as_begin_index   lookup.py:52-62, 358-369
//   morpheme_lookup                  lookup.py:212-279
//   lr_lookup                        lookup.py:171-210
//   MorphemeDictionary.lookup/check  dictionary.py:230-242, 304-315
//   analyze_morphology               lemmatizer.py:5-51
//   get_lemma_candidates             lemmatizer.py:53-112
// Node order is the reference's: lookup order within an eojeol, eojeols in
// sentence order, then a stable grouping by begin position.
//
// One string table keys everything the lookup asks a dictionary about: a
// string's tag bits (get_tags / check), its verb / adjective / eomi
// membership (analyze_morphology) and its rule pairs (rules.get), so each
// probe of a substring or candidate is one hash lookup.
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <memory>
#include <new>
#include <string>
#include <thread>
#include <string_view>
#include <vector>

#include "../../include/lattice_lookup.h"
#include "lt_error.h"
#include "lt_host.h"
#include "lt_lattice_store.h"

using lt::Arr;

namespace {

// ------------------------------------------------------- CPython str hash --
// CPython 3.10 hashes a str as SipHash-2-4 (Python/pyhash.c) of its canonical
// storage: 1, 2 or 4 bytes per code point by the string's largest code point
// (Objects/unicodeobject.c unicode_hash -> _Py_HashBytes); -1 maps to -2.
inline uint64_t rotl(uint64_t x, int b) { return (x << b) | (x >> (64 - b)); }

inline void half_round(uint64_t& a, uint64_t& b, uint64_t& c, uint64_t& d, int s, int t) {
  a += b;
  c += d;
  b = rotl(b, s) ^ a;
  d = rotl(d, t) ^ c;
  a = rotl(a, 32);
}

inline void double_round(uint64_t& v0, uint64_t& v1, uint64_t& v2, uint64_t& v3) {
  half_round(v0, v1, v2, v3, 13, 16);
  half_round(v2, v1, v0, v3, 17, 21);
  half_round(v0, v1, v2, v3, 13, 16);
  half_round(v2, v1, v0, v3, 17, 21);
}

uint64_t siphash24(uint64_t k0, uint64_t k1, const uint8_t* in, size_t sz) {
  uint64_t b = (uint64_t)sz << 56;
  uint64_t v0 = k0 ^ 0x736f6d6570736575ULL;
  uint64_t v1 = k1 ^ 0x646f72616e646f6dULL;
  uint64_t v2 = k0 ^ 0x6c7967656e657261ULL;
  uint64_t v3 = k1 ^ 0x7465646279746573ULL;
  while (sz >= 8) {
    uint64_t mi;
    memcpy(&mi, in, 8);                     // little-endian host
    in += 8;
    sz -= 8;
    v3 ^= mi;
    double_round(v0, v1, v2, v3);
    v0 ^= mi;
  }
  uint64_t t = 0;
  memcpy(&t, in, sz);
  b |= t;
  v3 ^= b;
  double_round(v0, v1, v2, v3);
  v0 ^= b;
  v2 ^= 0xff;
  double_round(v0, v1, v2, v3);
  double_round(v0, v1, v2, v3);
  return (v0 ^ v1) ^ (v2 ^ v3);
}

int64_t py_str_hash(const uint32_t* s, size_t n, uint64_t k0, uint64_t k1) {
  if (n == 0) return 0;
  uint32_t mx = 0;
  for (size_t i = 0; i < n; ++i) mx = std::max(mx, s[i]);
  const size_t kind = mx < 0x100 ? 1 : (mx < 0x10000 ? 2 : 4);
  uint8_t stack[64];
  std::vector<uint8_t> heap;
  uint8_t* buf = stack;
  if (n * kind > sizeof stack) {
    heap.resize(n * kind);
    buf = heap.data();
  }
  for (size_t i = 0; i < n; ++i) {
    const uint32_t c = s[i];
    if (kind == 1) buf[i] = (uint8_t)c;
    else if (kind == 2) { buf[2 * i] = (uint8_t)c; buf[2 * i + 1] = (uint8_t)(c >> 8); }
    else memcpy(buf + 4 * i, &c, 4);
  }
  int64_t x = (int64_t)siphash24(k0, k1, buf, n * kind);
  return x == -1 ? -2 : x;
}

// Iteration order of the set {a, b} that BUILD_SET makes (a added first) in
// a fresh 8-slot table (Objects/setobject.c set_add_entry, mask 7: no linear
// probes, perturbation on collision).  True when b comes first.
bool set2_second_first(int64_t ha, int64_t hb) {
  const size_t mask = 7;
  const size_t ia = (size_t)ha & mask;
  size_t i = (size_t)hb & mask, perturb = (size_t)hb;
  while (i == ia) {
    perturb >>= 5;
    i = (i * 5 + 1 + perturb) & mask;
  }
  return i < ia;
}

// ------------------------------------------------------------ utf-8 / 32 --
bool utf8_decode(const char* s, size_t n, std::vector<uint32_t>& out) {
  out.clear();
  const uint8_t* p = (const uint8_t*)s;
  size_t i = 0;
  while (i < n) {
    uint32_t c = p[i];
    int extra;
    if (c < 0x80) { extra = 0; }
    else if ((c >> 5) == 6) { extra = 1; c &= 0x1F; }
    else if ((c >> 4) == 14) { extra = 2; c &= 0x0F; }
    else if ((c >> 3) == 30) { extra = 3; c &= 0x07; }
    else return false;
    if (extra && i + extra >= n) return false;
    for (int k = 1; k <= extra; ++k) {
      if ((p[i + k] & 0xC0) != 0x80) return false;
      c = (c << 6) | (p[i + k] & 0x3F);
    }
    out.push_back(c);
    i += 1 + (size_t)extra;
  }
  return true;
}

void utf8_append(std::string& out, const uint32_t* s, size_t n) {
  for (size_t i = 0; i < n; ++i) {
    const uint32_t cp = s[i];
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
}

// ------------------------------------------------------------ string table --
constexpr uint8_t F_VERB = 1, F_ADJ = 2, F_EOMI = 4;

struct Info {
  uint64_t tags = 0;         // bit t: the string is a morph of dictionary tag t
  uint8_t flags = 0;         // F_VERB | F_ADJ | F_EOMI
  int32_t rule_lo = 0, rule_n = 0;
};

struct Span {
  uint32_t off = 0, len = 0;
};

// Sequence hash in three parts, so that a common prefix is hashed once: the
// state after a prefix (hs_feed from HS_INIT) continues with any suffix, and
// the length is folded in at the end (the lemmatizer hashes the stem w[:i] +
// each rule's stem, and each rule's eomi + the rest of the word).
constexpr uint64_t HS_INIT = 0x9E3779B97F4A7C15ull;
inline uint64_t hs_feed(uint64_t h, const uint32_t* s, uint32_t n) {
  for (uint32_t i = 0; i < n; ++i) {
    h ^= s[i];
    h *= 0xff51afd7ed558ccdull;
    h ^= h >> 29;
  }
  return h;
}
inline uint64_t hs_final(uint64_t h, uint32_t n) {
  h ^= (uint64_t)n * 0xC2B2AE3D27D4EB4Full;
  h *= 0xff51afd7ed558ccdull;
  h ^= h >> 31;
  return h ^ (h >> 32);
}
inline uint64_t seq_hash(const uint32_t* s, uint32_t n) { return hs_final(hs_feed(HS_INIT, s, n), n); }

class Table {
 public:
  std::vector<uint32_t> pool;                 // key code points (+ rule strings)
  std::vector<Span> keys;
  std::vector<Info> infos;

  void reserve(size_t n) {
    size_t cap = 16;
    while (cap < 2 * n + 16) cap <<= 1;
    slots_.assign(cap, 0);
    mask_ = cap - 1;
  }

  Info& get_or_add(const uint32_t* s, uint32_t n) {
    const uint64_t h = seq_hash(s, n);
    size_t i = (size_t)h & mask_;
    for (uint64_t v; (v = slots_[i]) != 0; i = (i + 1) & mask_)
      if (tag_of(v) == tag(h) && same(idx_of(v), s, n)) return infos[idx_of(v)];
    if (2 * (keys.size() + 1) > slots_.size()) {      // grow and re-place
      grow();
      return get_or_add(s, n);
    }
    slots_[i] = entry(h, keys.size());
    keys.push_back(Span{(uint32_t)pool.size(), n});
    pool.insert(pool.end(), s, s + n);
    infos.emplace_back();
    return infos.back();
  }

  // Most lookups miss (substrings that are no morpheme): a slot carries the
  // key's hash tag beside its index, so a probe compares the tag in the slot
  // array and touches the key's span and code points only on a tag match.
  const Info* find(const uint32_t* s, uint32_t n) const {
    const uint64_t h = seq_hash(s, n);
    size_t i = (size_t)h & mask_;
    for (uint64_t v; (v = slots_[i]) != 0; i = (i + 1) & mask_)
      if (tag_of(v) == tag(h) && same(idx_of(v), s, n)) return &infos[idx_of(v)];
    return nullptr;
  }
  // find() of the concatenation a + b; ha = hs_feed(HS_INIT, a, na)
  const Info* find2(uint64_t ha, const uint32_t* a, uint32_t na, const uint32_t* b, uint32_t nb) const {
    const uint64_t h = hs_final(hs_feed(ha, b, nb), na + nb);
    size_t i = (size_t)h & mask_;
    for (uint64_t v; (v = slots_[i]) != 0; i = (i + 1) & mask_) {
      if (tag_of(v) != tag(h)) continue;
      const Span& k = keys[idx_of(v)];
      const uint32_t* q = pool.data() + k.off;
      if (k.len == na + nb && std::equal(a, a + na, q) && std::equal(b, b + nb, q + na))
        return &infos[idx_of(v)];
    }
    return nullptr;
  }

 private:
  // slot: hash tag (high 32 bits of the key's hash) << 32 | index + 1; 0 = empty
  std::vector<uint64_t> slots_;
  size_t mask_ = 0;

  static uint32_t tag(uint64_t h) { return (uint32_t)(h >> 32); }
  static uint32_t tag_of(uint64_t v) { return (uint32_t)(v >> 32); }
  static size_t idx_of(uint64_t v) { return (size_t)(uint32_t)v - 1; }
  static uint64_t entry(uint64_t h, size_t idx) { return ((uint64_t)tag(h) << 32) | (uint64_t)(idx + 1); }
  bool same(size_t x, const uint32_t* s, uint32_t n) const {
    const Span& k = keys[x];
    return k.len == n && std::equal(s, s + n, pool.data() + k.off);
  }

  void grow() {
    std::vector<uint64_t> old;
    old.swap(slots_);
    slots_.assign(old.size() * 2, 0);
    mask_ = slots_.size() - 1;
    for (size_t x = 0; x < keys.size(); ++x) {
      const Span& k = keys[x];
      const uint64_t h = seq_hash(pool.data() + k.off, k.len);
      size_t i = (size_t)h & mask_;
      while (slots_[i] != 0) i = (i + 1) & mask_;
      slots_[i] = entry(h, x);
    }
  }
};

struct RulePair {
  Span stem, eomi;            // in Table::pool
  uint64_t eomi_hs = 0;       // hs_feed(HS_INIT, eomi): the prefix state of eomi + rest
};

struct Standalone {
  int32_t dict_tag;           // index into the dictionary's tags, -1: not a dictionary tag
  int32_t name;               // index into names
  bool is_noun;
};

// One lattice node while building (strings by reference).
struct WordRec {
  uint32_t w_off, w_len;      // surface: text[w_off .. +w_len)
  int32_t m0_off, m0_len;     // morph0 in the thread pool; m0_off < 0: the surface
  int32_t m1_off, m1_len;     // morph1 in the thread pool; m1_off < 0: None
  int32_t tag0, tag1;         // name indices; tag1 < 0: None
  int32_t len, b, e;
  bool is_l;
};

}  // namespace

struct lt_lexicon {
  Table table;
  std::vector<RulePair> rules;
  std::vector<std::string> names;     // UTF-8 tag names: dictionary tags, then literals
  int32_t n_dict_tags = 0;
  int32_t dict_noun = -1, dict_josa = -1;       // dictionary tag indices of 'Noun' / 'Josa'
  int32_t name_noun = 0, name_josa = 0, name_adj = 0, name_verb = 0, name_eomi = 0;
  std::vector<Standalone> standalones;
  int32_t max_len = 0;
  bool prefer_exact = true;
  uint64_t k0 = 0, k1 = 0;
};


namespace {

// ------------------------------------------------------------ the lookup --
struct Worker {
  const lt_lexicon& lx;
  const uint32_t* text;
  std::vector<uint32_t> pool;         // lemma strings of this worker
  std::vector<uint32_t> sbuf, ebuf;   // candidate stem / eomi
  std::vector<WordRec> tl, tr;        // lr_lookup's lset / rset

  Worker(const lt_lexicon& l, const uint32_t* t) : lx(l), text(t) {}

  const Info* find(const uint32_t* s, uint32_t n) const { return lx.table.find(s, n); }

  // Lookups of substrings of the current eojeol, memoised: the lemmatizer
  // and the lr / standalone scans probe the same (start, length) pairs many
  // times over (every substring's lemmatisation re-probes its 1-3 syllable
  // windows and its suffixes).  Eojeols longer than MEMO_MAX probe directly.
  static constexpr uint32_t MEMO_MAX = 48;
  uint32_t m_off = 0, m_n = 0;
  std::vector<const Info*> memo;
  std::vector<uint8_t> memo_ok;
  void begin_eojeol(uint32_t off, uint32_t n) {
    m_off = off;
    m_n = n <= MEMO_MAX ? n : 0;
    const size_t sz = (size_t)(m_n + 1) * (m_n + 1);
    if (memo.size() < sz) memo.resize(sz);
    memo_ok.assign(sz, 0);
  }
  // find(text + s, len) for a substring of the text
  const Info* find_t(uint32_t s, uint32_t len) {
    if (s >= m_off && len <= m_n && s - m_off <= m_n - len) {
      const size_t k = (size_t)(s - m_off) * (m_n + 1) + len;
      if (!memo_ok[k]) {
        memo[k] = find(text + s, len);
        memo_ok[k] = 1;
      }
      return memo[k];
    }
    return find(text + s, len);
  }

  static bool has(const Info* in, int32_t tag) { return tag >= 0 && in && ((in->tags >> tag) & 1u); }

  int32_t keep(const std::vector<uint32_t>& s) {
    const int32_t off = (int32_t)pool.size();
    pool.insert(pool.end(), s.begin(), s.end());
    return off;
  }

  // analyze_morphology (lemmatizer.py:43-51) of the candidate in sbuf/ebuf
  void consider(uint32_t w_off, uint32_t m, int32_t len, int32_t b, int32_t e, bool is_l,
                std::vector<WordRec>& out) {
    const Info* ei = find(ebuf.data(), (uint32_t)ebuf.size());
    if (!ei || !(ei->flags & F_EOMI)) return;
    const Info* si = find(sbuf.data(), (uint32_t)sbuf.size());
    if (!si || !(si->flags & (F_ADJ | F_VERB))) return;
    const int32_t so = keep(sbuf), eo = keep(ebuf);
    const int32_t sl = (int32_t)sbuf.size(), el = (int32_t)ebuf.size();
    if (si->flags & F_ADJ)
      out.push_back(WordRec{w_off, m, so, sl, eo, el, lx.name_adj, lx.name_eomi, len, b, e, is_l});
    if (si->flags & F_VERB)
      out.push_back(WordRec{w_off, m, so, sl, eo, el, lx.name_verb, lx.name_eomi, len, b, e, is_l});
  }

  // consider() of stem s1 + s2, eomi e1 + e2: the two lookups run on the
  // pieces (s1h, e1h: the hash prefix states of s1, e1); the candidate is
  // copied only when both succeed
  void consider_parts(uint64_t s1h, const uint32_t* s1, uint32_t n1, const uint32_t* s2, uint32_t n2,
                      uint64_t e1h, const uint32_t* e1, uint32_t m1, const uint32_t* e2, uint32_t m2,
                      uint32_t w_off, uint32_t m, int32_t len, int32_t b, int32_t e, bool is_l,
                      std::vector<WordRec>& out) {
    const Info* ei = lx.table.find2(e1h, e1, m1, e2, m2);
    if (!ei || !(ei->flags & F_EOMI)) return;
    const Info* si = lx.table.find2(s1h, s1, n1, s2, n2);
    if (!si || !(si->flags & (F_ADJ | F_VERB))) return;
    set_cand(s1, n1, s2, n2, e1, m1, e2, m2);
    consider(w_off, m, len, b, e, is_l, out);
  }

  // consider() of the split text[s .. s + sl) + text[s + sl .. s + sl + el)
  void consider_text(uint32_t s, uint32_t sl, uint32_t el, uint32_t w_off, uint32_t m, int32_t len,
                     int32_t b, int32_t e, bool is_l, std::vector<WordRec>& out) {
    const Info* ei = find_t(s + sl, el);
    if (!ei || !(ei->flags & F_EOMI)) return;
    const Info* si = find_t(s, sl);
    if (!si || !(si->flags & (F_ADJ | F_VERB))) return;
    set_cand(text + s, sl, nullptr, 0, text + s + sl, el, nullptr, 0);
    consider(w_off, m, len, b, e, is_l, out);
  }

  void set_cand(const uint32_t* s1, size_t n1, const uint32_t* s2, size_t n2,
                const uint32_t* e1, size_t m1, const uint32_t* e2, size_t m2) {
    sbuf.assign(s1, s1 + n1);
    sbuf.insert(sbuf.end(), s2, s2 + n2);
    ebuf.assign(e1, e1 + m1);
    ebuf.insert(ebuf.end(), e2, e2 + m2);
  }

  // MorphemeDictionary.lemmatize(word) words (dictionary.py:304-309) for the
  // surface text[w_off .. +m): get_lemma_candidates (lemmatizer.py:90-112)
  // filtered by analyze_morphology, in candidate order.
  void lemmatize(uint32_t w_off, uint32_t m, int32_t len, int32_t b, int32_t e, bool is_l,
                 std::vector<WordRec>& out) {
    const uint32_t* w = text + w_off;
    const std::vector<RulePair>& R = lx.rules;
    const uint32_t* P = lx.table.pool.data();
    uint64_t wh = HS_INIT;                       // hs_feed(HS_INIT, w, i): the stem prefix w[:i]
    for (uint32_t i = 0; i < m; wh = hs_feed(wh, w + i, 1), ++i) {
      // (l, r) = (word[:i+1], word[i+1:]), while i < max_i
      if (i + 1 < m) consider_text(w_off, i + 1, m - i - 1, w_off, m, len, b, e, is_l, out);
      // 1 syllable conjugation: the pairs of rules[c], |rules[c]| times over
      // (the nested loop of lemmatizer.py:100-101) -- every repetition emits
      // the same words, so one pass is scored and its words repeated
      if (const Info* ci = find_t(w_off + i, 1); ci && ci->rule_n > 0) {
        const size_t first = out.size();
        for (int32_t q = ci->rule_lo; q < ci->rule_lo + ci->rule_n; ++q) {
          const RulePair& rp = R[(size_t)q];
          consider_parts(wh, w, i, P + rp.stem.off, rp.stem.len, rp.eomi_hs, P + rp.eomi.off, rp.eomi.len,
                         w + i + 1, m - i - 1, w_off, m, len, b, e, is_l, out);
        }
        const size_t pass = out.size() - first;
        if (pass) out.reserve(out.size() + pass * (size_t)(ci->rule_n - 1));
        for (int32_t rep = 1; rep < ci->rule_n && pass; ++rep)
          for (size_t x = 0; x < pass; ++x) out.push_back(out[first + x]);
      }
      // 2 or 3 syllables conjugation: for conj in {word[i:i+2], word[i:i+3]}
      // (set iteration order, lemmatizer.py:107); eomi + r[1:].  The order
      // only matters when both surfaces have rules.
      const uint32_t n2 = std::min<uint32_t>(2, m - i), n3 = std::min<uint32_t>(3, m - i);
      const uint32_t* rest = w + std::min<uint32_t>(m, i + 2);
      const uint32_t nrest = m - std::min<uint32_t>(m, i + 2);
      const Info* c2 = find_t(w_off + i, n2);
      const Info* c3 = n3 != n2 ? find_t(w_off + i, n3) : nullptr;
      const Info* conj[2] = {c2 && c2->rule_n ? c2 : nullptr, c3 && c3->rule_n ? c3 : nullptr};
      if (conj[0] && conj[1] &&
          set2_second_first(py_str_hash(w + i, n2, lx.k0, lx.k1), py_str_hash(w + i, n3, lx.k0, lx.k1)))
        std::swap(conj[0], conj[1]);
      for (const Info* ci : conj) {
        if (!ci) continue;
        for (int32_t q = ci->rule_lo; q < ci->rule_lo + ci->rule_n; ++q) {
          const RulePair& rp = R[(size_t)q];
          consider_parts(wh, w, i, P + rp.stem.off, rp.stem.len, rp.eomi_hs, P + rp.eomi.off, rp.eomi.len, rest,
                         nrest, w_off, m, len, b, e, is_l, out);
        }
      }
    }
  }

  // MorphemeDictionary.lookup(word, b, is_l) (dictionary.py:304-315)
  void dict_lookup(uint32_t w_off, uint32_t n, int32_t b, bool is_l, std::vector<WordRec>& out) {
    if (const Info* in = find_t(w_off, n)) {
      for (int32_t t = 0; t < lx.n_dict_tags; ++t)
        if ((in->tags >> t) & 1u)
          out.push_back(WordRec{w_off, n, -1, 0, -1, 0, t, -1, (int32_t)n, b, b + (int32_t)n, is_l});
    }
    lemmatize(w_off, n, (int32_t)n, b, b + (int32_t)n, is_l, out);
  }

  void noun_josa(uint32_t e_off, uint32_t n, uint32_t i, int32_t offset, int32_t len, std::vector<WordRec>& out) {
    out.push_back(WordRec{e_off, i, -1, 0, -1, 0, lx.name_noun, -1, len, offset, offset + (int32_t)i, true});
    out.push_back(WordRec{e_off + i, n - i, -1, 0, -1, 0, lx.name_josa, -1, len, offset + (int32_t)i,
                          offset + (int32_t)n, false});
  }

  bool is_noun_josa(uint32_t e_off, uint32_t n, uint32_t i) {
    if (lx.dict_noun < 0 || lx.dict_josa < 0) return false;
    return has(find_t(e_off, i), lx.dict_noun) && has(find_t(e_off + i, n - i), lx.dict_josa);
  }

  // lr_lookup (lookup.py:171-210)
  void lr_lookup(uint32_t e_off, uint32_t n, int32_t offset, bool prefer, std::vector<WordRec>& out) {
    const size_t start = out.size();
    dict_lookup(e_off, n, offset, true, out);
    if (prefer && out.size() > start) return;
    for (uint32_t i = 1; i < n; ++i) {
      if (is_noun_josa(e_off, n, i)) {
        noun_josa(e_off, n, i, offset, (int32_t)n, out);
        continue;
      }
      tl.clear();
      dict_lookup(e_off, i, offset, true, tl);
      if (tl.empty()) continue;
      tr.clear();
      dict_lookup(e_off + i, n - i, offset + (int32_t)i, false, tr);
      if (tr.empty()) continue;
      out.insert(out.end(), tl.begin(), tl.end());
      out.insert(out.end(), tr.begin(), tr.end());
    }
  }

  // morpheme_lookup (lookup.py:212-279)
  void morpheme_lookup(uint32_t e_off, uint32_t n, int32_t offset, std::vector<WordRec>& out) {
    begin_eojeol(e_off, n);
    const size_t start = out.size();
    lr_lookup(e_off, n, offset, false, out);
    if (lx.prefer_exact && out.size() > start) return;
    const uint32_t max_len = lx.max_len <= 0 ? n : (uint32_t)lx.max_len;
    std::vector<uint8_t> noun_end(n + 1, 0);
    for (uint32_t i = 1; i < n; ++i)
      if (is_noun_josa(e_off, n, i)) noun_josa(e_off, n, i, offset, (int32_t)i, out);
    for (uint32_t b = 1; b < n; ++b) {
      const uint32_t e_hi = std::min(b + max_len, n);
      for (uint32_t e = b + 1; e <= e_hi; ++e) {
        const uint32_t so = e_off + b, sl = e - b;
        const Info* in = find_t(so, sl);
        const int32_t B = offset + (int32_t)b, E = offset + (int32_t)e;
        for (const Standalone& st : lx.standalones)
          if (has(in, st.dict_tag)) {
            out.push_back(WordRec{so, sl, -1, 0, -1, 0, st.name, -1, (int32_t)sl, B, E, false});
            if (st.is_noun) noun_end[e] = 1;
          }
        if (noun_end[b] && has(in, lx.dict_josa))
          out.push_back(WordRec{so, sl, -1, 0, -1, 0, lx.name_josa, -1, (int32_t)sl, B, E, false});
        lemmatize(so, sl, (int32_t)sl, B, E, false, out);
      }
    }
  }
};

// Compact columns of a range of sentences (one worker's share); lemma morphs
// in the chunk's pool.
struct Chunk {
  std::vector<uint32_t> w_off, w_len, m0_off, m0_len, m1_off, m1_len;
  std::vector<int16_t> tag0, tag1;
  std::vector<int32_t> len, e, b;
  std::vector<uint8_t> is_l;
  std::vector<uint32_t> pool;
  std::vector<int64_t> slot_n;      // words per begin slot, sentence-major
  std::vector<int64_t> sent_n;      // words per sentence
  int64_t field_cps[5] = {0, 0, 0, 0, 0};
  std::string err;
};

void run_chunk(const lt_lexicon& lx, const lt_text_desc& td, int32_t s0, int32_t s1, Chunk& ck) {
  Worker wk(lx, td.text);
  std::vector<WordRec> words, grouped;
  std::vector<int64_t> cnt;
  size_t max_name = 0;
  for (const std::string& nm : lx.names) max_name = std::max(max_name, nm.size());
  for (int32_t s = s0; s < s1; ++s) {
    const int64_t n = td.char_off[s + 1] - td.char_off[s];
    words.clear();
    int32_t offset = 0;
    for (int64_t j = td.sent_eoj[s]; j < td.sent_eoj[s + 1]; ++j) {
      const uint32_t eo = (uint32_t)td.eoj_off[j], el = (uint32_t)(td.eoj_off[j + 1] - td.eoj_off[j]);
      wk.morpheme_lookup(eo, el, offset, words);
      offset += (int32_t)el;
    }
    // bindex[word.b].append(word) (lookup.py:365-367): stable by begin
    cnt.assign((size_t)n + 1, 0);
    for (const WordRec& w : words) {
      if (w.b < 0 || w.b >= n) {
        ck.err = "word begins outside its sentence (eojeols longer than the sentence's characters)";
        return;
      }
      ++cnt[(size_t)w.b + 1];
    }
    for (int64_t x = 0; x < n; ++x) ck.slot_n.push_back(cnt[(size_t)x + 1]);
    for (int64_t x = 0; x < n; ++x) cnt[(size_t)x + 1] += cnt[(size_t)x];
    grouped.resize(words.size());
    for (const WordRec& w : words) grouped[(size_t)cnt[(size_t)w.b]++] = w;
    ck.sent_n.push_back((int64_t)words.size());
    for (const WordRec& w : grouped) {
      ck.w_off.push_back(w.w_off);
      ck.w_len.push_back(w.w_len);
      const bool own0 = w.m0_off >= 0, own1 = w.m1_off >= 0;
      ck.m0_off.push_back(own0 ? (uint32_t)w.m0_off : LT_NOREF);
      ck.m0_len.push_back(own0 ? (uint32_t)w.m0_len : 0u);
      ck.m1_off.push_back(own1 ? (uint32_t)w.m1_off : LT_NOREF);
      ck.m1_len.push_back(own1 ? (uint32_t)w.m1_len : 0u);
      ck.tag0.push_back((int16_t)w.tag0);
      ck.tag1.push_back((int16_t)(w.tag1 >= 0 ? w.tag1 : -1));
      ck.len.push_back(w.len);
      ck.e.push_back(w.e);
      ck.b.push_back(w.b);
      ck.is_l.push_back(w.is_l ? 1 : 0);
      ck.field_cps[0] += w.w_len;
      ck.field_cps[1] += own0 ? w.m0_len : w.w_len;
      ck.field_cps[2] += own1 ? w.m1_len : 0;
    }
    ck.field_cps[3] += (int64_t)(grouped.size() * max_name);
    ck.field_cps[4] += (int64_t)(grouped.size() * max_name);
  }
  ck.pool.swap(wk.pool);
}

// Where chunk c's pieces go in the merged arrays.
struct Base {
  int64_t words = 0, slots = 0, sents = 0, pool = 0;
};

// Copy chunk c into the merged arrays at base; frees the chunk.
void merge_chunk(Chunk& c, const Base& at, lt_lattices& L) {
  const int64_t W = (int64_t)c.len.size();
  auto cols = [&](auto& dst, const auto& src) {
    if (W) memcpy(dst.data() + at.words, src.data(), (size_t)W * sizeof(src[0]));
  };
  cols(L.w_off, c.w_off);
  cols(L.w_len, c.w_len);
  cols(L.m0_len, c.m0_len);
  cols(L.m1_len, c.m1_len);
  cols(L.tag0, c.tag0);
  cols(L.tag1, c.tag1);
  cols(L.len, c.len);
  cols(L.e, c.e);
  cols(L.b, c.b);
  cols(L.is_l, c.is_l);
  const uint32_t pb = (uint32_t)at.pool;                // rebase the pool references
  for (int64_t i = 0; i < W; ++i) {
    const uint32_t o0 = c.m0_off[(size_t)i], o1 = c.m1_off[(size_t)i];
    L.m0_off[at.words + i] = o0 == LT_NOREF ? LT_NOREF : o0 + pb;
    L.m1_off[at.words + i] = o1 == LT_NOREF ? LT_NOREF : o1 + pb;
  }
  if (!c.pool.empty()) memcpy(L.pool.data() + at.pool, c.pool.data(), c.pool.size() * 4);
  int64_t run = at.words;
  for (size_t x = 0; x < c.slot_n.size(); ++x) L.slot_off.data()[at.slots + (int64_t)x + 1] = (run += c.slot_n[x]);
  run = at.words;
  for (size_t x = 0; x < c.sent_n.size(); ++x) L.sent_words.data()[at.sents + (int64_t)x + 1] = (run += c.sent_n[x]);
  c = Chunk();
}

// UTF-8 of a node's string field (0 word, 1 morph0, 2 morph1, 3 tag0,
// 4 tag1) appended to out; false for None.
bool field_utf8(const lt_lattices& L, int field, int64_t i, std::string& out) {
  switch (field) {
    case 0: utf8_append(out, L.text.data() + L.w_off[i], L.w_len[i]); return true;
    case 1: {
      uint32_t n;
      const uint32_t* c = L.m0_cps(i, n);
      utf8_append(out, c, n);
      return true;
    }
    case 2:
      if (L.m1_off[i] == LT_NOREF) return false;
      utf8_append(out, L.pool.data() + L.m1_off[i], L.m1_len[i]);
      return true;
    case 3: out += L.names[(size_t)L.tag0[i]]; return true;
    default:
      if (L.tag1[i] < 0) return false;
      out += L.names[(size_t)L.tag1[i]];
      return true;
  }
}

// lt_lattices_view's UTF-8 columns (threads over node ranges: each range's
// blobs, then offsets rebased)
bool build_utf8(const lt_lattices& L) {
  std::unique_ptr<lt_lattices::Utf8> u(new (std::nothrow) lt_lattices::Utf8);
  if (!u) return false;
  const int64_t W = L.n_words;
  Arr<char>* blobs[5] = {&u->wb, &u->mb, &u->m1b, &u->tb, &u->t1b};
  Arr<int64_t>* offs[5] = {&u->woff, &u->moff, &u->m1off, &u->toff, &u->t1off};
  bool ok = true;
  for (Arr<int64_t>* a : offs) ok = ok && a->alloc(W + 1);
  ok = ok && u->m1null.alloc(W) && u->t1null.alloc(W) && u->len.alloc(W) && u->e.alloc(W) && u->b.alloc(W) &&
       u->is_l.alloc(W);
  if (!ok) return false;
  const int nt = (int)std::max<int64_t>(1, std::min<int64_t>(lt::host_threads(), W / 4096 + 1));
  std::vector<std::string> part((size_t)nt * 5);
  std::vector<std::thread> th;
  auto work = [&](int t) {
    const int64_t lo = W * t / nt, hi = W * (t + 1) / nt;
    for (int f = 0; f < 5; ++f) {
      std::string& o = part[(size_t)t * 5 + (size_t)f];
      int64_t* off = offs[f]->data();
      for (int64_t i = lo; i < hi; ++i) {
        const bool some = field_utf8(L, f, i, o);
        off[i + 1] = (int64_t)o.size();                  // part-relative, rebased below
        if (f == 2) u->m1null[i] = !some;
        if (f == 4) u->t1null[i] = !some;
      }
    }
    for (int64_t i = lo; i < hi; ++i) {
      u->len[i] = L.len[i];
      u->e[i] = L.e[i];
      u->b[i] = L.b[i];
      u->is_l[i] = L.is_l[i];
    }
  };
  try {
    for (int t = 1; t < nt; ++t) th.emplace_back(work, t);
    work(0);
    for (std::thread& x : th) x.join();
  } catch (...) {
    for (std::thread& x : th)
      if (x.joinable()) x.join();
    return false;
  }
  for (int f = 0; f < 5; ++f) {
    int64_t total = 0;
    for (int t = 0; t < nt; ++t) total += (int64_t)part[(size_t)t * 5 + (size_t)f].size();
    if (!blobs[f]->alloc(total)) return false;
    int64_t* off = offs[f]->data();
    off[0] = 0;
    int64_t base = 0;
    for (int t = 0; t < nt; ++t) {
      const std::string& o = part[(size_t)t * 5 + (size_t)f];
      const int64_t lo = W * t / nt, hi = W * (t + 1) / nt;
      if (!o.empty()) memcpy(blobs[f]->data() + base, o.data(), o.size());
      for (int64_t i = lo; i < hi; ++i) off[i + 1] += base;
      base += (int64_t)o.size();
    }
  }
  L.utf8 = std::move(u);
  return true;
}

}  // namespace

extern "C" {

int64_t lt_py_str_hash(const uint32_t* cps, int64_t n, uint64_t k0, uint64_t k1) {
  if (n < 0 || (n > 0 && !cps)) return 0;
  return py_str_hash(cps, (size_t)n, k0, k1);
}

int lt_py_set2_second_first(int64_t hash_a, int64_t hash_b) {
  return set2_second_first(hash_a, hash_b) ? 1 : 0;
}

lt_status lt_lexicon_create(const lt_lexicon_desc* d, lt_lexicon** out) {
  if (!d || !out) return lt::set_error(LT_EINVAL, "lt_lexicon_create: NULL argument");
  *out = nullptr;
  const int64_t T = d->tag.n;
  if (T < 0 || T > LT_LEXICON_MAX_TAGS)
    return lt::set_error(LT_EUNSUPPORTED, "lt_lexicon_create: %lld tags (at most %d)", (long long)T,
                         LT_LEXICON_MAX_TAGS);
  if (T > 0 && !d->morph_off) return lt::set_error(LT_EINVAL, "lt_lexicon_create: morph_off is NULL");
  if (d->rule_surface.n > 0 && !d->rule_off) return lt::set_error(LT_EINVAL, "lt_lexicon_create: rule_off is NULL");
  std::unique_ptr<lt_lexicon> lx(new (std::nothrow) lt_lexicon);
  if (!lx) return lt::set_error(LT_ENOMEM, "lt_lexicon_create: out of host memory");
  auto str = [](const lt_strings& t, int64_t i) {
    return std::string(t.data + t.off[i], (size_t)(t.off[i + 1] - t.off[i]));
  };
  std::vector<uint32_t> cp;
  auto decode = [&](const lt_strings& t, int64_t i) {
    return utf8_decode(t.data + t.off[i], (size_t)(t.off[i + 1] - t.off[i]), cp);
  };
  Table& tab = lx->table;
  tab.reserve((size_t)(d->morph.n + d->verbs.n + d->adjectives.n + d->eomis.n + d->rule_surface.n));
  // tags and their morphs (get_tags order = the dictionary's tag order)
  auto name_index = [&](const std::string& s) {
    for (size_t i = 0; i < lx->names.size(); ++i)
      if (lx->names[i] == s) return (int32_t)i;
    lx->names.push_back(s);
    return (int32_t)lx->names.size() - 1;
  };
  for (int64_t t = 0; t < T; ++t) {
    const std::string name = str(d->tag, t);
    for (size_t i = 0; i < lx->names.size(); ++i)
      if (lx->names[i] == name) return lt::set_error(LT_EINVAL, "lt_lexicon_create: duplicate tag");
    lx->names.push_back(name);
  }
  lx->n_dict_tags = (int32_t)T;
  for (int64_t t = 0; t < T; ++t)
    for (int64_t i = d->morph_off[t]; i < d->morph_off[t + 1]; ++i) {
      if (i < 0 || i >= d->morph.n) return lt::set_error(LT_EINVAL, "lt_lexicon_create: morph_off out of range");
      if (!decode(d->morph, i)) return lt::set_error(LT_EINVAL, "lt_lexicon_create: bad UTF-8");
      tab.get_or_add(cp.data(), (uint32_t)cp.size()).tags |= (uint64_t)1 << t;
    }
  const std::pair<const lt_strings*, uint8_t> sets[] = {
      {&d->verbs, F_VERB}, {&d->adjectives, F_ADJ}, {&d->eomis, F_EOMI}};
  for (const auto& st : sets)
    for (int64_t i = 0; i < st.first->n; ++i) {
      if (!decode(*st.first, i)) return lt::set_error(LT_EINVAL, "lt_lexicon_create: bad UTF-8");
      tab.get_or_add(cp.data(), (uint32_t)cp.size()).flags |= st.second;
    }
  // rules (surface -> pairs); the pair strings live in the table's pool
  for (int64_t r = 0; r < d->rule_surface.n; ++r) {
    if (d->rule_off[r] > d->rule_off[r + 1] || d->rule_off[r + 1] > d->rule_stem.n ||
        d->rule_stem.n != d->rule_eomi.n)
      return lt::set_error(LT_EINVAL, "lt_lexicon_create: rule_off out of range");
    const int32_t lo = (int32_t)lx->rules.size();
    for (int64_t q = d->rule_off[r]; q < d->rule_off[r + 1]; ++q) {
      RulePair rp;
      if (!decode(d->rule_stem, q)) return lt::set_error(LT_EINVAL, "lt_lexicon_create: bad UTF-8");
      rp.stem = Span{(uint32_t)tab.pool.size(), (uint32_t)cp.size()};
      tab.pool.insert(tab.pool.end(), cp.begin(), cp.end());
      if (!decode(d->rule_eomi, q)) return lt::set_error(LT_EINVAL, "lt_lexicon_create: bad UTF-8");
      rp.eomi = Span{(uint32_t)tab.pool.size(), (uint32_t)cp.size()};
      tab.pool.insert(tab.pool.end(), cp.begin(), cp.end());
      rp.eomi_hs = hs_feed(HS_INIT, cp.data(), (uint32_t)cp.size());
      lx->rules.push_back(rp);
    }
    if (!decode(d->rule_surface, r)) return lt::set_error(LT_EINVAL, "lt_lexicon_create: bad UTF-8");
    Info& in = tab.get_or_add(cp.data(), (uint32_t)cp.size());
    if (in.rule_n == 0) {                      // first entry wins (dict keys are unique anyway)
      in.rule_lo = lo;
      in.rule_n = (int32_t)lx->rules.size() - lo;
    }
  }
  // the tagset literals the lookup writes (tagset.py)
  auto dict_tag = [&](const char* s) {
    for (int32_t t = 0; t < (int32_t)T; ++t)
      if (lx->names[(size_t)t] == s) return t;
    return (int32_t)-1;
  };
  lx->dict_noun = dict_tag("Noun");
  lx->dict_josa = dict_tag("Josa");
  lx->name_noun = name_index("Noun");
  lx->name_josa = name_index("Josa");
  lx->name_adj = name_index("Adjective");
  lx->name_verb = name_index("Verb");
  lx->name_eomi = name_index("Eomi");
  for (int64_t i = 0; i < d->standalones.n; ++i) {
    const std::string s = str(d->standalones, i);
    Standalone st;
    st.dict_tag = -1;
    for (int32_t t = 0; t < (int32_t)T; ++t)
      if (lx->names[(size_t)t] == s) st.dict_tag = t;
    st.name = name_index(s);
    st.is_noun = s == "Noun";
    lx->standalones.push_back(st);
  }
  lx->max_len = d->max_len;
  lx->prefer_exact = d->prefer_exact_match != 0;
  lx->k0 = d->hash_k0;
  lx->k1 = d->hash_k1;
  *out = lx.release();
  return LT_OK;
}

lt_status lt_lexicon_destroy(lt_lexicon* lx) {
  delete lx;
  return LT_OK;
}

lt_status lt_lexicon_lookup(const lt_lexicon* lx, const lt_text_desc* td, int n_threads, lt_lattices** out) {
  if (!lx || !td || !out) return lt::set_error(LT_EINVAL, "lt_lexicon_lookup: NULL argument");
  *out = nullptr;
  const int32_t S = td->n_sent;
  if (S < 0) return lt::set_error(LT_EINVAL, "lt_lexicon_lookup: negative sentence count");
  if (S > 0 && (!td->sent_eoj || !td->char_off || !td->eoj_off))
    return lt::set_error(LT_EINVAL, "lt_lexicon_lookup: NULL arrays");
  for (int32_t s = 0; s < S; ++s) {
    if (td->sent_eoj[s + 1] < td->sent_eoj[s] || td->char_off[s + 1] < td->char_off[s])
      return lt::set_error(LT_EINVAL, "lt_lexicon_lookup: offsets decrease at sentence %d", s);
    int64_t total = 0;
    for (int64_t j = td->sent_eoj[s]; j < td->sent_eoj[s + 1]; ++j) {
      if (td->eoj_off[j + 1] < td->eoj_off[j]) return lt::set_error(LT_EINVAL, "lt_lexicon_lookup: eojeol offsets decrease");
      total += td->eoj_off[j + 1] - td->eoj_off[j];
    }
    if (total > td->char_off[s + 1] - td->char_off[s])
      return lt::set_error(LT_EINVAL, "lt_lexicon_lookup: sentence %d has more eojeol characters than characters", s);
    if (td->char_off[s + 1] - td->char_off[s] > (int64_t)1 << 30)
      return lt::set_error(LT_EUNSUPPORTED, "lt_lexicon_lookup: sentence %d too long", s);
  }
  if (S > 0 && td->char_off[0] != 0) return lt::set_error(LT_EINVAL, "lt_lexicon_lookup: char_off[0] != 0");
  if (S > 0 && (td->eoj_off[td->sent_eoj[S]] >= ((int64_t)1 << 32) || td->sent_eoj[0] < 0))
    return lt::set_error(LT_EUNSUPPORTED, "lt_lexicon_lookup: text too long for one call");
  int nt = n_threads > 0 ? n_threads : lt::host_threads();
  nt = std::max(1, std::min(nt, std::max(1, S / 16)));
  std::vector<Chunk> ck((size_t)nt);
  {
    std::vector<std::thread> th;
    for (int t = 0; t < nt; ++t) {
      const int32_t s0 = (int32_t)((int64_t)S * t / nt), s1 = (int32_t)((int64_t)S * (t + 1) / nt);
      if (t + 1 == nt) run_chunk(*lx, *td, s0, s1, ck[(size_t)t]);
      else th.emplace_back([&, s0, s1, t] { run_chunk(*lx, *td, s0, s1, ck[(size_t)t]); });
    }
    for (std::thread& x : th) x.join();
  }
  for (const Chunk& c : ck)
    if (!c.err.empty()) return lt::set_error(LT_EINVAL, "lt_lexicon_lookup: %s", c.err.c_str());
  std::unique_ptr<lt_lattices> L(new (std::nothrow) lt_lattices);
  if (!L) return lt::set_error(LT_ENOMEM, "lt_lexicon_lookup: out of host memory");
  const int64_t C = S > 0 ? td->char_off[S] : 0;
  const int64_t TX = S > 0 ? td->eoj_off[td->sent_eoj[S]] : 0;     // text code points
  // bases of the chunks in the merged arrays
  std::vector<Base> at(ck.size() + 1);
  for (size_t t = 0; t < ck.size(); ++t) {
    const Chunk& c = ck[t];
    Base& nx = at[t + 1];
    nx = at[t];
    nx.words += (int64_t)c.len.size();
    nx.slots += (int64_t)c.slot_n.size();
    nx.sents += (int64_t)c.sent_n.size();
    nx.pool += (int64_t)c.pool.size();
    for (int f = 0; f < 5; ++f) L->field_cps[f] += c.field_cps[f];
  }
  const Base& tot = at.back();
  if (tot.slots != C || tot.sents != S) return lt::set_error(LT_EINVAL, "lt_lexicon_lookup: slot count mismatch");
  if (tot.pool >= (int64_t)LT_NOREF) return lt::set_error(LT_EUNSUPPORTED, "lt_lexicon_lookup: too many lemmas for one call");
  const int64_t W = tot.words;
  bool ok = L->chars.alloc(C) && L->char_off.alloc(S + 1) && L->slot_off.alloc(C + 1) &&
            L->sent_words.alloc(S + 1) && L->text.alloc(TX) && L->pool.alloc(tot.pool);
  for (Arr<uint32_t>* a : {&L->w_off, &L->w_len, &L->m0_off, &L->m0_len, &L->m1_off, &L->m1_len}) ok = ok && a->alloc(W);
  ok = ok && L->tag0.alloc(W) && L->tag1.alloc(W) && L->len.alloc(W) && L->e.alloc(W) && L->b.alloc(W) &&
       L->is_l.alloc(W);
  if (!ok) return lt::set_error(LT_ENOMEM, "lt_lexicon_lookup: out of host memory");
  try {
    L->names = lx->names;
  } catch (...) {
    return lt::set_error(LT_ENOMEM, "lt_lexicon_lookup: out of host memory");
  }
  L->n_sent = S;
  L->n_words = W;
  if (C) memcpy(L->chars.data(), td->chars, (size_t)C * 4);
  if (TX) memcpy(L->text.data(), td->text, (size_t)TX * 4);
  if (S) memcpy(L->char_off.data(), td->char_off, (size_t)(S + 1) * 8);
  else L->char_off.data()[0] = 0;
  L->slot_off.data()[0] = 0;
  L->sent_words.data()[0] = 0;
  {
    std::vector<std::thread> th;
    for (size_t t = 0; t + 1 < ck.size(); ++t)
      th.emplace_back([&, t] { merge_chunk(ck[t], at[t], *L); });
    merge_chunk(ck.back(), at[ck.size() - 1], *L);
    for (std::thread& x : th) x.join();
  }
  *out = L.release();
  return LT_OK;
}

// str.isspace() of CPython 3.10 (Py_UNICODE_ISSPACE): the separators of
// str.split() without arguments
static inline bool py_isspace(uint32_t c) {
  if (c <= 0x20) return c == 0x20 || (c >= 0x09 && c <= 0x0D) || (c >= 0x1C && c <= 0x1F);
  if (c < 0x85) return false;
  return c == 0x85 || c == 0xA0 || c == 0x1680 || (c >= 0x2000 && c <= 0x200A) || c == 0x2028 ||
         c == 0x2029 || c == 0x202F || c == 0x205F || c == 0x3000;
}

lt_status lt_lexicon_lookup_sents(const lt_lexicon* lx, const uint32_t* text, const int64_t* sent_off,
                                  int32_t n_sent, int n_threads, lt_lattices** out) {
  if (!lx || !out || n_sent < 0 || (n_sent > 0 && (!sent_off || (!text && sent_off[n_sent] > 0))))
    return lt::set_error(LT_EINVAL, "lt_lexicon_lookup_sents: bad argument");
  *out = nullptr;
  const int32_t S = n_sent;
  if (S > 0 && sent_off[0] != 0) return lt::set_error(LT_EINVAL, "lt_lexicon_lookup_sents: sent_off[0] != 0");
  for (int32_t s = 0; s < S; ++s)
    if (sent_off[s + 1] < sent_off[s]) return lt::set_error(LT_EINVAL, "lt_lexicon_lookup_sents: offsets decrease");
  // pass 1 (threads): eojeols, eojeol characters and decode characters per sentence
  std::vector<int64_t> n_eoj((size_t)S + 1, 0), n_tx((size_t)S + 1, 0), n_ch((size_t)S + 1, 0);
  lt::parallel_ranges(S, [&](int, int64_t lo, int64_t hi) {
    for (int64_t s = lo; s < hi; ++s) {
      int64_t ne = 0, nt = 0, nc = 0;
      bool in = false;
      for (int64_t i = sent_off[s]; i < sent_off[s + 1]; ++i) {
        const uint32_t c = text[i];
        const bool sp = py_isspace(c);
        if (!sp) {
          ++nt;
          if (!in) ++ne;
        }
        in = !sp;
        nc += c != 0x20;
      }
      n_eoj[(size_t)s + 1] = ne;
      n_tx[(size_t)s + 1] = nt;
      n_ch[(size_t)s + 1] = nc;
    }
  }, 1024);
  for (int32_t s = 0; s < S; ++s) {
    n_eoj[(size_t)s + 1] += n_eoj[(size_t)s];
    n_tx[(size_t)s + 1] += n_tx[(size_t)s];
    n_ch[(size_t)s + 1] += n_ch[(size_t)s];
  }
  std::vector<uint32_t> tx((size_t)std::max<int64_t>(1, n_tx[(size_t)S])), ch((size_t)std::max<int64_t>(1, n_ch[(size_t)S]));
  std::vector<int64_t> eoj_off((size_t)n_eoj[(size_t)S] + 1);
  eoj_off[0] = 0;
  // pass 2 (threads): the eojeols' text back to back, their ends, the characters
  lt::parallel_ranges(S, [&](int, int64_t lo, int64_t hi) {
    for (int64_t s = lo; s < hi; ++s) {
      int64_t t = n_tx[(size_t)s], c = n_ch[(size_t)s], j = n_eoj[(size_t)s];
      bool in = false;
      for (int64_t i = sent_off[s]; i < sent_off[s + 1]; ++i) {
        const uint32_t x = text[i];
        const bool sp = py_isspace(x);
        if (sp && in) eoj_off[(size_t)++j] = t;        // an eojeol ends
        if (!sp) tx[(size_t)t++] = x;
        in = !sp;
        if (x != 0x20) ch[(size_t)c++] = x;
      }
      if (in) eoj_off[(size_t)++j] = t;
    }
  }, 1024);
  lt_text_desc td;
  td.n_sent = S;
  td.text = tx.data();
  td.eoj_off = eoj_off.data();
  td.sent_eoj = n_eoj.data();
  td.chars = ch.data();
  td.char_off = n_ch.data();
  return lt_lexicon_lookup(lx, &td, n_threads, out);
}

lt_status lt_lattices_columns(const lt_lattices* L, lt_lattice_columns* c) {
  if (!L || !c) return lt::set_error(LT_EINVAL, "lt_lattices_columns: NULL argument");
  c->n_sent = (int32_t)L->n_sent;
  c->n_words = L->n_words;
  c->chars = L->chars.data();
  c->char_off = L->char_off.data();
  c->slot_off = L->slot_off.data();
  c->sent_words = L->sent_words.data();
  c->len = L->len.data();
  c->b = L->b.data();
  c->e = L->e.data();
  c->is_l = L->is_l.data();
  return LT_OK;
}

lt_status lt_lattices_view(const lt_lattices* L, lt_lattice_view* v) {
  if (!L || !v) return lt::set_error(LT_EINVAL, "lt_lattices_view: NULL argument");
  std::call_once(L->utf8_once, [L] { L->utf8_ok = build_utf8(*L); });
  if (!L->utf8_ok) return lt::set_error(LT_ENOMEM, "lt_lattices_view: out of host memory");
  const lt_lattices::Utf8& u = *L->utf8;
  lt_lattice_desc& d = v->lattice;
  const int64_t W = L->n_words;
  auto view_of = [W](const Arr<char>& blob, const Arr<int64_t>& off, const uint8_t* null) {
    lt_strings s;
    s.data = blob.data();
    s.off = off.data();
    s.null = null;
    s.n = W;
    return s;
  };
  d.n_sent = (int32_t)L->n_sent;
  d.chars = L->chars.data();
  d.char_off = L->char_off.data();
  d.slot_off = L->slot_off.data();
  d.n_words = W;
  d.word = view_of(u.wb, u.woff, nullptr);
  d.morph0 = view_of(u.mb, u.moff, nullptr);
  d.tag0 = view_of(u.tb, u.toff, nullptr);
  d.morph1 = view_of(u.m1b, u.m1off, u.m1null.data());
  d.tag1 = view_of(u.t1b, u.t1off, u.t1null.data());
  d.len = u.len.data();
  d.e = u.e.data();
  d.is_l = u.is_l.data();
  v->b = u.b.data();
  v->sent_words = L->sent_words.data();
  return LT_OK;
}

lt_status lt_lattices_strings(const lt_lattices* L, int field, const int64_t* idx, int64_t n, char* out,
                              int64_t cap, int64_t* used) {
  if (!L || (n > 0 && !idx) || field < 0 || field > 4)
    return lt::set_error(LT_EINVAL, "lt_lattices_strings: bad argument");
  std::string buf;
  try {
    for (int64_t i = 0; i < n; ++i) {
      const int64_t v = idx[i];
      if (v < 0 || v >= L->n_words) return lt::set_error(LT_EINVAL, "lt_lattices_strings: index %lld", (long long)v);
      field_utf8(*L, field, v, buf);
      buf.push_back('\0');
    }
  } catch (...) {
    return lt::set_error(LT_ENOMEM, "lt_lattices_strings: out of memory");
  }
  const int64_t need = (int64_t)buf.size();
  if (used) *used = need;
  if (need > cap || (need > 0 && !out)) return lt::set_error(LT_EINVAL, "lt_lattices_strings: %lld bytes needed", (long long)need);
  if (need) memcpy(out, buf.data(), (size_t)need);
  return LT_OK;
}

lt_status lt_lattices_strings_coded(const lt_lattices* L, int field, const int64_t* idx, int64_t n,
                                    int32_t* codes, char* out, int64_t cap, int64_t* used,
                                    int64_t* n_unique) {
  if (!L || (n > 0 && (!idx || !codes)) || field < 0 || field > 4)
    return lt::set_error(LT_EINVAL, "lt_lattices_strings_coded: bad argument");
  for (int64_t i = 0; i < n; ++i)
    if (idx[i] < 0 || idx[i] >= L->n_words)
      return lt::set_error(LT_EINVAL, "lt_lattices_strings_coded: index %lld", (long long)idx[i]);
  std::string blob;
  int64_t nu = 0;
  try {
    if (field >= 3) {
      // tags: the lexicon's names, coded in first-appearance order
      const int16_t* tg = field == 3 ? L->tag0.data() : L->tag1.data();
      std::vector<int32_t> code_of(L->names.size(), -1);
      for (int64_t i = 0; i < n; ++i) {
        const int16_t t = tg[idx[i]];
        if (t < 0) {
          codes[i] = -1;
          continue;
        }
        int32_t& c = code_of[(size_t)t];
        if (c < 0) {
          const std::string& nm = L->names[(size_t)t];
          if (nm.find('\0') != std::string::npos)
            return lt::set_error(LT_EUNSUPPORTED, "lt_lattices_strings_coded: string with a NUL byte");
          c = (int32_t)nu++;
          blob += nm;
          blob.push_back('\0');
        }
        codes[i] = c;
      }
    } else {
      // code-point strings: open addressing over (hash, code) on the distinct
      // strings' (pointer, length); the table grows with the distinct strings
      struct Ref {
        const uint32_t* p;
        uint32_t n;
      };
      struct Slot {
        uint64_t h;                                  // 0: empty
        int32_t code;
      };
      std::vector<Ref> uniq;
      std::vector<Slot> tab(1024, Slot{0, 0});
      uint64_t mask = 1023;
      for (int64_t i = 0; i < n; ++i) {
        const int64_t v = idx[i];
        const uint32_t* p;
        uint32_t m;
        if (field == 0) {
          p = L->text.data() + L->w_off[v];
          m = L->w_len[v];
        } else if (field == 1) {
          p = L->m0_cps(v, m);
        } else {
          if (L->m1_off[v] == LT_NOREF) {
            codes[i] = -1;
            continue;
          }
          p = L->pool.data() + L->m1_off[v];
          m = L->m1_len[v];
        }
        uint64_t h = 0x9E3779B97F4A7C15ull ^ m;
        for (uint32_t k = 0; k < m; ++k) {
          h = (h ^ p[k]) * 0xBF58476D1CE4E5B9ull;
          h ^= h >> 31;
        }
        h |= 1ull;
        uint64_t j = h & mask;
        for (;; j = (j + 1) & mask) {
          if (tab[j].h == 0) {
            if (std::find(p, p + m, 0u) != p + m)
              return lt::set_error(LT_EUNSUPPORTED, "lt_lattices_strings_coded: string with a NUL byte");
            tab[j] = Slot{h, (int32_t)uniq.size()};
            uniq.push_back(Ref{p, m});
            utf8_append(blob, p, m);
            blob.push_back('\0');
            if (uniq.size() * 2 > tab.size()) {          // grow: re-place by the stored hashes
              std::vector<Slot> t2(tab.size() * 2, Slot{0, 0});
              const uint64_t m2 = t2.size() - 1;
              for (const Slot& x : tab)
                if (x.h) {
                  uint64_t q = x.h & m2;
                  while (t2[q].h) q = (q + 1) & m2;
                  t2[q] = x;
                }
              tab.swap(t2);
              mask = m2;
            }
            codes[i] = (int32_t)uniq.size() - 1;
            break;
          }
          const Ref& r = uniq[(size_t)tab[j].code];
          if (tab[j].h == h && r.n == m && std::equal(p, p + m, r.p)) {
            codes[i] = tab[j].code;
            break;
          }
        }
      }
      nu = (int64_t)uniq.size();
    }
  } catch (...) {
    return lt::set_error(LT_ENOMEM, "lt_lattices_strings_coded: out of memory");
  }
  const int64_t need = (int64_t)blob.size();
  if (used) *used = need;
  if (n_unique) *n_unique = nu;
  if (need > cap || (need > 0 && !out))
    return lt::set_error(LT_EINVAL, "lt_lattices_strings_coded: %lld bytes needed", (long long)need);
  if (need) memcpy(out, blob.data(), (size_t)need);
  return LT_OK;
}

int64_t lt_lattices_field_bytes(const lt_lattices* L, int field) {
  if (!L || field < 0 || field > 4) return 0;
  return field < 3 ? 4 * L->field_cps[field] : L->field_cps[field];     // UTF-8: at most 4 bytes per code point
}

lt_status lt_lattices_destroy(lt_lattices* L) {
  delete L;
  return LT_OK;
}

}  // extern "C"
