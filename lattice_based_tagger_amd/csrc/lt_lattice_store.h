// lt_lattice_store.h -- the native lattice builder's output (lt_lattices),
// shared by the builder (lt_lookup.cpp) and the packer (lt_packer.cpp).
//
// Nodes are kept compact: a node's strings are references -- the surface
// into the eojeol text, lemma morphs into the call's code-point pool, tags as
// indices into the lexicon's tag names -- so the lookup writes about 40 bytes
// per node instead of five UTF-8 strings and nine 64-bit columns, and the
// packer (lt_packer_pack_lattices) hashes code points it already has.  The
// UTF-8 columns of lt_lattice_desc are built only when asked for
// (lt_lattices_view), the path node strings per call (lt_lattices_strings*).
#pragma once
#include <cstdint>
#include <mutex>
#include <string>
#include <vector>

#include "lt_host.h"

constexpr uint32_t LT_NOREF = 0xFFFFFFFFu;      // morph0: the surface; morph1: None

struct lt_lattices {
  int64_t n_sent = 0, n_words = 0;
  lt::Arr<uint32_t> chars;                     // decode characters (sent.replace(' ', ''))
  lt::Arr<int64_t> char_off, slot_off, sent_words;
  lt::Arr<uint32_t> text;                      // the eojeols' code points (sent.split())
  lt::Arr<uint32_t> pool;                      // lemma morph code points
  std::vector<std::string> names;              // tag names (the lexicon's)
  // per node (bindex order)
  lt::Arr<uint32_t> w_off, w_len;              // surface text[w_off .. +w_len)
  lt::Arr<uint32_t> m0_off, m0_len;            // pool[m0_off .. +m0_len); LT_NOREF: the surface
  lt::Arr<uint32_t> m1_off, m1_len;            // LT_NOREF: None
  lt::Arr<int16_t> tag0, tag1;                 // names index; tag1 -1: None
  lt::Arr<int32_t> len, b, e;
  lt::Arr<uint8_t> is_l;
  // upper bounds of each string field's UTF-8 bytes (lt_lattices_field_bytes)
  int64_t field_cps[5] = {0, 0, 0, 0, 0};

  // lt_lattices_view's UTF-8 columns, built on first use
  struct Utf8 {
    lt::Arr<char> wb, mb, m1b, tb, t1b;
    lt::Arr<int64_t> woff, moff, m1off, toff, t1off;
    lt::Arr<uint8_t> m1null, t1null;
    lt::Arr<int64_t> len, e, b, is_l;
  };
  mutable std::once_flag utf8_once;
  mutable std::unique_ptr<Utf8> utf8;
  mutable bool utf8_ok = false;

  const uint32_t* m0_cps(int64_t i, uint32_t& n) const {
    if (m0_off[i] == LT_NOREF) {
      n = w_len[i];
      return text.data() + w_off[i];
    }
    n = m0_len[i];
    return pool.data() + m0_off[i];
  }
};
