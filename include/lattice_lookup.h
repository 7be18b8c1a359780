/* lattice_lookup.h -- C-ABI of the native lattice builder (liblt.so).
 *
 * the dictionary lookup in front of the decoder.  It
 * replaces, for whole corpora at once, what `Tagger.tag` does per sentence
 * before beam_search (lattice_tagger/tagger/tagger.py:72-74):
 *   - sentence_lookup / sentence_lookup_as_begin_index
 *     (lattice_tagger/dictionary/lookup.py:52-62, 358-369),
 *   - MorphemeLookup -> morpheme_lookup -> lr_lookup (lookup.py:99-132,
 *     171-279) with the defaults the reference Tagger uses (flatten=False),
 *   - MorphemeDictionary.lookup / check / get_tags / lemmatize
 *     (dictionary/dictionary.py:230-242, 304-315),
 *   - analyze_morphology / get_lemma_candidates (dictionary/lemmatizer.py:5-112).
 * Lattices come out in exactly the reference's node order, so the output
 * feeds lt_packer_pack (include/lattice_pack.h) and the decoder unchanged.
 *
 * Order hazards the caller resolves: the dictionary's
 * tag order (dict insertion order) and each rule tuple's order are passed in
 * as the Python objects hold them; the iteration order of the two-element set
 * {word[i:i+2], word[i:i+3]} (lemmatizer.py:107) depends on Python's str hash
 * and is reproduced from the SipHash-2-4 key of the Python process whose
 * behaviour is wanted (CPython 3.10's str hash; lt_py_str_hash exposes it for
 * the callers' self-check).
 *
 * Strings are lt_strings (UTF-8, see lattice_pack.h).
 */
#ifndef LATTICE_LOOKUP_H
#define LATTICE_LOOKUP_H

#include <stdint.h>
#include "lattice_pack.h"

#ifdef __cplusplus
extern "C" {
#endif

#define LT_LEXICON_MAX_TAGS 64

typedef struct {
  /* tag_to_morphs in the dictionary's iteration order (get_tags order,
   * dictionary.py:241-242); morphs of tag t are morph[morph_off[t] .. morph_off[t+1]) */
  lt_strings tag;                 /* [n_tags] (<= LT_LEXICON_MAX_TAGS) */
  const int64_t* morph_off;       /* [n_tags + 1] */
  lt_strings morph;
  /* MorphemeDictionary.verbs / adjectives / eomis (dictionary.py:300-302) */
  lt_strings verbs, adjectives, eomis;
  /* rules: surface -> (stem, eomi) pairs in the tuple's order (dictionary.py:366-377) */
  lt_strings rule_surface;        /* [n_rules] */
  const int64_t* rule_off;        /* [n_rules + 1] */
  lt_strings rule_stem, rule_eomi;
  /* MorphemeLookup parameters (lookup.py:100-114): standalone tags in order,
   * max_len (<= 0: the eojeol length), prefer_exact_match */
  lt_strings standalones;
  int32_t max_len;
  int32_t prefer_exact_match;
  /* SipHash-2-4 key (CPython _Py_HashSecret.siphash k0, k1) */
  uint64_t hash_k0, hash_k1;
} lt_lexicon_desc;

/* Sentences, already split the way the reference splits them: eojeols of
 * sentence s are [sent_eoj[s], sent_eoj[s+1]) (sent.split(), lookup.py:58),
 * eojeol j is text[eoj_off[j] .. eoj_off[j+1]); the sentence's decode
 * characters (sent.replace(' ', ''), tagger.py:72) are
 * chars[char_off[s] .. char_off[s+1]).  All UTF-32 code points. */
typedef struct {
  int32_t n_sent;
  const uint32_t* text;
  const int64_t* eoj_off;         /* [n_eoj + 1] */
  const int64_t* sent_eoj;        /* [n_sent + 1] */
  const uint32_t* chars;
  const int64_t* char_off;        /* [n_sent + 1] */
} lt_text_desc;

/* The lattices: `lattice` as lt_packer_pack consumes it (bindex order:
 * nodes grouped by begin, lookup order within a begin), plus each node's
 * begin `b` and each sentence's node count (0 with n_s > 0 is the reference's
 * empty bindex, on which beam_search raises IndexError, lookup.py:362-363). */
typedef struct {
  lt_lattice_desc lattice;
  const int64_t* b;               /* [n_words] */
  const int64_t* sent_words;      /* [n_sent + 1] word offsets per sentence */
} lt_lattice_view;

typedef struct lt_lexicon lt_lexicon;
typedef struct lt_lattices lt_lattices;

lt_status lt_lexicon_create(const lt_lexicon_desc* desc, lt_lexicon** out);
lt_status lt_lexicon_destroy(lt_lexicon* lexicon);
/* Host only.  n_threads <= 0: OMP_NUM_THREADS, else the hardware concurrency. */
lt_status lt_lexicon_lookup(const lt_lexicon* lexicon, const lt_text_desc* text, int n_threads,
                            lt_lattices** out);
/* The UTF-8 columns of lt_lattice_view are built on the first call (the
 * builder keeps nodes as references into the text, a lemma pool and the tag
 * names); lt_packer_pack_lattices (lattice_pack.h) and the calls below read
 * the compact form directly. */
/* The same from raw sentences: sentence s is text[sent_off[s] ..
 * sent_off[s+1]) (UTF-32); its eojeols are sent.split() (runs of CPython
 * str.isspace() characters separate them, lookup.py:58) and its decode
 * characters sent.replace(' ', '') (tagger.py:72). */
lt_status lt_lexicon_lookup_sents(const lt_lexicon* lexicon, const uint32_t* text, const int64_t* sent_off,
                                  int32_t n_sent, int n_threads, lt_lattices** out);
lt_status lt_lattices_view(const lt_lattices* lattices, lt_lattice_view* view);

/* Offsets and the integer node columns, without building any string column
 * (valid while the lattices live). */
typedef struct {
  int32_t n_sent;
  int64_t n_words;
  const uint32_t* chars;          /* [char_off[n_sent]] */
  const int64_t* char_off;        /* [n_sent + 1] */
  const int64_t* slot_off;        /* [char_off[n_sent] + 1] */
  const int64_t* sent_words;      /* [n_sent + 1] */
  const int32_t* len;             /* [n_words] */
  const int32_t* b;
  const int32_t* e;
  const uint8_t* is_l;
} lt_lattice_columns;
lt_status lt_lattices_columns(const lt_lattices* lattices, lt_lattice_columns* columns);
lt_status lt_lattices_destroy(lt_lattices* lattices);
/* Bulk string extraction for re-materialising nodes: field 0..4 = word,
 * morph0, morph1, tag0, tag1; the strings of nodes idx[0..n) are written to
 * out back to back, each followed by a NUL byte (a None value writes just
 * the NUL).  cap: bytes available; *used receives the bytes written (or
 * needed, with LT_EINVAL, when cap is too small). */
lt_status lt_lattices_strings(const lt_lattices* lattices, int field, const int64_t* idx, int64_t n,
                              char* out, int64_t cap, int64_t* used);
/* The same strings dictionary-coded: codes[i] is the index of node idx[i]'s
 * string among the distinct strings (first-appearance order), -1 for None;
 * the distinct strings are written to out NUL-terminated, *n_unique of them.
 * cap >= the field's blob bytes + n always suffices; a smaller cap that
 * does not fit fails with LT_EINVAL and *used = the bytes needed.  A string
 * holding a NUL byte fails with LT_EUNSUPPORTED (use lt_lattices_strings'
 * offsets instead). */
lt_status lt_lattices_strings_coded(const lt_lattices* lattices, int field, const int64_t* idx, int64_t n,
                                    int32_t* codes, char* out, int64_t cap, int64_t* used,
                                    int64_t* n_unique);
/* Bytes of one string field's blob (the cap bound above, less n). */
int64_t lt_lattices_field_bytes(const lt_lattices* lattices, int field);

/* CPython 3.10 hash() of the str with these code points under SipHash key
 * (k0, k1) -- test hook for the set-order reproduction. */
int64_t lt_py_str_hash(const uint32_t* cps, int64_t n, uint64_t k0, uint64_t k1);
/* 1 when the set {a, b} (a added first, BUILD_SET) of two unequal strs with
 * these hashes iterates b first in CPython 3.10 -- test hook. */
int lt_py_set2_second_first(int64_t hash_a, int64_t hash_b);

#ifdef __cplusplus
}
#endif
#endif /* LATTICE_LOOKUP_H */
