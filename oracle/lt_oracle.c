/*
 * TEST INFRASTRUCTURE ONLY -- C restatement of the reference decoder over the
 * packed batch format of include/lattice_decode.h.  Used by tests/ (parity of
 * the HIP kernel on large batches) and by bench.py's cpu_baseline leg.  Never
 * linked into the product library.
 *
 * Restates:
 *   beam_search            lattice_tagger/beam/beam.py:5-61
 *     candidate order      beam.py:31-42 (begin ascending, beam rank, bindex order)
 *     unknown-run skip     beam.py:43-45
 *     Beam.append          beam.py:83-86 (stable sort on -score, keep k)
 *     Sequence.add         beam.py:112-116
 *     EOS append           beam.py:59-61 (score + 0)
 *   BeamScoreFunctions     beam/score_funcs.py:50-54 (pre-summed node terms
 *                          + trigram + post node terms, in order)
 *   SimpleTrigramFeatureScore.score  score_funcs.py:137-144
 *   trigram_encoder        features/feature.py:76-121
 *   numpy pairwise sum     (score_funcs.py:144; numpy pairwise_sum order)
 * Independent of the product's data structures: key presence is a binary
 * search over the sorted key array (no hash table, no pre-filter masks) and
 * the beam is a full stable sort of every grown hypothesis.  Implicit Unknown
 * candidates (lt_batch_desc.n_unk: an empty span in range holds the
 * synthesised Unknown of beam.py:36-38) are enumerated in their span's place
 * and reported by their negative path code.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/lattice_decode.h"

#define F_UNK (1u << 16)
#define F_CTX (1u << 17)
#define F_HAS4 (1u << 18)
#define F_HAS5 (1u << 19)
#define F_HAS6 (1u << 20)

typedef struct {
  uint32_t cls, a, b, c;
  double coef;
} okey;

typedef struct {
  okey* keys;
  int64_t n;
} omodel;

static int key_cmp(const void* x, const void* y) {
  const okey* p = (const okey*)x;
  const okey* q = (const okey*)y;
  if (p->cls != q->cls) return p->cls < q->cls ? -1 : 1;
  if (p->a != q->a) return p->a < q->a ? -1 : 1;
  if (p->b != q->b) return p->b < q->b ? -1 : 1;
  if (p->c != q->c) return p->c < q->c ? -1 : 1;
  return 0;
}

static int lookup(const omodel* m, uint32_t cls, uint32_t a, uint32_t b, uint32_t c, double* coef) {
  if (a == 0 || b == 0) return 0;
  okey k = {cls, a, b, c, 0.0};
  const okey* hit = (const okey*)bsearch(&k, m->keys, (size_t)m->n, sizeof(okey), key_cmp);
  if (!hit) return 0;
  *coef = hit->coef;
  return 1;
}

typedef struct {
  double score;
  int32_t node;      /* last node (local index) */
  int32_t prev;      /* second-last node, -1 = None */
  int32_t depth;
  int32_t ppos, prank;
  int32_t unk;       /* num_unk > 0 */
} ohyp;

typedef struct {
  double score;
  int64_t gen;
  int32_t node, prev, depth, ppos, prank, unk;
} ogrown;

static int grown_cmp(const void* x, const void* y) {
  /* sorted(key=-score) is stable: order by score desc, then generation index */
  const ogrown* p = (const ogrown*)x;
  const ogrown* q = (const ogrown*)y;
  if (p->score > q->score) return -1;
  if (p->score < q->score) return 1;
  return p->gen < q->gen ? -1 : (p->gen > q->gen ? 1 : 0);
}

static double numpy_sum(const double* v, int m) {
  if (m < 8) {
    double s = 0.0;
    for (int i = 0; i < m; ++i) s += v[i];
    return s;
  }
  double r[8];
  for (int i = 0; i < 8; ++i) r[i] = v[i];
  int i = 8;
  for (; i < m - (m % 8); i += 8)
    for (int j = 0; j < 8; ++j) r[j] += v[i + j];
  double s = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  for (; i < m; ++i) s += v[i];
  return s;
}

/* A candidate word of sentence `nb` by its path code (lattice_decode.h):
 * x >= 0 local node x; x <= -2 the implicit Unknown of span entry -2 - x
 * (n_unk: the synthesised Word of an empty span, beam.py:36-38), whose record
 * is entry d - 1 of the unk_* arrays, d = SS - (entry mod SS). */
typedef struct {
  int32_t w, m, t;
  uint32_t f;
  double pre, f4, f5, f6;
  int64_t at;     /* node index into node_post, or -(d) for unk_post */
} onode;

static void node_at(const lt_batch_desc* d, int64_t nb, int SS, int32_t x, onode* o) {
  if (x >= 0) {
    const int64_t i = nb + x;
    o->w = d->node_word[i]; o->m = d->node_morph0[i]; o->t = d->node_tag[i]; o->f = d->node_mask[i];
    o->pre = d->node_pre[i]; o->f4 = d->node_f4[i]; o->f5 = d->node_f5[i]; o->f6 = d->node_f6[i];
    o->at = i;
  } else {
    const int dd = SS - ((-2 - x) % SS);
    const int i = dd - 1;
    o->w = d->unk_word[i]; o->m = d->unk_morph0[i]; o->t = d->unk_tag[i]; o->f = d->unk_mask[i];
    o->pre = d->unk_pre[i]; o->f4 = d->unk_f4[i]; o->f5 = d->unk_f5[i]; o->f6 = d->unk_f6[i];
    o->at = -(int64_t)dd;
  }
}

static double post_term(const lt_batch_desc* d, const onode* o, int t) {
  return o->at >= 0 ? d->node_post[(int64_t)t * d->n_nodes + o->at]
                    : d->unk_post[(int64_t)t * d->n_unk + (-o->at - 1)];
}

static int decode_sentence(const omodel* m, const lt_batch_desc* d, int s, int k, int32_t* count,
                           int32_t* length, double* score, int32_t* codes, int64_t code_base,
                           int64_t* n_exp, int64_t* n_tup, int64_t* n_hit) {
  const int n = d->sent_n[s];
  const int64_t nb = d->sent_node_off[s];
  const int32_t* ss = d->span_start + d->sent_span_off[s];
  ohyp* H = (ohyp*)malloc(sizeof(ohyp) * (size_t)(n + 1) * (size_t)k);
  int32_t* cnt = (int32_t*)calloc((size_t)n + 1, sizeof(int32_t));
  size_t gcap = 1024;
  ogrown* G = (ogrown*)malloc(sizeof(ogrown) * gcap);
  if (!H || !cnt || !G) { free(H); free(cnt); free(G); return -1; }
  ohyp bos = {0.0, 0, -1, 0, -1, -1, 0};
  H[0] = bos;
  cnt[0] = 1;
  const int SS = d->max_len <= LT_MAX_SPAN ? LT_MAX_SPAN : d->max_len;   /* span slots per position */
  for (int e = 1; e <= n; ++e) {
    const int bmin = e - d->max_len > 0 ? e - d->max_len : 0;
    size_t ng = 0;
    int64_t gen = 0;
    for (int b = bmin; b < e; ++b) {
      const int dd = e - b;
      const int j = SS - dd;
      const int32_t lo = ss[(int64_t)(e - 1) * SS + j], hi = ss[(int64_t)(e - 1) * SS + j + 1];
      /* no node in the span: its implicit Unknown (beam.py:36-38), by code */
      const int imp = lo == hi && d->n_unk > 0;
      const int32_t xlo = imp ? -2 - ((e - 1) * SS + j) : lo, xhi = imp ? xlo + 1 : hi;
      for (int r = 0; r < cnt[b]; ++r) {
        const ohyp* h = &H[(size_t)b * k + r];
        for (int32_t x = xlo; x < xhi; ++x) {
          const int64_t gi = gen++;
          onode X, J, I;
          node_at(d, nb, SS, x, &X);
          if (h->unk && (X.f & F_UNK) && bmin < b) continue;
          double tri = 0.0;
          if (d->has_trigram) {
            const int jn = h->node, in = h->prev;
            node_at(d, nb, SS, jn, &J);
            if (in != -1) node_at(d, nb, SS, in, &I);
            double v[9];
            int mm = 0;
            double c;
            int tup = 6;
            if (lookup(m, 0, J.w, X.w, X.t, &c)) v[mm++] = c;
            if (lookup(m, 1, J.w, X.t, 0, &c)) v[mm++] = c;
            if (lookup(m, 2, J.t, X.w, X.t, &c)) v[mm++] = c;
            if (lookup(m, 3, J.t, X.t, 0, &c)) v[mm++] = c;
            if (X.f & F_HAS4) v[mm++] = X.f4;
            if (X.f & F_HAS5) v[mm++] = X.f5;
            if (J.f & F_UNK) {
              ++tup;
              if (J.f & F_HAS6) v[mm++] = J.f6;
            }
            if (in != -1) {
              ++tup;
              if (I.w != 0 && lookup(m, 7, I.w, J.w, X.w, &c)) v[mm++] = c;
            }
            if (X.f & F_CTX) {
              if (J.f & F_CTX) {
                ++tup;
                if (lookup(m, 8, J.m, X.m, 0, &c)) v[mm++] = c;
              } else if (in != -1 && (I.f & F_CTX)) {
                ++tup;
                if (lookup(m, 8, I.m, X.m, 0, &c)) v[mm++] = c;
              }
            }
            tri = numpy_sum(v, mm);
            *n_tup += tup;
            *n_hit += mm;
          }
          double inc = X.pre + tri;
          for (int t = 0; t < d->n_post; ++t) inc += post_term(d, &X, t);
          if (ng == gcap) {
            gcap *= 2;
            ogrown* G2 = (ogrown*)realloc(G, sizeof(ogrown) * gcap);
            if (!G2) { free(H); free(cnt); free(G); return -1; }
            G = G2;
          }
          ogrown* g = &G[ng++];
          g->score = h->score + inc;
          g->gen = gi;
          g->node = x;
          g->prev = h->node;
          g->depth = h->depth + 1;
          g->ppos = b;
          g->prank = r;
          g->unk = (X.f & F_UNK) ? 1 : 0;
          ++*n_exp;
        }
      }
    }
    qsort(G, ng, sizeof(ogrown), grown_cmp);
    const int keep = (int)(ng < (size_t)k ? ng : (size_t)k);
    for (int t = 0; t < keep; ++t) {
      ohyp* o = &H[(size_t)e * k + t];
      o->score = G[t].score;
      o->node = G[t].node;
      o->prev = G[t].prev;
      o->depth = G[t].depth;
      o->ppos = G[t].ppos;
      o->prank = G[t].prank;
      o->unk = G[t].unk;
    }
    cnt[e] = keep;
  }
  count[s] = cnt[n];
  for (int t = 0; t < cnt[n]; ++t) {
    const ohyp* f = &H[(size_t)n * k + t];
    score[(int64_t)s * k + t] = f->score + 0.0;
    length[(int64_t)s * k + t] = f->depth;
    int32_t* out = codes + code_base + (int64_t)t * n;
    int pos = n, rank = t;
    for (int step = f->depth - 1; step >= 0; --step) {
      const ohyp* h = &H[(size_t)pos * k + rank];
      out[step] = h->node;
      pos = h->ppos;
      rank = h->prank;
    }
  }
  free(H);
  free(cnt);
  free(G);
  return 0;
}

/* Decodes sentences [s0, s1) of the batch.  Output layout = lt_result with
 * beam k (codes of sentence s at k * sum_{s'<s} n_{s'}).  Returns 0 or -1. */
int lto_decode(const lt_model_desc* md, const lt_batch_desc* d, int k, int s0, int s1,
               int32_t* count, int32_t* length, double* score, int32_t* codes,
               int64_t* expansions, int64_t* feature_tuples, int64_t* present, int nthreads) {
  if (k < 1 || s0 < 0 || s1 > d->n_sent || s0 > s1) return -1;
  omodel m;
  m.n = md->n_keys;
  m.keys = (okey*)malloc(sizeof(okey) * (size_t)(m.n > 0 ? m.n : 1));
  if (!m.keys) return -1;
  for (int64_t i = 0; i < m.n; ++i) {
    m.keys[i].a = md->keys[4 * i];
    m.keys[i].b = md->keys[4 * i + 1];
    m.keys[i].c = md->keys[4 * i + 2];
    m.keys[i].cls = md->keys[4 * i + 3];
    m.keys[i].coef = md->coefs[i];
  }
  qsort(m.keys, (size_t)m.n, sizeof(okey), key_cmp);
  int64_t* base = (int64_t*)malloc(sizeof(int64_t) * ((size_t)d->n_sent + 1));
  if (!base) { free(m.keys); return -1; }
  base[0] = 0;
  for (int s = 0; s < d->n_sent; ++s) base[s + 1] = base[s] + d->sent_n[s];
  int64_t tot_exp = 0, tot_tup = 0, tot_hit = 0;
  int err = 0;
  (void)nthreads;
#pragma omp parallel for schedule(dynamic, 16) reduction(+ : tot_exp, tot_tup, tot_hit) num_threads(nthreads > 0 ? nthreads : 1)
  for (int s = s0; s < s1; ++s) {
    int64_t ex = 0, tu = 0, hi = 0;
    if (decode_sentence(&m, d, s, k, count, length, score, codes, (int64_t)k * base[s], &ex, &tu, &hi))
      err = 1;
    tot_exp += ex;
    tot_tup += tu;
    tot_hit += hi;
  }
  if (expansions) *expansions = tot_exp;
  if (feature_tuples) *feature_tuples = tot_tup;
  if (present) *present = tot_hit;
  free(base);
  free(m.keys);
  return err ? -1 : 0;
}
