// lt_decode.hip -- batched lattice beam decoder for gfx950 (MI355X).
//
// Restates, one sentence per lane group, the reference decoder
//   beam_search            lattice_tagger/beam/beam.py:5-61
//   Beam.append            beam.py:83-86  (stable sort by -score, keep k)
//   Sequence.add           beam.py:112-116
// scored by the lowered composite
//   BeamScoreFunctions     beam/score_funcs.py:50-54 (ordered sum)
//   SimpleTrigramFeatureScore.score  score_funcs.py:137-144
//   trigram_encoder        features/feature.py:76-121
//
// Execution model:
//  * a group of G lanes (G = 16/32/64, inside one wave64) owns one sentence;
//    256-thread blocks hold 256/G sentences; no block-level barriers.
//  * the frontier -- beams of the last 9 end positions -- lives in LDS as a
//    ring; each hypothesis entry caches the fields of its last two nodes, so
//    scoring an expansion reads the candidate node from HBM and the
//    hypothesis from LDS only.
//  * expansions of end position e are enumerated in the reference's
//    generation order g (begin ascending, hypothesis rank, candidate order);
//    lane l takes g = l, l+G, ...; ties are broken by lower g exactly as
//    Python's stable sort does.
//  * trigram features: classes 4/5/6 arrive pre-resolved per node; classes
//    0,1,2,3,7,8 are probed in an open-addressing table (32 B slots), all
//    probes of an expansion issued before any is resolved.  The present
//    coefficients are summed in numpy's pairwise order (H7).
//  * top-k: every lane keeps its own top-k of the expansions it scored
//    (registers), then k rounds of group argmax merge them.
//  * backpointers (4 B per beam entry) go to HBM; the final backtrace walks
//    them per mature.
#include <hip/hip_runtime.h>
#include <math.h>
#include "lt_common.h"
#include "lt_internal.h"

using namespace lt;

namespace {

constexpr uint32_t INV = 0xFFFFFFFFu;

struct alignas(16) Entry {
  double score;     // path score
  double f6;        // coefficient of (6, min(8, wj.len)) when wj has F_HAS6
  int32_t node;     // local node index of wj (the last node)
  int32_t jword, jmorph, jtag;
  uint32_t jmask;   // wj mask + flags
  int32_t iword, imorph;
  uint32_t imask;   // wi mask + flags, F_WI when wi exists
  int32_t depth;    // words on the path, BOS excluded
  int32_t pad[3];
};
static_assert(sizeof(Entry) == 64, "Entry must be 64 B");

__device__ __forceinline__ bool better(double s1, uint32_t g1, double s2, uint32_t g2) {
  // (score desc, generation index asc); INV never wins.
  if (g2 == INV) return g1 != INV;
  if (g1 == INV) return false;
  return (s1 > s2) || (s1 == s2 && g1 < g2);
}

template <int G>
__device__ __forceinline__ void group_argmax(double& s, uint32_t& g) {
#pragma unroll
  for (int off = G / 2; off >= 1; off >>= 1) {
    double os = __shfl_xor(s, off, G);
    uint32_t og = __shfl_xor(g, off, G);
    if (better(os, og, s, g)) { s = os; g = og; }
  }
}

template <int G>
__device__ __forceinline__ unsigned long long group_sum(unsigned long long v) {
#pragma unroll
  for (int off = G / 2; off >= 1; off >>= 1) v += __shfl_xor(v, off, G);
  return v;
}

// Probe the table for key (a,b,c,cls); returns true and the coefficient if
// present.  `first` is the already-loaded slot at the home index.
__device__ __forceinline__ bool resolve(const Slot* __restrict__ tab, uint32_t tmask,
                                        uint32_t h, Slot first, uint32_t a, uint32_t b,
                                        uint32_t c, uint32_t cls1, double& coef) {
  Slot sl = first;
  for (;;) {
    if (sl.cls1 == cls1 && sl.a == a && sl.b == b && sl.c == c) { coef = sl.coef; return true; }
    if (sl.cls1 == EMPTY) return false;
    h = (h + 1u) & tmask;
    sl = tab[h];
  }
}

__device__ __forceinline__ Slot load_slot(const Slot* __restrict__ tab, uint32_t h) {
  const uint4* p = reinterpret_cast<const uint4*>(tab + h);
  uint4 k = p[0];
  uint4 v = p[1];
  Slot s;
  s.a = k.x; s.b = k.y; s.c = k.z; s.cls1 = k.w;
  s.coef = __hiloint2double((int)v.y, (int)v.x);
  s.pad = 0;
  return s;
}

// Sum of the present features in numpy's pairwise order
// (numpy pairwise_sum: n < 8 -> ((0.0 + a0) + a1) + ...;
//  8 <= n < 16 -> r = a[0:8], ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)), then + a8...).
__device__ __forceinline__ double numpy_sum9(const double (&v)[9], const bool (&pr)[9]) {
  int m = 0;
#pragma unroll
  for (int q = 0; q < 9; ++q) m += pr[q] ? 1 : 0;
  if (m < 8) {
    double s = 0.0;
#pragma unroll
    for (int q = 0; q < 9; ++q) s = pr[q] ? s + v[q] : s;
    return s;
  }
  // m is 8 or 9: at most one feature is missing; compact in order.
  int miss = 9;
#pragma unroll
  for (int q = 8; q >= 0; --q) if (!pr[q]) miss = q;
  double r[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) r[q] = (q < miss) ? v[q] : v[q + 1];
  double s = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  if (m == 9) s += v[8];
  return s;
}

template <int KT, int G, bool COUNT>
__global__ void __launch_bounds__(256)
lt_decode_k(DecodeParams p) {
  constexpr int SPB = 256 / G;               // sentences per block
  static_assert(KT <= G, "beam width must not exceed the lane group");
  __shared__ Entry ring[SPB][RING][KT];
  __shared__ int32_t cnt[SPB][RING];

  const int grp = threadIdx.x / G;
  const int gl = threadIdx.x % G;
  const int slot = blockIdx.x * SPB + grp;
  if (slot >= p.n_sent) return;
  const int s = p.order[slot];
  const int n = p.sent_n[s];
  const int64_t nbase = p.node_off[s];
  const int32_t* __restrict__ ssp = p.span_start + p.span_off[s];
  uint32_t* __restrict__ bp = p.bp + p.bp_off[s];
  const int k = p.k;
  const int bstride = p.bp_stride;
  const Slot* __restrict__ tab = p.table;
  const uint32_t tmask = p.tmask;
  const int has_tri = p.has_tri;

  Entry (&R)[RING][KT] = ring[grp];
  unsigned long long n_exp = 0, n_tup = 0, n_probe = 0;

  if (gl == 0) {                             // beam[0] = [BOS] (beam.py:21-23)
    Entry e0;
    e0.score = 0.0;
    e0.f6 = p.nf6[nbase];
    e0.node = 0;
    e0.jword = p.nword[nbase];
    e0.jmorph = p.nmorph[nbase];
    e0.jtag = p.ntag[nbase];
    e0.jmask = p.nmask[nbase];
    e0.iword = 0; e0.imorph = 0; e0.imask = 0;
    e0.depth = 0;
    e0.pad[0] = e0.pad[1] = e0.pad[2] = 0;
    R[0][0] = e0;
    cnt[grp][0] = 1;
  }
  __builtin_amdgcn_wave_barrier();

  for (int e = 1; e <= n; ++e) {
    const int dmax = min(e, p.max_len);
    const int32_t* sse = ssp + (e - 1) * MAX_SPAN;
    int ss[MAX_SPAN + 1];
#pragma unroll
    for (int j = 0; j <= MAX_SPAN; ++j) ss[j] = sse[j];
    // expansions per span slot j (d = 8 - j, begin b = e - d ascending)
    int pre[MAX_SPAN + 1];
    pre[0] = 0;
#pragma unroll
    for (int j = 0; j < MAX_SPAN; ++j) {
      const int d = MAX_SPAN - j;
      const int c = (d <= dmax) ? cnt[grp][(e - d) % RING] : 0;
      pre[j + 1] = pre[j] + c * (ss[j + 1] - ss[j]);
    }
    const int X = pre[MAX_SPAN];

    // lane-local top-k of this lane's expansions
    double ls[KT];
    uint32_t lg[KT];
#pragma unroll
    for (int q = 0; q < KT; ++q) { ls[q] = -INFINITY; lg[q] = INV; }

    for (int g = gl; g < X; g += G) {
      int j = 0;
#pragma unroll
      for (int q = 1; q < MAX_SPAN; ++q) j = (g >= pre[q]) ? q : j;
      const int m = ss[j + 1] - ss[j];
      const int local = g - pre[j];
      const int r = local / m;
      const int i = local - r * m;
      const int d = MAX_SPAN - j;
      const Entry& h = R[(e - d) % RING][r];
      const int64_t gn = nbase + ss[j] + i;
      const uint32_t km = p.nmask[gn];
      const uint32_t jm = h.jmask;
      // skip successive unknown words (beam.py:43-45): num_unk > 0 <=> wj is Unk
      if ((jm & F_UNK) && (km & F_UNK) && (d < dmax)) continue;

      double tri = 0.0;
      if (has_tri) {
        const uint32_t kw = (uint32_t)p.nword[gn], kmo = (uint32_t)p.nmorph[gn],
                       kt = (uint32_t)p.ntag[gn];
        const uint32_t jw = (uint32_t)h.jword, jmo = (uint32_t)h.jmorph, jt = (uint32_t)h.jtag;
        const uint32_t im = h.imask;
        const bool has_i = (im & F_WI) != 0;
        // keys of the probed classes, in feature order 0,1,2,3,7,8
        uint32_t ka[6], kb[6], kc[6], kcls[6];
        bool need[6];
        ka[0] = jw;  kb[0] = kw; kc[0] = kt; kcls[0] = 1;
        need[0] = (jm & J0A) && (km & K0B) && (km & K0C);
        ka[1] = jw;  kb[1] = kt; kc[1] = 0;  kcls[1] = 2;
        need[1] = (jm & J1A) && (km & K1B);
        ka[2] = jt;  kb[2] = kw; kc[2] = kt; kcls[2] = 3;
        need[2] = (jm & J2A) && (km & K2B) && (km & K2C);
        ka[3] = jt;  kb[3] = kt; kc[3] = 0;  kcls[3] = 4;
        need[3] = (jm & J3A) && (km & K3B);
        ka[4] = (uint32_t)h.iword; kb[4] = jw; kc[4] = kw; kcls[4] = 8;
        need[4] = has_i && (im & I7A) && (jm & J7B) && (km & K7C);
        // class 8: (wj.morph0 | wi.morph0, wk.morph0) (feature.py:113-119)
        bool emit8 = false;
        kb[5] = kmo; kc[5] = 0; kcls[5] = 9; ka[5] = 0; need[5] = false;
        if (km & F_CTX) {
          if (jm & F_CTX) {
            emit8 = true; ka[5] = jmo; need[5] = (jm & J8A) && (km & K8B);
          } else if (has_i && (im & F_CTX)) {
            emit8 = true; ka[5] = (uint32_t)h.imorph; need[5] = (im & I8A) && (km & K8B);
          }
        }
        uint32_t hh[6];
        Slot first[6];
#pragma unroll
        for (int q = 0; q < 6; ++q) {
          hh[q] = key_hash(ka[q], kb[q], kc[q], kcls[q] - 1u) & tmask;
          first[q].a = first[q].b = first[q].c = first[q].cls1 = 0u;
          first[q].coef = 0.0;
          if (need[q]) first[q] = load_slot(tab, hh[q]);
        }
        double v[9];
        bool pr[9];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          double cf = 0.0;
          pr[q] = need[q] && resolve(tab, tmask, hh[q], first[q], ka[q], kb[q], kc[q], kcls[q], cf);
          v[q] = cf;
        }
        pr[4] = (km & F_HAS4) != 0; v[4] = p.nf4[gn];
        pr[5] = (km & F_HAS5) != 0; v[5] = p.nf5[gn];
        pr[6] = (jm & F_HAS6) != 0; v[6] = h.f6;
        {
          double cf = 0.0;
          pr[7] = need[4] && resolve(tab, tmask, hh[4], first[4], ka[4], kb[4], kc[4], kcls[4], cf);
          v[7] = cf;
          cf = 0.0;
          pr[8] = need[5] && resolve(tab, tmask, hh[5], first[5], ka[5], kb[5], kc[5], kcls[5], cf);
          v[8] = cf;
        }
        tri = numpy_sum9(v, pr);
        if (COUNT) {
          n_tup += 6 + ((jm & F_UNK) ? 1 : 0) + (has_i ? 1 : 0) + (emit8 ? 1 : 0);
#pragma unroll
          for (int q = 0; q < 6; ++q) n_probe += need[q] ? 1 : 0;
        }
      }
      // inc = ((0 + pre...) + tri) + post...   (score_funcs.py:50-54)
      double inc = p.npre[gn] + tri;
      for (int t = 0; t < p.n_post; ++t) inc += p.npost[(int64_t)t * p.n_nodes + gn];
      const double sc = h.score + inc;       // Sequence.add (beam.py:115)
      if (COUNT) ++n_exp;

      // insert (sc, g) into the lane-local sorted list; g grows per lane, so
      // an equal score lands after the earlier expansion (stable).
      if (better(sc, (uint32_t)g, ls[KT - 1], lg[KT - 1])) {
        ls[KT - 1] = sc; lg[KT - 1] = (uint32_t)g;
#pragma unroll
        for (int q = KT - 1; q > 0; --q) {
          if (better(ls[q], lg[q], ls[q - 1], lg[q - 1])) {
            double ts = ls[q]; ls[q] = ls[q - 1]; ls[q - 1] = ts;
            uint32_t tg = lg[q]; lg[q] = lg[q - 1]; lg[q - 1] = tg;
          }
        }
      }
    }

    // merge: k rounds of group argmax over the lanes' list heads (beam.py:85)
    double sel_s = 0.0;
    uint32_t sel_g = INV;
    int nsel = 0;
    for (int t = 0; t < k; ++t) {
      double bs = ls[0];
      uint32_t bg = lg[0];
      group_argmax<G>(bs, bg);
      if (bg == INV) break;
      if (lg[0] == bg) {
#pragma unroll
        for (int q = 0; q < KT - 1; ++q) { ls[q] = ls[q + 1]; lg[q] = lg[q + 1]; }
        ls[KT - 1] = -INFINITY; lg[KT - 1] = INV;
      }
      if (gl == t) { sel_s = bs; sel_g = bg; }
      ++nsel;
    }

    // lanes t < nsel materialise beam[e][t] (Sequence.add, beam.py:112-116)
    Entry ne;
    uint32_t bpv = 0;
    const bool writer = gl < nsel;
    if (writer) {
      const int g = (int)sel_g;
      int j = 0;
#pragma unroll
      for (int q = 1; q < MAX_SPAN; ++q) j = (g >= pre[q]) ? q : j;
      const int m = ss[j + 1] - ss[j];
      const int local = g - pre[j];
      const int r = local / m;
      const int i = local - r * m;
      const int d = MAX_SPAN - j;
      const Entry& h = R[(e - d) % RING][r];
      const int node = ss[j] + i;
      const int64_t gn = nbase + node;
      ne.score = sel_s;
      ne.f6 = p.nf6[gn];
      ne.node = node;
      ne.jword = p.nword[gn];
      ne.jmorph = p.nmorph[gn];
      ne.jtag = p.ntag[gn];
      ne.jmask = p.nmask[gn];
      ne.iword = h.jword;
      ne.imorph = h.jmorph;
      ne.imask = h.jmask | F_WI;
      ne.depth = h.depth + 1;
      ne.pad[0] = ne.pad[1] = ne.pad[2] = 0;
      bpv = bp_pack((uint32_t)node, (uint32_t)d, (uint32_t)r);
    }
    __builtin_amdgcn_wave_barrier();
    if (writer) {
      R[e % RING][gl] = ne;
      bp[(int64_t)e * bstride + gl] = bpv;
    }
    if (gl == 0) cnt[grp][e % RING] = nsel;
    __builtin_amdgcn_wave_barrier();
  }

  // matures = beam[n] + EOS (beam.py:59-61); backtrace per mature rank
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  const int nm = cnt[grp][n % RING];
  if (gl == 0) p.out_count[s] = nm;
  if (gl >= nm && gl < k) {                  // unused mature slots read as empty
    p.out_score[(int64_t)s * k + gl] = 0.0;
    p.out_len[(int64_t)s * k + gl] = 0;
  }
  if (gl < nm) {
    const Entry& f = R[n % RING][gl];
    const int64_t o = (int64_t)s * k + gl;
    p.out_score[o] = f.score + 0.0;
    p.out_len[o] = f.depth;
    int32_t* codes = p.out_codes + (int64_t)k * p.cum_n[s] + (int64_t)gl * n;
    int pos = n, rank = gl;
    for (int step = f.depth - 1; step >= 0; --step) {
      const uint32_t v = bp[(int64_t)pos * bstride + rank];
      codes[step] = (int32_t)bp_node(v);
      pos -= (int)bp_d(v);
      rank = (int)bp_rank(v);
    }
  }
  if (COUNT) {
    n_exp = group_sum<G>(n_exp);
    n_tup = group_sum<G>(n_tup);
    n_probe = group_sum<G>(n_probe);
    if (gl == 0) {
      atomicAdd(p.counters + 0, n_exp);
      atomicAdd(p.counters + 1, n_tup);
      atomicAdd(p.counters + 2, n_probe);
    }
  }
}

template <int KT, int G, bool COUNT>
hipError_t launch_t(const DecodeParams& p, hipStream_t st) {
  constexpr int SPB = 256 / G;
  const int blocks = (p.n_sent + SPB - 1) / SPB;
  if (blocks == 0) return hipSuccess;
  hipLaunchKernelGGL((lt_decode_k<KT, G, COUNT>), dim3(blocks), dim3(256), 0, st, p);
  return hipGetLastError();
}

template <bool COUNT>
hipError_t launch_k(const DecodeParams& p, int kt, hipStream_t st) {
  switch (kt) {
    case 1: return launch_t<1, 16, COUNT>(p, st);
    case 2: return launch_t<2, 32, COUNT>(p, st);
    case 4: return launch_t<4, 32, COUNT>(p, st);
    case 8: return launch_t<8, 64, COUNT>(p, st);
    case 16: return launch_t<16, 64, COUNT>(p, st);
    case 32: return launch_t<32, 64, COUNT>(p, st);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace

namespace lt {

int beam_template_for(int k) {
  if (k <= 1) return 1;
  if (k <= 2) return 2;
  if (k <= 4) return 4;
  if (k <= 8) return 8;
  if (k <= 16) return 16;
  if (k <= 32) return 32;
  return -1;
}

hipError_t launch_decode(const DecodeParams& p, hipStream_t st, bool count) {
  const int kt = beam_template_for(p.k);
  return count ? launch_k<true>(p, kt, st) : launch_k<false>(p, kt, st);
}

}  // namespace lt
