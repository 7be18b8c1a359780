# A/B of library builds on the bench, interleaved to average out box drift.
#   LIBS    tags of experiment builds: tag "base" is the in-tree liblt.so, any
#           other tag T is lattice_based_tagger_amd/_lib/liblt_T.so, built
#           beforehand on the CPU side, e.g.
#             python -m lattice_based_tagger_amd._build -DBM_DEDUP=0 -o lattice_based_tagger_amd/_lib/liblt_nodedup.so
#   KS      beams (default 1), ROUNDS interleaved passes (default 2),
#   STEPS   timed steps per line (default 10), SENT sentences (default 65536).
# One line per (round, k, tag): kernel ms, sentences/s; the raw JSON lines in
# gpurun_out/ab/<tag>_k<k>_r<round>.jsonl.
#   gpurun -- 'LIBS="base nodedup" KS="5 16" bash tools/gpu_ab.sh'
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/ab
mkdir -p $O
export PYTHONUNBUFFERED=1
cd $R
for RD in $(seq 1 ${ROUNDS:-2}); do
for K in ${KS:-1}; do
for T in ${LIBS:-base}; do
  if [ "$T" = base ]; then LIB=$R/lattice_based_tagger_amd/_lib/liblt.so; else LIB=$R/lattice_based_tagger_amd/_lib/liblt_$T.so; fi
  F=$O/${T}_k${K}_r$RD.jsonl
  LT_LIBRARY=$LIB timeout -k 10 300 python3 -u bench.py --steps ${STEPS:-10} --warmup 2 --k $K --extra-k '' \
    --sentences ${SENT:-65536} --no-cpu-baseline --no-check > $F.log 2>&1 || { echo AB_FAIL $T $K; tail -20 $F.log; exit 1; }
  tail -1 $F.log > $F
  python3 -c "import json;d=json.load(open('$F'));r=d['roofline'];print('r$RD $T k=$K', round(d['value']), 'sents/s kernel_ms', round(r['avg_kernel_ms'],4), 'frac', round(r['frac'],4), 'fresh_ms', (d.get('fresh_batch') or {}).get('ms_per_step'))"
done
done
done
