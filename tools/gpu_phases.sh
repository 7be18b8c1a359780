# Phase stamps of lt_viterbi_pk (k=1) and lt_beam_hw (k=2..8) (diagnostic
# build, -DPK_PHASES): per-wave cycles spent in each part of the macro-step /
# position (lt_decode.hip PK_STAMP), from the counting call of bench.py,
# beside the shipping library's bench line.
#   LIBS="phases ..." (liblt_<tag>.so), PKS (beams of the stamped runs),
#   KS (beams of the plain bench)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
export PYTHONUNBUFFERED=1
cd $R
for T in ${LIBS:-phases}; do
for PK in ${PKS:-1}; do
LT_LIBRARY=$R/lattice_based_tagger_amd/_lib/liblt_$T.so timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 1 --k $PK --extra-k '' --no-cpu-baseline --no-check > gpurun_out/phases_${T}_k$PK.log 2>&1 || { echo PHASES_FAIL $T; tail -30 gpurun_out/phases_${T}_k$PK.log; exit 1; }
grep PK_PHASES gpurun_out/phases_${T}_k$PK.log
done
done
for K in ${KS:-1}; do
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 3 --k $K --no-cpu-baseline > gpurun_out/bench_k$K.log 2>&1 || { echo BENCH_FAIL; tail -30 gpurun_out/bench_k$K.log; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/bench_k$K.log').read().strip().splitlines()[-1]);print('k=$K', round(d['value']), 'sents/s ms/step', round(d['ms_per_step'],3), 'kernel_ms', round(d['roofline']['avg_kernel_ms'],3), 'frac', round(d['roofline']['frac'],4))"
done
