# A/B of experiment builds: for each LIBS tag (lattice_based_tagger_amd/_lib/liblt_<tag>.so)
# and each beam in KS, one short bench line (kernel ms, sentences/s).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
export PYTHONUNBUFFERED=1
cd $R
for K in ${KS:-1}; do
for T in ${LIBS}; do
LT_LIBRARY=$R/lattice_based_tagger_amd/_lib/liblt_$T.so timeout -k 10 300 python3 -u bench.py --steps ${STEPS:-10} --warmup 2 --k $K --extra-k '' --no-cpu-baseline --no-check > gpurun_out/ab_${T}_k$K.log 2>&1 || { echo AB_FAIL $T $K; tail -20 gpurun_out/ab_${T}_k$K.log; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/ab_${T}_k$K.log').read().strip().splitlines()[-1]);print('$T k=$K', round(d['value']), 'kernel_ms', round(d['roofline']['avg_kernel_ms'],4), 'frac', round(d['roofline']['frac'],4))"
done
done
