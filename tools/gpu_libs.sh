# A/B of experiment builds (LT_LIBRARY=_lib/liblt_<tag>.so) on the k=1 bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
export PYTHONUNBUFFERED=1
cd $R
for T in ${LIBS}; do
LT_LIBRARY=$R/lattice_based_tagger_amd/_lib/liblt_$T.so timeout -k 10 600 python3 -u bench.py --steps 10 --warmup 2 --k ${K:-1} --no-cpu-baseline > gpurun_out/bench_lib_$T.log 2>&1 || { echo BENCH_FAIL $T; tail -30 gpurun_out/bench_lib_$T.log; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/bench_lib_$T.log').read().strip().splitlines()[-1]);print('$T', round(d['value']), 'sents/s kernel_ms', round(d['roofline']['avg_kernel_ms'],3), 'frac', round(d['roofline']['frac'],4))"
done
