# parity tests, then beam benches for the default kernel and LT_BEAM=v1
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
export PYTHONUNBUFFERED=1
cd $R
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -30 gpurun_out/smoke.log; exit 1; }
if [ -z "$NOTEST" ]; then
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
fi
for K in ${KS:-5 16}; do
for V in ${BV:-v2 v1}; do
LT_BEAM=$V timeout -k 10 600 python3 -u bench.py --steps 5 --warmup 1 --k $K --no-cpu-baseline > gpurun_out/bench_b_${V}_k$K.log 2>&1 || { echo BENCH_FAIL $V $K; tail -30 gpurun_out/bench_b_${V}_k$K.log; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/bench_b_${V}_k$K.log').read().strip().splitlines()[-1]);print('$V k=$K', round(d['value']), 'sents/s kernel_ms', round(d['roofline']['avg_kernel_ms'],3), 'frac', round(d['roofline']['frac'],4))"
done
done
