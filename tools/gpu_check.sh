# Development check on the GPU box: smoke, selected -m gpu tests ($TESTS,
# default all), one bench line per $KS (default 1).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -30 gpurun_out/smoke.log; exit 1; }
timeout -k 10 900 python3 -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
for K in ${KS:-1}; do
timeout -k 10 600 python3 -u bench.py --steps 20 --warmup 3 --k $K ${BENCH_ARGS:---no-cpu-baseline} > gpurun_out/bench_k$K.log 2>&1 || { echo BENCH_FAIL; tail -30 gpurun_out/bench_k$K.log; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/bench_k$K.log').read().strip().splitlines()[-1]);print('k=$K', round(d['value']), 'sents/s ms/step', round(d['ms_per_step'],3), 'kernel_ms', round(d['roofline']['avg_kernel_ms'],3), 'frac', round(d['roofline']['frac'],4), 'kfrac', round(d['roofline']['kernel_bytes_frac'],4), 'd2h', d['d2h']['bytes_per_step'], d['check'])"
done
