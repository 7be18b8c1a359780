# final-state check: smoke, the GPU suite, one default bench line (k=1 + extras, CPU baselines off)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/final
export PYTHONUNBUFFERED=1
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -30 gpurun_out/final/smoke.log; exit 1; }
echo SMOKE_OK
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/final/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -60 gpurun_out/final/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/final/pytest_gpu.log
timeout -k 10 600 python3 -u bench.py --no-cpu-baseline > gpurun_out/final/bench.log 2>&1 || { echo BENCH_FAIL; tail -30 gpurun_out/final/bench.log; exit 1; }
tail -1 gpurun_out/final/bench.log > gpurun_out/final/bench.jsonl
python3 -c "import json;d=json.load(open('gpurun_out/final/bench.jsonl'));r=d['roofline'];print('k=1', round(d['value']), 'kernel_ms', round(r['avg_kernel_ms'],4), 'frac', round(r['frac'],4), 'fresh', d['fresh_batch']['ms_per_step'], 'sched_ms', d['host']['sched_ms'], {k: round(v['avg_kernel_ms'],3) for k, v in d['extra'].items()})"
