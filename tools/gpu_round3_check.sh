# Round-3 development check: every -m gpu test, the default bench line (k=1
# headline + k=5/16 extras), and the k=1 phase stamps of the diagnostic build.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -30 gpurun_out/smoke.log; exit 1; }
timeout -k 10 900 python3 -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 400 python3 -u bench.py ${BENCH_ARGS} > gpurun_out/bench_default.log 2>&1 || { echo BENCH_FAIL; tail -30 gpurun_out/bench_default.log; exit 1; }
python3 -c "
import json;d=json.loads(open('gpurun_out/bench_default.log').read().strip().splitlines()[-1])
print('k=1', round(d['value']), round(d['ms_per_step'],3), round(d['roofline']['avg_kernel_ms'],3), round(d['roofline']['frac'],3))
for k,v in (d.get('extra') or {}).items(): print(k, round(v['value']), round(v['ms_per_step'],3), round(v['avg_kernel_ms'],3), round(v['roofline']['frac'],3), v['kernel'])
cb = d.get('cpu_baseline') or {}
print('cpu', cb.get('value'), (d.get('cpu_baseline_c') or {}).get('value'))"
if [ -f lattice_based_tagger_amd/_lib/liblt_phases.so ]; then
LT_LIBRARY=$PWD/lattice_based_tagger_amd/_lib/liblt_phases.so timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 1 --k 1 --no-cpu-baseline --no-check --extra-k '' > gpurun_out/phases.log 2>&1 || { echo PHASES_FAIL; tail -30 gpurun_out/phases.log; exit 1; }
grep PK_PHASES gpurun_out/phases.log
fi
