set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_gather.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_parity.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_parity.log; exit 1; }
tail -3 gpurun_out/pytest_parity.log
timeout -k 10 400 python3 -u bench.py > gpurun_out/bench_default.log 2>&1 || { echo BENCH_FAIL; tail -30 gpurun_out/bench_default.log; exit 1; }
python3 -c "
import json;d=json.loads(open('gpurun_out/bench_default.log').read().strip().splitlines()[-1])
print('k=1', round(d['value']), round(d['ms_per_step'],3), round(d['roofline']['avg_kernel_ms'],3), round(d['roofline']['frac'],3))
for k,v in d['extra'].items(): print(k, round(v['value']), round(v['ms_per_step'],3), round(v['avg_kernel_ms'],3), round(v['roofline']['frac'],3), v['kernel'])
print(d['cpu_baseline']['value'], d['cpu_baseline_c']['value'])"
