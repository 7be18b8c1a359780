# Beam kernels: parity tests, then kernel time per beam width (pk = one sentence per wave, pw = packed).
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_bc.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_bc.log; exit 1; }
tail -1 gpurun_out/pytest_bc.log
for K in ${KS:-2 5 16}; do
for V in ${VS:-pk pw}; do
LT_BEAM=$V timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 2 --k $K --no-cpu-baseline > gpurun_out/bench_${V}_k$K.log 2>&1 || { echo BENCH_FAIL; tail -30 gpurun_out/bench_${V}_k$K.log; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/bench_${V}_k$K.log').read().strip().splitlines()[-1]);print('$V k=$K', round(d['value']), 'kernel_ms', round(d['roofline']['avg_kernel_ms'],3), 'frac', round(d['roofline']['frac'],4), d['roofline']['kernel'])"
done
done
