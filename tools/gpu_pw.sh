# Beam kernel A/B: parity tests for the beam widths, then bench k=5 (and k=2, 4) with
# the packed-wave kernel and with LT_BEAM=pk (one sentence per wave).
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_tagger.py tests/test_gpu_gather.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_pw.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_pw.log; exit 1; }
tail -2 gpurun_out/pytest_pw.log
for K in ${KS:-5 2 4}; do
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 2 --k $K --no-cpu-baseline > gpurun_out/bench_pw_k$K.log 2>&1 || { echo BENCH_FAIL; tail -30 gpurun_out/bench_pw_k$K.log; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/bench_pw_k$K.log').read().strip().splitlines()[-1]);print('pw k=$K', round(d['value']), 'kernel_ms', round(d['roofline']['avg_kernel_ms'],3), 'frac', round(d['roofline']['frac'],4), d['roofline']['kernel'])"
LT_BEAM=pk timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 2 --k $K --no-cpu-baseline > gpurun_out/bench_pk_k$K.log 2>&1 || { echo BENCH_FAIL; tail -30 gpurun_out/bench_pk_k$K.log; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/bench_pk_k$K.log').read().strip().splitlines()[-1]);print('pk k=$K', round(d['value']), 'kernel_ms', round(d['roofline']['avg_kernel_ms'],3), 'frac', round(d['roofline']['frac'],4), d['roofline']['kernel'])"
done
