# Half-wave beam kernel A/B: parity (LT_BEAM=hw for the beam tests), then k=5/4/8 timings vs pk.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
LT_BEAM=hw timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_tagger.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_hw.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_hw.log; exit 1; }
tail -1 gpurun_out/pytest_hw.log
for K in ${KS:-5 4 8}; do
for V in hw pk; do
LT_BEAM=$V timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 2 --k $K --no-cpu-baseline > gpurun_out/bench_${V}_k$K.log 2>&1 || { echo BENCH_FAIL; tail -30 gpurun_out/bench_${V}_k$K.log; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/bench_${V}_k$K.log').read().strip().splitlines()[-1]);print('$V k=$K', round(d['value']), 'kernel_ms', round(d['roofline']['avg_kernel_ms'],3), 'frac', round(d['roofline']['frac'],4), d['roofline']['kernel'])"
done
done
