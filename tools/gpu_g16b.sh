set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_tagger.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_g.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_g.log; exit 1; }
tail -1 gpurun_out/pytest_g.log
for V in "0 2" "0 3" "16 4" "32 4" "0 5" "0 8"; do set -- $V
if [ "$1" = "0" ]; then unset LT_BEAM_G; else export LT_BEAM_G=$1; fi
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 2 --k $2 --no-cpu-baseline > gpurun_out/bench_g$1_k$2.log 2>&1 || { echo BENCH_FAIL; tail -30 gpurun_out/bench_g$1_k$2.log; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/bench_g$1_k$2.log').read().strip().splitlines()[-1]);print('G=$1 k=$2', round(d['value']), 'kernel_ms', round(d['roofline']['avg_kernel_ms'],3), 'frac', round(d['roofline']['frac'],4))"
done
