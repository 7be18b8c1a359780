set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -30 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
for V in "hw 2" "def 2" "def 3" "def 5"; do set -- $V; 
LT_BEAM=$1 timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 2 --k $2 --no-cpu-baseline > gpurun_out/bench_$1_k$2.log 2>&1 || { echo BENCH_FAIL; tail -30 gpurun_out/bench_$1_k$2.log; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/bench_$1_k$2.log').read().strip().splitlines()[-1]);print('$1 k=$2', round(d['value']), 'kernel_ms', round(d['roofline']['avg_kernel_ms'],3), 'frac', round(d['roofline']['frac'],4), d['roofline']['kernel'])"
done
