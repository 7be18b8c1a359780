set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -30 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
TAG=r01c KS="2 5" bash $R/tools/gpu_profile_final.sh || exit 1
cd $R
for K in 3 8; do
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 2 --k $K --no-cpu-baseline > gpurun_out/bench_k$K.log 2>&1 || { echo BENCH_FAIL; tail -30 gpurun_out/bench_k$K.log; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/bench_k$K.log').read().strip().splitlines()[-1]);print('k=$K', round(d['value']), 'kernel_ms', round(d['roofline']['avg_kernel_ms'],3), 'frac', round(d['roofline']['frac'],4), d['roofline']['kernel'])"
done
