set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -30 gpurun_out/smoke.log; exit 1; }
echo SMOKE_OK
timeout -k 10 900 python3 -u -m pytest tests -m gpu --maxfail 6 -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 600 python3 -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_k1.log 2>&1 || { echo BENCH_FAIL; tail -30 gpurun_out/bench_k1.log; exit 1; }
tail -c 3000 gpurun_out/bench_k1.log
