# Full GPU check: smoke, every -m gpu test, tagger end-to-end bench, bench k=1.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -30 gpurun_out/smoke.log; exit 1; }
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python3 -u tools/bench_tagger.py --sentences 65536 --k 1 --threads 16 > gpurun_out/bench_tagger_k1.log 2>&1 || { echo TB_FAIL; tail -30 gpurun_out/bench_tagger_k1.log; exit 1; }
tail -1 gpurun_out/bench_tagger_k1.log
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 3 > gpurun_out/bench_default.log 2>&1 || { echo BENCH_FAIL; tail -30 gpurun_out/bench_default.log; exit 1; }
tail -1 gpurun_out/bench_default.log
