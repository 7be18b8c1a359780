set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 200 python3 -u -m pytest tests/test_gpu_parity.py -k several_launches -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_split.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/pytest_split.log; exit 1; }
tail -1 gpurun_out/pytest_split.log
timeout -k 10 300 python3 -u tools/bench_tagger.py --sentences 65536 --k 1 --threads 16 > gpurun_out/bench_tagger_k1.log 2>&1 || { echo TB_FAIL; tail -30 gpurun_out/bench_tagger_k1.log; exit 1; }
tail -1 gpurun_out/bench_tagger_k1.log
timeout -k 10 300 python3 -u tools/bench_tagger.py --sentences 65536 --k 5 --threads 16 > gpurun_out/bench_tagger_k5.log 2>&1 || { echo TB_FAIL; tail -30 gpurun_out/bench_tagger_k5.log; exit 1; }
tail -1 gpurun_out/bench_tagger_k5.log
