set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_tagger.py tests/test_gpu_gather.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_tagger.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_tagger.log; exit 1; }
tail -6 gpurun_out/pytest_tagger.log
