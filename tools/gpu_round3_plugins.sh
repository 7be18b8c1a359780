set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_plugins.py tests/test_gpu_debug.py tests/test_gpu_parity.py tests/test_evaluate.py tests/test_gpu_wide.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_plugins.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_plugins.log; exit 1; }
tail -2 gpurun_out/pytest_plugins.log
KS="16 5 2" LIBS="bb1 bb0 bb1 bb0" bash tools/gpu_ab.sh
