# A/B of the bit-scan 8-9 term sum ("sum9") against HEAD ("base"), then the
# parity suites (the golden 'dense' set holds 8- and 9-term expansions).
set -o pipefail
KS="5 1 16 2" LIBS="base sum9 base sum9" bash tools/gpu_ab.sh || exit 1
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_plugins.py tests/test_gpu_api.py tests/test_gpu_debug.py tests/test_gpu_wide.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_sum9.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_sum9.log; exit 1; }
tail -1 gpurun_out/pytest_sum9.log
