# A/B of the span starts through LDS in lt_beam_hw ("ss") against the bit-scan
# sum build ("sum9"), then the beam parity tests.
set -o pipefail
KS="5 2 4 3 8" LIBS="sum9 ss sum9 ss" bash tools/gpu_ab.sh || exit 1
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_plugins.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_ss.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_ss.log; exit 1; }
tail -1 gpurun_out/pytest_ss.log
