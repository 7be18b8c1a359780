set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -30 gpurun_out/smoke.log; exit 1; }
timeout -k 10 900 python3 -u -m pytest ${TESTS:-tests/test_gpu_parity.py tests/test_gpu_plugins.py} -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_k1.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_k1.log; exit 1; }
tail -2 gpurun_out/pytest_k1.log
KS="${KS:-1}" LIBS="${LIBS:-bb1 sch bb1 sch}" bash tools/gpu_ab.sh
