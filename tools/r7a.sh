# parity suite + interleaved A/B (old = HEAD build, base = working tree)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python3 -u -m pytest tests -m gpu --maxfail 6 -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
LIBS="${LIBS:-old base}" KS="${KS:-1 5 16}" ROUNDS=${ROUNDS:-2} bash tools/gpu_ab.sh
