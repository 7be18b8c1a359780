# GPU suite at the bit-window class-3 index, A/B against the build before it (prevd3),
# and the two-rank bench path on one GPU with each rank copying its own results (--gather 0)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python3 -u -m pytest tests -m gpu --maxfail 6 -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
LIBS="prevd3 base" KS="1 2 3" ROUNDS=2 bash tools/gpu_ab.sh || exit 1
TAG=_local ARGS="--gather 0" bash tools/gpu_rehearse_n2.sh
