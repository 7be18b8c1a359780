# GPU suite + A/B: k=1 record DMA early in the macro-step and asm argmax atomics
# (base) against asm atomics only (asmonly) and neither (k1old); lt_beam_pk's
# single-round ranking by list position (base) against the generation compare (pkold)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python3 -u -m pytest tests -m gpu --maxfail 6 -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
LIBS="k1old asmonly base" KS="1" ROUNDS=2 bash tools/gpu_ab.sh || exit 1
LIBS="pkold base" KS="16 12" ROUNDS=2 bash tools/gpu_ab.sh
