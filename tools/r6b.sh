# round 6 call b: the k=1 lane-pair pre-reduction (PK_PAIR_MAX=1) against the
# current build -- its parity first, then the GPU suite, an interleaved A/B and
# SQ / LDS counters of both
set -o pipefail
mkdir -p gpurun_out/r6b
export PYTHONUNBUFFERED=1
LT_LIBRARY=$PWD/lattice_based_tagger_amd/_lib/liblt_pair.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r6b/pytest_pair_parity.log 2>&1 && tail -2 gpurun_out/r6b/pytest_pair_parity.log &&
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r6b/pytest_gpu.log 2>&1 && tail -2 gpurun_out/r6b/pytest_gpu.log &&
LIBS="base pair" KS="1" ROUNDS=3 STEPS=20 timeout -k 10 600 bash tools/gpu_ab.sh > gpurun_out/r6b/ab.log 2>&1 && cat gpurun_out/r6b/ab.log &&
OUT=r6b/sq LIBS="base pair" KS=1 timeout -k 10 400 bash tools/gpu_sq_ab.sh > gpurun_out/r6b/sq.log 2>&1 && cat gpurun_out/r6b/sq.log && echo ALL_DONE
