set -o pipefail
mkdir -p gpurun_out/r6a
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r6a/pytest_gpu.log 2>&1 && tail -3 gpurun_out/r6a/pytest_gpu.log &&
LIBS="head base nod3x" KS="1 5 16" ROUNDS=2 STEPS=10 timeout -k 10 900 bash tools/gpu_ab.sh > gpurun_out/r6a/ab.log 2>&1 && cat gpurun_out/r6a/ab.log &&
OUT=r6a/sq LIBS="head base nod3x atom1" KS=1 timeout -k 10 600 bash tools/gpu_sq_ab.sh > gpurun_out/r6a/sq1.log 2>&1 &&
OUT=r6a/sq LIBS="head base" KS="5 16" timeout -k 10 600 bash tools/gpu_sq_ab.sh > gpurun_out/r6a/sq2.log 2>&1 && echo ALL_DONE
