# round 6 call f: nontemporal result stores at k=1 (K1_OUT_NT) and
# nontemporal HBM backpointer stores in every decoder (BM_BP_AUX=2) against
# the current build
set -o pipefail
mkdir -p gpurun_out/r6f
export PYTHONUNBUFFERED=1
LIBS="base outnt bpnt" KS="1 5 16" ROUNDS=2 STEPS=20 timeout -k 10 1000 bash tools/gpu_ab.sh > gpurun_out/r6f/ab.log 2>&1; rc=$?; cat gpurun_out/r6f/ab.log; [ $rc -eq 0 ] && echo ALL_DONE
