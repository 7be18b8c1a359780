# round 6 call c: Tagger end to end with the four-stage pipeline (GPU Tagger
# tests first), the k=1 step against the batch size (multi-GPU model,
# DESIGN section 7) and the packed-result D2H at N = 1
set -o pipefail
mkdir -p gpurun_out/r6c
export PYTHONUNBUFFERED=1
TESTS=1 KS="1 5" timeout -k 10 900 bash tools/gpu_tagger_e2e.sh > gpurun_out/r6c/tagger.log 2>&1 && cat gpurun_out/r6c/tagger.log &&
cp gpurun_out/bench_tagger_k1.log gpurun_out/r6c/ && cp gpurun_out/bench_tagger_k5.log gpurun_out/r6c/ &&
for S in 8192 16384 32768 65536 131072; do
  timeout -k 10 300 python3 -u bench.py --sentences $S --steps 20 --warmup 3 --extra-k '' --no-cpu-baseline --no-check > gpurun_out/r6c/sweep_$S.log 2>&1 || { echo SWEEP_FAIL $S; tail -5 gpurun_out/r6c/sweep_$S.log; exit 1; }
  tail -1 gpurun_out/r6c/sweep_$S.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('S=$S', 'step_ms', round(d['ms_per_step'],4), 'kernel_ms', round(d['roofline']['avg_kernel_ms'],4), 'd2h_B', d['d2h']['bytes_per_step'])"
done &&
for M in padded packed padded packed; do
  timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 3 --extra-k '' --no-cpu-baseline --no-check --d2h $M > gpurun_out/r6c/d2h_$M.log 2>&1 || { echo D2H_FAIL $M; tail -5 gpurun_out/r6c/d2h_$M.log; exit 1; }
  tail -1 gpurun_out/r6c/d2h_$M.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('d2h=$M', 'step_ms', round(d['ms_per_step'],4), 'kernel_ms', round(d['roofline']['avg_kernel_ms'],4), 'd2h_B', d['d2h']['bytes_per_step'])"
done && echo ALL_DONE
