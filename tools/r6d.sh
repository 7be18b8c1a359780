# round 6 call d: the GPU suite with several-trigram composites (golden set
# multitri, general kernel, evaluate, debug dump), then the N = 1 step with
# packed results over the SDMA copy against the padded results
set -o pipefail
mkdir -p gpurun_out/r6d
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r6d/pytest_gpu.log 2>&1; rc=$?; tail -5 gpurun_out/r6d/pytest_gpu.log; [ $rc -eq 0 ] &&
for M in padded packed padded packed; do
  timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 3 --extra-k '' --no-cpu-baseline --no-check --d2h $M > gpurun_out/r6d/d2h_$M.log 2>&1 || { echo D2H_FAIL $M; tail -5 gpurun_out/r6d/d2h_$M.log; exit 1; }
  tail -1 gpurun_out/r6d/d2h_$M.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('d2h=$M', 'step_ms', round(d['ms_per_step'],4), 'kernel_ms', round(d['roofline']['avg_kernel_ms'],4), 'd2h_B', d['d2h']['bytes_per_step'])"
done && echo ALL_DONE
