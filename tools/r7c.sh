# GPU suite + A/B: k=1 steady and fresh-batch steps with the fused fill on /
# off against the deadnp build, then k=5 / 16 / 2
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/ab
export PYTHONUNBUFFERED=1
timeout -k 10 900 python3 -u -m pytest tests -m gpu --maxfail 6 -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
L=$GRAFT_REPO_ROOT/lattice_based_tagger_amd/_lib
run() {  # tag lib fused k round
  F=gpurun_out/ab/$1_k$4_r$5.jsonl
  LT_K1_FUSED_FILL=$3 LT_LIBRARY=$2 timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 2 --k $4 --extra-k '' \
    --sentences 65536 --no-cpu-baseline --no-check > $F.log 2>&1 || { echo AB_FAIL $1 $4; tail -20 $F.log; exit 1; }
  tail -1 $F.log > $F
  python3 -c "import json;d=json.load(open('$F'));r=d['roofline'];fb=d.get('fresh_batch') or {};print('r$5 $1 k=$4', round(d['value']), 'ms', round(d['ms_per_step'],4), 'kernel_ms', round(r['avg_kernel_ms'],4), 'fresh_ms', fb.get('ms_per_step'), 'prep_ms', fb.get('prep_ms_last'))"
}
for R in 1 2; do
  run deadnp $L/liblt_deadnp.so 1 1 $R || exit 1
  run fused $L/liblt.so 1 1 $R || exit 1
  run nofuse $L/liblt.so 0 1 $R || exit 1
done
for R in 1 2; do for K in 5 16 2; do
  run deadnp $L/liblt_deadnp.so 1 $K $R || exit 1
  run base $L/liblt.so 1 $K $R || exit 1
done; done
