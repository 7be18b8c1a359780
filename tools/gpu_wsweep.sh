# lt_viterbi_pk sentences-per-wave (W) at strong-scaling shard sizes.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
for S in 8192 16384 32768; do
for W in pk4 pk5 default; do
LT_VITERBI=$W timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-check --sentences $S > gpurun_out/w_${S}_$W.log 2>&1 || { echo FAIL; tail -20 gpurun_out/w_${S}_$W.log; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/w_${S}_$W.log').read().strip().splitlines()[-1]);print('S=$S W=$W', round(d['value']), 'ms/step', round(d['ms_per_step'],4), 'kernel_ms', round(d['roofline']['avg_kernel_ms'],4))"
done; done
