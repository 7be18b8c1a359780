# k=1 kernel variants: bench each (LT_VITERBI=...) after smoke + parity tests.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
export PYTHONUNBUFFERED=1
cd $R
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -30 gpurun_out/smoke.log; exit 1; }
if [ -z "$NOTEST" ]; then
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
fi
# a variant is LT_VITERBI[+nod3][+hot][+kN]
for V in ${VARIANTS:-row16 pk6}; do
VK=${V%%+*}; D3=1; HOT=0; KK=1
case "$V" in *+nod3*) D3=0;; esac
case "$V" in *+hot*) HOT=1;; esac
case "$V" in *+k*) KK=${V##*+k};; esac
LT_D3=$D3 LT_HOT=$HOT LT_VITERBI=$VK timeout -k 10 600 python3 -u bench.py --steps 10 --warmup 2 --k $KK --no-cpu-baseline > gpurun_out/bench_v_$V.log 2>&1 || { echo BENCH_FAIL $V; tail -30 gpurun_out/bench_v_$V.log; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/bench_v_$V.log').read().strip().splitlines()[-1]);print('$V', round(d['value']), 'sents/s kernel_ms', round(d['roofline']['avg_kernel_ms'],3), 'frac', round(d['roofline']['frac'],4))"
done
