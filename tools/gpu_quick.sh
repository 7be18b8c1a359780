# Quick perf check: smoke, bench (k list), one TA/SQ counter pass.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
export PYTHONUNBUFFERED=1
cd $R
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -30 gpurun_out/smoke.log; exit 1; }
for K in ${KS:-1}; do
timeout -k 10 600 python3 -u bench.py --steps 10 --warmup 2 --k $K --no-cpu-baseline > gpurun_out/bench_k$K.log 2>&1 || { echo BENCH_FAIL; tail -30 gpurun_out/bench_k$K.log; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/bench_k$K.log').read().strip().splitlines()[-1]);print('k=$K', round(d['value']), 'sents/s kernel_ms', round(d['roofline']['avg_kernel_ms'],3), 'frac', round(d['roofline']['frac'],4))"
done
if [ -n "$PROF" ]; then
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc TA_BUSY_avr TA_TA_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum -T --output-format csv -d $R/gpurun_out/prof_q -o run -- python3 $R/bench.py --no-cpu-baseline --steps 2 --warmup 1 --k ${PROFK:-1} > $R/gpurun_out/prof_q.log 2>&1 && python3 $R/tools/summarize_prof.py $R/gpurun_out/prof_q lt_
fi
