# Kernel trace of the bench step (decode + pack + slab copy) at k=1.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 3 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/bench_step.log 2>&1 || { echo BENCH_FAIL; tail -30 gpurun_out/bench_step.log; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/bench_step.log').read().strip().splitlines()[-1]);print(round(d['value']), 'sents/s ms/step', round(d['ms_per_step'],3), 'kernel_ms', round(d['roofline']['avg_kernel_ms'],3))"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_step -o run -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-check ${BENCH_ARGS} > $R/gpurun_out/prof_step.log 2>&1 || { echo PROF_FAIL; tail -20 $R/gpurun_out/prof_step.log; exit 1; }
find $R/gpurun_out/prof_step -name "*kernel_stats.csv" | head -1 | xargs cut -d, -f1-8 | head -20
