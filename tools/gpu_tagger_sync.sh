# Host synchronisation inside Tagger.tag_batch (round-3 verdict: the k=1
# schedule must not block a chunk): a rocprofv3 kernel + HIP runtime trace of
# one tools/bench_tagger.py run, summarised per HIP call (count, total ms) and
# per kernel (tools/sync_summary.py).  Output gpurun_out/tagger_sync/.
#   gpurun -- 'K=1 bash tools/gpu_tagger_sync.sh'
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/tagger_sync
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export PYTHONUNBUFFERED=1
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d $O/trace -o run -- \
  python3 $R/tools/bench_tagger.py --sentences ${SENT:-16384} --k ${K:-1} --threads 16 --reps 1 --api-reps 1 \
  > $O/bench.log 2> $O/bench.err || { echo TRACE_FAIL; tail -20 $O/bench.log $O/bench.err; exit 1; }
python3 $R/tools/sync_summary.py $O/trace > $O/summary.txt || exit 1
cat $O/summary.txt
