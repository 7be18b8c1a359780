# Profile set of the bench in one gpurun call (TAG names the output):
#   1. rocprofv3 kernel trace of the default bench line (k=1 headline, fresh
#      batch, k=5 / k=16 extras) -> per-kernel stats with the warm-up launches
#      dropped (tools/kstats.py: the first WARM dispatches of every kernel);
#   2. separate FETCH_SIZE and WRITE_SIZE counter passes per k (KS) ->
#      traffic.json (tools/traffic_summary.py, tagged with bench.LAYOUT).
# Run:  gpurun -- 'TAG=r04 bash tools/gpu_prof.sh'
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r04}
O=$R/gpurun_out/prof_$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export PYTHONUNBUFFERED=1
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/trace -o run -- \
  python3 $R/bench.py --steps ${STEPS:-20} --warmup ${WARM:-3} --no-cpu-baseline > $O/bench_traced.log 2>&1 \
  || { echo TRACE_FAIL; tail -20 $O/bench_traced.log; exit 1; }
python3 $R/tools/kstats.py $O/trace ${WARM:-3} $O/kernel_stats.csv || exit 1
tail -1 $O/bench_traced.log > $O/bench_traced.jsonl
for K in ${KS:-1 5 16}; do
  KN=$(python3 -c "import sys; sys.path.insert(0,'$R'); from lattice_based_tagger_amd import _capi; print(_capi.load().lt_kernel_name($K).decode())")
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $C -T --output-format csv -d $O/${C}_k$K -o run -- \
      python3 $R/bench.py --steps 2 --warmup 1 --k $K --extra-k "" --no-cpu-baseline > $O/${C}_k$K.log 2>&1 \
      || { echo PMC_FAIL $C $K; tail -5 $O/${C}_k$K.log; exit 1; }
  done
  python3 $R/tools/traffic_summary.py $O/traffic.json $O/FETCH_SIZE_k$K $O/WRITE_SIZE_k$K $KN $K 65536 1000000 0 || exit 1
done
echo PROF_OK
