# Round profile set for the committed bench numbers: rocprofv3 kernel-trace
# stats of bench.py per k, then separate FETCH_SIZE / WRITE_SIZE passes per k
# (-> profiles/<tag>_traffic.json via tools/traffic_summary.py).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r01}
O=$R/gpurun_out/final_$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for K in ${KS:-1 5 16}; do
  KN=$(python3 -c "import sys; sys.path.insert(0,'$R'); from lattice_based_tagger_amd import _capi; print(_capi.load().lt_kernel_name($K).decode())")
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/trace_k$K -o run -- python3 $R/bench.py --steps ${TRACE_STEPS:-10} --warmup 2 --k $K --extra-k "" --no-cpu-baseline > $O/trace_k$K.log 2>&1 || { echo TRACE_FAIL $K; tail -5 $O/trace_k$K.log; exit 1; }
  timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d $O/fetch_k$K -o run -- python3 $R/bench.py --steps 2 --warmup 1 --k $K --extra-k "" --no-cpu-baseline > $O/fetch_k$K.log 2>&1 || { echo FETCH_FAIL $K; tail -5 $O/fetch_k$K.log; exit 1; }
  timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -T --output-format csv -d $O/write_k$K -o run -- python3 $R/bench.py --steps 2 --warmup 1 --k $K --extra-k "" --no-cpu-baseline > $O/write_k$K.log 2>&1 || { echo WRITE_FAIL $K; tail -5 $O/write_k$K.log; exit 1; }
  python3 $R/tools/traffic_summary.py $O/traffic.json $O/fetch_k$K $O/write_k$K $KN $K 65536 1000000 0 || exit 1
done
