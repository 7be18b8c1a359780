# Round-3 evidence run, second session (part A): smoke, every -m gpu test,
# rocprofv3 kernel-trace stats and FETCH_SIZE / WRITE_SIZE traffic per k
# (profiles/${TAG}_traffic.json, read by the bench line), the default bench
# line (k=1 headline + k=5/16 extras, CPU baselines), k=1 phase stamps.
# Part B: tools/gpu_round3b_counters.sh.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r03b}
cd $R && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -30 gpurun_out/smoke.log; exit 1; }
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
TAG=$TAG KS="1 5 16" bash tools/gpu_profile_final.sh || { echo PROFILE_FAIL; exit 1; }
cp gpurun_out/final_$TAG/traffic.json profiles/${TAG}_traffic.json
python3 -c "import json; [print(e['kernel'], e['k'], e['traffic_bytes_per_launch']) for e in json.load(open('profiles/${TAG}_traffic.json'))]"
timeout -k 10 400 python3 -u bench.py > gpurun_out/bench_default.log 2>&1 || { echo BENCH_FAIL; tail -30 gpurun_out/bench_default.log; exit 1; }
tail -1 gpurun_out/bench_default.log | cut -c1-300
if [ -f lattice_based_tagger_amd/_lib/liblt_phases.so ]; then
LT_LIBRARY=$R/lattice_based_tagger_amd/_lib/liblt_phases.so timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 1 --k 1 --extra-k '' --no-cpu-baseline --no-check > gpurun_out/phases.log 2>&1 || { echo PHASES_FAIL; tail -30 gpurun_out/phases.log; exit 1; }
grep PK_PHASES gpurun_out/phases.log
fi
