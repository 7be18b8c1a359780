# The round's evidence, first half (gpu_evidence.sh split in two calls of
# < 20 min): smoke, every -m gpu test, the profile set (tools/gpu_prof.sh)
#   gpurun --timeout 1200 -- 'TAG=r06 bash tools/gpu_evidence_a.sh'
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r06}
O=$R/gpurun_out/evidence_$TAG
mkdir -p $O
cd $R
export PYTHONUNBUFFERED=1
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 \
  || { echo SMOKE_FAIL; tail -30 $O/smoke.log; exit 1; }
echo SMOKE_OK
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > $O/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -60 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
cd $R && TAG=$TAG bash tools/gpu_prof.sh || exit 1
cp $R/gpurun_out/prof_$TAG/traffic.json $O/traffic.json
echo EVIDENCE_A_OK
