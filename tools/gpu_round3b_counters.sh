# Round-3 evidence run, second session (part B): the counter set of the
# shipping kernels at k = 1, 5, 16 (tools/gpu_counters.sh), then
# Tagger.tag_batch end to end at k = 1, 5.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
KS="1 5 16" CALIB=0 bash tools/gpu_counters.sh || { echo COUNTERS_FAIL; exit 1; }
bash tools/gpu_tagger_e2e.sh
