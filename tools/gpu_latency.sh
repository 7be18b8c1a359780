# Tagger.tag latency (one sentence per call) with a per-phase breakdown.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python3 -u tools/bench_tag_latency.py > gpurun_out/tag_latency.log 2>&1 || { echo LAT_FAIL; tail -30 gpurun_out/tag_latency.log; exit 1; }
tail -1 gpurun_out/tag_latency.log
