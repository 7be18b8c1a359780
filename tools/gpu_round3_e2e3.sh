# Tagger e2e diagnostics: batch-create phase timings (LT_TIMING=1) of one
# pipelined tag_batch call, then the pipeline chunk sweep.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
LT_TIMING=1 timeout -k 10 300 python3 -u tools/bench_tagger.py --sentences 65536 --k 1 --threads 16 --reps 1 --api-reps 2 > gpurun_out/tagger_timing.log 2> gpurun_out/tagger_timing.err || { echo TIMING_FAIL; tail -20 gpurun_out/tagger_timing.err; exit 1; }
grep LT_TIMING gpurun_out/tagger_timing.err | tail -4
python3 -c "import json;d=json.loads(open('gpurun_out/tagger_timing.log').read().strip().splitlines()[-1]);print([round(x) for x in d['tag_batch_api_runs_sentences_per_s']], {p: round(v, 3) for p, v in d['phase_s'].items()})"
bash tools/gpu_tagger_chunks.sh
