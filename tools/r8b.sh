# Tagger.tag_batch first call after the per-phase breakdown: glibc heap trim check
# (MALLOC_TRIM_THRESHOLD_ raised so free() does not hand the heap top back to the kernel)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/tagger_calls
export PYTHONUNBUFFERED=1
MALLOC_TRIM_THRESHOLD_=17179869184 timeout -k 10 300 python3 -u tools/bench_tagger.py --sentences 65536 --k 1 --threads 16 --reps 2 --api-reps 5 > gpurun_out/tagger_calls/k1_default_notrim.log 2>&1 || { echo TB_FAIL; tail -20 gpurun_out/tagger_calls/k1_default_notrim.log; exit 1; }
tail -1 gpurun_out/tagger_calls/k1_default_notrim.log > gpurun_out/tagger_calls/k1_default_notrim.jsonl
python3 -c "import json;d=json.load(open('gpurun_out/tagger_calls/k1_default_notrim.jsonl'));print('notrim', [round(x) for x in d['tag_batch_api_runs_sentences_per_s']]);[print(s) for s in d['tag_batch_api_call_stats']]"
