# Tagger.tag_batch per-call stage times (last_stats): the first timed call against the warm ones,
# after the per-phase breakdown (default order) and right after the warm-up (--api-first)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/tagger_calls
export PYTHONUNBUFFERED=1
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_tagger.py -m gpu -q --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/tagger_calls/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/tagger_calls/pytest.log; exit 1; }
tail -1 gpurun_out/tagger_calls/pytest.log
for MODE in default api_first; do
  F=""; [ $MODE = api_first ] && F="--api-first"
  timeout -k 10 300 python3 -u tools/bench_tagger.py --sentences 65536 --k 1 --threads 16 --reps 2 --api-reps 5 $F > gpurun_out/tagger_calls/k1_$MODE.log 2>&1 || { echo TB_FAIL; tail -20 gpurun_out/tagger_calls/k1_$MODE.log; exit 1; }
  tail -1 gpurun_out/tagger_calls/k1_$MODE.log > gpurun_out/tagger_calls/k1_$MODE.jsonl
  python3 -c "import json;d=json.load(open('gpurun_out/tagger_calls/k1_$MODE.jsonl'));print('$MODE', [round(x) for x in d['tag_batch_api_runs_sentences_per_s']]);[print(s) for s in d['tag_batch_api_call_stats']]"
done
