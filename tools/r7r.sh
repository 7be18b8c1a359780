# GPU suite (the lexicon's new hashing end to end through Tagger.tag_batch) and Tagger end to end
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/tagger_lk
export PYTHONUNBUFFERED=1
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/tagger_lk/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -60 gpurun_out/tagger_lk/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/tagger_lk/pytest_gpu.log
for K in 1 5; do
  timeout -k 10 300 python3 -u tools/bench_tagger.py --sentences 65536 --k $K --threads 16 --reps 2 --api-reps 5 > gpurun_out/tagger_lk/k$K.log 2>&1 || { echo TB_FAIL; tail -20 gpurun_out/tagger_lk/k$K.log; exit 1; }
  tail -1 gpurun_out/tagger_lk/k$K.log > gpurun_out/tagger_lk/tagger_e2e_k$K.jsonl
  python3 -c "import json;d=json.load(open('gpurun_out/tagger_lk/tagger_e2e_k$K.jsonl'));print('k=$K', [round(x) for x in d['tag_batch_api_runs_sentences_per_s']], {p: round(v, 3) for p, v in d['phase_s'].items()})"
done
