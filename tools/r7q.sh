# Tagger.tag_batch end to end at the final build: five timed calls each at k = 1 and 5
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/tagger_final
export PYTHONUNBUFFERED=1
for K in 1 5; do
  timeout -k 10 300 python3 -u tools/bench_tagger.py --sentences 65536 --k $K --threads 16 --reps 2 --api-reps 5 > gpurun_out/tagger_final/k$K.log 2>&1 || { echo TB_FAIL; tail -20 gpurun_out/tagger_final/k$K.log; exit 1; }
  tail -1 gpurun_out/tagger_final/k$K.log > gpurun_out/tagger_final/tagger_e2e_k$K.jsonl
  python3 -c "import json;d=json.load(open('gpurun_out/tagger_final/tagger_e2e_k$K.jsonl'));print('k=$K', [round(x) for x in d['tag_batch_api_runs_sentences_per_s']], {p: round(v, 3) for p, v in d['phase_s'].items()})"
done
