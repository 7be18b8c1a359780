# Tagger end-to-end bench (k = 1, 5): per-phase times and three timed
# tag_batch calls each -> profiles-ready JSON lines.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for K in 1 5; do
timeout -k 10 300 python3 -u tools/bench_tagger.py --sentences 65536 --k $K --threads 16 --reps 2 --api-reps 3 > gpurun_out/bench_tagger_k$K.log 2>&1 || { echo TB_FAIL; tail -30 gpurun_out/bench_tagger_k$K.log; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/bench_tagger_k$K.log').read().strip().splitlines()[-1]);print('k=$K', [round(x) for x in d['tag_batch_api_runs_sentences_per_s']])"
done
