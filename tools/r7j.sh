# Tagger.tag_batch: five timed calls right after the warm-up (--api-first) and after the phase breakdown
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/tagger_order
export PYTHONUNBUFFERED=1
for K in 1 5; do
  for MODE in first after; do
    F=""; [ $MODE = first ] && F=--api-first
    timeout -k 10 300 python3 -u tools/bench_tagger.py --sentences 65536 --k $K --threads 16 --reps 1 --api-reps 5 $F > gpurun_out/tagger_order/k${K}_$MODE.log 2>&1 || { echo TB_FAIL; tail -20 gpurun_out/tagger_order/k${K}_$MODE.log; exit 1; }
    python3 -c "import json;d=json.loads(open('gpurun_out/tagger_order/k${K}_$MODE.log').read().strip().splitlines()[-1]);print('k=$K $MODE', [round(x) for x in d['tag_batch_api_runs_sentences_per_s']])"
  done
done
