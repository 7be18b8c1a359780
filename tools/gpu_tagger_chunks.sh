# Tagger.tag_batch throughput against the pipeline chunk (k = 1; unique text).
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for CH in ${CHUNKS:-2048 4096 8192 16384}; do
timeout -k 10 300 python3 -u tools/bench_tagger.py --sentences 65536 --k ${K:-1} --threads 16 --reps 1 --api-reps 3 --chunk $CH > gpurun_out/tagger_chunk_$CH.log 2>&1 || { echo TB_FAIL $CH; tail -20 gpurun_out/tagger_chunk_$CH.log; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/tagger_chunk_$CH.log').read().strip().splitlines()[-1]);print('chunk $CH', [round(x) for x in d['tag_batch_api_runs_sentences_per_s']])"
done
