set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_tagger.py tests/test_gpu_gather.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_tagger.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_tagger.log; exit 1; }
tail -1 gpurun_out/pytest_tagger.log
for K in 1 5; do
timeout -k 10 300 python3 -u tools/bench_tagger.py --sentences 65536 --k $K --reps 2 > gpurun_out/bench_tagger_k$K.log 2>&1 || { echo TB_FAIL; tail -30 gpurun_out/bench_tagger_k$K.log; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/bench_tagger_k$K.log').read().strip().splitlines()[-1]);print('k=$K api', round(d['tag_batch_api_sentences_per_s']), 'phases', {k: round(v,3) for k,v in d['phase_s'].items()})"
done
