# Tagger end to end on the GPU box: tagger + packer GPU tests, then the
# per-phase bench at k = 1 and 5.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_tagger.py tests/test_gpu_parity.py -k "tagger or several_launches" -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_tagger.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/pytest_tagger.log; exit 1; }
tail -1 gpurun_out/pytest_tagger.log
for K in 1 5; do
timeout -k 10 300 python3 -u tools/bench_tagger.py --sentences 65536 --k $K --threads 16 > gpurun_out/bench_tagger_k$K.log 2>&1 || { echo TB_FAIL; tail -30 gpurun_out/bench_tagger_k$K.log; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/bench_tagger_k$K.log').read().strip().splitlines()[-1]);print('k=$K', {p: round(v,3) for p,v in d['phase_s'].items()}, 'api', round(d['tag_batch_api_sentences_per_s']))"
done
