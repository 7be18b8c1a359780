# Round-end check: smoke, every -m gpu test, the default bench line, the
# Tagger end-to-end bench at k = 1 and 5.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -30 gpurun_out/smoke.log; exit 1; }
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 400 python3 -u bench.py > gpurun_out/bench_default.log 2>&1 || { echo BENCH_FAIL; tail -30 gpurun_out/bench_default.log; exit 1; }
tail -1 gpurun_out/bench_default.log | cut -c1-400
for K in 1 5; do
timeout -k 10 300 python3 -u tools/bench_tagger.py --sentences 65536 --k $K --threads 16 --reps 2 --api-reps 3 > gpurun_out/bench_tagger_k$K.log 2>&1 || { echo TB_FAIL; tail -30 gpurun_out/bench_tagger_k$K.log; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/bench_tagger_k$K.log').read().strip().splitlines()[-1]);print('k=$K', {p: round(v,3) for p,v in d['phase_s'].items()}, 'api', [round(x) for x in d['tag_batch_api_runs_sentences_per_s']])"
done
