# Tagger end-to-end bench (k = 1, 5): per-phase times and three timed
# tag_batch calls each -> profiles-ready JSON lines.  TEXT=unique (default:
# fresh sentences, tools/bench_tagger.py) or golden; PROFILE=1 adds a cProfile
# of one call (stderr of the log).  TESTS=1 first runs the GPU Tagger tests.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
if [ -n "$TESTS" ]; then
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_tagger.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_tagger.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_tagger.log; exit 1; }
tail -1 gpurun_out/pytest_tagger.log
fi
for K in ${KS:-1 5}; do
timeout -k 10 300 python3 -u tools/bench_tagger.py --sentences 65536 --k $K --threads 16 --reps 2 --api-reps 3 --text ${TEXT:-unique} ${PROFILE:+--profile} > gpurun_out/bench_tagger_k$K.log 2> gpurun_out/bench_tagger_k$K.err || { echo TB_FAIL; tail -30 gpurun_out/bench_tagger_k$K.log gpurun_out/bench_tagger_k$K.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/bench_tagger_k$K.log').read().strip().splitlines()[-1]);print('k=$K', [round(x) for x in d['tag_batch_api_runs_sentences_per_s']], {p: round(v, 3) for p, v in d['phase_s'].items()})"
done
