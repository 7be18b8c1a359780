# Tagger end-to-end bench with a cProfile of the caller thread, plus chunk-size variants.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python3 -u tools/bench_tagger.py --sentences 65536 --k 1 --threads 16 --reps 1 --profile > gpurun_out/bench_tagger_prof.log 2> gpurun_out/bench_tagger_prof.err || { echo TB_FAIL; tail -30 gpurun_out/bench_tagger_prof.err; exit 1; }
tail -1 gpurun_out/bench_tagger_prof.log | cut -c1-300
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_tagger.py tests/test_lookup.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_tagger.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/pytest_tagger.log; exit 1; }
tail -1 gpurun_out/pytest_tagger.log
for C in 4096 16384; do
timeout -k 10 300 python3 -u tools/bench_tagger.py --sentences 65536 --k 1 --threads 16 --reps 1 --chunk $C > gpurun_out/bench_tagger_c$C.log 2>&1 || { echo TB_FAIL; tail -30 gpurun_out/bench_tagger_c$C.log; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/bench_tagger_c$C.log').read().strip().splitlines()[-1]);print('chunk $C api', round(d['tag_batch_api_sentences_per_s']))"
done
