# round 6 call e: the fresh-batch step with nontemporal schedule-row stores
# in the fill (K1_FILL_AUX=2) against the current build, then
# Tagger.tag_batch with the four-stage pipeline against the three-stage one
# (LT_TAGGER_STAGES), interleaved, five timed calls each
set -o pipefail
mkdir -p gpurun_out/r6e
export PYTHONUNBUFFERED=1
LIBS="base fillnt" KS="1" ROUNDS=3 STEPS=20 timeout -k 10 600 bash tools/gpu_ab.sh > gpurun_out/r6e/ab.log 2>&1 && cat gpurun_out/r6e/ab.log &&
for RD in 1 2; do
for ST in 3 4; do
for K in 1 5; do
  LT_TAGGER_STAGES=$ST timeout -k 10 300 python3 -u tools/bench_tagger.py --sentences 65536 --k $K --threads 16 --reps 1 --api-reps 5 --text unique > gpurun_out/r6e/st${ST}_k${K}_r$RD.log 2> gpurun_out/r6e/st${ST}_k${K}_r$RD.err || { echo TB_FAIL; tail -20 gpurun_out/r6e/st${ST}_k${K}_r$RD.err; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/r6e/st${ST}_k${K}_r$RD.log').read().strip().splitlines()[-1]);print('r$RD stages=$ST k=$K', [round(x) for x in d['tag_batch_api_runs_sentences_per_s']])"
done
done
done
echo ALL_DONE
