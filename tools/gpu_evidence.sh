# The round's evidence in one gpurun call (TAG names it): smoke, every -m gpu
# test, the default bench line (CPU baselines included), the profile set
# (tools/gpu_prof.sh: kernel-trace stats without warm-up launches, FETCH_SIZE /
# WRITE_SIZE passes per k) and Tagger.tag_batch end to end at k = 1 and 5
# (tools/gpu_tagger_e2e.sh).  Everything lands in gpurun_out/evidence_$TAG/
# (and gpurun_out/prof_$TAG/) for copying into profiles/$TAG/.
#   gpurun --timeout 1200 -- 'TAG=r04 bash tools/gpu_evidence.sh'
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r04}
O=$R/gpurun_out/evidence_$TAG
mkdir -p $O
cd $R
export PYTHONUNBUFFERED=1
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 \
  || { echo SMOKE_FAIL; tail -30 $O/smoke.log; exit 1; }
echo SMOKE_OK
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > $O/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -60 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
# the profile set first: its PMC traffic summary goes where bench.py reads it
# (profiles/<TAG>_traffic.json), so the default line below carries this
# build's fabric bytes
cd $R && TAG=$TAG bash tools/gpu_prof.sh || exit 1
cp $R/gpurun_out/prof_$TAG/traffic.json $R/profiles/${TAG}_traffic.json
cp $R/gpurun_out/prof_$TAG/traffic.json $O/traffic.json
# round 6: the SQ counter set per k (VALU / LDS instructions, LDS bank
# conflicts, VALU busy) -> the issue roofline bench.py reads
# (profiles/**/sq_summary*.json, tied to this source by its hash)
cd $R && OUT=evidence_$TAG/sq LIBS=base KS="${KS:-1 5 16}" timeout -k 10 900 bash tools/gpu_sq_ab.sh > $O/sq.log 2>&1 \
  || { echo SQ_FAIL; tail -20 $O/sq.log; exit 1; }
mkdir -p $R/profiles/$TAG
python3 $R/tools/sq_summary.py $O/sq base $R/profiles/$TAG/sq_summary.json || exit 1
cp $R/profiles/$TAG/sq_summary.json $O/sq_summary.json
cd $R
timeout -k 10 600 python3 -u bench.py > $O/bench_default.log 2>&1 || { echo BENCH_FAIL; tail -30 $O/bench_default.log; exit 1; }
tail -1 $O/bench_default.log > $O/bench_default.jsonl
python3 -c "import json;d=json.load(open('$O/bench_default.jsonl'));r=d['roofline'];print('k=1', round(d['value']), 'sents/s kernel_ms', round(r['avg_kernel_ms'],4), 'frac', round(r['frac'],4), 'traffic', r['traffic'], 'fresh_ms', d['fresh_batch']['ms_per_step'], {k: (v['avg_kernel_ms'], v['value']) for k, v in d['extra'].items()})"
cd $R && bash tools/gpu_tagger_e2e.sh || exit 1
for K in 1 5; do tail -1 $R/gpurun_out/bench_tagger_k$K.log > $O/tagger_e2e_k$K.jsonl; done
echo EVIDENCE_OK
