# The round's evidence, second half: the SQ counter set per k (-> the issue
# roofline, profiles/$TAG/sq_summary.json), the default bench line (CPU
# baselines included; it reads profiles/${TAG}_traffic.json and the SQ
# summary), Tagger.tag_batch end to end at k = 1 and 5
#   gpurun --timeout 1200 -- 'TAG=r06 bash tools/gpu_evidence_b.sh'
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r06}
O=$R/gpurun_out/evidence_$TAG
mkdir -p $O
cd $R
export PYTHONUNBUFFERED=1
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
echo EVIDENCE_B_OK
