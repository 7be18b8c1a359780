# SQ counter set at the final source (the issue roofline's same_build), then the default bench line
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/evidence_r06d
mkdir -p $O
cd $R
export PYTHONUNBUFFERED=1
OUT=evidence_r06d/sq LIBS=base KS="1 5 16" timeout -k 10 900 bash tools/gpu_sq_ab.sh > $O/sq.log 2>&1 || { echo SQ_FAIL; tail -20 $O/sq.log; exit 1; }
mkdir -p $R/profiles/r06
python3 $R/tools/sq_summary.py $O/sq base $R/profiles/r06/sq_summary.json || exit 1
cp $R/profiles/r06/sq_summary.json $O/sq_summary.json
timeout -k 10 600 python3 -u bench.py > $O/bench_default.log 2>&1 || { echo BENCH_FAIL; tail -30 $O/bench_default.log; exit 1; }
tail -1 $O/bench_default.log > $O/bench_default.jsonl
python3 -c "import json;d=json.load(open('$O/bench_default.jsonl'));r=d['roofline'];print('k=1', round(d['value']), 'kernel_ms', round(r['avg_kernel_ms'],4), 'frac', round(r['frac'],4), 'issue', r['issue']['frac'], r['issue']['same_build'], 'fresh', d['fresh_batch']['ms_per_step'], {k: round(v['avg_kernel_ms'],3) for k, v in d['extra'].items()})"
