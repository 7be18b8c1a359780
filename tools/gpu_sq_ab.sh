# SQ counter A/B of library builds: one rocprofv3 --pmc pass per (tag, k) over
# tools/prof_decode.py (the bench batch; a counting launch, then warm-up and
# timed decodes), the per-dispatch table of each under gpurun_out/$OUT/.
#   LIBS  tags as tools/gpu_ab.sh ("base" = the in-tree liblt.so, T = _lib/liblt_T.so)
#   KS    beams (default 1); PMC the counters of the pass (at most 8 SQ_)
#   gpurun -- 'LIBS="head base" KS="1 5" bash tools/gpu_sq_ab.sh'
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${OUT:-sq_ab}
mkdir -p $O
export PYTHONUNBUFFERED=1
PMC=${PMC:-"SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES"}
cd /tmp && export TMPDIR=/tmp
for K in ${KS:-1}; do
for T in ${LIBS:-base}; do
  if [ "$T" = base ]; then LIB=$R/lattice_based_tagger_amd/_lib/liblt.so; else LIB=$R/lattice_based_tagger_amd/_lib/liblt_$T.so; fi
  LT_LIBRARY=$LIB timeout -s KILL 150 rocprofv3 --pmc $PMC -T --output-format csv -d $O/${T}_k$K -o run -- python3 $R/tools/prof_decode.py --k $K --steps 2 --warmup 1 > $O/${T}_k$K.log 2>&1 || { echo PASS_FAIL $T k=$K; tail -5 $O/${T}_k$K.log; exit 1; }
  python3 $R/tools/pmc_table.py $O/${T}_k$K lt_ > $O/${T}_k$K.txt
  echo "== $T k=$K"; grep -v "lt_strip\|lt_k1_sched" $O/${T}_k$K.txt
done
done
echo SQ_AB_DONE
