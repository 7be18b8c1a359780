# SQ/LDS counter passes on one bench configuration (k=${PROFK:-1}).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
i=0
for G in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
         "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU" \
         "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS" ${EXTRA_PMC:+"$EXTRA_PMC"}; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $G -T --output-format csv -d $R/gpurun_out/sqroot${TAG}/p$i -o run -- python3 $R/bench.py --no-cpu-baseline --steps 2 --warmup 1 --k ${PROFK:-1} > $R/gpurun_out/sq${TAG}_$i.log 2>&1 || { echo PASS_$i FAIL; tail -5 $R/gpurun_out/sq${TAG}_$i.log; exit 1; }
done
python3 $R/tools/pmc_table.py $R/gpurun_out/sqroot${TAG} lt_
