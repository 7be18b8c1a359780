# Counter list + VALU breakdown / stall passes for the current kernel.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r01e}; shift || true
ARGS="$@"
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
run() {
  local name=$1; shift
  timeout -k 10 400 rocprofv3 "$@" -T --output-format csv -d $OUT/$name -o run -- \
    python3 $R/bench.py --no-cpu-baseline --steps 2 --warmup 1 $ARGS > $OUT/$name.log 2>&1
  local rc=$?
  echo "pass $name rc=$rc"; tail -1 $OUT/$name.log | cut -c1-150
  return $rc
}
run trace --kernel-trace --stats || exit 1
run v1 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_CVT SQ_WAVES || true
run v2 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC || true
run v3 --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_INSTS_SENDMSG SQ_WAVES || true
run v4 --pmc SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS SQ_ACCUM_PREV_HIRES SQ_WAVES || true
run t1 --pmc TA_BUSY_avr TA_TA_BUSY_sum TD_BUSY_avr TCP_TOTAL_CACHE_ACCESSES_sum || true
run t2 --pmc TCC_REQ_sum TCC_READ_sum TCC_HIT_sum TCC_MISS_sum || true
exit 0
