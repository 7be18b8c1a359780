# Stall / latency counters of the decode kernel (separate PMC passes).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r01b}; shift || true
ARGS="$@"
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
run() {
  local name=$1; shift
  timeout -k 10 400 rocprofv3 "$@" -T --output-format csv -d $OUT/$name -o run -- \
    python3 $R/bench.py --no-cpu-baseline --steps 2 --warmup 1 $ARGS > $OUT/$name.log 2>&1
  local rc=$?
  echo "pass $name rc=$rc"; tail -1 $OUT/$name.log | cut -c1-200
  return $rc
}
run sq1 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD || exit 1
run sq2 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_INSTS_SMEM || exit 1
run tcp --pmc TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum || exit 1
run tcc --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum || exit 1
run grbm --pmc GRBM_GUI_ACTIVE GRBM_COUNT || exit 1
