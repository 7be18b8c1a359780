# rocprofv3 passes over bench.py (kernel trace + separate PMC passes).
# Usage on the GPU box: bash tools/gpu_prof.sh <tag> [bench args...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r01}; shift || true
ARGS="$@"
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
run() {  # name, steps, rocprof args...
  local name=$1; EXTRA="--steps $2 --warmup 1"; shift 2
  timeout -k 10 400 rocprofv3 "$@" -T --output-format csv -d $OUT/$name -o run -- \
    python3 $R/bench.py --no-cpu-baseline $ARGS $EXTRA > $OUT/$name.log 2>&1
  local rc=$?
  echo "pass $name rc=$rc"; tail -2 $OUT/$name.log
  return $rc
}
run trace 10 --kernel-trace --stats || exit 1
run fetch 2 --pmc FETCH_SIZE || exit 1
run write 2 --pmc WRITE_SIZE || exit 1
run sq 2 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY || exit 1
run tcc 2 --pmc TCC_HIT_sum TCC_MISS_sum || exit 1
ls -R $OUT | head -50
