# k=1 record DMA with each lane fetching its own record halves (K1_DMA_DIRECT, `direct`) against the
# permuted packed stream (base): parity of direct, interleaved bench lines, SQ counters of both
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
LT_LIBRARY=$GRAFT_REPO_ROOT/lattice_based_tagger_amd/_lib/liblt_direct.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_direct.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_direct.log; exit 1; }
tail -1 gpurun_out/pytest_direct.log
LIBS="base direct" KS="1" ROUNDS=3 bash tools/gpu_ab.sh || exit 1
OUT=sq_direct LIBS="base direct" KS="1" timeout -k 10 600 bash tools/gpu_sq_ab.sh
