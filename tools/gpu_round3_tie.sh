# Round-3 check of the tie-probe ranking: every -m gpu test with the product
# library, then interleaved A/B lines (kernel ms) of HEAD's build
# (liblt_head.so), the product build (liblt.so) and the build without the tie
# probe (liblt_notie.so) at k = 2, 5, 16.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -30 gpurun_out/smoke.log; exit 1; }
timeout -k 10 900 python3 -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
cp lattice_based_tagger_amd/_lib/liblt.so lattice_based_tagger_amd/_lib/liblt_tie.so
for rep in 1 2; do
KS="${KS:-2 5 16}" LIBS="${LIBS:-head tie notie}" STEPS=20 bash tools/gpu_ab.sh || exit 1
done
