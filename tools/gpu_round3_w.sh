# Round-3 k=1 sentences per wave (W) A/B: the product build (W = 6, LDS
# backpointer window 87) against W = 6 / window 64, W = 7 / 64, W = 8 / 40
# (the window shrinks so four 4-wave blocks still fit a CU's LDS), two
# interleaved rounds of short bench lines.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
cp lattice_based_tagger_amd/_lib/liblt.so lattice_based_tagger_amd/_lib/liblt_cur.so
for rep in 1 2; do
KS=1 LIBS="${LIBS:-cur w6b64 w7 w8}" STEPS=20 bash tools/gpu_ab.sh || exit 1
done
