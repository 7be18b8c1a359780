# Round-3 k=1 experiment: table size (LT_TABLE_LOAD: the cuckoo table's
# maximum load factor, 0.45 by default -> fewer flagged primaries, so fewer
# macro-steps that need a second memory round trip) against the record DMA's
# place in the macro-step (liblt_edma.so: PK_EARLY_DMA=1, issued behind the
# primary probes).  One short bench line per (library, load factor).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
cp lattice_based_tagger_amd/_lib/liblt.so lattice_based_tagger_amd/_lib/liblt_cur.so
for rep in 1 2; do
for L in 0.45 0.2 0.1 0.05; do
for T in ${LIBS:-cur edma}; do
LT_TABLE_LOAD=$L LT_LIBRARY=$R/lattice_based_tagger_amd/_lib/liblt_$T.so timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 3 --k 1 --extra-k '' --no-cpu-baseline --no-check > gpurun_out/tab_${T}_$L.log 2>&1 || { echo TAB_FAIL $T $L; tail -20 gpurun_out/tab_${T}_$L.log; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/tab_${T}_$L.log').read().strip().splitlines()[-1]);print('$T load=$L', round(d['value']), 'kernel_ms', round(d['roofline']['avg_kernel_ms'],4), 'loads', d['ops_per_launch']['table_slot_loads'])"
done
done
done
# the beams share the table: their time at the default and a low load factor,
# and the product library against HEAD's
for K in 2 5 16; do
for L in 0.45 0.1; do
for T in cur head; do
LT_TABLE_LOAD=$L LT_LIBRARY=$R/lattice_based_tagger_amd/_lib/liblt_$T.so timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 2 --k $K --extra-k '' --no-cpu-baseline --no-check > gpurun_out/tabk_${T}_${L}_$K.log 2>&1 || { echo TABK_FAIL $T $L $K; tail -20 gpurun_out/tabk_${T}_${L}_$K.log; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/tabk_${T}_${L}_$K.log').read().strip().splitlines()[-1]);print('$T k=$K load=$L', round(d['value']), 'kernel_ms', round(d['roofline']['avg_kernel_ms'],4))"
done
done
done
