set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/counters_beam
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python3 $R/tools/prof_decode.py --k 1 --steps 1 --cache /tmp/ltw > $O/gen.log 2>&1 || { echo GEN_FAIL; tail -5 $O/gen.log; exit 1; }
cd /tmp && export TMPDIR=/tmp
for K in 5 16; do
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS -T --output-format csv -d $O/k$K/p1 -o run -- python3 $R/tools/prof_decode.py --k $K --steps 3 --cache /tmp/ltw > $O/k${K}_p1.log 2>&1 || { echo PASS_FAIL; tail -5 $O/k${K}_p1.log; exit 1; }
timeout -s KILL 150 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/k$K/trace -o run -- python3 $R/tools/prof_decode.py --k $K --steps 3 --cache /tmp/ltw > $O/k${K}_t.log 2>&1 || { echo TRACE_FAIL; exit 1; }
python3 $R/tools/pmc_table.py $O/k$K lt_ > $O/k$K.txt
cat $O/k$K.txt | grep -v strip
grep -h "lt_beam" $O/k$K/trace/*kernel_stats.csv | head -3
done
