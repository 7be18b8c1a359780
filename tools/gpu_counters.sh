# Counter set of the shipping decode kernels (round 2): per beam k in $KS,
# separate rocprofv3 --pmc passes (SQ issue / wait / instruction mix, LDS
# bank conflicts, TA busy, TCC hit / miss / fabric requests, FETCH_SIZE,
# WRITE_SIZE) of tools/prof_decode.py, plus the FETCH_SIZE calibration
# microkernels (tools/fetch_calib).  Output under gpurun_out/counters/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${OUT:-counters}      # OUT: output dir; LT_LIBRARY: the library; NPASS: first N passes only
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python3 $R/tools/prof_decode.py --k 1 --steps 1 --cache /tmp/ltw > $O/gen.log 2>&1 || { echo GEN_FAIL; tail -5 $O/gen.log; exit 1; }
cd /tmp && export TMPDIR=/tmp
rocprofv3 -L > $O/pmc_list.txt 2>&1 || true
PASSES=("SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS"
        "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS TA_TA_BUSY_sum TA_BUSY_avr"
        "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum"
        "TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_REQ_sum"
        "FETCH_SIZE"
        "WRITE_SIZE")
for K in ${KS:-1 2 5 16}; do
  i=0
  for G in "${PASSES[@]}"; do
    i=$((i+1))
    [ $i -gt ${NPASS:-99} ] && break
    timeout -s KILL 150 rocprofv3 --pmc $G -T --output-format csv -d $O/k$K/p$i -o run -- python3 $R/tools/prof_decode.py --k $K --steps 3 --cache /tmp/ltw > $O/k${K}_p$i.log 2>&1 || { echo PASS_FAIL k=$K p=$i; tail -5 $O/k${K}_p$i.log; exit 1; }
  done
  python3 $R/tools/pmc_table.py $O/k$K lt_ > $O/k$K.txt
done
if [ "${CALIB:-1}" = 1 ] && [ -x $R/tools/fetch_calib ]; then
  i=0
  for G in "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum" "TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_REQ_sum" "TA_TA_BUSY_sum GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $G -T --output-format csv -d $O/calib/p$i -o run -- $R/tools/fetch_calib > $O/calib_p$i.log 2>&1 || { echo CALIB_FAIL $i; tail -5 $O/calib_p$i.log; exit 1; }
  done
  timeout -s KILL 120 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/calib/trace -o run -- $R/tools/fetch_calib > $O/calib_trace.log 2>&1 || { echo CALIB_TRACE_FAIL; exit 1; }
  python3 $R/tools/pmc_table.py $O/calib calib_ dispatch > $O/calib.txt
  cp $O/calib_p1.log $O/calib_dispatches.jsonl
fi
echo COUNTERS_DONE
