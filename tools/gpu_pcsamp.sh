# PC sampling (host trap) of the decode kernels: which instructions the waves
# sit on.  Output under gpurun_out/pcs/k$K.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/pcs
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python3 $R/tools/prof_decode.py --k 1 --steps 1 --cache /tmp/ltw > $O/gen.log 2>&1 || { echo GEN_FAIL; tail -5 $O/gen.log; exit 1; }
cd /tmp && export TMPDIR=/tmp
for K in ${KS:-5}; do
  timeout -s KILL 120 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time --pc-sampling-interval ${PCI:-50} --output-format csv -d $O/k$K -o run -- python3 $R/tools/prof_decode.py --k $K --steps 3 --cache /tmp/ltw > $O/k$K.log 2>&1 || { echo PCS_FAIL k=$K; tail -20 $O/k$K.log; exit 1; }
  ls -la $O/k$K
done
echo PCS_DONE
