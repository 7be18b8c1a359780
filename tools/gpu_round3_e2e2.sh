# Tagger e2e after the compact-lattice change + the multiply-rate microbenchmark.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 tools/valu_rate.hip -o gpurun_out/valu_rate > /dev/null 2>&1 || { echo BUILD_FAIL; exit 1; }
timeout -k 10 60 gpurun_out/valu_rate > gpurun_out/valu_rate.txt 2>&1 || { echo VALU_FAIL; cat gpurun_out/valu_rate.txt; exit 1; }
cat gpurun_out/valu_rate.txt
TESTS=1 bash tools/gpu_tagger_e2e.sh
