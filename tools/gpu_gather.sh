# RCCL gather check on the one-GPU box: gather tests, both library load
# orders, then bench with the in-step gather at N=1 (single-rank communicator).
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_gather.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gather.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_gather.log; exit 1; }
tail -4 gpurun_out/pytest_gather.log
timeout -k 10 120 python3 -u tools/gather_check.py > gpurun_out/gather_check1.log 2>&1 || { echo CHECK1_FAIL; tail -20 gpurun_out/gather_check1.log; exit 1; }
tail -1 gpurun_out/gather_check1.log
timeout -k 10 120 python3 -u tools/gather_check.py --torch-first > gpurun_out/gather_check2.log 2>&1 || { echo CHECK2_FAIL; tail -20 gpurun_out/gather_check2.log; exit 1; }
tail -1 gpurun_out/gather_check2.log
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 2 --k 1 --no-cpu-baseline --gather 1 > gpurun_out/bench_gather.log 2>&1 || { echo BENCH_FAIL; tail -30 gpurun_out/bench_gather.log; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/bench_gather.log').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_step'], d['gather'])"
