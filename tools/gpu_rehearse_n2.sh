# Two ranks on the one-GPU box (both on GPU 0): exercises the N>1 bench path
# (gloo barriers, max-over-ranks timing, the gather setup and its
# every-rank-or-none fallback -- RCCL refuses two ranks on one GPU).
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 240 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 1 > gpurun_out/bench_n2.log 2>&1
rc=$?
tail -5 gpurun_out/bench_n2.log | cut -c1-600
exit $rc
