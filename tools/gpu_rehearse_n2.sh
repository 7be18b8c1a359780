# Two ranks on the one-GPU box (both on GPU 0): exercises the N>1 bench path
# (the host group's barriers, max-over-ranks timing, the strong split of one
# batch and rank 0's check).  RCCL refuses two ranks on one GPU, so with the
# default RCCL gather every rank reports the failed setup and exits 3 (by
# design: no silent fallback); ARGS="--gather 0" times the ranks each copying
# their own results.  ARGS: extra bench.py arguments.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 2 ${ARGS} > gpurun_out/bench_n2${TAG}.log 2>&1
rc=$?
grep -v "^{" gpurun_out/bench_n2${TAG}.log | tail -4 | cut -c1-300
python3 -c "import json;d=json.loads([l for l in open('gpurun_out/bench_n2${TAG}.log') if l.startswith('{')][-1]);print(d['n_gpus'], d['scaling'], round(d['value']), 'ms/step', round(d['ms_per_step'],3), 'kernel_ms', round(d['roofline']['avg_kernel_ms'],3), d['config']['sentences_rank0'], d['check'], d['gather'])"
exit $rc
