# k=1 kernel time against the batch size (tail / fill of the grid): one bench
# line per size, kernel ms and ns per sentence.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for N in ${SIZES:-8192 16384 24576 32768 49152 65536 131072 262144}; do
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 2 --k ${K:-1} --sentences $N --no-cpu-baseline --no-check > gpurun_out/sweep_$N.log 2>&1 || { echo FAIL $N; tail -20 gpurun_out/sweep_$N.log; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/sweep_$N.log').read().strip().splitlines()[-1]);km=d['roofline']['avg_kernel_ms'];print($N, 'kernel_ms', round(km,4), 'ns/sent', round(km*1e6/$N,2), 'ms/step', round(d['ms_per_step'],4))"
done
