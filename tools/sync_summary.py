"""HIP runtime calls and kernels of a rocprofv3 trace (--hip-runtime-trace,
--kernel-trace, csv): per HIP function the call count and total wall ms, the
synchronising calls first; per kernel the dispatch count and total ms.

    python tools/sync_summary.py TRACE_DIR
"""
import collections
import csv
import glob
import os
import sys

SYNC = ('hipStreamSynchronize', 'hipDeviceSynchronize', 'hipEventSynchronize', 'hipStreamWaitEvent',
        'hipMalloc', 'hipFree', 'hipHostMalloc', 'hipHostFree', 'hipMemcpy')


def table(files, key):
    out = collections.defaultdict(lambda: [0, 0])
    for f in files:
        for r in csv.DictReader(open(f)):
            t = out[r[key]]
            t[0] += 1
            t[1] += int(r['End_Timestamp']) - int(r['Start_Timestamp'])
    return out


def main():
    root = sys.argv[1]
    api = table(glob.glob(os.path.join(root, '**', '*hip_api_trace.csv'), recursive=True), 'Function')
    ker = table(glob.glob(os.path.join(root, '**', '*kernel_trace.csv'), recursive=True), 'Kernel_Name')
    if not api and not ker:
        raise SystemExit('no trace under %s' % root)
    print('HIP calls (synchronising / allocating first): count, total ms')
    for name, (n, ns) in sorted(api.items(), key=lambda x: (not x[0].startswith(SYNC), -x[1][1])):
        print('  %-40s %8d %10.3f' % (name, n, ns / 1e6))
    print('kernels: dispatches, total ms')
    for name, (n, ns) in sorted(ker.items(), key=lambda x: -x[1][1]):
        print('  %-60s %8d %10.3f' % (name[:60], n, ns / 1e6))


if __name__ == '__main__':
    main()
