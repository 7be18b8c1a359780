#!/usr/bin/env python3
"""Host-code profile of Tagger.tag_batch's C++ stages on unique synthetic text
(CPU container; tools/pcprof.c samples the process's PCs on SIGPROF):
lookup and pack of --sentences, samples resolved per function with
addr2line -f -i (inlined frames: the outermost caller).

    gcc -O2 -shared -fPIC tools/pcprof.c -o tools/pcprof.so -ldl
    python tools/pcprof.py [--stage lookup|pack|both] [--sentences 16384] [--threads 8]
"""
import argparse
import collections
import ctypes
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests'))
sys.path.insert(0, os.path.join(ROOT, 'tools'))

from bench_tagger import unique_text  # noqa: E402
from golden_io import load  # noqa: E402
from test_lookup import _fixture, fixture_lexicon  # noqa: E402
from lattice_based_tagger_amd.beam import lowered_model  # noqa: E402
from lattice_based_tagger_amd.native_packer import packer_for  # noqa: E402


def resolve(path):
    by_lib = collections.defaultdict(list)
    total = 0
    for line in open(path):
        c, lib, off = line.split()
        c = int(c)
        total += c
        by_lib[lib].append((int(off, 16), c))
    out = collections.Counter()
    for lib, items in by_lib.items():
        if lib in ('?', 'dropped') or not os.path.exists(lib):
            for _, c in items:
                out[os.path.basename(lib)] += c
            continue
        addrs = '\n'.join(hex(o) for o, _ in items)
        # llvm-symbolizer: the innermost inlined frame's file:line per address
        r = subprocess.run(['/opt/rocm/lib/llvm/bin/llvm-symbolizer', '--obj=' + lib, '--no-inlines',
                            '--output-style=GNU', '-f=none'],
                           input=addrs, capture_output=True, text=True)
        lines = [l for l in r.stdout.splitlines() if l.strip()]
        for (o, c), ln in zip(items, lines):
            out['%s:%s' % (os.path.basename(lib), os.path.basename(ln.split(' ')[0]))] += c
    return out, total


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--sentences', type=int, default=16384)
    ap.add_argument('--threads', type=int, default=8)
    ap.add_argument('--stage', default='both')
    ap.add_argument('--top', type=int, default=40)
    a = ap.parse_args()
    if os.environ.get('LT_LIBRARY'):
        print('library', os.environ['LT_LIBRARY'])
    prof = ctypes.CDLL(os.path.join(ROOT, 'tools', 'pcprof.so'))
    entry = _fixture()['base']
    lex = fixture_lexicon(entry)
    model = lowered_model(load('base')[0].funcs)
    npk = packer_for(model)
    sents = unique_text(entry['sentences'], a.sentences, 7)
    lat = lex.lookup(sents, n_threads=a.threads)                   # warm
    npk.pack_lattices(lat, max_len=8)
    prof.pcprof_start(2000)
    t0 = time.perf_counter()
    for _ in range(3):
        if a.stage in ('lookup', 'both'):
            lat = lex.lookup(sents, n_threads=a.threads)
        if a.stage in ('pack', 'both'):
            npk.pack_lattices(lat, max_len=8)
    dt = time.perf_counter() - t0
    prof.pcprof_stop(b'/tmp/pcprof.txt')
    out, total = resolve('/tmp/pcprof.txt')
    print('%d samples over %.2f s wall' % (total, dt))
    for name, c in out.most_common(a.top):
        print('%6.2f%%  %s' % (100.0 * c / total, name))


if __name__ == '__main__':
    main()
