"""Per-basic-block instruction counts of one kernel's main loop (no GPU):
compiles lt_decode.hip to gfx950 assembly and prints, for the kernel whose
mangled name contains NAME, each block of the outermost loop with its VALU /
SALU / LDS / VMEM counts and its first instructions.

    python tools/isa_blocks.py [NAME] [-DX=Y ...] [--all]
"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, 'lattice_based_tagger_amd', 'csrc', 'lt_decode.hip')


def asm(defines=()):
    out = '/tmp/lt_isa.s'
    subprocess.run(['/opt/rocm/bin/hipcc', '--offload-arch=gfx950', '-O3', '-std=c++17', '-fPIC',
                    '-ffp-contract=off', '-I' + os.path.join(ROOT, 'include'), '--cuda-device-only', '-S',
                    SRC, '-o', out] + ['-D' + d for d in defines], check=True, capture_output=True)
    return open(out).read().splitlines()


def kernel(lines, name):
    start = next(i for i, l in enumerate(lines) if re.match(r'^_Z\w*' + name + r'\w*:', l))
    end = next(i for i in range(start, len(lines)) if 's_endpgm' in lines[i])
    return lines[start:end + 1]


def main():
    args = sys.argv[1:]
    name = next((a for a in args if not a.startswith('-')), 'lt_viterbi_pkILi6ELb1ELb0E')
    defs = [a[2:] for a in args if a.startswith('-D')]
    body = kernel(asm(defs), name)
    blocks, cur = [], None
    for l in body:
        m = re.match(r'^(\.LBB\w+|; %bb\.\d+):', l)
        if m:
            cur = {'name': m.group(1), 'loop': 'Loop' in l, 'ins': []}
            blocks.append(cur)
            continue
        if cur is None:
            cur = {'name': 'entry', 'loop': False, 'ins': []}
            blocks.append(cur)
        t = l.strip()
        if t and not t.startswith(';') and not t.startswith('.'):
            cur['ins'].append(t.split()[0])
    tot = {'v': 0, 's': 0, 'ds': 0, 'vm': 0}
    for b in blocks:
        if not b['loop'] and '--all' not in args:
            continue
        c = {'v': sum(i.startswith('v_') for i in b['ins']), 's': sum(i.startswith('s_') for i in b['ins']),
             'ds': sum(i.startswith('ds_') for i in b['ins']),
             'vm': sum(i.startswith(('buffer_', 'global_')) for i in b['ins'])}
        for k in tot:
            tot[k] += c[k]
        print('%-14s v=%3d s=%3d ds=%2d vm=%2d  %s' % (b['name'], c['v'], c['s'], c['ds'], c['vm'],
                                                      ' '.join(b['ins'][:6])))
    print('total', tot)


if __name__ == '__main__':
    main()
