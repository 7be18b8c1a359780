"""Kernel resource usage (VGPRs, SGPRs, LDS, occupancy) of a HIP source for
gfx950, from the compiler's kernel-resource-usage remarks (no GPU needed).

    python tools/kres.py [SRC] [-DNAME=V ...] [--filter SUBSTR]
"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def usage(src, defines=(), flt=''):
    cmd = ['/opt/rocm/bin/hipcc', '--offload-arch=gfx950', '-O3', '-std=c++17', '-fPIC', '-ffp-contract=off',
           '-I' + os.path.join(ROOT, 'include'), '-c', src, '-o', '/dev/null',
           '-Rpass-analysis=kernel-resource-usage', '--cuda-device-only'] + ['-D' + d for d in defines]
    err = subprocess.run(cmd, capture_output=True, text=True).stderr
    rows, cur = [], None
    for line in err.splitlines():
        m = re.search(r'remark: (.*?) \[-Rpass', line)
        if not m:
            continue
        t = m.group(1).strip()
        if t.startswith('Function Name:'):
            name = subprocess.run(['c++filt'], input=t.split(':', 1)[1].strip(), capture_output=True,
                                  text=True).stdout.strip()
            name = name.replace('(anonymous namespace)::', '').replace('(lt::DecodeParams)', '')
            cur = {'name': name}
            rows.append(cur)
        elif cur is not None and ':' in t:
            k, v = t.split(':', 1)
            cur[k.strip()] = v.strip()
    return [r for r in rows if flt in r['name']]


if __name__ == '__main__':
    args = sys.argv[1:]
    src = next((a for a in args if not a.startswith('-')),
               os.path.join(ROOT, 'lattice_based_tagger_amd', 'csrc', 'lt_decode.hip'))
    defs = [a[2:] for a in args if a.startswith('-D')]
    flt = args[args.index('--filter') + 1] if '--filter' in args else ''
    for r in usage(src, defs, flt):
        print('%-48s VGPR %4s  SGPR %4s  LDS %6s  spill %s/%s  waves/SIMD %s' % (
            r['name'][:48], r.get('VGPRs', '?'), r.get('SGPRs', '?'), r.get('LDS Size [bytes/block]', '?'),
            r.get('VGPRs Spill', '?'), r.get('SGPRs Spill', '?'), r.get('Occupancy [waves/SIMD]', '?')))
