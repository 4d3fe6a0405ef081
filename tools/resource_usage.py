#!/usr/bin/env python3
"""Per-kernel register / scratch / occupancy table of one dispatch unit (hipcc's
kernel-resource-usage remarks, device-only compile; nothing runs).

    python tools/resource_usage.py [MAXY RMAX] [-DNAME=VALUE ...] [--filter resolve]
"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, 'land_trendr_amd', 'csrc', 'lt_dispatch_unit.hip')


def main(argv):
    pos = [a for a in argv if not a.startswith('-')]
    defs = [a for a in argv if a.startswith('-D')]
    flt = None
    if '--filter' in argv:
        flt = argv[argv.index('--filter') + 1]
        pos = [a for a in pos if a != flt]
    maxy, rmax = (pos + ['32', '4'])[:2] if len(pos) < 2 else pos[:2]
    with tempfile.TemporaryDirectory() as td:
        cmd = ['/opt/rocm/bin/hipcc', '-x', 'hip', '--offload-arch=gfx950', '-O3', '-ffp-contract=off',
               '-std=c++17', '-fPIC', '-Wno-unused-result', f'-DLT_UNIT_MAXY={maxy}',
               f'-DLT_UNIT_RMAX={rmax}', *defs, '--cuda-device-only',
               '-Rpass-analysis=kernel-resource-usage', '-c', '-o', os.path.join(td, 'u.o'), SRC]
        r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode:
        sys.stderr.write(r.stderr[-4000:])
        return r.returncode
    rows, cur = [], None
    for line in r.stderr.splitlines():
        m = re.search(r'remark:\s+(.*?)\s*\[-Rpass', line)
        if not m:
            continue
        txt = m.group(1)
        if txt.startswith('Function Name:'):
            cur = {'name': txt.split(':', 1)[1].strip()}
            rows.append(cur)
        elif cur is not None and ':' in txt:
            k, v = txt.split(':', 1)
            cur[k.strip()] = v.strip()
    keys = ['VGPRs', 'AGPRs', 'VGPRs Spill', 'SGPRs Spill', 'ScratchSize [bytes/lane]',
            'Occupancy [waves/SIMD]', 'LDS Size [bytes/block]']
    print('kernel'.ljust(58), *[k.split(' [')[0][:12].rjust(12) for k in keys])
    for row in rows:
        if flt and flt not in row['name']:
            continue
        print(row['name'][:58].ljust(58), *[str(row.get(k, '')).rjust(12) for k in keys])
    return 0


if __name__ == '__main__':
    sys.exit(main(sys.argv[1:]))
