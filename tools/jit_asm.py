"""Post-compile A/B variants of a JIT module (timing experiments, not the product): the source
lt_jit_source gives for a bench config is compiled with hipcc to assembly (the hiprtc prelude
replaced by the HIP headers), optionally rewritten, assembled and linked into a code object named
lt_src_<FNV-1a of the source>.co, which a run with LT_JIT_OVERRIDE_DIR=<dir> loads instead of
compiling that source (lt_jit.h compile).

    python tools/jit_asm.py c2 --out build/override/e64 --rewrite e64
rewrites: none (the hipcc build as it is: the control), e64 (every v_cndmask_b32_e32 on VCC as
its VOP3 form naming vcc: the e32 form reading VCC measured 16 cycles on gfx950,
profiles/r05_run2/valu_peak2.json)."""
import argparse
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'tools'))
sys.path.insert(0, ROOT)
LLVM = '/opt/rocm/lib/llvm/bin'


def fnv1a(b):
    h = 1469598103934665603
    for c in b:
        h ^= c
        h = (h * 1099511628211) & 0xFFFFFFFFFFFFFFFF
    return h


def rewrite_e64(asm):
    pat = re.compile(r'v_cndmask_b32_e32 (v\d+), ([^,]+), (v\d+), vcc\b')
    return pat.sub(r'v_cndmask_b32_e64 \1, \2, \3, vcc', asm)


def main():
    import jit_isa
    ap = argparse.ArgumentParser()
    ap.add_argument('config', nargs='?', default='c2')
    ap.add_argument('--out', required=True)
    ap.add_argument('--rewrite', default='none', choices=['none', 'e64'])
    a = ap.parse_args()
    src = jit_isa.jit_source(a.config)
    i = src.index('namespace std {')
    j = src.index('}\n', i) + 2
    hsrc = '#include <hip/hip_runtime.h>\n#include <stdint.h>\n#include <type_traits>\n' + src[j:]
    os.makedirs(a.out, exist_ok=True)
    base = os.path.join(a.out, a.config)
    with open(base + '.hip', 'w') as fh:
        fh.write(hsrc)
    subprocess.check_call(['/opt/rocm/bin/hipcc', '-x', 'hip', '--offload-arch=gfx950',
                           '--cuda-device-only', '-S', '-O3', '-ffp-contract=off', '-std=c++17',
                           '-I', os.path.join(ROOT, 'land_trendr_amd', 'csrc'),
                           '-I', os.path.join(ROOT, 'include'), '-w', '-o', base + '.s',
                           base + '.hip'])
    asm = open(base + '.s').read()
    n0 = asm.count('v_cndmask_b32_e32')
    if a.rewrite == 'e64':
        asm = rewrite_e64(asm)
    with open(base + '.s', 'w') as fh:
        fh.write(asm)
    subprocess.check_call([LLVM + '/clang', '-x', 'assembler', '-target', 'amdgcn-amd-amdhsa',
                           '-mcpu=gfx950', '-c', base + '.s', '-o', base + '.o'])
    name = os.path.join(a.out, 'lt_src_%016x.co' % fnv1a(src.encode()))
    subprocess.check_call([LLVM + '/ld.lld', '-shared', base + '.o', '-o', name])
    print('%s: %s (%s; e32 selects %d -> %d)' % (a.config, name, a.rewrite, n0,
                                                  asm.count('v_cndmask_b32_e32')))


if __name__ == '__main__':
    main()
