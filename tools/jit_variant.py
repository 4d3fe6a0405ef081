"""Override code objects for A/B runs of a bench config's JIT module, compiled with hiprtc like
the product (lt_jit.h) but with extra compiler options, e.g. LLVM switches that change the code
generator's scheduling of waits (debugging aid, not the product):

    python tools/jit_variant.py c3 --out build/override/fz --define LT_PASSB_SLOTS=0 \\
        --opt=-mllvm --opt=-amdgpu-waitcnt-forcezero

writes <out>/lt_src_<FNV-1a of the source>.co; a run with LT_JIT_OVERRIDE_DIR=<out> (and the same
LT_JIT_DEFINES) loads it instead of compiling that source. --defines are passed the way
LT_JIT_DEFINES passes them (part of the generated source, so of its hash). --hdr-root builds it
from modified copies of the kernel headers (A/B of a source change without rebuilding the
library: the generated source, and so the override's name, does not include the headers).
"""
import argparse
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'tools'))
sys.path.insert(0, ROOT)


def compile_rtc(src, opts, arch='gfx950', hdr_root=ROOT):
    import __graft_entry__ as ge
    rtc = ctypes.CDLL('/opt/rocm/lib/libhiprtc.so')
    names, texts = [], []
    for rel in ge.JIT_HEADERS:
        with open(os.path.join(hdr_root, rel)) as fh:
            texts.append(fh.read().replace('#include "../../include/lt_abi.h"',
                                           '#include "lt_abi.h"').encode())
        names.append(os.path.basename(rel).encode())
    prog = ctypes.c_void_p()
    n = len(names)
    rc = rtc.hiprtcCreateProgram(ctypes.byref(prog), src.encode(), b'lt_jit.hip', n,
                                 (ctypes.c_char_p * n)(*texts), (ctypes.c_char_p * n)(*names))
    if rc != 0:
        raise RuntimeError('hiprtcCreateProgram %d' % rc)
    o = [b'--offload-arch=' + arch.encode(), b'-O3', b'-ffp-contract=off', b'-std=c++17']
    o += [x.encode() for x in opts]
    rc = rtc.hiprtcCompileProgram(prog, len(o), (ctypes.c_char_p * len(o))(*o))
    if rc != 0:
        sz = ctypes.c_size_t()
        rtc.hiprtcGetProgramLogSize(prog, ctypes.byref(sz))
        log = ctypes.create_string_buffer(sz.value + 1)
        rtc.hiprtcGetProgramLog(prog, log)
        raise RuntimeError('hiprtc: ' + log.value.decode()[:4000])
    sz = ctypes.c_size_t()
    rtc.hiprtcGetCodeSize(prog, ctypes.byref(sz))
    code = ctypes.create_string_buffer(sz.value)
    rtc.hiprtcGetCode(prog, code)
    rtc.hiprtcDestroyProgram(ctypes.byref(prog))
    return code.raw


def main():
    import jit_asm
    import jit_isa
    ap = argparse.ArgumentParser()
    ap.add_argument('config', nargs='?', default='c3')
    ap.add_argument('--out', required=True)
    ap.add_argument('--define', action='append', default=[])
    ap.add_argument('--opt', action='append', default=[])
    ap.add_argument('--hdr-root', default=ROOT,
                    help='a tree holding modified copies of the kernel headers (same layout): the '
                         'override is built from them, the library and its build hash stay as '
                         'they are')
    ap.add_argument('--sub', action='append', default=[],
                    help='OLD=>NEW: a text substitution in the generated source before compiling '
                         '(e.g. another __launch_bounds__); the override keeps the name of the '
                         'unmodified source, so the runtime loads it in its place')
    a = ap.parse_args()
    if a.define:
        os.environ['LT_JIT_DEFINES'] = ','.join(a.define)
    src = jit_isa.jit_source(a.config)
    csrc = src
    for sub in a.sub:
        old, new = sub.split('=>')
        if old not in csrc:
            raise SystemExit('--sub: %r not in the generated source' % old)
        csrc = csrc.replace(old, new)
    code = compile_rtc(csrc, a.opt, hdr_root=a.hdr_root)
    os.makedirs(a.out, exist_ok=True)
    name = os.path.join(a.out, 'lt_src_%016x.co' % jit_asm.fnv1a(src.encode()))
    with open(name, 'wb') as fh:
        fh.write(code)
    asm = subprocess.check_output(['/opt/rocm/lib/llvm/bin/llvm-objdump', '-d', '--mcpu=gfx950',
                                   name]).decode()
    h = jit_isa.histogram(asm)
    print('%s: %s (%d bytes; opts %s; %d s_waitcnt, %d instructions in lt_jit_analyze)'
          % (a.config, name, len(code), a.opt, h.get('s_waitcnt', 0), sum(h.values())))


if __name__ == '__main__':
    main()
