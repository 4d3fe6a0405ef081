"""Build the JIT analyze / resolve module bench.py runs for a config ON THE HOST (no GPU: hiprtc
cross-compiles for gfx950) and disassemble it: the source lt_jit_source returns for bench's scene,
params and 'B1 - B2', compiled with hiprtc from the kernel headers as __graft_entry__.embed_headers
stores them, with lt_jit.h's options. Writes <out>/<config>.hip, .co, .s (llvm-objdump) and prints
the static instruction histogram of lt_jit_analyze.

    python tools/jit_isa.py c2 [--out build/isa] [--define NAME=VALUE ...]
"""
import argparse
import collections
import ctypes
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def jit_source(cfg_name, pixels=64, flags=None):
    """flags None: bench.py's launch (spec + scene + its output fields)."""
    import bench
    from land_trendr_amd import _abi
    from land_trendr_amd.index_eqn import IndexProgram
    from land_trendr_amd.scene import build_scene, parse_date
    from land_trendr_amd.settings import compile_params
    from land_trendr_amd.synth import make_scene
    c = bench.CONFIGS[cfg_name]
    sc = make_scene(pixels, n_years=c['years'], k_min=c['k'][0], k_max=c['k'][1],
                    mask_prob=c['mask'], seed=c['seed'], device='cpu')
    meta = build_scene(sc.dates, parse_date(bench.TARGET))
    params, _ = compile_params(c['line_cost'], c['rules'], c['mode'])
    prog = IndexProgram('B1 - B2', band_dtype='int16').to_c()
    lib = _abi.load_lib()
    if flags is None:
        fields = ['status', 'matched', 'class_val', 'onset_year', 'duration', 'magnitude']
        if c['trendline']:
            fields += bench.TRENDLINE_FIELDS
        mask = 0
        for f in fields:
            mask |= _abi.LT_FIELD_BITS[f]
        flags = (_abi.LT_JIT_SRC_SPEC | _abi.LT_JIT_SRC_SCENE | _abi.LT_JIT_SRC_FIELDS |
                 (mask << 8))
    scn = meta.to_c()
    args = (ctypes.byref(scn), ctypes.byref(params), ctypes.byref(prog),
            1 if c['mask'] > 0 else 0, 1 if c['trendline'] else 0, flags)
    n = lib.lt_jit_source(*args, None, 0)
    if n < 0:
        raise RuntimeError('lt_jit_source failed (%d)' % n)
    buf = ctypes.create_string_buffer(n + 1)
    lib.lt_jit_source(*args, buf, n + 1)
    return buf.value.decode()


def hiprtc_compile(src, arch='gfx950'):
    import __graft_entry__ as ge
    rtc = ctypes.CDLL('/opt/rocm/lib/libhiprtc.so')
    names, texts = [], []
    for rel in ge.JIT_HEADERS:
        with open(os.path.join(ROOT, rel)) as fh:
            texts.append(fh.read().replace('#include "../../include/lt_abi.h"',
                                           '#include "lt_abi.h"').encode())
        names.append(os.path.basename(rel).encode())
    prog = ctypes.c_void_p()
    n = len(names)
    rc = rtc.hiprtcCreateProgram(ctypes.byref(prog), src.encode(), b'lt_jit.hip', n,
                                 (ctypes.c_char_p * n)(*texts), (ctypes.c_char_p * n)(*names))
    if rc != 0:
        raise RuntimeError('hiprtcCreateProgram %d' % rc)
    opts = [b'--offload-arch=' + arch.encode(), b'-O3', b'-ffp-contract=off', b'-std=c++17']
    rc = rtc.hiprtcCompileProgram(prog, len(opts), (ctypes.c_char_p * len(opts))(*opts))
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


def histogram(asm, kernel='lt_jit_analyze'):
    """Static opcode counts of one kernel in llvm-objdump output."""
    lines, on = [], False
    for ln in asm.splitlines():
        if re.match(r'^[0-9a-f]+ <%s>:' % kernel, ln):
            on = True
            continue
        if on and re.match(r'^[0-9a-f]+ <.*>:', ln):
            break
        if on:
            m = re.match(r'^\s+([sv]_\w+|ds_\w+|global_\w+|buffer_\w+|scratch_\w+|flat_\w+)', ln)
            if m:
                lines.append(m.group(1))
    return collections.Counter(lines)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('config', nargs='?', default='c2')
    ap.add_argument('--out', default=os.path.join(ROOT, 'build', 'isa'))
    ap.add_argument('--define', action='append', default=[])
    ap.add_argument('--top', type=int, default=40)
    a = ap.parse_args()
    src = jit_source(a.config)
    if a.define:  # A/B switches, as LT_JIT_DEFINES adds them
        src = ''.join('#define %s\n' % d.replace('=', ' ', 1) for d in a.define) + src
    os.makedirs(a.out, exist_ok=True)
    base = os.path.join(a.out, a.config)
    with open(base + '.hip', 'w') as fh:
        fh.write(src)
    code = hiprtc_compile(src)
    with open(base + '.co', 'wb') as fh:
        fh.write(code)
    asm = subprocess.check_output(['/opt/rocm/lib/llvm/bin/llvm-objdump', '-d',
                                   '--mcpu=gfx950', base + '.co']).decode()
    with open(base + '.s', 'w') as fh:
        fh.write(asm)
    h = histogram(asm)
    valu = sum(v for k, v in h.items() if k.startswith('v_'))
    salu = sum(v for k, v in h.items() if k.startswith('s_'))
    print('%s: %d instructions (%d VALU, %d SALU) in lt_jit_analyze' % (a.config, sum(h.values()),
                                                                         valu, salu))
    for k, v in h.most_common(a.top):
        print('%6d  %s' % (v, k))


if __name__ == '__main__':
    main()
