"""Patch the scratch (private segment) size of the kernels in a code object WITHOUT changing a
single instruction (debugging aid for the wrong-result variants, DESIGN.md § Wrong-result
variants): the per-lane private segment size is rewritten in both places the runtime and the
hardware read it from,
  * the AMDGPU metadata note (msgpack `.private_segment_fixed_size`, which HIP copies into the
    dispatch packet's private_segment_size, i.e. each wave's scratch slot), and
  * the kernel descriptor `<kernel>.kd` (amd_kernel_code_t-successor, u32 at byte 4).
A wave whose code reads or writes past its declared private segment then lands in its own padding
instead of the neighbouring wave's slot: if a wrong-result variant becomes correct with the same
code and a larger slot, an access beyond the declared size is the cause.

    python tools/co_patch.py IN.co OUT.co --private 2048 [--kernel lt_jit_analyze]
    python tools/co_patch.py IN.co OUT.co --vgprs 168   (occupancy only: 3 waves per SIMD)

--vgprs rewrites COMPUTE_PGM_RSRC1's granulated VGPR count (kd byte 48, bits 5:0, granules of 8
on gfx950) and the metadata's .vgpr_count: the same code then gets more registers than it uses,
so fewer waves share a SIMD (a lower occupancy with the LDS, scratch and code unchanged).

    python tools/co_patch.py IN.co OUT.co --waitcnt lgkm [--range 0x3b00:0x9000] [--kernel K]

--waitcnt makes waits stricter in place, each instruction keeping its address: every `s_waitcnt`
(SOPP, one 32-bit word on gfx950) gets its lgkmcnt field (LDS, scalar memory, messages: bits
11:8), its vmcnt field (vector memory: bits 3:0 and 15:14) or both set to 0, so the wave waits
there for every outstanding access of that kind. A stricter wait can only make the code slower,
never change what it computes: if a wrong-result variant becomes correct with every lgkm wait at
zero and identical code otherwise, a wait that let an LDS or scalar-memory result be used before
it arrived (or a hazard those accesses hide) is the cause; --range (virtual addresses, hex) and
--kernel narrow it down by bisection.
"""
import argparse
import re
import struct
import subprocess

READELF = '/opt/rocm/lib/llvm/bin/llvm-readelf'
KEY = b'\xbb.private_segment_fixed_size'  # msgpack fixstr of 27 bytes


def kd_offsets(path):
    """{kernel name: file offset of its .kd} (the .rodata section's file offset == its address)."""
    out = subprocess.check_output([READELF, '-s', '-S', '--wide', path]).decode()
    sec = {}
    for ln in out.splitlines():
        f = ln.split()
        if len(f) > 6 and f[1] == '.rodata' or (len(f) > 6 and f[2:3] == ['.rodata']):
            # [ 6] .rodata PROGBITS addr off size ...
            g = ln.split(']')[1].split()
            sec['rodata'] = (int(g[2], 16), int(g[3], 16))
    res = {}
    for ln in out.splitlines():
        f = ln.split()
        if len(f) == 8 and f[7].endswith('.kd'):
            addr = int(f[1], 16)
            a0, o0 = sec['rodata']
            res[f[7][:-3]] = addr - a0 + o0
    return res


def kernel_meta_ranges(data):
    """(name, start, end) of each kernel's metadata map in the note, by the `.name` keys: the
    `.private_segment_fixed_size` key between one kernel's neighbours belongs to it (the map's
    keys are written sorted, `.name` before `.private_segment_fixed_size`)."""
    names = []
    i = data.find(b'\xa5.name')
    while i >= 0:
        j = i + 6
        ln = data[j] & 0x1f if (data[j] & 0xe0) == 0xa0 else data[j + 1]
        s = j + 1 if (data[j] & 0xe0) == 0xa0 else j + 2
        names.append((data[s:s + ln].decode(), i))
        i = data.find(b'\xa5.name', i + 1)
    return names


def patch_vgprs(data, names, vgprs, kernels, kds):
    key = b'\xab.vgpr_count'
    pos = data.find(key)
    while pos >= 0:
        owner = [n for n, i in names if i < pos]
        owner = owner[-1] if owner else None
        v = pos + len(key)
        if (kernels is None or owner in kernels):
            if data[v] == 0xcc:
                data[v + 1] = vgprs
            elif data[v] < 0x80 and vgprs < 0x80:
                data[v] = vgprs
            else:
                raise SystemExit('vgpr_count encoding %02x' % data[v])
        pos = data.find(key, pos + 1)
    for k, off in kds.items():
        if kernels is None or k in kernels:
            r1 = struct.unpack('<I', data[off + 48:off + 52])[0]
            r1 = (r1 & ~0x3f) | ((vgprs + 7) // 8 - 1)
            data[off + 48:off + 52] = struct.pack('<I', r1)


OBJDUMP = '/opt/rocm/lib/llvm/bin/llvm-objdump'
WAIT_CLEAR = {'lgkm': 0x0F00, 'vm': 0xC00F, 'all': 0xCF0F}


def func_ranges(path):
    """{kernel name: (start, end)} virtual address ranges of the FUNC symbols."""
    out = subprocess.check_output([READELF, '-s', '--wide', path]).decode()
    res = {}
    for ln in out.splitlines():
        f = ln.split()
        if len(f) == 8 and f[3] == 'FUNC':
            a = int(f[1], 16)
            res[f[7]] = (a, a + int(f[2]))
    return res


def text_section(path):
    """(address, file offset, size) of .text."""
    out = subprocess.check_output([READELF, '-S', '--wide', path]).decode()
    for ln in out.splitlines():
        if '] .text ' in ln:
            g = ln.split(']')[1].split()
            return int(g[2], 16), int(g[3], 16), int(g[4], 16)
    raise SystemExit('no .text in %s' % path)


def patch_waitcnt(data, path, kind, lo=None, hi=None, kernels=None):
    """Zero the `kind` counter fields of every s_waitcnt in [lo, hi) (and in `kernels`); returns
    (waits seen in range, waits changed)."""
    addr0, off0, size = text_section(path)
    fr = func_ranges(path)
    asm = subprocess.check_output([OBJDUMP, '-d', '--mcpu=gfx950', path]).decode()
    seen = changed = 0
    for m in re.finditer(r'\ts_waitcnt [^\n]*// ([0-9A-F]+): ([0-9A-F]{8})\n', asm):
        a, word = int(m.group(1), 16), int(m.group(2), 16)
        if (lo is not None and a < lo) or (hi is not None and a >= hi):
            continue
        if kernels is not None and not any(fr[k][0] <= a < fr[k][1] for k in kernels):
            continue
        assert addr0 <= a < addr0 + size and word >> 16 == 0xBF8C, (hex(a), hex(word))
        o = a - addr0 + off0
        assert struct.unpack('<I', data[o:o + 4])[0] == word, hex(a)
        new = word & ~WAIT_CLEAR[kind]
        seen += 1
        if new != word:
            data[o:o + 4] = struct.pack('<I', new)
            changed += 1
    return seen, changed


def patch_accum(data, accum, kernels, kds):
    """COMPUTE_PGM_RSRC3 ACCUM_OFFSET (kd byte 44, bits 5:0, granules of 4): the first unified
    register of the wave's AGPRs; the AGPR count is the allocation minus it."""
    for k, off in kds.items():
        if kernels is None or k in kernels:
            r3 = struct.unpack('<I', data[off + 44:off + 48])[0]
            r3 = (r3 & ~0x3f) | (accum // 4 - 1)
            data[off + 44:off + 48] = struct.pack('<I', r3)


def patch(src, dst, private, kernels=None, vgprs=None, waitcnt=None, rng=(None, None), accum=None):
    data = bytearray(open(src, 'rb').read())
    if waitcnt is not None:
        seen, changed = patch_waitcnt(data, src, waitcnt, rng[0], rng[1], kernels)
        print('s_waitcnt: %d in range, %d made stricter (%s -> 0)' % (seen, changed, waitcnt))
    names = kernel_meta_ranges(bytes(data))
    done = []
    if vgprs is not None:
        patch_vgprs(data, names, vgprs, kernels, kd_offsets(src))
    if accum is not None:
        patch_accum(data, accum, kernels, kd_offsets(src))
    pos = data.find(KEY) if private is not None else -1
    while pos >= 0:
        # the owning kernel: the last `.name` before this key
        owner = [n for n, i in names if i < pos]
        owner = owner[-1] if owner else None
        v = pos + len(KEY)
        if kernels is None or owner in kernels:
            if data[v] == 0xcd:  # uint16
                old = struct.unpack('>H', data[v + 1:v + 3])[0]
                data[v + 1:v + 3] = struct.pack('>H', private)
            elif data[v] == 0xcc:  # uint8: only a value that still fits
                old = data[v + 1]
                if private > 255:
                    raise SystemExit('uint8 size %d: cannot widen in place' % old)
                data[v + 1] = private
            else:  # positive fixint: only when the new value also fits
                old = data[v]
                if private > 127:
                    raise SystemExit('fixint size %d: cannot widen in place' % old)
                data[v] = private
            done.append((owner, old))
        pos = data.find(KEY, pos + 1)
    for k, off in kd_offsets(src).items():
        if private is not None and (kernels is None or k in kernels):
            data[off + 4:off + 8] = struct.pack('<I', private)
    open(dst, 'wb').write(bytes(data))
    return done


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('src')
    ap.add_argument('dst')
    ap.add_argument('--private', type=int, default=None, help='bytes per lane')
    ap.add_argument('--vgprs', type=int, default=None, help='VGPRs per lane (multiple of 8)')
    ap.add_argument('--accum', type=int, default=None,
                    help='ACCUM_OFFSET (multiple of 4): where the AGPRs start in the allocation')
    ap.add_argument('--kernel', action='append', default=None)
    ap.add_argument('--waitcnt', choices=sorted(WAIT_CLEAR), default=None,
                    help='set this counter of every s_waitcnt to 0 (stricter waits, same code)')
    ap.add_argument('--range', default=None, help='LO:HI virtual addresses (hex) for --waitcnt')
    a = ap.parse_args()
    rng = (None, None)
    if a.range:
        lo, hi = a.range.split(':')
        rng = (int(lo, 16) if lo else None, int(hi, 16) if hi else None)
    done = patch(a.src, a.dst, a.private, set(a.kernel) if a.kernel else None, a.vgprs,
                 a.waitcnt, rng, a.accum)
    print('patched %s -> %s: private %s (%s), vgprs %s'
          % (a.src, a.dst, a.private, ', '.join('%s was %d' % d for d in done), a.vgprs))


if __name__ == '__main__':
    main()
