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
"""
import argparse
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


def patch(src, dst, private, kernels=None, vgprs=None):
    data = bytearray(open(src, 'rb').read())
    names = kernel_meta_ranges(bytes(data))
    done = []
    if vgprs is not None:
        patch_vgprs(data, names, vgprs, kernels, kd_offsets(src))
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
    ap.add_argument('--kernel', action='append', default=None)
    a = ap.parse_args()
    done = patch(a.src, a.dst, a.private, set(a.kernel) if a.kernel else None, a.vgprs)
    print('patched %s -> %s: private %s (%s), vgprs %s'
          % (a.src, a.dst, a.private, ', '.join('%s was %d' % d for d in done), a.vgprs))


if __name__ == '__main__':
    main()
