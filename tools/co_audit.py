#!/usr/bin/env python3
"""Static bounds audit of a JIT (or any gfx950) code object: does any instruction of a kernel
touch a register or a private / LDS byte outside what the kernel descriptor allocates?

    python tools/co_audit.py build/override/s0/lt_src_<hash>.co [--json out.json]

Per kernel it reports
  - the highest VGPR / AGPR / SGPR index the instructions name, against the allocation in the
    kernel descriptor (compute_pgm_rsrc1 granules: 8 VGPRs, 8 SGPRs on gfx9; rsrc3 accum_offset
    for the AGPR base) — a wave that names a register past its allocation would read or write
    a co-resident wave's registers;
  - every scratch access with a constant address (SGPR base or `off`, plus the instruction
    offset) against private_segment_fixed_size, and the scratch accesses whose address is a VGPR
    (per-lane dynamic offsets: listed for a source audit, their bound is not static);
  - the largest ds_* instruction offset against group_segment_fixed_size.
Nothing runs on a GPU. Used for the wrong-result variants (DESIGN.md § Wrong-result variants).
"""
import json
import re
import struct
import subprocess
import sys

LLVM = '/opt/rocm/lib/llvm/bin/'
SIZES = {'byte': 1, 'ubyte': 1, 'sbyte': 1, 'short': 2, 'ushort': 2, 'sshort': 2, 'dword': 4,
         'dwordx2': 8, 'dwordx3': 12, 'dwordx4': 16}


def descriptors(co):
    """name -> dict from the 64-byte kernel descriptors (<name>.kd in .rodata)."""
    data = open(co, 'rb').read()
    secs = subprocess.check_output([LLVM + 'llvm-readelf', '-SW', co]).decode()
    rodata = None
    for ln in secs.splitlines():
        m = re.match(r'\s*\[\s*\d+\]\s+\.rodata\s+\S+\s+([0-9a-f]+)\s+([0-9a-f]+)', ln)
        if m:
            rodata = (int(m.group(1), 16), int(m.group(2), 16))
    out = {}
    syms = subprocess.check_output([LLVM + 'llvm-readelf', '-sW', co]).decode()
    for ln in syms.splitlines():
        p = ln.split()
        if len(p) < 8 or not p[-1].endswith('.kd') or rodata is None:
            continue
        o = rodata[1] + int(p[1], 16) - rodata[0]
        kd = data[o:o + 64]
        group, private = struct.unpack_from('<II', kd, 0)
        rsrc3, rsrc1, rsrc2 = struct.unpack_from('<III', kd, 44)
        out[p[-1][:-3]] = {
            'group_segment': group, 'private_segment': private,
            'vgprs': ((rsrc1 & 63) + 1) * 8, 'sgprs': (((rsrc1 >> 6) & 15) + 1) * 8,
            'accum_offset': ((rsrc3 & 63) + 1) * 4, 'private_enabled': bool(rsrc2 & 1)}
    return out


def audit_asm(asm, desc):
    """desc: the descriptors(); asm: llvm-objdump -d text. Returns {kernel: report}."""
    rep, kern = {}, None
    for ln in asm.splitlines():
        m = re.match(r'^[0-9a-f]+ <([\w.]+)>:', ln)
        if m:
            kern = m.group(1) if m.group(1) in desc else None
            if kern:
                rep[kern] = {'max_v': -1, 'max_a': -1, 'max_s': -1, 'scratch_const': [],
                             'scratch_vgpr_addressed': [], 'max_ds_offset': 0}
            continue
        if kern is None:
            continue
        body = ln.split('//')[0].strip()
        addr = ln.split('//')[1].split(':')[0].strip() if '//' in ln else ''
        if not body:
            continue
        r = rep[kern]
        for t, hi in re.findall(r'\b([vas])\[\d+:(\d+)\]', body):
            r['max_' + t] = max(r['max_' + t], int(hi))
        for t, i in re.findall(r'(?<![\w\[:])([vas])(\d+)\b', body):
            r['max_' + t] = max(r['max_' + t], int(i))
        m = re.match(r'scratch_(load|store)_(\w+?)(?:_d16\w*)?\s+(.*)', body)
        if m:
            kind, ty, ops = m.groups()
            size = SIZES.get(ty, 4)
            ops = [x.strip() for x in ops.split(',')]
            off = re.search(r'offset:(-?\d+)', body)
            off = int(off.group(1)) if off else 0
            vaddr = ops[0] if kind == 'store' else ops[1]
            if vaddr.startswith('v'):
                r['scratch_vgpr_addressed'].append({'pc': addr, 'insn': body})
            else:
                r['scratch_const'].append({'pc': addr, 'lo': off, 'hi': off + size,
                                           'sgpr_base': ops[-1].split()[0] != 'off',
                                           'insn': body})
        m = re.match(r'ds_\w+.*offset(?:1)?:(\d+)', body)
        if m:
            r['max_ds_offset'] = max(r['max_ds_offset'], int(m.group(1)))
    for k, r in rep.items():
        d = desc[k]
        r.update(d)
        # SGPR allocation includes VCC (and the XNACK mask pair where enabled)
        r['vgpr_within'] = r['max_v'] < min(d['vgprs'], d['accum_offset'] if r['max_a'] >= 0
                                            else d['vgprs'])
        r['agpr_within'] = r['max_a'] < 0 or d['accum_offset'] + r['max_a'] < d['vgprs']
        r['sgpr_within'] = r['max_s'] + 2 < d['sgprs']
        const = [s for s in r['scratch_const'] if not s['sgpr_base']]
        r['scratch_const_max_hi'] = max([s['hi'] for s in const] or [0])
        r['scratch_const_within'] = r['scratch_const_max_hi'] <= d['private_segment']
        r['n_scratch_sgpr_addressed'] = sum(s['sgpr_base'] for s in r['scratch_const'])
        r['ds_offset_within'] = r['max_ds_offset'] < d['group_segment']
        r['scratch_const'] = len(r['scratch_const'])
    return rep


def main(argv):
    co = argv[0]
    asm = subprocess.check_output([LLVM + 'llvm-objdump', '-d', '--mcpu=gfx950', co]).decode()
    rep = audit_asm(asm, descriptors(co))
    for k, r in rep.items():
        print('%s: v%d/%d a%d s%d/%d (%s) private %d B/lane, constant scratch offsets < %d, '
              '%d SGPR-based, %d VGPR-addressed; ds offset <= %d of %d' % (
                  k, r['max_v'], r['vgprs'], r['max_a'], r['max_s'], r['sgprs'],
                  'within' if r['vgpr_within'] and r['agpr_within'] and r['sgpr_within']
                  else 'OUTSIDE', r['private_segment'], r['scratch_const_max_hi'],
                  r['n_scratch_sgpr_addressed'], len(r['scratch_vgpr_addressed']),
                  r['max_ds_offset'], r['group_segment']))
        for s in r['scratch_vgpr_addressed']:
            print('    %s  %s' % (s['pc'], s['insn']))
    if '--json' in argv:
        with open(argv[argv.index('--json') + 1], 'w') as fh:
            json.dump(rep, fh, indent=1)


if __name__ == '__main__':
    main(sys.argv[1:])
