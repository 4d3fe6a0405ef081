"""CPU smoke tests of the diagnostics in tools/ that run without a GPU: the deferral diagnostic
(tools/defer_diag.py: the kernels' host build of the lazy DP + the reference's binary64 DP, used
for DESIGN.md § 2. resolve) on a small c2 scene."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_defer_diag_classifies_the_deferred_columns():
    out = subprocess.check_output([sys.executable, os.path.join(ROOT, 'tools', 'defer_diag.py'),
                                   '--config', 'c2', '--pixels', '1500', '--examples', '2'],
                                  cwd=ROOT, timeout=300)
    d = json.loads(out)
    st = d['stats']
    assert st['pixels'] == 1500 and st['columns'] > 1500 * 20
    # about one pixel in a hundred defers (the GPU: 1.17 % of the c2 scene); every ambiguous
    # column on a deferred path is classified as an exact or a near tie
    assert 0 < st['deferred'] < 60
    kinds = d['ambiguous_columns_on_deferred_paths']
    assert sum(kinds.values()) == st.get('exact_tie_columns', 0) + st.get('near_tie_columns', 0)
    assert sum(kinds.values()) >= st['deferred']


def test_dp_lockstep_model_counts_starts_per_column():
    """tools/dp_lockstep_model.py (DESIGN.md § The DP's lockstep cost): the wave prices at least
    the lanes' mean, and a budget of one start per column defers most pixels."""
    out = subprocess.check_output([sys.executable, os.path.join(ROOT, 'tools',
                                                                'dp_lockstep_model.py'),
                                   '--config', 'c2', '--pixels', '640'], cwd=ROOT, timeout=300)
    d = json.loads(out)
    assert d['pixels'] == 640 and d['columns'] > 0
    assert d['wave_starts_per_column'] >= d['lane_mean_starts_per_column'] > 0.5
    assert d['budget']['1']['deferred_frac'] > d['budget']['3']['deferred_frac']


def test_co_patch_rewrites_only_the_resource_fields(tmp_path):
    """tools/co_patch.py (DESIGN.md § Wrong-result variants, round 6) on a small gfx950 code
    object: the private segment size and the VGPR allocation change in the metadata and the kernel
    descriptor; the instructions do not."""
    sys.path.insert(0, os.path.join(ROOT, 'tools'))
    import jit_isa  # hiprtc, as the JIT modules are built
    src = ('extern "C" __global__ void k(int* a, int n) {\n'
           '  int t[40];\n'
           '  for (int i = 0; i < 40; i++) t[(i * 7 + threadIdx.x) % 40] = i + n;\n'
           '  a[threadIdx.x] = t[(threadIdx.x + n) % 40];\n}\n')
    co = str(tmp_path / 'k.co')
    with open(co, 'wb') as f:
        f.write(jit_isa.hiprtc_compile(src))
    out = str(tmp_path / 'p.co')
    subprocess.check_call([sys.executable, os.path.join(ROOT, 'tools', 'co_patch.py'), co, out,
                           '--private', '248', '--vgprs', '120'], timeout=60)
    ro = '/opt/rocm/lib/llvm/bin/llvm-readelf'
    notes = subprocess.check_output([ro, '--notes', out]).decode()
    assert '.private_segment_fixed_size: 248' in notes and '.vgpr_count:     120' in notes
    dis = [subprocess.check_output(['/opt/rocm/lib/llvm/bin/llvm-objdump', '-d', '--mcpu=gfx950',
                                    f]).decode().split('\n', 3)[3] for f in (co, out)]
    assert dis[0] == dis[1]


def test_co_patch_waitcnt_only_tightens_waits(tmp_path):
    """co_patch.py --waitcnt: every s_waitcnt of the kernel gets the chosen counter at 0, in
    place; every other instruction and every address stays as it was."""
    sys.path.insert(0, os.path.join(ROOT, 'tools'))
    import jit_isa
    src = ('extern "C" __global__ void k(const double* a, double* b, int n) {\n'
           '  __shared__ double s[64];\n'
           '  s[threadIdx.x] = a[threadIdx.x] * a[threadIdx.x + n];\n'
           '  __syncthreads();\n'
           '  b[threadIdx.x] = s[(threadIdx.x + n) & 63] + a[threadIdx.x + 2 * n];\n}\n')
    co = str(tmp_path / 'k.co')
    with open(co, 'wb') as f:
        f.write(jit_isa.hiprtc_compile(src))
    od = '/opt/rocm/lib/llvm/bin/llvm-objdump'
    for kind, pat in (('lgkm', 'lgkmcnt(0)'), ('vm', 'vmcnt(0)')):
        out = str(tmp_path / ('%s.co' % kind))
        subprocess.check_call([sys.executable, os.path.join(ROOT, 'tools', 'co_patch.py'), co,
                               out, '--waitcnt', kind], timeout=60)
        d0, d1 = [subprocess.check_output([od, '-d', '--mcpu=gfx950', f]).decode()
                  .split('\n', 3)[3].splitlines() for f in (co, out)]
        assert len(d0) == len(d1)
        n_wait = 0
        for x, y in zip(d0, d1):
            if 's_waitcnt' in x:
                n_wait += 1
                assert pat in y, y
                assert x.split('//')[1].split(':')[0] == y.split('//')[1].split(':')[0]
            else:
                assert x == y
        assert n_wait > 0


def test_co_audit_reads_descriptor_and_bounds(tmp_path):
    """tools/co_audit.py (DESIGN.md § Wrong-result variants, round 6): the allocation it reads from
    the kernel descriptor agrees with the code object's metadata, and a private array indexed by a
    lane's own value shows up as a VGPR-addressed scratch access."""
    sys.path.insert(0, os.path.join(ROOT, 'tools'))
    import co_audit
    import jit_isa
    src = ('extern "C" __global__ void k(int* a, int n) {\n'
           '  int t[40];\n'
           '  for (int i = 0; i < 40; i++) t[(i * 7 + threadIdx.x) % 40] = i + n;\n'
           '  a[threadIdx.x] = t[(threadIdx.x + n) % 40];\n}\n')
    co = str(tmp_path / 'k.co')
    with open(co, 'wb') as f:
        f.write(jit_isa.hiprtc_compile(src))
    desc = co_audit.descriptors(co)
    notes = subprocess.check_output(['/opt/rocm/lib/llvm/bin/llvm-readelf', '--notes', co]).decode()
    assert '.private_segment_fixed_size: %d' % desc['k']['private_segment'] in notes
    assert '.vgpr_count:     %d' % desc['k']['vgprs'] in notes or desc['k']['vgprs'] % 8 == 0
    asm = subprocess.check_output(['/opt/rocm/lib/llvm/bin/llvm-objdump', '-d', '--mcpu=gfx950',
                                   co]).decode()
    r = co_audit.audit_asm(asm, desc)['k']
    assert r['vgpr_within'] and r['sgpr_within'] and r['scratch_const_within']
    assert r['scratch_vgpr_addressed'], 'the dynamically indexed array lives in scratch'


def test_co_patch_accum_moves_only_the_agpr_split(tmp_path):
    """co_patch.py --vgprs / --accum (DESIGN.md § Wrong-result variants, run 25, there 136 / 136):
    the descriptor's allocation and AGPR split change, the instructions do not (a small kernel:
    its metadata holds the count in one byte, so the patch stays below 128 here)."""
    sys.path.insert(0, os.path.join(ROOT, 'tools'))
    import co_audit
    import jit_isa
    src = 'extern "C" __global__ void k(double* a) { a[threadIdx.x] = a[threadIdx.x] * 3.0 + 1.0; }\n'
    co = str(tmp_path / 'k.co')
    with open(co, 'wb') as f:
        f.write(jit_isa.hiprtc_compile(src))
    out = str(tmp_path / 'p.co')
    subprocess.check_call([sys.executable, os.path.join(ROOT, 'tools', 'co_patch.py'), co, out,
                           '--vgprs', '120', '--accum', '112'], timeout=60)
    d = co_audit.descriptors(out)['k']
    assert d['vgprs'] == 120 and d['accum_offset'] == 112
    dis = [subprocess.check_output(['/opt/rocm/lib/llvm/bin/llvm-objdump', '-d', '--mcpu=gfx950',
                                    f]).decode().split('\n', 3)[3] for f in (co, out)]
    assert dis[0] == dis[1]
