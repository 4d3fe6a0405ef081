"""Host-side pieces of bench.py and of the kernels' integer shortcuts that need no GPU.

- bench.pmc_summary: a committed PMC summary counts only for the kernel build it was taken on
  (its '_build' = _abi.build_hash()); bench.py refuses any other (roofline.pmc_refused).
- bench.valu_peak: the headline peak is the measured mix rate of profiles/r05_valu_peak.json.
- The int16 despike step of lt_fast.h: "not monotone with both |steps| >= K" restated as
  "one step >= K and the other <= -K" (K >= 1), against the reference's form
  (/root/reference/utils.py:556-582: x <= y <= z or x >= y >= z, |y - x| > sd, |y - z| > sd).
"""
import json
import os

import bench
from land_trendr_amd._abi import build_hash


def _write(path, build):
    with open(path, 'w') as f:
        json.dump({'_build': build, '_pixels_per_launch': 64,
                   'analyze': {'SQ_INSTS_VALU': 640.0}}, f)


def test_pmc_summary_prefers_this_build_and_marks_others(tmp_path, monkeypatch):
    prof = tmp_path / 'profiles'
    prof.mkdir()
    monkeypatch.setattr(bench, 'ROOT', str(tmp_path))
    _write(prof / 'r04_pmc_c2.json', 'another-build')
    _write(prof / 'r03_pmc_c2.json', 'older-build')
    d = bench.pmc_summary('c2', 'this-build')
    assert d['_path'] == os.path.join('profiles', 'r04_pmc_c2.json')  # newest, not matching
    assert d['_matches_build'] is False
    _write(prof / 'r03_pmc_c2.json', 'this-build')
    d = bench.pmc_summary('c4', 'this-build')  # c4 runs c2's kernel instance
    assert d['_path'] == os.path.join('profiles', 'r03_pmc_c2.json')
    assert d['_matches_build'] is True
    assert bench.per_px(d, 'analyze', 'SQ_INSTS_VALU') == 10.0


def test_committed_pmc_summaries_carry_a_build_hash():
    for c in ('c2', 'c3', 'c5'):
        d = bench.pmc_summary(c, build_hash())
        assert d is not None and d.get('_build'), c
        assert len(d['_build']) == 16


def test_valu_peak_is_the_measured_mix_rate():
    """The headline peak is the mix at full occupancy (8 waves per SIMD); the rate
    at the kernel's own 4 waves is reported beside it."""
    peak, src, cyc = bench.valu_peak()
    assert src == 'profiles/r05_valu_peak.json'
    assert 590.0 < peak < 640.0
    assert 500.0 < cyc['mix_c2_at_4_waves_g_per_s'] < peak
    assert 4.0 < cyc['mix_c2'] < 4.6 and 2.0 < cyc['add_u32'] < 2.6


def test_despike_step_as_four_compares():
    def reference(d1, d2, k):
        mono = (d1 >= 0 and d2 >= 0) or (d1 <= 0 and d2 <= 0)
        return (not mono) and min(abs(d1), abs(d2)) >= k

    def kernel(d1, d2, k):
        return (d1 >= k and d2 <= -k) or (d1 <= -k and d2 >= k)

    for k in range(1, 9):
        for d1 in range(-20, 21):
            for d2 in range(-20, 21):
                assert reference(d1, d2, k) == kernel(d1, d2, k), (d1, d2, k)
    for d1, d2 in ((65535, -65535), (-65535, 65535), (1, -65535), (65535, 0)):
        for k in (1, 2, 32767, 65535):
            assert reference(d1, d2, k) == kernel(d1, d2, k)
