"""The CPU oracle (oracle/lt_oracle.c) against the reference's own outputs (tests/golden/).

This pins the oracle: every later GPU parity claim is made against it and the same goldens.
"""
import os

import numpy as np
import pytest

import golden_io
from oracle import oracle


def test_lstsq_matches_reference_bitwise():
    z = dict(np.load(os.path.join(golden_io.GOLDEN, 'lstsq.npz')))
    bad = 0
    for t in range(len(z['m'])):
        m = int(z['m'][t])
        rc, s, c, r = oracle.lstsq(z['x'][t, :m], z['y'][t, :m])
        assert rc == 0
        want = (z['slope'][t], z['icpt'][t], z['ssr'][t])
        if not all(golden_io._bits_equal(a, b) for a, b in zip((s, c, r), want)):
            bad += 1
    assert bad == 0, '%d of %d segments differ from np.linalg.lstsq' % (bad, len(z['m']))


def test_reference_least_squares_known_answer():
    # tests/utils_test.py:172-177 (reference's own expectation, 7 decimals)
    rc, m, c, ssr = oracle.lstsq([0, 1, 2, 3, 4], [1, 2.1, 3, 4.4, 4.7])
    assert rc == 0
    assert round(m - 0.96999999999999997, 7) == 0
    assert round(c - 1.1000000000000008, 7) == 0
    assert round(ssr - 0.24300000000000019, 7) == 0


@pytest.mark.parametrize('name', golden_io.scene_names())
def test_oracle_scene_bit_exact(name):
    g = golden_io.GoldenScene(name)
    out = oracle.analyze_tile(g.scene, g.params, g.values, g.valid, n_threads=4)
    bad = golden_io.compare(g, out)
    assert not bad, '\n'.join(bad[:40])
