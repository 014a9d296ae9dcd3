"""The converged stream of MODEL_SPEC 4.5 (trm.roche.bspot, CVModel.py:288).

The oracle's bspot (table inside its domain, fine RK4 outside) against an
independent high-accuracy integration (scipy DOP853, tools/gen_stream_table.py)
on random (q, r); continuity across the table's edge; the miss and
start-region status codes.  The GPU side is checked against the oracle in
tests/test_gpu_parity.py::test_roche_primitives.
"""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
gst = pytest.importorskip("gen_stream_table")
from oracle.oracle import Oracle  # noqa: E402

S_TOP = gst.SB[-1]


@pytest.fixture(scope="module")
def orc():
    return Oracle()


def test_table_matches_converged_integration(orc):
    rng = np.random.default_rng(20261016)
    perr = verr = 0.0
    for q in np.exp(rng.uniform(np.log(gst.Q_LO), np.log(gst.Q_HI), 10)):
        st = gst.Stream(q)
        for s in np.concatenate([rng.uniform(0.0, S_TOP, 4), [1e-3, S_TOP - 1e-9]]):
            rad = st.rmin + (st.r0 - st.rmin) * s * s
            got = np.array(orc.bspot(q, rad))
            ref = st.at_radius(rad)
            perr = max(perr, np.abs(got[:2] - ref[:2]).max())
            verr = max(verr, np.abs(got[2:] - ref[2:]).max())
    assert perr < 1e-12, perr
    assert verr < 2e-11, verr


@pytest.mark.parametrize("q", [0.0015, 0.3, 6.0])
def test_fine_rk4_outside_the_table(orc, q):
    """q beyond [QLO, QHI], or r in the start region s > S_TOP: fine RK4."""
    st = gst.Stream(q)
    for s in (0.5, 0.97):
        rad = st.rmin + (st.r0 - st.rmin) * s * s
        got = np.array(orc.bspot(q, rad))
        ref = st.at_radius(rad)
        assert np.abs(got[:2] - ref[:2]).max() < 1e-11
        assert np.abs(got[2:] - ref[2:]).max() < 1e-9


def test_continuous_across_the_table_edge(orc):
    q = 0.1037
    st = gst.Stream(q)
    r_in = st.rmin + (st.r0 - st.rmin) * (S_TOP - 1e-12) ** 2
    r_out = st.rmin + (st.r0 - st.rmin) * (S_TOP + 1e-12) ** 2
    a, b = np.array(orc.bspot(q, r_in)), np.array(orc.bspot(q, r_out))
    assert np.abs(a[:2] - b[:2]).max() < 1e-11
    assert np.abs(a[2:] - b[2:]).max() < 1e-9


def test_misses_and_start_region(orc):
    q = 0.2
    st = gst.Stream(q)
    with pytest.raises(ValueError):
        orc.bspot(q, st.rmin * (1.0 - 1e-6))  # inside periastron: the stream misses
    orc.bspot(q, st.rmin * (1.0 + 1e-6))
    with pytest.raises(ValueError):
        orc.bspot(q, 0.5 * (st.r0 + orc.xl1(q)))  # between the start point and L1
