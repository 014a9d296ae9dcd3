"""The converged stream of MODEL_SPEC 4.5 (trm.roche.bspot, CVModel.py:288).

The oracle's bspot (table for q in [QLO, QHI], fine RK4 outside) against an
independent high-accuracy integration (scipy DOP853, tools/gen_stream_table.py)
on random (q, r); continuity across the table's q edges; the miss and
start-region status codes; the table's xl1 and findphi(q, 90) series against
the oracle's solvers.  The GPU side is checked against the oracle in
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
        for s in np.concatenate([rng.uniform(0.0, S_TOP, 4), rng.uniform(0.95, 1.0, 2), [1e-3, 1.0 - 1e-9]]):
            rad = st.rmin + (st.r0 - st.rmin) * s * s
            got = np.array(orc.bspot(q, rad))
            ref = st.at_radius(rad)
            perr = max(perr, np.abs(got[:2] - ref[:2]).max())
            verr = max(verr, np.abs(got[2:] - ref[2:]).max())
    assert perr < 1e-12, perr
    assert verr < 2e-11, verr


@pytest.mark.parametrize("q", [0.0015, 6.0])
def test_fine_rk4_outside_the_table(orc, q):
    """q beyond [QLO, QHI]: fine RK4."""
    st = gst.Stream(q)
    for s in (0.5, 0.97):
        rad = st.rmin + (st.r0 - st.rmin) * s * s
        got = np.array(orc.bspot(q, rad))
        ref = st.at_radius(rad)
        assert np.abs(got[:2] - ref[:2]).max() < 1e-11
        assert np.abs(got[2:] - ref[2:]).max() < 1e-9


@pytest.mark.parametrize("qe", [gst.Q_LO, gst.Q_HI])
def test_continuous_across_the_table_edge(orc, qe):
    """Table just inside [QLO, QHI], fine RK4 just outside."""
    for s in (0.3, 0.9):
        st = gst.Stream(qe)
        rad = st.rmin + (st.r0 - st.rmin) * s * s
        a = np.array(orc.bspot(qe * (1.0 - 1e-13), rad))
        b = np.array(orc.bspot(qe * (1.0 + 1e-13), rad))
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


def test_q_series_match_the_solvers(orc):
    """xl1(q) and findphi(q, 90) series of the table vs the oracle's root finders."""
    from numpy.polynomial import chebyshev as C
    lqb = np.linspace(np.log(gst.Q_LO), np.log(gst.Q_HI), gst.NQ + 1)
    hdr = open(gst.OUT).read()

    def arr(name):
        line = [l for l in hdr.splitlines() if l.startswith("#define %s {" % name)][0]
        return np.array([float(v) for v in line.split("{", 1)[1].rsplit("}", 1)[0].split(",")])
    xl1c = arr("LFG_ST_XL1").reshape(gst.NQ, -1)
    phic = arr("LFG_ST_PHI90").reshape(gst.NQ, -1)
    for q in np.exp(np.random.default_rng(5).uniform(np.log(gst.Q_LO), np.log(gst.Q_HI), 40)):
        iq = min(gst.NQ - 1, int((np.log(q) - lqb[0]) / (lqb[1] - lqb[0])))
        xq = 2.0 * (np.log(q) - lqb[iq]) / (lqb[iq + 1] - lqb[iq]) - 1.0
        assert abs(C.chebval(xq, xl1c[iq]) - orc.xl1(q)) < 1e-14
        assert abs(C.chebval(xq, phic[iq]) - orc.findphi(q, 90.0)) < 1e-12
