"""The CPU oracle: known answers and physical properties of MODEL_SPEC.md,
plus the plausibility anchor against the reference's real data."""
import json
import os

import numpy as np
import pytest

from tests.helpers import TRUTH14, TRUTH18, ECL1, phase_grid

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def test_xl1_known_answers(oracle):
    assert abs(oracle.xl1(1.0) - 0.5) < 1e-14
    qs = np.geomspace(0.01, 10, 40)
    x = np.array([oracle.xl1(q) for q in qs])
    assert np.all(np.diff(x) < 0)                       # L1 moves toward the WD as q grows
    for q, xl in zip(qs, x):                            # dPhi/dx = 0 there
        cA, cB, mu = 2 / (1 + q), 2 * q / (1 + q), q / (1 + q)
        assert abs(cA / xl**2 - cB / (1 - xl)**2 - 2 * (xl - mu)) < 1e-9
    assert abs(oracle.xl1(1 / 3.) + oracle.xl1(3.) - 1.0) < 1e-13   # q <-> 1/q mirror
    assert np.isnan(oracle.xl1(-0.1))


@pytest.mark.parametrize("q", [0.05, 0.1037, 0.3, 1.0])
@pytest.mark.parametrize("inc", [86.0, 88.0, 89.9])
def test_findi_inverts_findphi(oracle, q, inc):
    dphi = oracle.findphi(q, inc)
    assert 0 < dphi < 0.2
    assert abs(oracle.findi(q, dphi) - inc) < 1e-8


def test_findphi_monotone_and_limits(oracle):
    q = 0.1037
    d = [oracle.findphi(q, i) for i in (82, 84, 86, 88, 90)]
    assert np.all(np.diff(d) > 0)
    with pytest.raises(ValueError):
        oracle.findi(q, d[-1] + 1e-4)                   # wider than i = 90 allows
    with pytest.raises(ValueError):
        oracle.findphi(0.05, 75.0)                      # WD centre never eclipsed


def test_bspot_stream(oracle):
    q = 0.1037
    x1 = oracle.xl1(q)
    prev = None
    for r in np.linspace(0.25, 0.6, 8) * x1:
        x, y, vx, vy = oracle.bspot(q, r)
        assert abs(np.hypot(x, y) - r) < 1e-10          # lands on the requested radius
        assert y > 0 and vx < 0                         # Coriolis deflects the stream to +y
        assert x * vy - y * vx > 0                      # prograde (L_z > 0)
        if prev is not None:
            assert np.arctan2(y, x) < prev              # impact azimuth falls with radius
        prev = np.arctan2(y, x)
    with pytest.raises(ValueError):
        oracle.bspot(q, 0.01)                           # inside the stream's periastron


def test_wd_centre_eclipse_symmetric(oracle):
    # the WD-centre contacts are at -dphi/2, +dphi/2 (README.md:30)
    st, a, b, w, don, geo = oracle.elements(TRUTH18)
    assert st == 0
    q, dphi = TRUTH18[4], TRUTH18[5]
    assert abs(geo[2] - oracle.findi(q, dphi)) < 1e-12
    # mirror tiles of the WD (y -> -y) have mirrored intervals
    wd_a, wd_b = a[:400], b[:400]
    k0 = 4 * 9 * 9          # outer ring start
    nk = 4 * 19
    for j in range(nk):
        jm = (nk // 2 - 1 - j) % nk
        assert abs(wd_a[k0 + j] + wd_b[k0 + jm]) < 1e-11
    # every WD tile's interval brackets the WD-centre interval edge region
    assert np.all(wd_a < 0) and np.all(wd_b > 0)
    assert abs(np.mean(wd_b - wd_a) - dphi) < 0.2 * dphi


@pytest.mark.parametrize("pars", [TRUTH18, ECL1, TRUTH14])
def test_flux_normalisation_and_components(oracle, pars):
    x, w = phase_grid(600, -0.5, 0.5)
    st, (f, ywd, yd, ys, yrs) = oracle.flux(pars, x, w, components=True)
    assert st == 0
    np.testing.assert_allclose(ywd + yd + ys + yrs, f, rtol=1e-13, atol=1e-16)
    out = np.abs(x) > 0.2
    np.testing.assert_allclose(ywd[out], pars[0], rtol=1e-13)        # uneclipsed WD = wdFlux
    np.testing.assert_allclose(yd[out], pars[1], rtol=1e-13)         # uneclipsed disc = dFlux
    assert ys.max() <= pars[2] * (1 + 1e-12)                          # sFlux is maximum light
    assert yrs.max() <= pars[3] * (1 + 5e-3)    # tile discretisation: max ~ quadrature
    st, (f2, _, _, _, yrs2) = oracle.flux(pars, np.array([0.25 + pars[13]]), np.array([0.0]),
                                          components=True)
    assert abs(yrs2[0] - pars[3]) < 1e-14                             # donor normalised at quadrature
    assert np.all(ywd >= -1e-15) and ywd.min() < 1e-3 * pars[0]       # WD fully eclipsed at phase 0


def test_subbinning_converges(oracle):
    x, w = phase_grid(200)
    ref = oracle.flux(TRUTH18, x, w, nsub=81)[1]
    errs = [np.max(np.abs(oracle.flux(TRUTH18, x, w, nsub=s)[1] - ref)) for s in (1, 3, 9, 27)]
    assert all(e2 < e1 for e1, e2 in zip(errs, errs[1:]))
    assert errs[-1] < 1e-6
    # S = 1 is the native path; WD and disc are S-independent (exact overlap)
    _, c1 = oracle.flux(TRUTH18, x, w, nsub=1, components=True)
    _, c5 = oracle.flux(TRUTH18, x, w, nsub=5, components=True)
    np.testing.assert_allclose(c1[1], c5[1], atol=1e-14)
    np.testing.assert_allclose(c1[2], c5[2], atol=1e-14)


def test_phase_offset_shifts_curve(oracle):
    x, w = phase_grid(300)
    p = list(TRUTH18)
    p[13] = 0.0
    f0 = oracle.flux(p, x, w)[1]
    p[13] = 0.01
    f1 = oracle.flux(p, x + 0.01, w)[1]
    np.testing.assert_allclose(f0, f1, atol=1e-12)


@pytest.mark.parametrize("bad,status", [({4: -0.1}, 1), ({5: 0.5}, 2), ({8: 0.0}, 3),
                                         ({6: 1.5}, 3), ({6: 0.02}, 4), ({9: -1.0}, 3),
                                         ({0: float('nan')}, 5)])
def test_invalid_parameters(oracle, bad, status):
    p = list(TRUTH18)
    for k, v in bad.items():
        p[k] = v
    x, w = phase_grid(50)
    st, f = oracle.flux(p, x, w)
    assert st == status
    assert np.all(np.isnan(f))


def test_point_evaluation(oracle):
    # w = 0: visibility is a step function; exposure smoothing only averages it
    x = np.linspace(-0.05, 0.05, 101)
    st, f0 = oracle.flux(TRUTH18, x, np.zeros_like(x))
    st, fw = oracle.flux(TRUTH18, x, np.full_like(x, 1e-7))
    assert np.max(np.abs(f0 - fw)) < 1e-3


def test_plausibility_against_reference_data(oracle):
    """Anchor of the model to the reference's real data: the parameters in the
    reference's example input were fitted with real lfit, so a faithful model
    should reproduce those light curves.  Eclipses 1-5 give chi^2/N of 1.5-3.5
    (the residual is flickering, which the reference's GP absorbed); eclipse 0
    is an outlier fit (rdisc = 0.295) and is not asserted."""
    r = json.load(open(os.path.join(GOLD, "routing.json")))
    lcs = np.load(os.path.join(GOLD, "lightcurves.npz"))
    names = r["names"]
    start = dict(zip(names, r["start"]))
    out = {}
    for e in r["eclipses"]:
        lab, band = e["label"], e["band"]
        pars = []
        for pn in e["cv_parnames"]:
            key = "%s_%s" % (pn, lab) if "%s_%s" % (pn, lab) in start else (
                "%s_%s" % (pn, band) if "%s_%s" % (pn, band) in start else "%s_core" % pn)
            pars.append(start[key])
        x, y, ye, w = (lcs["%s_%s" % (k, lab)] for k in ("x", "y", "ye", "w"))
        st, f = oracle.flux(pars, x, w)
        assert st == 0
        out[lab] = np.sum(((y - f) / ye) ** 2) / len(x)
    for lab in "12345":
        assert out[lab] < 5.0, out
