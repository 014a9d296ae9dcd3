"""lfit's component objects (PyWhiteDwarf / PyDisc / PySpot / PyDonor,
testCV.py:27-49; MODEL_SPEC 5.6).

CPU: the oracle's components, at inc = findi(q, dphi) and phase x - phi0,
times the flux parameters, are the oracle's CV components (testCV.py:65's
sum), for the default grids; grid-size rules.
GPU: the HIP components against the oracle's on default and caller-chosen
grids (1e-9 relative), against the CV path's components, and the lfit error
behaviour on invalid input."""
import numpy as np
import pytest

from tests.helpers import ECL1, TRUTH18, phase_grid

# testCV.py:17-40's demo values
DEMO = dict(q=0.1, inc=86.9, rwd_a=0.01, ulimb=0.4, rdisc=0.6, dexp=0.2, az=157.0, fis=0.2, scale=0.039,
            exp1=2.0, exp2=1.0, tilt=120.0, yaw=1.0)


def _split(pars):
    """CV parameters -> (q, dphi, phi0, flux parameters, per-kind component parameters)."""
    p = list(pars) + ([2.0, 1.0, 90.0, 0.0] if len(pars) == 14 else [])
    wdf, df, sf, rsf, q, dphi, rdisc, ul, rwd, scale, az, fis, dexp, phi0, e1, e2, tilt, yaw = p
    cps = {0: [rwd, ul], 1: [rwd, rdisc, dexp], 2: [rdisc, az, fis, scale, e1, e2, tilt, yaw], 3: []}
    return q, dphi, phi0, (wdf, df, sf, rsf), cps


GRIDS = {0: (0, 0), 1: (20, 50), 2: (100, 0), 3: (20, 20)}


@pytest.mark.parametrize("pars", [TRUTH18, ECL1, TRUTH18[:14]])
def test_oracle_components_sum_to_the_cv(oracle, pars):
    x, w = phase_grid(300)
    q, dphi, phi0, fl, cps = _split(pars)
    inc = oracle.findi(q, dphi)
    st, comps = oracle.flux(pars, x, w, components=True)
    assert st == 0
    total = np.zeros_like(x)
    for kind in range(4):
        s, y = oracle.component(kind, cps[kind], q, inc, x - phi0, w, *GRIDS[kind])
        assert s == 0
        np.testing.assert_allclose(fl[kind] * y, comps[1 + kind], rtol=1e-12, atol=1e-15)
        total += fl[kind] * y
    np.testing.assert_allclose(total, comps[0], rtol=1e-12)


def test_oracle_component_normalisation(oracle):
    """Unit flux at maximum light: WD and disc out of eclipse = 1, the donor
    = 1 at quadrature, the spot's beaming peaks at 1."""
    x = np.array([-0.25, 0.25, 0.4])
    d = DEMO
    xl1 = oracle.xl1(d["q"])
    for kind, cp in ((0, [d["rwd_a"] / xl1, d["ulimb"]]), (1, [d["rwd_a"] / xl1, d["rdisc"], d["dexp"]])):
        st, y = oracle.component(kind, cp, d["q"], d["inc"], x, None, 20, 50)
        assert st == 0
        np.testing.assert_allclose(y, 1.0, rtol=1e-14)
    st, y = oracle.component(3, [], d["q"], d["inc"], np.array([0.25, -0.25]), None, 20, 20)
    np.testing.assert_allclose(y, 1.0, rtol=1e-14)
    ph = np.linspace(-0.5, 0.5, 2001)
    st, y = oracle.component(2, [d["rdisc"], d["az"], d["fis"], d["scale"], 2.0, 1.0, 90.0, 0.0], d["q"],
                             d["inc"], ph, None, 100)
    assert st == 0 and 0.99 < y.max() <= 1.0 + 1e-12


def test_grid_rules():
    from lfit_python_amd.lfit import disc_grid, donor_grid
    assert disc_grid(1000) == (20, 50) and donor_grid(400) == (20, 20)
    assert disc_grid(250) == (10, 25) and donor_grid(100) == (10, 10)
    nr, naz = disc_grid(777)
    assert abs(nr * naz - 777) <= nr


@pytest.mark.gpu
@pytest.mark.parametrize("pars", [TRUTH18, ECL1, TRUTH18[:14]])
def test_gpu_components_match_oracle_and_cv(oracle, pars):
    from lfit_python_amd import lfit
    x, w = phase_grid(300)
    q, dphi, phi0, fl, cps = _split(pars)
    inc = oracle.findi(q, dphi)
    _, comps, _ = None, None, None
    f, st, cv = lfit.flux_batch(np.asarray(pars)[None, :], x, w, components=True)
    cv = cv[:, 0].cpu().numpy()
    objs = [lfit.PyWhiteDwarf(*cps[0]), lfit.PyDisc(q, *cps[1]),
            lfit.PySpot(q, *cps[2][:4], exp1=cps[2][4], exp2=cps[2][5], tilt=cps[2][6], yaw=cps[2][7],
                        complex=True),
            lfit.PyDonor(q)]
    for kind, obj in enumerate(objs):
        y = obj.calcFlux(q, inc, x - phi0, w)
        _, ref = oracle.component(kind, cps[kind], q, inc, x - phi0, w, *GRIDS[kind])
        np.testing.assert_allclose(y, ref, rtol=1e-9, atol=1e-12)
        # the CV pipeline's component (sweep accumulation, symmetric solves)
        np.testing.assert_allclose(fl[kind] * y, cv[kind], rtol=1e-9, atol=1e-12)


@pytest.mark.gpu
@pytest.mark.parametrize("npts", [100, 250, 777, 4000])
def test_gpu_caller_chosen_grids_match_oracle(oracle, npts):
    from lfit_python_amd import lfit
    d = DEMO
    xl1 = oracle.xl1(d["q"])
    phi = np.linspace(-0.5, 0.5, 1000)                       # testCV.py:20-21
    width = np.mean(np.diff(phi)) * np.ones_like(phi) / 2.0
    disc = lfit.PyDisc(d["q"], d["rwd_a"] / xl1, d["rdisc"], d["dexp"], npts)
    donor = lfit.PyDonor(d["q"], npts)
    for kind, obj, cp in ((1, disc, [d["rwd_a"] / xl1, d["rdisc"], d["dexp"]]), (3, donor, [])):
        y = obj.calcFlux(d["q"], d["inc"], phi, width)
        _, ref = oracle.component(kind, cp, d["q"], d["inc"], phi, width, obj.n1, obj.n2)
        np.testing.assert_allclose(y, ref, rtol=1e-9, atol=1e-12)
    # testCV.py's spot and WD, complex spot with its tilt and yaw
    spot = lfit.PySpot(d["q"], d["rdisc"], d["az"], d["fis"], d["scale"], exp1=d["exp1"], exp2=d["exp2"],
                       tilt=d["tilt"], yaw=d["yaw"], complex=True)
    y = spot.calcFlux(d["q"], d["inc"], phi, width)
    _, ref = oracle.component(2, spot._cpars(), d["q"], d["inc"], phi, width, 100)
    np.testing.assert_allclose(y, ref, rtol=1e-9, atol=1e-12)
    wd = lfit.PyWhiteDwarf(d["rwd_a"] / xl1, d["ulimb"])
    y = wd.calcFlux(d["q"], d["inc"], phi, width)
    _, ref = oracle.component(0, wd._cpars(), d["q"], d["inc"], phi, width)
    np.testing.assert_allclose(y, ref, rtol=1e-9, atol=1e-12)


@pytest.mark.gpu
def test_gpu_component_errors_raise_like_lfit():
    from lfit_python_amd import lfit
    x = np.linspace(-0.2, 0.2, 50)
    with pytest.raises(lfit.LfitError):
        lfit.PyDisc(0.1, 0.02, 1.5, 0.5).calcFlux(0.1, 86.0, x)     # rdisc beyond L1
    with pytest.raises(lfit.LfitError):
        lfit.PyWhiteDwarf(0.02, 0.3).calcFlux(-0.1, 86.0, x)       # q <= 0
    with pytest.raises(lfit.LfitError):
        lfit.PySpot(0.1, 0.5, 120.0, 0.2, 0.04).calcFlux(0.1, 95.0, x)  # inclination out of (0, 90]
