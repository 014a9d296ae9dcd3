"""The fair CPU baseline (cpu_baseline/lfg_cpu.cpp: the GPU path's algorithm
compiled for the host) against the oracle: same ln_prob to 1e-10 on the
BASELINE config shapes, with prior-rejected and invalid walkers.  It is a
timed baseline only (bench.py), so this is what makes its number comparable."""
import numpy as np
import pytest

from lfit_python_amd import batch, synthetic


@pytest.fixture(scope="module")
def port(tmp_path_factory):
    from cpu_baseline import cpu
    path = cpu.build(out=str(tmp_path_factory.mktemp("cpu") / "liblfg_cpu.so"))
    return cpu.CpuPort(path)


def _flux(oracle):
    return lambda p, x, w, nsub: oracle.flux(p, x, w, nsub=nsub)[1]


@pytest.mark.parametrize("cfg", ["c1_simple", "c2_complex", "c3_tree", "c5_subbins"])
def test_port_matches_oracle(oracle, port, cfg):
    f = _flux(oracle)
    if cfg == "c1_simple":
        m, nsub = synthetic.config_single(300, complex_bs=False, flux_fn=f), 1
    elif cfg == "c2_complex":
        m, nsub = synthetic.config_single(300, flux_fn=f), 1
    elif cfg == "c3_tree":
        m, nsub = synthetic.config_tree(2, 200, flux_fn=f), 1
    else:
        m, nsub = synthetic.config_single(1500, flux_fn=f, nsub=5), 5
    t = batch.compile_tree(m, nsub=nsub)
    rng = np.random.default_rng(12)
    p0 = np.array(m.dynasty_par_vals)
    walk = p0 * (1.0 + 0.01 * rng.standard_normal((24, p0.size)))
    names = m.dynasty_par_names
    walk[1, [i for i, n in enumerate(names) if n.startswith("az")][0]] = 200.0   # outside its prior
    walk[2, 0] = np.nan
    ref, _, _ = oracle.lnprob_batch(walk, t, nsub=nsub, nthreads=4)
    got, used = port.lnprob_batch(walk, t, nthreads=4)
    assert used >= 1
    assert np.array_equal(np.isfinite(got), np.isfinite(ref))
    assert np.isneginf(got[1]) and np.isneginf(got[2])
    fin = np.isfinite(ref)
    assert fin.sum() >= 16
    np.testing.assert_allclose(got[fin], ref[fin], rtol=1e-10, atol=1e-8)


def test_port_gp_tree_matches_reference(oracle, port):
    """The reference's useGP = 1 example tree (6 eclipses, real light curves):
    the port's serial Kalman filter and its changepoint recompute (walkers
    that trip the 120 % cache rule are among the golden ones) against the
    reference's own ln_prob (tests/golden/lnprob_gp.npz) and the oracle's
    dense GP likelihood."""
    import os
    from lfit_python_amd import cvmodel
    gold = os.path.join(os.path.dirname(__file__), "golden")
    d = np.load(os.path.join(gold, "lnprob_gp.npz"))
    m = cvmodel.construct_model(os.path.join(gold, "ref_test_data", "mcmc_input.dat"))
    t = batch.compile_tree(m)
    assert t.gp
    got, _ = port.lnprob_batch(d["walkers"], t, nthreads=4)
    ref, _, _ = oracle.lnprob_batch(d["walkers"], t, nthreads=4)
    assert np.array_equal(np.isfinite(got), np.isfinite(d["ln_prob"]))
    fin = np.isfinite(got)
    np.testing.assert_allclose(got[fin], d["ln_prob"][fin], rtol=1e-9)
    np.testing.assert_allclose(got[fin], ref[fin], rtol=1e-9)


def test_cpu_twins_match_oracle_and_batch(oracle, port):
    """The lfg_cpu_* twins (cpu_baseline/lfg_cpu.h): lfg_cpu_lnlike and
    lfg_cpu_flux of one eclipse against the oracle's flux and chi^2
    (SimpleEclipse.chisq, CVModel.py:157-178), lfg_cpu_lnprob against the
    batch form bench.py times, with an invalid parameter set among them."""
    from tests.helpers import random_pars, phase_grid
    pars = random_pars(12, complex_bs=True, seed=5)
    pars[3, 4] = -1.0  # q < 0: LFG_ST_BAD_Q
    x, w = phase_grid(300)
    rng = np.random.default_rng(3)
    _, f0 = oracle.flux(pars[0], x, w)
    y = f0 + 0.004 * rng.standard_normal(x.size)
    ye = np.full(x.size, 0.004)
    ll, st = port.lnlike(pars, x, w, y, ye, nthreads=4)
    fl, st2 = port.flux(pars, x, w, nthreads=4)
    assert st[3] == 1 and st2[3] == 1 and np.isneginf(ll[3]) and np.isnan(fl[3]).all()
    ok = st == 0
    assert ok.sum() >= 8
    for i in np.flatnonzero(ok):
        _, fo = oracle.flux(pars[i], x, w)
        np.testing.assert_allclose(fl[i], fo, rtol=1e-9, atol=1e-12)
        chi = np.sum(((y - fo) / ye) ** 2)
        assert abs(ll[i] - (-0.5 * chi)) <= 1e-9 * max(1.0, 0.5 * chi)
    m = synthetic.config_single(300, flux_fn=_flux(oracle))
    t = batch.compile_tree(m)
    p0 = np.array(m.dynasty_par_vals)
    walk = p0 * (1.0 + 0.01 * rng.standard_normal((16, p0.size)))
    np.testing.assert_array_equal(port.lnprob(walk, t, nthreads=4), port.lnprob_batch(walk, t, nthreads=4)[0])
