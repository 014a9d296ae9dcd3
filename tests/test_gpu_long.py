"""GPU: k_pair's LONG variant -- eclipses longer than one 512-point tile and
sub-binned exposures (the reference's lc.w exposure path with sub-samples,
/root/reference/CVModel.py:29-30, :64; BASELINE config 5) in one launch per
half-step: the element phase keeps its results in LDS, per-pair breakpoint
tables replace the two-kernel hand-off, and the points are dealt in blocks
of 64 to waves by estimated cost, each wave taking a range of blocks with its
lanes interleaved (a step of a wave reads 64 consecutive points).  Every case against the oracle (oracle.lnprob_batch, the
flux -> chi^2 restatement of MODEL_SPEC 3, 5) at LNP_RTOL, through lfg_lnprob
(compiled trees) and lfg_lnlike."""
import ctypes

import numpy as np
import pytest

from tests.test_gpu_lnprob import LNP_RTOL, _same

pytestmark = pytest.mark.gpu

CASES = [  # (points, sub-bins, data order)
    (1300, 1, "sorted"),      # three tiles' worth, S = 1
    (2000, 5, "sorted"),      # config 5's exposure model at a fifth of its points
    (700, 3, "shuffled"),
    (600, 2, "descending"),   # negative widths: point evaluation (MODEL_SPEC 3)
    (1000, 1, "wrap"),        # phases through +-0.5 after phi0
    (300, 4, "ragged"),       # one tile, sub-bins, ragged widths
    (800, 3, "nan_width"),
]


def _lightcurve(npts, kind, rng):
    from lfit_python_amd.synthetic import phase_grid
    if kind == "wrap":
        x, w = phase_grid(npts, 0.45, 1.1)
    else:
        x, w = phase_grid(npts)
    if kind == "shuffled":
        p = rng.permutation(npts)
        x, w = x[p], w[p]
    elif kind == "descending":
        x = x[::-1].copy()
        w = np.mean(np.diff(x)) * np.ones_like(x) / 2.0
    elif kind == "ragged":
        w = w * rng.uniform(0.3, 3.0, npts)
    elif kind == "nan_width":
        w = w.copy()
        w[npts // 3] = np.nan
    return x, w


def _model(oracle, npts, nsub, kind, E=1):
    from lfit_python_amd import synthetic
    from lfit_python_amd.synthetic import NOISE
    rng = np.random.default_rng(npts + nsub)
    m = synthetic.config_single(300, nsub=nsub) if E == 1 else synthetic.config_tree(1, 300, nsub=nsub)
    for k, lf in enumerate(m.leaves()):
        x, w = _lightcurve(npts, kind if k == 0 else "sorted", rng)
        lf.lc.x, lf.lc.w = x, w
        lf.lc.ye = NOISE * np.ones_like(x)
        st, f = oracle.flux(lf.cv_parlist, x, np.where(np.isnan(w), np.nanmean(w), w), nsub=nsub)
        assert st == 0
        lf.lc.y = f + NOISE * rng.standard_normal(f.shape)
    return m


def _walkers(m, W, seed):
    rng = np.random.default_rng(seed)
    p0 = np.array(m.dynasty_par_vals)
    return p0 * (1.0 + 0.01 * rng.standard_normal((W, p0.size)))


@pytest.mark.parametrize("npts,nsub,kind", CASES)
def test_long_lnprob_matches_oracle(oracle, npts, nsub, kind):
    import torch
    from lfit_python_amd import _native, batch
    m = _model(oracle, npts, nsub, kind)
    t = batch.compile_tree(m, nsub=nsub)
    ev = batch.LnProbEvaluator(t)
    assert _native.lib().lfg_layout(ctypes.byref(ev.ctree)) == (1 if (nsub == 1 and npts <= 512) else 2)
    W = 48
    walk = _walkers(m, W, 7)
    lle = torch.empty((W, 1), dtype=torch.float64, device="cuda")
    got = ev(torch.as_tensor(walk, device="cuda"), lnlike_e=lle).cpu().numpy()
    ref, rlle, _ = oracle.lnprob_batch(walk, t, nsub=nsub)
    if kind == "nan_width":
        assert np.all(np.isneginf(got)) and np.all(np.isneginf(ref))
    else:
        assert np.isfinite(ref).sum() >= W // 2
        fin = np.isfinite(ref)
        _same(lle.cpu().numpy()[fin], rlle[fin], LNP_RTOL)
    _same(got, ref, LNP_RTOL)


@pytest.mark.parametrize("npts,nsub,kind", [(1300, 1, "sorted"), (2000, 5, "sorted"), (700, 3, "shuffled")])
def test_long_lnlike_matches_oracle(oracle, npts, nsub, kind):
    """lfg_lnlike (no tree) on the LONG path"""
    from lfit_python_amd.lfit import lnlike_batch
    m = _model(oracle, npts, nsub, kind)
    leaf = m.leaves()[0]
    W = 40
    walk = _walkers(m, W, 9)
    pars = np.empty((W, 18))
    for i in range(W):
        m.dynasty_par_vals = walk[i]
        pars[i] = leaf.cv_parlist
    lc = leaf.lc
    got, st = lnlike_batch(pars, lc.x, lc.y, lc.ye, width=lc.w, nsub=nsub)
    got, st = got.cpu().numpy(), st.cpu().numpy()
    ref = np.empty(W)
    for i in range(W):
        s, f = oracle.flux(pars[i], lc.x, lc.w, nsub=nsub)
        assert s == st[i]
        ref[i] = -np.inf if (s != 0 or np.any(np.isnan(f))) else -0.5 * np.sum(((lc.y - f) / lc.ye) ** 2)
    assert np.isfinite(ref).sum() >= W // 2
    _same(got, ref, LNP_RTOL)


def test_long_three_eclipse_tree(oracle):
    """a 3-band tree of 1 500-point, S = 3 eclipses (E = 3: the LONG pairs,
    then k_combine_walkers)"""
    import torch
    from lfit_python_amd import batch
    m = _model(oracle, 1500, 3, "sorted", E=3)
    t = batch.compile_tree(m, nsub=3)
    assert t.E == 3
    W = 24
    walk = _walkers(m, W, 3)
    got = batch.LnProbEvaluator(t)(torch.as_tensor(walk, device="cuda")).cpu().numpy()
    ref, _, _ = oracle.lnprob_batch(walk, t, nsub=3)
    assert np.isfinite(ref).sum() >= W // 2
    _same(got, ref, LNP_RTOL)


def test_long_spec_chain_equals_plain_chain():
    """The fused speculative chain on the LONG path (candidates formed by the
    previous launch, the snapshot, the in-kernel acceptance) equals the plain
    chain (k_setup + the same kernel), bit for bit; and the deferred-acceptance
    shard path (two workspaces) equals both"""
    import torch
    from lfit_python_amd import batch, sampler, synthetic
    from tests.test_gpu_fold import _rank_chains
    from tests.test_gpu_multirank import _flux_fn
    m = synthetic.config_single(2000, flux_fn=_flux_fn, nsub=5)
    t = batch.compile_tree(m, nsub=5)
    ev = batch.LnProbEvaluator(t)
    W = 128
    p0 = np.array(m.dynasty_par_vals)
    init = p0 * (1.0 + 1e-3 * np.random.default_rng(2).standard_normal((W, p0.size)))
    out = []
    for spec in (True, False):
        S = sampler.EnsembleSampler(W, t.ndim, ev, seed=19)
        S.spec = spec
        S.set_state(init)
        lnp0 = S.lnp.clone()
        S.run_mcmc(None, 3)
        out.append((S.chain_dev.cpu().numpy(), S.lnprob_dev.cpu().numpy(), S.naccept.cpu().numpy()))
    for a, b in zip(*out):
        np.testing.assert_array_equal(a, b)
    got, _, _ = _rank_chains(t, init, lnp0, 19, 3, 2)
    for a, b in zip(got, out[0]):
        np.testing.assert_array_equal(a, b)
    assert torch.isfinite(torch.as_tensor(out[0][1])).all()


def test_long_equal_shares_beyond_block_table(oracle):
    """180 000 points: more blocks of 64 than the spent LDS holds for the
    cost partition (2 800 ints), so the waves take equal shares of the blocks
    (k_pair LONG's fallback); S = 1, against the oracle"""
    import torch
    from lfit_python_amd import _native, batch
    npts = 180000
    assert (npts + 63) // 64 + 1 > 2800
    m = _model(oracle, npts, 1, "sorted")
    t = batch.compile_tree(m, nsub=1)
    ev = batch.LnProbEvaluator(t)
    assert _native.lib().lfg_layout(ctypes.byref(ev.ctree)) == 2
    W = 8
    walk = _walkers(m, W, 5)
    got = ev(torch.as_tensor(walk, device="cuda")).cpu().numpy()
    ref, _, _ = oracle.lnprob_batch(walk, t, nsub=1)
    assert np.isfinite(ref).sum() >= W // 2
    _same(got, ref, LNP_RTOL)

