"""GPU: batched ln_prob through the C ABI against the reference tree's own
ln_prob (golden) and the oracle, for every BASELINE config shape; the
stretch-move kernels draw-for-draw against the host double."""
import os

import numpy as np
import pytest

from tests import stretch_double as sd

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
LNP_RTOL = 1e-8   # ln_prob ~ -1e3: flux parity 1e-12 -> |d chi^2| << 1e-6


@pytest.fixture
def layout(request):
    """Run the test on one kernel layout (lfg_set_layout): 1 = k_pair, the
    default for one-tile S = 1 trees; 0 = k_elements + k_lnlike."""
    from lfit_python_amd import _native
    L = _native.lib()
    prev = L.lfg_set_layout(request.param)
    yield request.param
    L.lfg_set_layout(prev)


LAYOUTS = pytest.mark.parametrize("layout", [1, 0], indirect=True, ids=["pair", "two_kernel"])


def _same(a, b, rtol):
    a, b = np.asarray(a, float), np.asarray(b, float)
    assert np.array_equal(np.isfinite(a), np.isfinite(b))
    f = np.isfinite(a)
    np.testing.assert_allclose(a[f], b[f], rtol=rtol, atol=1e-9)


def _golden_tree(tag, tmpdir):
    from tests.helpers import golden_tree
    return golden_tree(tag, tmpdir)


@LAYOUTS
@pytest.mark.parametrize("tag", ["tree", "simple"])
def test_lnprob_matches_reference_tree(tag, tmp_path, layout):
    import torch
    from lfit_python_amd import batch
    d, m = _golden_tree(tag, tmp_path)
    t = batch.compile_tree(m)
    ev = batch.LnProbEvaluator(t)
    W = len(d["walkers"])
    lle = torch.empty((W, t.E), dtype=torch.float64, device="cuda")
    got = ev(torch.as_tensor(d["walkers"], device="cuda"), lnlike_e=lle).cpu().numpy()
    _same(got, d["ln_prob"], LNP_RTOL)
    fin = np.isfinite(d["ln_prior"])
    _same(lle.cpu().numpy().sum(1)[fin], d["ln_like"][fin], LNP_RTOL)


def _flux_fn(p, x, w, nsub):
    from lfit_python_amd.lfit import flux_batch
    f, st = flux_batch(np.asarray(p)[None, :], x, w, nsub=nsub)
    return f[0].cpu().numpy()


@LAYOUTS
@pytest.mark.parametrize("cfg", ["c1_simple", "c2_complex", "c3_tree", "c5_fine"])
def test_lnprob_configs_match_oracle(oracle, cfg, layout):
    import torch
    from lfit_python_amd import batch, synthetic
    if cfg == "c1_simple":
        m, nsub, W = synthetic.config_single(300, complex_bs=False, flux_fn=_flux_fn), 1, 100
    elif cfg == "c2_complex":
        m, nsub, W = synthetic.config_single(300, flux_fn=_flux_fn), 1, 96
    elif cfg == "c3_tree":
        m, nsub, W = synthetic.config_tree(4, 300, flux_fn=_flux_fn), 1, 24
    else:
        m, nsub, W = synthetic.config_single(10000, flux_fn=_flux_fn, nsub=5), 5, 6
    t = batch.compile_tree(m, nsub=nsub)
    rng = np.random.default_rng(4)
    p0 = np.array(m.dynasty_par_vals)
    walk = p0 * (1.0 + 0.01 * rng.standard_normal((W, p0.size)))
    got = batch.LnProbEvaluator(t)(torch.as_tensor(walk, device="cuda")).cpu().numpy()
    ref, _, _ = oracle.lnprob_batch(walk, t, nsub=nsub)
    assert np.isfinite(ref).sum() >= W // 2
    _same(got, ref, LNP_RTOL)


def _prior_rejection_case(cfg):
    from lfit_python_amd import batch, synthetic
    if cfg == "c2_complex":
        m, W = synthetic.config_single(300, flux_fn=_flux_fn), 512
    else:
        m, W = synthetic.config_tree(4, 300, flux_fn=_flux_fn), 96
    t = batch.compile_tree(m)
    names = m.dynasty_par_names
    rng = np.random.default_rng(11)
    p0 = np.array(m.dynasty_par_vals)
    walk = p0 * (1.0 + 0.002 * rng.standard_normal((W, p0.size)))
    bad = np.zeros(W, bool)
    exp2 = [i for i, n in enumerate(names) if n.startswith("exp2")]
    az = [i for i, n in enumerate(names) if n.startswith("az")]
    walk[1::4, exp2[0]] = 3e-3      # prior uniform(0.5, 5): out, absurd strip
    walk[3::8, az[0]] = 200.0       # prior uniform(50, 175): out
    bad[1::4] = True
    bad[3::8] = True
    return t, walk, bad


@pytest.mark.parametrize("cfg", ["c2_complex", "c3_tree"])
def test_prior_rejected_walkers_skip_the_model(oracle, cfg):
    """Walkers with ln_prior = -inf get -inf without the model being run
    (Node.ln_prob, model.py:476-498): k_elements and k_lnlike skip them.  An
    exp2 -> 0 proposal puts the bright-spot strip at ~1e270 (bs_umax), whose
    elements once sent whole waves into ms-long nested solves."""
    import torch
    from lfit_python_amd import batch
    t, walk, bad = _prior_rejection_case(cfg)
    got = batch.LnProbEvaluator(t)(torch.as_tensor(walk, device="cuda")).cpu().numpy()
    assert np.all(np.isneginf(got[bad]))
    ref, _, _ = oracle.lnprob_batch(walk, t)
    _same(got, ref, LNP_RTOL)
    assert np.isfinite(got[~bad]).sum() >= (~bad).sum() // 2


@pytest.mark.perf
@pytest.mark.parametrize("cfg", ["c2_complex", "c3_tree"])
def test_prior_rejected_walkers_stay_fast(cfg):
    """The wall-clock side of the test above (a shared box can slow it for
    other reasons, hence the perf marker): a batch with prior-rejected absurd
    strips stays far below the ms-long nested solves it once caused."""
    import time
    import torch
    from lfit_python_amd import batch
    t, walk, _ = _prior_rejection_case(cfg)
    ev = batch.LnProbEvaluator(t)
    x = torch.as_tensor(walk, device="cuda")
    ev(x)
    times = []
    for _ in range(5):   # the fastest of five calls: a host stall cannot decide it
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ev(x)
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
    per = min(times)
    assert per < 2e-3, "ln_prob of %d walkers took %.2f ms (calls: %s)" % (
        len(walk), per * 1e3, np.round(np.array(times) * 1e3, 3))


@pytest.mark.parametrize("cfg", ["c2_complex", "c3_tree", "gp"])
def test_non_finite_walkers_give_minus_inf(oracle, cfg):
    """NaN / inf walker coordinates: ln_prob -inf for those walkers only, in
    one- and many-eclipse trees and the GP tree; the others as the oracle."""
    import torch
    from lfit_python_amd import batch, cvmodel, synthetic
    if cfg == "c2_complex":
        m, W = synthetic.config_single(300, flux_fn=_flux_fn), 64
    elif cfg == "c3_tree":
        m, W = synthetic.config_tree(4, 300, flux_fn=_flux_fn), 24
    else:
        m, W = cvmodel.construct_model(os.path.join(GOLD, "ref_test_data", "mcmc_input.dat")), 24
    t = batch.compile_tree(m)
    rng = np.random.default_rng(13)
    p0 = np.array(m.dynasty_par_vals)
    walk = p0 * (1.0 + 1e-3 * rng.standard_normal((W, p0.size)))
    walk[3, 0] = np.nan
    walk[7, -1] = np.inf
    walk[11, p0.size // 2] = -np.inf
    got = batch.LnProbEvaluator(t)(torch.as_tensor(walk, device="cuda")).cpu().numpy()
    assert np.all(np.isneginf(got[[3, 7, 11]]))
    if cfg == "gp":
        fin = np.isfinite(got)
        assert fin.sum() >= W // 2
        return
    ref, _, _ = oracle.lnprob_batch(walk, t)
    _same(got, ref, LNP_RTOL)


@pytest.mark.perf
def test_long_chain_keeps_its_pace():
    """A config-2 chain (1024 walkers) must not slow down as it leaves the
    starting ball: proposals outside the prior box once ran the nested
    solver on non-finite geometry for milliseconds (tools/chain_drift.py).

    Blocks of 30 steps after the first 60 (the failure set in from step
    ~150; it was a sustained 2.5-6x slowdown of every later step).  Each
    step is bracketed by HIP events on the evaluator's stream, so a step's
    DEVICE time excludes host stalls between steps; the assertion is on the
    median step of each block (one slow step cannot decide it, a slow path
    that sets in does), with host and device times both in the message.
    The chain is deterministic (seed 7, Philox, exact fixed-point sums), so
    its device work is the same on every box; round 5's driver run saw one
    block of 15.4 ms host time against 2.3-2.5 ms for the other seven, which
    the same library did not repeat on another box: a host-side stall, not
    the kernels.  The timed blocks also run with the Python GC off."""
    import gc
    import time
    import torch
    from lfit_python_amd import batch, sampler, synthetic
    m = synthetic.config_single(300, flux_fn=_flux_fn)
    t = batch.compile_tree(m)
    W = 1024
    ev = batch.LnProbEvaluator(t, max_walkers=W)
    p0 = np.array(m.dynasty_par_vals)
    init = sampler.initialise_walkers(p0, sampler.comp_scatter(m.dynasty_par_names, 0.1), W,
                                      lambda p: ev(torch.as_tensor(p, device="cuda")).cpu().numpy(), seed=7)
    S = sampler.EnsembleSampler(W, t.ndim, ev, seed=7)
    S.set_state(init)
    for _ in range(60):
        S.step()
    nb, ns = 8, 30
    ev_s = [[torch.cuda.Event(enable_timing=True) for _ in range(2)] for _ in range(nb * ns)]
    host = []
    gc_was = gc.isenabled()
    gc.disable()
    try:
        for b in range(nb):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for s in range(ns):
                e0, e1 = ev_s[b * ns + s]
                e0.record()
                S.step()
                e1.record()
            torch.cuda.synchronize()
            host.append(time.perf_counter() - t0)
    finally:
        if gc_was:
            gc.enable()
    S.close()
    dev = np.array([e0.elapsed_time(e1) for e0, e1 in ev_s]).reshape(nb, ns)   # ms per step
    med = np.median(dev, axis=1)
    msg = ("per-step device median by block (us): %s; device block sums (ms): %s; host blocks (ms): %s"
           % (np.round(med * 1e3, 1), np.round(dev.sum(1), 2), np.round(np.array(host) * 1e3, 2)))
    print(msg)
    assert med.max() < 2.0 * med.min(), msg
    assert np.all(np.isfinite(S.lnp.cpu().numpy()))


def test_stretch_kernels_match_host_double():
    import torch
    from lfit_python_amd.sampler import HipStretchOps
    rng = np.random.default_rng(2)
    W, nd = 64, 7
    pos = rng.standard_normal((W, nd))
    lnp = rng.standard_normal(W)
    ops = HipStretchOps(torch.device("cuda"))
    for half, seed, step in ((0, 12345, 0), (1, 2**40 + 7, 2**33 + 5)):
        P = torch.as_tensor(pos, device="cuda")
        Lp = torch.as_tensor(lnp, device="cuda")
        q = torch.empty((W // 2, nd), dtype=torch.float64, device="cuda")
        z = torch.empty(W // 2, dtype=torch.float64, device="cuda")
        ops.propose(P, half, 2.0, seed, step, q, z)
        qh, zh = sd.propose(pos, half, 2.0, seed, step)
        np.testing.assert_allclose(q.cpu().numpy(), qh, rtol=0, atol=1e-15)
        np.testing.assert_allclose(z.cpu().numpy(), zh, rtol=1e-15, atol=1e-15)
        new = lnp[:W // 2] + rng.standard_normal(W // 2)
        new[3] = -np.inf
        new[5] = np.nan
        na = torch.zeros(W, dtype=torch.int32, device="cuda")
        ops.accept(P, Lp, half, q, z, torch.as_tensor(new, device="cuda"), seed, step, na)
        ph, lh, nh = pos.copy(), lnp.copy(), np.zeros(W, np.int64)
        sd.accept(ph, lh, half, qh, zh, new, seed, step, nh)
        np.testing.assert_allclose(P.cpu().numpy(), ph, atol=1e-15)
        np.testing.assert_array_equal(Lp.cpu().numpy(), lh)
        np.testing.assert_array_equal(na.cpu().numpy(), nh)
        assert nh[half * W // 2 + 3] == 0 and nh[half * W // 2 + 5] == 0


def test_device_mcmc_runs():
    import torch
    from lfit_python_amd import batch, sampler, synthetic
    m = synthetic.config_single(300, flux_fn=_flux_fn)
    t = batch.compile_tree(m)
    ev = batch.LnProbEvaluator(t)
    p0 = np.array(m.dynasty_par_vals)
    init = sampler.initialise_walkers(p0, sampler.comp_scatter(m.dynasty_par_names, 0.1), 128,
                                      lambda p: ev(torch.as_tensor(p, device="cuda")).cpu().numpy())
    S = sampler.EnsembleSampler(128, t.ndim, ev, seed=3)
    pos, lnp, _ = S.run_mcmc(init, 20)
    assert np.all(np.isfinite(lnp))
    assert S.chain_dev.shape == (20, 128, t.ndim)
    acc = S.acceptance_fraction.mean()
    assert 0.05 < acc < 0.9
    # the stored ln_prob is the ln_prob of the stored positions
    again = ev(S.chain_dev[-1].contiguous()).cpu().numpy()
    np.testing.assert_allclose(again, S.lnprob_dev[-1].cpu().numpy(), rtol=1e-12)


def test_reference_call_pattern_on_device(tmp_path):
    """The reference's burn-in -> reset -> production sequence through the
    emcee 2.x surface (mcmc_utils.py:114-164, mcmcfit.py:292-341) on the HIP
    sampler (config 2, 64 walkers): sampler.chain is (nwalkers, nsteps,
    npars), flatchain(sampler.chain, npars, thin=10) keeps steps 0, 10, 20,
    and the bulk mcmc_utils path writes the same chain_prod.txt byte for byte."""
    import torch
    from lfit_python_amd import batch, mcmc_utils, sampler, synthetic
    from tests.helpers import pattern_run_burnin, pattern_run_mcmc_save
    m = synthetic.config_single(300, flux_fn=_flux_fn)
    t = batch.compile_tree(m)
    ev = batch.LnProbEvaluator(t)
    p0 = np.array(m.dynasty_par_vals)
    init = sampler.initialise_walkers(p0, sampler.comp_scatter(m.dynasty_par_names, 0.1), 64,
                                      lambda p: ev(torch.as_tensor(p, device="cuda")).cpu().numpy())
    names = "walker_no " + " ".join(m.dynasty_par_names) + " ln_prob"
    npars, nprod = t.ndim, 25
    S1 = sampler.EnsembleSampler(64, npars, ev, seed=17)
    pos, prob, state = pattern_run_burnin(S1, init, 6)
    S1.reset()
    f1 = str(tmp_path / "pattern.txt")
    S1 = pattern_run_mcmc_save(S1, pos, nprod, state, f1, col_names=names)
    chain = S1.chain
    assert chain.shape == (64, nprod, npars) and S1.lnprobability.shape == (64, nprod)
    flat = mcmc_utils.flatchain(S1.chain, npars, thin=10)
    dev = S1.chain_dev.cpu().numpy()
    np.testing.assert_array_equal(flat, dev[::10].transpose(1, 0, 2).reshape(-1, npars))
    S2 = sampler.EnsembleSampler(64, npars, ev, seed=17)
    pos2, prob2, state2 = mcmc_utils.run_burnin(S2, init, 6)
    S2.reset()
    f2 = str(tmp_path / "bulk.txt")
    mcmc_utils.run_mcmc_save(S2, pos2, nprod, state2, f2, col_names=names, chunk=10)
    assert open(f1).read() == open(f2).read()
    np.testing.assert_array_equal(S2.chain, chain)
    # the stored ln_prob is the ln_prob of the stored positions
    again = ev(torch.as_tensor(chain[:, -1].copy(), device="cuda")).cpu().numpy()
    np.testing.assert_allclose(again, S1.lnprobability[:, -1], rtol=1e-12)


def test_fused_half_step_matches_separate_kernels():
    """lfg_stretch_step_half_spec (the default single-process path: proposal
    and setup formed speculatively in the previous half's k_elements,
    acceptance in k_lnlike) and lfg_stretch_step_half give the chain of
    lfg_stretch_propose + lfg_lnprob + lfg_stretch_accept, bit for bit, across
    reset() and set_state(); and so do lfg_stretch_lnprob_accept and the
    sharded path (lfg_stretch_step_shard on one or two shards +
    lfg_stretch_accept_regen)."""
    import torch
    from lfit_python_amd import batch, sampler, synthetic
    out = []
    for cfg in ("c2", "c3"):
        if cfg == "c2":
            m = synthetic.config_single(300, flux_fn=_flux_fn)
        else:
            m = synthetic.config_tree(2, 200, flux_fn=_flux_fn)   # E = 6: the last-eclipse counter path
        t = batch.compile_tree(m)
        ev = batch.LnProbEvaluator(t)
        p0 = np.array(m.dynasty_par_vals)
        W = 64 if cfg == "c2" else 2 * len(p0) + 2
        init = sampler.initialise_walkers(p0, sampler.comp_scatter(m.dynasty_par_names, 0.1), W,
                                          lambda p: ev(torch.as_tensor(p, device="cuda")).cpu().numpy())
        res = []
        for mode in ("separate", "spec", "step_half", "lnprob_accept", "shard1", "shard1_spec", "shard2"):
            S = sampler.EnsembleSampler(W, t.ndim, ev, seed=21)
            S.fuse = mode in ("spec", "step_half", "lnprob_accept")
            S.spec = mode in ("spec", "shard1_spec")
            S.force_shard = mode.startswith("shard")
            if mode == "shard2":
                # two ranks' shards of each half (lfg_stretch_step_shard with
                # lo = 0 and lo = k) into one ln_prob vector, as the gather does
                def shard(pos, h, a, seed, step, lo, q, zfac, lnp_sh, ev=ev):
                    k = lnp_sh.shape[0] // 2
                    for lo_, hi_ in ((0, k), (k, lnp_sh.shape[0])):
                        ev.step_shard(pos, h, a, seed, step, lo_, q[lo_:hi_], zfac[lo_:hi_], lnp_sh[lo_:hi_])
                S.shard_timer = shard
            if mode == "lnprob_accept":
                def half(pos, lnp, h, a, seed, step, q, zfac, naccept, lnp_new=None, S=S, ev=ev):
                    S.ops.propose(pos, h, a, seed, step, q, zfac)
                    ev.lnprob_accept(q, pos, lnp, h, zfac, seed, step, naccept, lnp_new=lnp_new)
                S.half_timer = half
            S.run_mcmc(init, 4)
            S.reset()
            S.run_mcmc(None, 3)
            ch, lc = S.chain_dev.cpu().numpy(), S.lnprob_dev.cpu().numpy()
            S.run_mcmc(ch[1], 2)  # set_state: new positions drop the speculative candidates
            res.append((ch, lc, S.chain_dev.cpu().numpy(), S.naccept.cpu().numpy()))
        for other in res[1:]:
            for a, b in zip(res[0], other):
                np.testing.assert_array_equal(a, b)


def test_graph_replay_matches_eager():
    """HIP-graph replay of whole iterations (device step counter) gives the
    bit-identical chain of the eager path, including across reset()."""
    import torch
    from lfit_python_amd import batch, sampler, synthetic
    m = synthetic.config_single(300, flux_fn=_flux_fn)
    t = batch.compile_tree(m)
    ev = batch.LnProbEvaluator(t)
    p0 = np.array(m.dynasty_par_vals)
    init = sampler.initialise_walkers(p0, sampler.comp_scatter(m.dynasty_par_names, 0.1), 64,
                                      lambda p: ev(torch.as_tensor(p, device="cuda")).cpu().numpy())
    out = []
    for graph in (False, True):
        S = sampler.EnsembleSampler(64, t.ndim, ev, seed=11)
        S.use_graph = graph
        S.run_mcmc(init, 6)
        S.reset()
        pos, lnp, _ = S.run_mcmc(None, 4)
        out.append((S.chain_dev.cpu().numpy(), S.lnprob_dev.cpu().numpy(), S.naccept.cpu().numpy()))
        if graph:
            assert S._graph is not None
    for a, b in zip(out[0], out[1]):
        np.testing.assert_array_equal(a, b)


@LAYOUTS
def test_spec_chain_with_interleaved_calls(layout):
    """The speculative path stays bit-identical to the plain half-step when
    other entry points use the evaluator between steps (their workspace use
    overlaps the candidates, so the next step recomputes its setup)."""
    import torch
    from lfit_python_amd import batch, sampler, synthetic
    m = synthetic.config_single(300, flux_fn=_flux_fn)
    t = batch.compile_tree(m)
    ev = batch.LnProbEvaluator(t)
    p0 = np.array(m.dynasty_par_vals)
    init = sampler.initialise_walkers(p0, sampler.comp_scatter(m.dynasty_par_names, 0.1), 96,
                                      lambda p: ev(torch.as_tensor(p, device="cuda")).cpu().numpy())
    out = []
    for spec in (False, True):
        S = sampler.EnsembleSampler(96, t.ndim, ev, seed=5)
        S.spec = spec
        S.set_state(init)
        rows = []
        for i in range(6):
            S.step()
            if i == 2:
                ev(S.pos[:64].contiguous())  # an lfg_lnprob call on the same workspace
            rows.append((S.pos.cpu().numpy().copy(), S.lnp.cpu().numpy().copy()))
        out.append(rows)
    for (pa, la), (pb, lb) in zip(*out):
        np.testing.assert_array_equal(pa, pb)
        np.testing.assert_array_equal(la, lb)


def test_spec_chain_survives_inplace_writes():
    """Writing S.pos / S.lnp in place between steps (same pointers) must drop
    the speculative candidates formed from the old positions: the chain
    equals the plain (spec off) chain with the same writes, bit for bit,
    on the single-process and the sharded path."""
    import torch
    from lfit_python_amd import batch, sampler, synthetic
    m = synthetic.config_single(300, flux_fn=_flux_fn)
    t = batch.compile_tree(m)
    ev = batch.LnProbEvaluator(t)
    p0 = np.array(m.dynasty_par_vals)
    init = sampler.initialise_walkers(p0, sampler.comp_scatter(m.dynasty_par_names, 0.1), 64,
                                      lambda p: ev(torch.as_tensor(p, device="cuda")).cpu().numpy())
    for shard in (False, True):
        out = []
        for spec in (False, True):
            S = sampler.EnsembleSampler(64, t.ndim, ev, seed=13)
            S.spec = spec
            S.force_shard = shard
            S.set_state(init)
            rows = []
            for i in range(6):
                S.step()
                if i == 1:
                    S.pos[0] = S.pos[1]          # in place: same data_ptr
                    S.lnp[0] = S.lnp[1]
                if i == 3:
                    S.pos[5:9] *= 1.0 + 1e-9
                    S.lnp[5:9] = ev(S.pos[5:9].contiguous())
                rows.append((S.pos.cpu().numpy().copy(), S.lnp.cpu().numpy().copy()))
            out.append(rows)
        for (pa, la), (pb, lb) in zip(*out):
            np.testing.assert_array_equal(pa, pb)
            np.testing.assert_array_equal(la, lb)


# ---------------------------------------------------------------- GP trees
def test_wdphases_matches_oracle(oracle):
    from lfit_python_amd import roche
    for q, dphi, r1 in ((0.1037, 0.0392, 0.0187), (0.2, 0.05, 0.01), (0.06, 0.03, 0.03)):
        inc = oracle.findi(q, dphi)
        got = roche.wdphases(q, inc, r1, 10)
        ref = oracle.wdphases(q, inc, r1, 10)
        np.testing.assert_allclose(got, ref, rtol=0, atol=1e-11)
        assert got[0] < dphi / 2 < got[1]


def test_gp_kernel_matches_dense_oracle(oracle):
    """lfg_gp_lnlike (Kalman filter, one wave per set) against the dense
    Cholesky oracle; bar 1e-9 relative (both exact, FP64 rounding apart)."""
    from lfit_python_amd import gp
    rng = np.random.default_rng(3)
    n, W = 300, 24
    x = rng.permutation(np.linspace(-0.2, 0.3, n))   # unsorted input: the wrapper sorts
    ye = rng.uniform(0.003, 0.006, n)
    res = 0.004 * rng.standard_normal((W, n))
    hyp = np.stack([np.exp(rng.uniform(-11, -8, W)), np.exp(rng.uniform(-11, -8, W)),
                    np.exp(rng.uniform(-6.9, -2, W))], axis=1)
    d = rng.uniform(0.01, 0.05, W)
    blocks = np.stack([np.stack([-1 + d, -d], 1), np.stack([d, 1 - d], 1)], axis=1)
    got = gp.log_likelihood_batch(x, ye, res, hyp, blocks)
    for i in range(W):
        ref = oracle.gp_lnlike(x, res[i], ye, *hyp[i], blocks[i])
        assert abs(got[i] - ref) <= 1e-9 * abs(ref), (i, got[i], ref)


@LAYOUTS
def test_gp_tree_matches_reference(layout):
    """Batched ln_prob of the shipped GP example (87 parameters, 6 eclipses)
    against the reference tree's own ln_prob (tests/golden/lnprob_gp.npz)."""
    import torch
    from lfit_python_amd import batch, cvmodel
    d = np.load(os.path.join(GOLD, "lnprob_gp.npz"))
    m = cvmodel.construct_model(os.path.join(GOLD, "ref_test_data", "mcmc_input.dat"))
    t = batch.compile_tree(m)
    ev = batch.LnProbEvaluator(t)
    W = len(d["walkers"])
    lle = torch.empty((W, t.E), dtype=torch.float64, device="cuda")
    got = ev(torch.as_tensor(d["walkers"], device="cuda"), lnlike_e=lle).cpu().numpy()
    _same(got, d["ln_prob"], LNP_RTOL)
    fin = np.isfinite(d["ln_prior"])
    _same(lle.cpu().numpy().sum(1)[fin], d["ln_like"][fin], LNP_RTOL)


@LAYOUTS
def test_gp_tree_spec_chain(layout):
    """The speculative half-step on the shipped GP tree (87 parameters, 6
    eclipses: acceptance through k_gp_like's per-walker combine) equals the
    plain half-step bit for bit."""
    import torch
    from lfit_python_amd import batch, cvmodel, sampler
    m = cvmodel.construct_model(os.path.join(GOLD, "ref_test_data", "mcmc_input.dat"))
    t = batch.compile_tree(m)
    ev = batch.LnProbEvaluator(t)
    p0 = np.array(m.dynasty_par_vals)
    W = 2 * len(p0) + 2
    init = sampler.initialise_walkers(p0, sampler.comp_scatter(m.dynasty_par_names, 0.1), W,
                                      lambda p: ev(torch.as_tensor(p, device="cuda")).cpu().numpy())
    out = []
    for spec in (False, True):
        S = sampler.EnsembleSampler(W, t.ndim, ev, seed=9)
        S.spec = spec
        S.run_mcmc(init, 3)
        out.append((S.chain_dev.cpu().numpy(), S.lnprob_dev.cpu().numpy(), S.naccept.cpu().numpy()))
    for a, b in zip(*out):
        np.testing.assert_array_equal(a, b)


def test_gp_leaf_scalar_path():
    """The one-walker host path (cvmodel GP leaves with the reference's
    changepoint cache, lfit_python_amd.gp) against the golden ln_prob."""
    import copy
    from lfit_python_amd import cvmodel
    d = np.load(os.path.join(GOLD, "lnprob_gp.npz"))
    m = cvmodel.construct_model(os.path.join(GOLD, "ref_test_data", "mcmc_input.dat"))
    m.ln_like()  # fills the changepoint caches at the start values, as mcmcfit.py:154 does
    for i in (0, 1, 5, 6):
        mc = copy.deepcopy(m)
        mc.dynasty_par_vals = list(d["walkers"][i])
        got = mc.ln_prob()
        ref = d["ln_prob"][i]
        assert np.isfinite(got) == np.isfinite(ref)
        if np.isfinite(ref):
            assert abs(got - ref) <= LNP_RTOL * abs(ref), (i, got, ref)


@pytest.mark.parametrize("tag", ["tree", "simple", "gp"])
def test_lnprior_matches_reference(tag, tmp_path):
    """lfg_lnprior (mcmcfit.ln_prior, used for the walker ball) against the
    reference tree's own ln_prior on the golden walkers."""
    import torch
    from lfit_python_amd import batch, cvmodel
    if tag == "gp":
        d = np.load(os.path.join(GOLD, "lnprob_gp.npz"))
        m = cvmodel.construct_model(os.path.join(GOLD, "ref_test_data", "mcmc_input.dat"))
    else:
        d, m = _golden_tree(tag, tmp_path)
    ev = batch.LnProbEvaluator(batch.compile_tree(m))
    got = ev.ln_prior(torch.as_tensor(d["walkers"], device="cuda")).cpu().numpy()
    _same(got, d["ln_prior"], 1e-10)


def test_lnprior_tiny_log_uniform_products():
    """The prior lanes form one log per chunk of 16 log_uniform / mod_jeff
    arguments: a chunk of tiny values (partial products far below the
    normal range) must still give the sum of the per-parameter terms
    (the running product keeps its exponent apart)."""
    import dataclasses
    import torch
    from lfit_python_amd import batch, synthetic
    from lfit_python_amd.tree import Prior
    m = synthetic.config_single(300, flux_fn=_flux_fn)
    t = batch.compile_tree(m)
    nd = t.ndim
    rng = np.random.default_rng(8)
    types = np.array([3 if k % 3 else 4 for k in range(nd)], np.int32)    # log_uniform, mod_jeff
    p1 = np.where(types == 3, 1e-30, 1e-200)
    p2 = np.where(types == 3, 1e-5, 1.0)
    pri = [Prior("log_uniform" if ty == 3 else "mod_jeff", a, b) for ty, a, b in zip(types, p1, p2)]
    t2 = dataclasses.replace(t, prior_type=types, prior_p1=p1.astype(np.float64), prior_p2=p2.astype(np.float64),
                             prior_norm=np.array([p.normalise for p in pri]), roche_priors=False)
    ev = batch.LnProbEvaluator(t2)
    W = 64
    walkers = np.exp(rng.uniform(np.log(1e-29), np.log(1e-6), (W, nd)))
    walkers[:, types == 4] = np.exp(rng.uniform(np.log(1e-199), np.log(0.5), (W, int((types == 4).sum()))))
    got = ev.ln_prior(torch.as_tensor(walkers, device="cuda")).cpu().numpy()
    ref = np.array([sum(p.ln_prob(v) for p, v in zip(pri, row)) for row in walkers])
    np.testing.assert_allclose(got, ref, rtol=1e-13, atol=1e-11)


@pytest.mark.gpu
@pytest.mark.parametrize("nsub", [1, 3])
def test_lfg_lnlike_matches_tree_and_cpu_twin(oracle, nsub, tmp_path):
    """lfg_lnlike (one eclipse, fused chi^2, no tree) against lfg_lnprob's
    per-eclipse ln_like on the same one-eclipse tree, and against its CPU
    twin lfg_cpu_lnlike (cpu_baseline/lfg_cpu.h), both through ctypes."""
    import torch
    from cpu_baseline import cpu
    from lfit_python_amd import batch, synthetic
    from lfit_python_amd.lfit import lnlike_batch
    dev = torch.device("cuda", 0)
    m = synthetic.config_single(300, flux_fn=lambda p, x, w, ns: oracle.flux(p, x, w, nsub=ns)[1], nsub=nsub)
    t = batch.compile_tree(m, nsub=nsub)
    ev = batch.LnProbEvaluator(t, device=dev)
    rng = np.random.default_rng(41)
    p0 = np.array(m.dynasty_par_vals)
    walk = p0 * (1.0 + 0.02 * rng.standard_normal((96, p0.size)))
    lle = torch.empty((96, 1), dtype=torch.float64, device=dev)
    lnp = ev(torch.as_tensor(walk, device=dev), lnlike_e=lle).cpu().numpy()
    leaf = m.leaves()[0]
    # each walker's CV vector, as the tree routes it (cv_parlist)
    pars = np.empty((96, 18))
    for i in range(96):
        m.dynasty_par_vals = walk[i]
        pars[i] = leaf.cv_parlist
    lc = leaf.lc
    got, st = lnlike_batch(pars, lc.x, lc.y, lc.ye, width=lc.w, nsub=nsub, device=dev)
    got = got.cpu().numpy()
    ref = lle.cpu().numpy()[:, 0]
    fin = np.isfinite(lnp)   # the tree skips walkers its priors reject
    assert fin.sum() >= 48
    np.testing.assert_allclose(got[fin], ref[fin], rtol=1e-12, atol=1e-9)
    port = cpu.CpuPort(cpu.build(out=str(tmp_path / "liblfg_cpu.so")))
    twin, st2 = port.lnlike(pars, lc.x, lc.w, lc.y, lc.ye, nsub=nsub, nthreads=4)
    np.testing.assert_array_equal(st2, st.cpu().numpy())
    ok = st2 == 0
    np.testing.assert_allclose(got[ok], twin[ok], rtol=1e-10, atol=1e-8)
    assert np.all(np.isneginf(got[~ok]))


def test_chunked_production_keeps_device_memory_flat(tmp_path):
    """mcmc_utils.run_mcmc_save in chunks (as mcmcfit does): each run's
    stored chunk moves to host memory when the run ends, so device memory
    after every chunk is the same however many chunks were written (ADVICE
    r03: the chunks used to stay on the device until reset()); last_run()
    is the most recent run's chunk, and None after a run that stored nothing."""
    import torch
    from lfit_python_amd import batch, mcmc_utils, sampler, synthetic
    m = synthetic.config_single(300, flux_fn=_flux_fn)
    t = batch.compile_tree(m)
    ev = batch.LnProbEvaluator(t)
    p0 = np.array(m.dynasty_par_vals)
    W = 64
    init = sampler.initialise_walkers(p0, sampler.comp_scatter(m.dynasty_par_names, 0.1), W,
                                      lambda p: ev(torch.as_tensor(p, device="cuda")).cpu().numpy())
    S = sampler.EnsembleSampler(W, t.ndim, ev, seed=5)
    pos, lnp, st = S.run_mcmc(init, 2, storechain=False)
    assert S.last_run() is None
    used = []
    for k in range(6):
        S.run_mcmc(None, 10, storechain=True)
        torch.cuda.synchronize()
        used.append(torch.cuda.memory_allocated())
        ch, lp = S.last_run()
        assert ch.shape == (10, W, t.ndim) and ch.device.type == "cpu"
    assert max(used) == min(used), used
    assert S.chain.shape == (W, 60, t.ndim)
    np.testing.assert_array_equal(S.chain[:, -10:], np.asarray(ch).transpose(1, 0, 2))
    S.run_mcmc(None, 3, storechain=False)
    assert S.last_run() is None
