"""GPU: the sharded half-step with the acceptance deferred into the next
launch (lfg_stretch_step_shard_fold / lfg_stretch_apply_verdicts).

Per half-step a rank runs ONE k_pair launch -- it applies the other half's
gathered verdicts of the half-step before, chooses each pair's speculative
candidate by them, evaluates its shard and leaves the shard's verdicts -- and
the exchange; k_accept_regen's launch is gone (the reference's analogue is
the pool.map fan-out of /root/reference/mcmcfit.py:273-288).  Every chain
here must be bit-identical to the single-process fused chain: the rows the
speculative lanes read through a pending verdict are re-formed exactly as the
apply writes them."""
import numpy as np
import pytest

from tests.test_gpu_fullsize import _check_against_oracle, _ensemble
from tests.test_gpu_lnprob import LAYOUTS, layout  # noqa: F401  (fixture)

pytestmark = pytest.mark.gpu


def _fused_chain(t, ev, init, seed, iters):
    from lfit_python_amd import sampler
    S = sampler.EnsembleSampler(init.shape[0], t.ndim, ev, seed=seed)
    S.set_state(init)
    lnp0 = S.lnp.clone()
    S.run_mcmc(None, iters)
    return (S.chain_dev.cpu().numpy(), S.lnprob_dev.cpu().numpy(), S.naccept.cpu().numpy()), lnp0


def _rank_chains(t, init, lnp0, seed, iters, R, evs=None, check_verdicts=True, layouts=None):
    """R evaluators (R ranks' workspaces), each holding the whole ensemble and
    running lfg_stretch_step_shard_fold on walkers k n .. (k+1) n - 1 of every
    half; the verdict shards concatenated as the all_gather hands them over.
    A step's state is recorded once its last verdicts are applied: right
    after the next step's half-0 launches (or after the final flush).
    layouts: optional lfg_set_layout value per half-step (2 it + half)."""
    import torch
    from lfit_python_amd import _native, batch
    W = init.shape[0]
    n = W // 2 // R
    f64 = dict(dtype=torch.float64, device="cuda")
    evs = evs or [batch.LnProbEvaluator(t, max_walkers=W // 2) for _ in range(R)]
    pos = [torch.as_tensor(init, **f64).contiguous() for _ in range(R)]
    lnp = [lnp0.clone() for _ in range(R)]
    nacc = [torch.zeros(W, dtype=torch.int32, device="cuda") for _ in range(R)]
    q = [torch.empty((n, t.ndim), **f64) for _ in range(R)]
    zf = [torch.empty(n, **f64) for _ in range(R)]
    lsh = [torch.empty(n, **f64) for _ in range(R)]
    vsh = [torch.empty(n, **f64) for _ in range(R)]
    V = [None, None]
    chain, lchain, spec_used = [], [], 0

    def record():
        for k in range(1, R):
            assert torch.equal(pos[k], pos[0]) and torch.equal(lnp[k], lnp[0]) and torch.equal(nacc[k], nacc[0])
        chain.append(pos[0].cpu().numpy())
        lchain.append(lnp[0].cpu().numpy())

    for it in range(iters):
        for half in (0, 1):
            vprev = V[1 - half]
            if layouts is not None:
                _native.lib().lfg_set_layout(int(layouts[2 * it + half]))
            for k in range(R):
                key = evs[k]._spec_key
                spec_used += int(key is not None and key[-2:] == (half, it) and vprev is not None)
                evs[k].step_shard_fold(pos[k], lnp[k], half, 2.0, seed, it, k * n, q[k], zf[k], lsh[k], vprev,
                                       vsh[k], nacc[k])
            if half == 0 and it > 0:
                record()   # step it - 1's state: its half-1 verdicts were applied just now
            V[half] = torch.cat(vsh)
            if check_verdicts:
                # a verdict is the evaluated ln_prob or NaN (rejected)
                lall, vall = torch.cat(lsh), V[half]
                acc = ~torch.isnan(vall)
                assert torch.equal(vall[acc], lall[acc])
    for k in range(R):   # the flush of the last half
        evs[k].apply_verdicts(pos[k], lnp[k], 1, 2.0, seed, iters - 1, V[1], nacc[k])
    record()
    return (np.stack(chain), np.stack(lchain), nacc[0].cpu().numpy()), spec_used, (torch.cat(q), torch.cat(lsh))


def test_config4_eight_rank_fold_workspaces(oracle):
    """The path an N = 8 run of config 4 takes with the deferred acceptance,
    rank by rank: 8 evaluators (8 workspaces), each holding the whole 16 384
    walkers, running lfg_stretch_step_shard_fold on its 1 024 walkers of the
    half (every launch applies the other half's 8 192 verdicts, 8 rows per
    workgroup).  Bit-identical on all ranks and to the fused chain; every half
    after the first runs on its candidates; the last half's proposals match
    the oracle."""
    m, t, ev0, init = _ensemble("c4")
    ref, lnp0 = _fused_chain(t, ev0, init, 29, 3)
    got, spec_used, (q, lsh) = _rank_chains(t, init, lnp0, 29, 3, 8)
    assert spec_used == 8 * (2 * 3 - 1)
    for a, b in zip(got, ref):
        np.testing.assert_array_equal(a, b)
    assert np.isfinite(lsh.cpu().numpy()).sum() > q.shape[0] // 4
    _check_against_oracle(oracle, t, q.cpu().numpy(), lsh.cpu().numpy(), 1, nsubset=64)


@LAYOUTS
@pytest.mark.parametrize("R", [1, 2])
def test_fold_config2_matches_fused(R, layout):
    """config 2 (1 024 walkers), one or two ranks' workspaces, on the k_pair
    layout (one launch per half) and the two-kernel layout (the fallback:
    apply, the shard's kernels, the verdict kernel)"""
    m, t, ev0, init = _ensemble("c2", seed=3)
    ref, lnp0 = _fused_chain(t, ev0, init, 17, 4)
    got, spec_used, _ = _rank_chains(t, init, lnp0, 17, 4, R)
    assert spec_used == R * (2 * 4 - 1)
    for a, b in zip(got, ref):
        np.testing.assert_array_equal(a, b)


def test_fold_layout_switch_between_halves_matches_fused():
    """lfg_set_layout between the halves of a deferred-acceptance chain (the
    contract include/lfg.h states): a two-kernel half-step followed by a fold
    k_pair half-step whose speculative lanes read the snapshot of the rows
    through the pending verdicts.  The two-kernel fallback leaves the same
    snapshot a fold k_pair launch leaves, so the chain follows the fused one
    whatever the switch pattern: positions and acceptance counts bit-identical,
    ln_prob to 1e-12 (the two layouts' sums differ in the last bits; a stale
    snapshot gives wrong candidates, i.e. different positions)."""
    from lfit_python_amd import _native
    m, t, ev0, init = _ensemble("c2", seed=3)
    init = init[:256]
    ref, lnp0 = _fused_chain(t, ev0, init, 19, 5)
    pattern = [1, 0, 1, 0, 0, 1, 1, 0, 1, 1]   # pair / two-kernel per half-step
    prev = _native.lib().lfg_set_layout(1)
    try:
        for R in (1, 2):
            got, _, _ = _rank_chains(t, init, lnp0, 19, 5, R, layouts=pattern)
            np.testing.assert_array_equal(got[0], ref[0])
            np.testing.assert_array_equal(got[2], ref[2])
            np.testing.assert_allclose(got[1], ref[1], rtol=1e-12, atol=0)
    finally:
        _native.lib().lfg_set_layout(prev)


def test_fold_e6_tree_fallback_matches_fused():
    """A 3-band x 2-eclipse tree (E = 6): the fold's fallback (the pending
    verdicts applied by their own launch, the shard's k_pair and
    k_combine_walkers, the verdicts from ln_prob) over two workspaces"""
    import torch
    from lfit_python_amd import batch, synthetic
    from tests.test_gpu_multirank import _flux_fn
    m = synthetic.config_tree(2, 200, flux_fn=_flux_fn)
    t = batch.compile_tree(m)
    ev0 = batch.LnProbEvaluator(t)
    W = 64
    rng = np.random.default_rng(17)
    p0 = np.array(m.dynasty_par_vals)
    init = p0 * (1.0 + 1e-3 * rng.standard_normal((W, p0.size)))
    ref, lnp0 = _fused_chain(t, ev0, init, 23, 3)
    got, _, _ = _rank_chains(t, init, lnp0, 23, 3, 2)
    for a, b in zip(got, ref):
        np.testing.assert_array_equal(a, b)
    assert torch.cuda.is_available()


def test_sampler_fold_path_matches_fused_with_stored_chain_and_breaks():
    """EnsembleSampler on the sharded path (force_shard, one rank) takes the
    fold: its stored chain (records deferred until a step's last verdicts are
    applied), lnprob and acceptance counters equal the fused chain's, across
    two run_mcmc calls, a sample() generator left early and S.pos reads in
    between (each flushes)."""
    from lfit_python_amd import sampler
    m, t, ev0, init = _ensemble("c2", seed=5)
    init = init[:256]
    S0 = sampler.EnsembleSampler(256, t.ndim, ev0, seed=41)
    S0.set_state(init)
    S0.run_mcmc(None, 7)
    ref = (S0.chain, S0.lnprobability, S0.naccepted)
    S = sampler.EnsembleSampler(256, t.ndim, ev0, seed=41)
    S.force_shard = True
    S.set_state(init)
    S.run_mcmc(None, 3)
    assert S._pending is None          # run_mcmc ends flushed
    p_mid = S.pos.cpu().numpy()
    np.testing.assert_array_equal(p_mid, S.chain[:, -1])
    for i, _ in enumerate(S.sample(iterations=3)):
        if i == 1:
            break                      # the generator left early: 2 steps stored
    S.run_mcmc(None, 2)
    got = (S.chain, S.lnprobability, S.naccepted)
    assert got[0].shape == ref[0].shape
    for a, b in zip(got, ref):
        np.testing.assert_array_equal(a, b)
    assert S._V is not None            # the fold path ran


def test_emulated_rank_fold_keeps_other_shards_still():
    """--emulate-rank K/N on the fold path: only rank K's shard of each half
    can move; the other shards' verdicts stay NaN"""
    import torch
    from lfit_python_amd import sampler
    m, t, ev0, init = _ensemble("c2", seed=9)
    S = sampler.EnsembleSampler(1024, t.ndim, ev0, seed=3)
    S.set_state(init)
    S.emulate_rank(1, 4)
    S.force_exchange = False
    before = S.pos.clone()
    S.run_mcmc(None, 4, storechain=False)
    after = S.pos
    moved = torch.any(after != before, dim=1).cpu().numpy()
    ns, n = 512, 128
    own = np.zeros(1024, bool)
    own[n:2 * n] = True
    own[ns + n:ns + 2 * n] = True
    assert moved[own].any() and not moved[~own].any()
    assert torch.isnan(S._V[0][:n]).all() and torch.isnan(S._V[0][2 * n:]).all()
