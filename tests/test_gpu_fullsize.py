"""GPU: the BASELINE configs at their real walker counts, through the same
fused launch path bench.py times (lfg_stretch_step_half / _shard), checked
against the CPU oracle.

* configs 2, 3, 5 at W = 1024, 2048, 4096: one half-step's proposals q and
  their ln_prob.  Every proposal's finite/-inf pattern against the oracle
  (on the tree with each light curve cut to its first 8 points: the pattern
  depends only on priors and geometry), a seeded subset of 32 proposals'
  ln_prob at the full tree to 1e-8;
* config 4 (the 16384-walker ensemble): the chain of 8 emulated rank shards
  (lfg_stretch_step_shard at lo = k x 1024, the shard vectors concatenated
  as the all_gather does, lfg_stretch_accept_regen) is bit-identical to the
  single-process chain, and 64 proposals' ln_prob match the oracle;
* the multi-rank code path with two real ranks (gloo, both on cuda:0) gives
  the single-rank chain bit for bit.
"""
import copy
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
LNP_RTOL = 1e-8


def _flux_fn(p, x, w, nsub):
    from lfit_python_amd.lfit import flux_batch
    f, _ = flux_batch(np.asarray(p)[None, :], x, w, nsub=nsub)
    return f[0].cpu().numpy()


def _model(cfg):
    from lfit_python_amd import synthetic
    if cfg == "c3":
        return synthetic.config_tree(4, 300, flux_fn=_flux_fn), 1, 2048
    if cfg == "c5":
        return synthetic.config_single(10000, flux_fn=_flux_fn, nsub=5), 5, 4096
    if cfg == "c4":
        return synthetic.config_single(300, flux_fn=_flux_fn), 1, 16384
    return synthetic.config_single(300, flux_fn=_flux_fn), 1, 1024


def _ensemble(cfg, seed=7):
    import torch
    from lfit_python_amd import batch, sampler
    m, nsub, W = _model(cfg)
    t = batch.compile_tree(m, nsub=nsub)
    ev = batch.LnProbEvaluator(t, max_walkers=W)
    p0 = np.array(m.dynasty_par_vals)
    init = sampler.initialise_walkers(p0, sampler.comp_scatter(m.dynasty_par_names, 0.1), W,
                                      lambda p: ev(torch.as_tensor(p, device="cuda")).cpu().numpy(), seed=seed)
    return m, t, ev, init


def _short_tree(t, k=8):
    """The compiled tree with every eclipse's data cut to its first k points."""
    s = copy.copy(t)
    offs, xs, ys, yes, ws = [0], [], [], [], []
    for e in range(t.E):
        a, b = t.offsets[e], min(t.offsets[e + 1], t.offsets[e] + k)
        for dst, src in ((xs, t.x), (ys, t.y), (yes, t.ye), (ws, t.w)):
            dst.append(src[a:b])
        offs.append(offs[-1] + b - a)
    s.x, s.y, s.ye, s.w = (np.concatenate(v) for v in (xs, ys, yes, ws))
    s.offsets = np.asarray(offs, np.int32)
    return s


def _check_against_oracle(oracle, t, q, lnp, nsub, nsubset=32, seed=11):
    # the finite pattern of every proposal (priors, Roche priors, geometry)
    ref_short, _, _ = oracle.lnprob_batch(q, _short_tree(t), nsub=nsub)
    np.testing.assert_array_equal(np.isfinite(lnp), np.isfinite(ref_short))
    # full ln_prob of a seeded subset of the finite ones
    fin = np.flatnonzero(np.isfinite(lnp))
    pick = np.random.default_rng(seed).choice(fin, size=min(nsubset, len(fin)), replace=False)
    ref, _, _ = oracle.lnprob_batch(q[pick], t, nsub=nsub)
    np.testing.assert_allclose(lnp[pick], ref, rtol=LNP_RTOL, atol=1e-9)


@pytest.mark.parametrize("cfg", ["c2", "c3", "c5"])
def test_full_size_half_step_matches_oracle(oracle, cfg):
    from lfit_python_amd import sampler
    m, t, ev, init = _ensemble(cfg)
    W = init.shape[0]
    S = sampler.EnsembleSampler(W, t.ndim, ev, seed=5)
    S.set_state(init)
    S.step()  # one whole iteration, then the half-step under test
    pos_before = S.pos.cpu().numpy()
    S.step()
    q, lnp = S.q.cpu().numpy(), S.lnp_new.cpu().numpy()   # half 1's proposals and their ln_prob
    assert q.shape == (W // 2, t.ndim)
    # the proposals are the stretch move of the ensemble as it stood (k_setup's inline proposal)
    assert np.all(np.isfinite(q))
    _check_against_oracle(oracle, t, q, lnp, t.nsub)
    # accepted walkers of half 1 took exactly their proposal and its ln_prob
    pos, lp = S.pos.cpu().numpy(), S.lnp.cpu().numpy()
    moved = np.any(pos[W // 2:] != pos_before[W // 2:], axis=1)
    np.testing.assert_array_equal(pos[W // 2:][moved], q[moved])
    np.testing.assert_array_equal(lp[W // 2:][moved], lnp[moved])


def test_config4_eight_shards_bit_identical(oracle):
    import torch
    from lfit_python_amd import sampler
    m, t, ev, init = _ensemble("c4")
    W, nranks = 16384, 8
    shard = W // 2 // nranks   # 1024 walkers of each half per rank
    chains = []
    for mode in ("fused", "shards"):
        S = sampler.EnsembleSampler(W, t.ndim, ev, seed=13)
        if mode == "shards":
            S.force_shard = True
            got = {}

            def eight(pos, h, a, seed, step, lo, q, zfac, lnp_sh, S=S, got=got):
                # lnp_sh is the [W/2] gathered vector of the one-rank sampler:
                # fill it shard by shard as 8 ranks and the all_gather would
                assert lnp_sh.shape[0] == W // 2
                for k in range(nranks):
                    sl = slice(k * shard, (k + 1) * shard)
                    S.ev.step_shard(pos, h, a, seed, step, k * shard, q[sl], zfac[sl], lnp_sh[sl])
                got["q"], got["lnp"] = q.clone(), lnp_sh.clone()
            S.shard_timer = eight
        S.set_state(init)
        S.run_mcmc(None, 3)
        chains.append((S.chain_dev.cpu().numpy(), S.lnprob_dev.cpu().numpy(), S.naccept.cpu().numpy()))
    for a, b in zip(*chains):
        np.testing.assert_array_equal(a, b)
    q, lnp = got["q"].cpu().numpy(), got["lnp"].cpu().numpy()
    assert torch.isfinite(got["lnp"]).sum() > W // 4
    _check_against_oracle(oracle, t, q, lnp, 1, nsubset=64)


def test_config4_eight_rank_workspaces_spec_path(oracle):
    """The path a real N = 8 run of config 4 takes, rank by rank: 8
    evaluators (one workspace each, as 8 processes have), each holding the
    whole 16 384-walker ensemble, running lfg_stretch_step_shard_spec on its
    1 024 walkers of the half (lo = k x 1024), the shard vectors concatenated
    as ncclAllGather would, then lfg_stretch_accept_regen_spec over the whole
    half on every rank.  From the second half-step on, every rank's shard
    takes its setup from the candidates its previous k_elements formed.  The
    chain is bit-identical on all 8 ranks and to the single-process fused
    chain; 64 proposals of the last half match the oracle."""
    import torch
    from lfit_python_amd import batch, sampler
    m, t, ev0, init = _ensemble("c4")
    W, R, iters = 16384, 8, 3
    n = W // 2 // R
    S = sampler.EnsembleSampler(W, t.ndim, ev0, seed=29)
    S.set_state(init)
    lnp_init = S.lnp.clone()
    S.run_mcmc(None, iters)
    ref = (S.chain_dev.cpu().numpy(), S.lnprob_dev.cpu().numpy(), S.naccept.cpu().numpy())
    del S
    f64 = dict(dtype=torch.float64, device="cuda")
    evs = [batch.LnProbEvaluator(t, max_walkers=W // 2) for _ in range(R)]
    pos = [torch.as_tensor(init, **f64).contiguous() for _ in range(R)]
    lnp = [lnp_init.clone() for _ in range(R)]
    nacc = [torch.zeros(W, dtype=torch.int32, device="cuda") for _ in range(R)]
    q = [torch.empty((n, t.ndim), **f64) for _ in range(R)]
    zf = [torch.empty(n, **f64) for _ in range(R)]
    lsh = [torch.empty(n, **f64) for _ in range(R)]
    chain, lchain, spec_used = [], [], 0
    for it in range(iters):
        for half in (0, 1):
            for k in range(R):
                key = evs[k]._spec_key
                spec_used += int(key is not None and key[-3:] == (half, it, "accepted"))
                evs[k].step_shard(pos[k], half, 2.0, 29, it, k * n, q[k], zf[k], lsh[k], spec=True)
            lnp_new = torch.cat(lsh)                 # what the all_gather hands every rank
            for k in range(R):
                evs[k].accept_regen(pos[k], lnp[k], half, 2.0, 29, it, lnp_new, nacc[k], n)
        for k in range(1, R):
            assert torch.equal(pos[k], pos[0]) and torch.equal(lnp[k], lnp[0])
        chain.append(pos[0].cpu().numpy())
        lchain.append(lnp[0].cpu().numpy())
    assert spec_used == R * (2 * iters - 1)          # every half but the first ran on candidates
    np.testing.assert_array_equal(np.stack(chain), ref[0])
    np.testing.assert_array_equal(np.stack(lchain), ref[1])
    np.testing.assert_array_equal(nacc[0].cpu().numpy(), ref[2])
    qa = torch.cat(q).cpu().numpy()
    assert torch.isfinite(lnp_new).sum() > W // 4
    _check_against_oracle(oracle, t, qa, lnp_new.cpu().numpy(), 1, nsubset=64)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, port, init, out):
    import torch
    import torch.distributed as dist
    from lfit_python_amd import batch, sampler, synthetic
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=2)
    try:
        m = synthetic.config_single(300, flux_fn=_flux_fn)
        t = batch.compile_tree(m)
        ev = batch.LnProbEvaluator(t)
        S = sampler.EnsembleSampler(init.shape[0], t.ndim, ev, seed=17)
        assert S.world == 2 and S.fuse_shard
        S.set_state(init)
        S.run_mcmc(None, 4)
        out[rank] = (S.chain_dev.cpu().numpy(), S.lnprob_dev.cpu().numpy())
        S.close()
    finally:
        dist.destroy_process_group()


def test_two_real_ranks_hip_shards_match_single_rank():
    """Two ranks (gloo; both on the one GPU of the box) run the multi-rank
    HIP path: lfg_stretch_step_shard on their own shard, all_gather of
    ln_prob, lfg_stretch_accept_regen.  Their chains equal the single-rank
    fused chain bit for bit."""
    import torch.multiprocessing as mp
    from lfit_python_amd import sampler
    m, t, ev, init = _ensemble("c2", seed=3)
    init = init[:256]
    S = sampler.EnsembleSampler(256, t.ndim, ev, seed=17)
    S.set_state(init)
    S.run_mcmc(None, 4)
    ref = (S.chain_dev.cpu().numpy(), S.lnprob_dev.cpu().numpy())
    out = mp.Manager().dict()
    mp.start_processes(_rank, args=(_free_port(), init, out), nprocs=2, join=True, start_method="spawn")
    for r in (0, 1):
        np.testing.assert_array_equal(out[r][0], ref[0])
        np.testing.assert_array_equal(out[r][1], ref[1])
