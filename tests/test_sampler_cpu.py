"""Sampler host logic on CPU: stretch-move semantics, walker initialisation,
and the multi-rank path (gloo, world_size 2) -- sharded ln_prob with an
all_gather per half-step must reproduce the single-rank chain exactly."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from lfit_python_amd.sampler import EnsembleSampler, comp_scatter, initialise_walkers
from tests import stretch_double as sd
from tests.helpers import pattern_run_burnin as _pattern_run_burnin
from tests.helpers import pattern_run_mcmc_save as _pattern_run_mcmc_save

NDIM, W, STEPS = 5, 16, 30


class GaussLnProb:
    """Stand-in evaluator: correlated Gaussian, -inf outside a box."""
    device = torch.device("cpu")

    def __init__(self):
        rng = np.random.default_rng(3)
        A = rng.standard_normal((NDIM, NDIM))
        self.P = torch.as_tensor(A @ A.T / NDIM + np.eye(NDIM))
        self.calls = []

    def __call__(self, x, out=None):
        self.calls.append(x.shape[0])
        v = -0.5 * torch.einsum("ni,ij,nj->n", x, self.P, x)
        v = torch.where((x.abs() < 4).all(1), v, torch.tensor(-np.inf, dtype=torch.float64))
        if out is not None:
            out.copy_(v)
            return out
        return v


def _p0():
    return np.random.default_rng(7).standard_normal((W, NDIM)) * 0.1


def _run_single():
    ev = GaussLnProb()
    S = EnsembleSampler(W, NDIM, ev, seed=99, ops=sd.TorchCpuOps())
    S.set_state(_p0())
    S.run_mcmc(None, STEPS)
    return S.chain_dev.numpy(), S.lnprob_dev.numpy(), ev.calls


def test_stretch_move_matches_numpy_reference():
    chain, lnp, calls = _run_single()
    assert set(calls[1:]) == {W // 2}                      # one batched call per half-step
    ev = GaussLnProb()
    pos = _p0()
    lp = ev(torch.as_tensor(pos)).numpy()
    nacc = np.zeros(W, np.int64)
    for it in range(STEPS):
        for half in (0, 1):
            q, zf = sd.propose(pos, half, 2.0, 99, it)
            new = ev(torch.as_tensor(q)).numpy()
            sd.accept(pos, lp, half, q, zf, new, 99, it, nacc)
        np.testing.assert_array_equal(chain[it], pos)
        np.testing.assert_array_equal(lnp[it], lp)
    assert 0.1 < nacc.mean() / STEPS < 0.9


def test_proposal_distribution():
    # z = ((a-1)u+1)^2/a has density ~ 1/sqrt(z) on [1/a, a]
    pos = np.random.default_rng(0).standard_normal((4096, 2))
    _, zf = sd.propose(pos, 0, 2.0, 5, 0)
    z = np.exp(zf)                                  # ndim - 1 = 1
    assert z.min() >= 0.5 and z.max() <= 2.0
    cdf = lambda t: (np.sqrt(2 * t) - 1) / (np.sqrt(2) - np.sqrt(0.5)) / np.sqrt(2)  # noqa: E731
    for t in (0.7, 1.0, 1.5):
        assert abs(np.mean(z < t) - (np.sqrt(t) - np.sqrt(0.5)) / (np.sqrt(2) - np.sqrt(0.5))) < 0.03
    del cdf


def _worker(rank, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=2)
    try:
        ev = GaussLnProb()
        S = EnsembleSampler(W, NDIM, ev, seed=99, ops=sd.TorchCpuOps())
        assert S.world == 2 and S.shard == W // 4
        S.set_state(_p0())
        S.run_mcmc(None, STEPS)
        out[rank] = (S.chain_dev.numpy().copy(), S.lnprob_dev.numpy().copy(), list(ev.calls))
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_two_rank_gloo_matches_single_rank():
    chain1, lnp1, _ = _run_single()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(_free_port(), out), nprocs=2, join=True)
    for r in (0, 1):
        chain, lnp, calls = out[r]
        np.testing.assert_array_equal(chain, chain1)    # replicated RNG: identical ensembles
        np.testing.assert_array_equal(lnp, lnp1)
        assert set(calls[1:]) == {W // 4}               # each rank evaluates its shard only


def test_initialise_walkers_resamples_invalid():
    p = np.array([1.0, 2.0, 3.0])
    calls = []

    def lnp(x):
        calls.append(len(x))
        return np.where(x[:, 0] > 1.05, -np.inf, 0.0)
    p0 = initialise_walkers(p, 0.1, 64, lnp, seed=1)
    assert p0.shape == (64, 3)
    assert np.all(p0[:, 0] <= 1.05)
    assert len(calls) >= 2


def test_comp_scatter_factors():
    names = ["q_core", "dphi_core", "ulimb_g", "ln_tau_gp_core", "az_0"]
    s = comp_scatter(names, 0.1)
    np.testing.assert_allclose(s, [0.1, 0.02, 1e-7, 0.1, 0.1])


def test_odd_walkers_rejected():
    with pytest.raises(ValueError):
        EnsembleSampler(15, NDIM, GaussLnProb(), ops=sd.TorchCpuOps())


def test_reset_keeps_the_random_stream():
    """reset() clears the counters but not the Philox counter: production
    draws continue the burn-in's stream instead of replaying it (the
    reference passes the burn-in RNG state on, mcmc_utils.py:135-183)."""
    ev = GaussLnProb()
    S = EnsembleSampler(W, NDIM, ev, seed=99, ops=sd.TorchCpuOps())
    S.run_mcmc(_p0(), 4, storechain=False)
    S.reset()
    assert S.iteration == 0 and S.random_state == 4 and int(S.naccept.sum()) == 0
    S.run_mcmc(None, 3)
    # the numpy double, steps 0..3 then 4..6 of one stream
    pos = _p0()
    lp = GaussLnProb()(torch.as_tensor(pos)).numpy()
    nacc = np.zeros(W, np.int64)
    for it in range(7):
        for half in (0, 1):
            q, zf = sd.propose(pos, half, 2.0, 99, it)
            sd.accept(pos, lp, half, q, zf, GaussLnProb()(torch.as_tensor(q)).numpy(), 99, it, nacc)
        if it >= 4:
            np.testing.assert_array_equal(S.chain_dev[it - 4].numpy(), pos)
    # replaying step 0 after the reset would have drawn the burn-in's z
    assert not np.array_equal(sd.propose(pos, 0, 2.0, 99, 0)[1], sd.propose(pos, 0, 2.0, 99, 4)[1])


def test_mcmc_utils_burnin_then_saved_production(tmp_path):
    from lfit_python_amd import mcmc_utils
    ev = GaussLnProb()
    S = EnsembleSampler(W, NDIM, ev, seed=99, ops=sd.TorchCpuOps())
    pos, prob, state = mcmc_utils.run_burnin(S, _p0(), 4)
    assert state == 4
    S.reset()
    names = ["p%d" % i for i in range(NDIM)]
    f = str(tmp_path / "chain_prod.txt")
    mcmc_utils.run_mcmc_save(S, pos, 5, state, f, col_names="walker_no " + " ".join(names) + " ln_prob", chunk=2)
    lines = open(f).read().splitlines()
    assert lines[0] == "walker_no p0 p1 p2 p3 p4 ln_prob" and len(lines) == 1 + 5 * W
    # rows in the reference's format: '{k:4d} {values} {ln_prob:f}'
    first = lines[1].split()
    assert lines[1].startswith("   0 ") and len(first) == NDIM + 2
    c = mcmc_utils.readchain(f)
    assert c.shape == (W, 5, NDIM + 1)
    np.testing.assert_array_equal(c[:, -1, :NDIM], S.pos.numpy())  # repr() round-trips exactly
    np.testing.assert_array_equal(mcmc_utils.readchain_dask(f), c)
    flat = mcmc_utils.flatchain(c, NDIM + 1, nskip=1, thin=2)
    assert flat.shape == (W * 2, NDIM + 1)
    np.testing.assert_array_equal(flat[:2], c[0, 1::2])


def test_initialise_walkers_reference_signature():
    from lfit_python_amd import mcmc_utils
    calls = []

    def ln_prior(p, model):  # mcmcfit.ln_prior(param_vector, model): one vector
        calls.append(model)
        return -np.inf if p[0] > 1.05 else 0.0
    p0 = mcmc_utils.initialise_walkers(np.array([1.0, 2.0]), 0.1, 32, ln_prior, "m", seed=2)
    assert p0.shape == (32, 2) and np.all(p0[:, 0] <= 1.05) and set(calls) == {"m"}


# ---- emcee 2.x surface: the reference's own call patterns over the sampler
def test_reference_call_pattern_and_flatchain(tmp_path):
    """The reference's burn-in -> reset -> production -> flatchain sequence
    (mcmcfit.py:292-341) through sample(): sampler.chain is
    (nwalkers, nsteps, npars), flatchain(sampler.chain, npars, thin=10)
    keeps every 10th step, and the bulk mcmc_utils path writes the same file
    and chain byte for byte."""
    from lfit_python_amd import mcmc_utils
    names = "walker_no " + " ".join("p%d" % i for i in range(NDIM)) + " ln_prob"
    nprod = 25
    S1 = EnsembleSampler(W, NDIM, GaussLnProb(), seed=99, ops=sd.TorchCpuOps())
    pos, prob, state = _pattern_run_burnin(S1, _p0(), 4)
    assert state == 4 and pos.shape == (W, NDIM) and prob.shape == (W,)
    S1.reset()
    f1 = str(tmp_path / "pattern.txt")
    S1 = _pattern_run_mcmc_save(S1, pos, nprod, state, f1, col_names=names)
    assert S1.chain.shape == (W, nprod, NDIM) and S1.lnprobability.shape == (W, nprod)
    assert S1.iterations == nprod and S1.flatchain.shape == (W * nprod, NDIM)
    flat = mcmc_utils.flatchain(S1.chain, NDIM, thin=10)
    assert flat.shape == (W * 3, NDIM)
    steps = S1.chain_dev.numpy()[::10]                    # steps 0, 10, 20 of production
    np.testing.assert_array_equal(flat, steps.transpose(1, 0, 2).reshape(-1, NDIM))
    np.testing.assert_array_equal(mcmc_utils.flatchain(S1.chain_dev.permute(1, 0, 2), NDIM, thin=10), flat)
    # the stored production steps are the stretch move's (numpy double),
    # continuing the burn-in's random stream
    p, lp = _p0(), None
    lp = GaussLnProb()(torch.as_tensor(p)).numpy()
    nacc = np.zeros(W, np.int64)
    for it in range(4 + nprod):
        for half in (0, 1):
            q, zf = sd.propose(p, half, 2.0, 99, it)
            sd.accept(p, lp, half, q, zf, GaussLnProb()(torch.as_tensor(q)).numpy(), 99, it, nacc)
        if it >= 4:
            np.testing.assert_array_equal(S1.chain[:, it - 4], p)
            # (production starts from set_state's batched ln_prob: rounding apart)
            np.testing.assert_allclose(S1.lnprobability[:, it - 4], lp, rtol=1e-14)
    # the bulk path: same file, same chain
    S2 = EnsembleSampler(W, NDIM, GaussLnProb(), seed=99, ops=sd.TorchCpuOps())
    pos2, prob2, state2 = mcmc_utils.run_burnin(S2, _p0(), 4)
    np.testing.assert_array_equal(pos2, pos)
    S2.reset()
    f2 = str(tmp_path / "bulk.txt")
    mcmc_utils.run_mcmc_save(S2, pos2, nprod, state2, f2, col_names=names, chunk=7)
    assert open(f1).read() == open(f2).read()
    np.testing.assert_array_equal(S2.chain, S1.chain)
    np.testing.assert_array_equal(S2.lnprobability, S1.lnprobability)
    c = mcmc_utils.readchain(f1)
    np.testing.assert_array_equal(c[:, :, :NDIM], S1.chain)
    # readflatchain: a headerless whitespace table
    f3 = str(tmp_path / "flat.txt")
    np.savetxt(f3, flat)
    np.testing.assert_array_equal(mcmc_utils.readflatchain(f3), flat)


def test_sample_thin_and_accumulation():
    """emcee 2.x storage rules: sample() with thin keeps steps i % thin == 0,
    successive runs append to the chain, reset() empties it"""
    S = EnsembleSampler(W, NDIM, GaussLnProb(), seed=4, ops=sd.TorchCpuOps())
    rows = []
    for pos, prob, state in S.sample(_p0(), iterations=7, thin=3):
        rows.append(pos)
    assert S.chain.shape == (W, 3, NDIM)
    for j, i in enumerate((0, 3, 6)):
        np.testing.assert_array_equal(S.chain[:, j], rows[i])
    S.run_mcmc(None, 2)
    assert S.chain.shape == (W, 5, NDIM) and state == 7 and S.random_state == 9
    S.run_mcmc(None, 2, storechain=False)
    assert S.chain.shape == (W, 5, NDIM)
    S.reset()
    assert S.chain.shape == (W, 0, NDIM) and S.iterations == 0


def _save_worker(rank, port, path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=2)
    try:
        from lfit_python_amd import mcmc_utils
        S = EnsembleSampler(W, NDIM, GaussLnProb(), seed=99, ops=sd.TorchCpuOps())
        pos, prob, state = mcmc_utils.run_burnin(S, _p0(), 3)
        S.reset()
        mcmc_utils.run_mcmc_save(S, pos, 5, state, path, col_names="walker_no a b c d e ln_prob", chunk=2)
    finally:
        dist.destroy_process_group()


def test_two_rank_run_mcmc_save_writes_once(tmp_path):
    """Every rank runs the production steps, rank 0 alone writes the file:
    1 header line + nSteps * W rows."""
    path = str(tmp_path / "chain_prod.txt")
    mp.spawn(_save_worker, args=(_free_port(), path), nprocs=2, join=True)
    lines = open(path).read().splitlines()
    assert len(lines) == 1 + 5 * W
    S = EnsembleSampler(W, NDIM, GaussLnProb(), seed=99, ops=sd.TorchCpuOps())
    from lfit_python_amd import mcmc_utils
    pos, prob, state = mcmc_utils.run_burnin(S, _p0(), 3)
    S.reset()
    one = str(tmp_path / "one.txt")
    mcmc_utils.run_mcmc_save(S, pos, 5, state, one, col_names="walker_no a b c d e ln_prob")
    assert open(one).read() == open(path).read()


def test_sample_generator_left_early_keeps_its_steps():
    """A sample() generator the caller leaves early (break -> GeneratorExit)
    keeps the steps it ran in the chain and no unwritten rows (ADVICE r04:
    the end-of-run handling now runs in a finally); a later run appends."""
    ev = GaussLnProb()
    S = EnsembleSampler(W, NDIM, ev, seed=5, ops=sd.TorchCpuOps())
    S.set_state(_p0())
    for i, (pos, lnp, _) in enumerate(S.sample(iterations=10, thin=2)):
        last = pos
        if i == 4:
            break                       # 5 steps ran: steps 0, 2, 4 stored
    assert S.chain.shape == (W, 3, NDIM)
    np.testing.assert_array_equal(S.chain[:, -1], last)
    assert S.last_run()[0].shape == (3, W, NDIM)
    S.run_mcmc(None, 4)
    assert S.chain.shape == (W, 7, NDIM)
    # the host chunks were replaced by one concatenation: a second read is the same object
    assert S._concat() is S._concat() and len(S._chunks) == 1
