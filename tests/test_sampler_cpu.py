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
    return S.chain.numpy(), S.lnprob_chain.numpy(), ev.calls


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
        out[rank] = (S.chain.numpy().copy(), S.lnprob_chain.numpy().copy(), list(ev.calls))
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
    S.run_mcmc(_p0(), 4, store=False)
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
            np.testing.assert_array_equal(S.chain[it - 4].numpy(), pos)
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
