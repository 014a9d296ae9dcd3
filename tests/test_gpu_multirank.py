"""GPU: the multi-rank sampler path (walker shards, one all_gather of ln_prob
per half-step, lfg_stretch_step_shard(_spec) + lfg_stretch_accept_regen(_spec))
with two real ranks sharing cuda:0 over gloo, against the single-rank fused
chain, for a single eclipse, a six-eclipse tree (the per-walker combine after
the likelihood kernels) and the reference's GP example.  The reference's analogue is the pool.map fan-out of mcmcfit.py:273-288;
the chains must be bit-identical whatever the rank count."""
import os
import socket
import tempfile

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _flux_fn(p, x, w, nsub):
    from lfit_python_amd.lfit import flux_batch
    f, st = flux_batch(np.asarray(p)[None, :], x, w, nsub=nsub)
    return f[0].cpu().numpy()


def _model(kind, tmp=None):
    """config 2's single eclipse, a 3-band x 2-eclipse tree (E = 6: the shard
    path's k_combine_walkers), or the reference's useGP = 1 example (E = 6)."""
    from lfit_python_amd import cvmodel, synthetic
    if kind == "single":
        return synthetic.config_single(300, flux_fn=_flux_fn)
    if kind == "tree":
        return synthetic.config_tree(2, 200, flux_fn=_flux_fn)
    gold = os.path.join(os.path.dirname(__file__), "golden", "ref_test_data", "mcmc_input.dat")
    return cvmodel.construct_model(gold)


def _init(m, W):
    p0 = np.array(m.dynasty_par_vals)
    rng = np.random.default_rng(17)
    return p0 * (1.0 + 1e-3 * rng.standard_normal((W, p0.size)))


def _chain(spec, world=1, rank=0, kind="single"):
    import torch
    from lfit_python_amd import batch, sampler
    m = _model(kind)
    t = batch.compile_tree(m)
    ev = batch.LnProbEvaluator(t, device=torch.device("cuda", 0))
    W = 64 if kind == "single" else 32
    S = sampler.EnsembleSampler(W, t.ndim, ev, seed=23)
    S.spec = spec
    S.run_mcmc(_init(m, W), 4 if kind == "single" else 3)
    out = (S.chain_dev.cpu().numpy(), S.lnprob_dev.cpu().numpy(), S.naccept.cpu().numpy())
    S.close()
    return out


def _rank_main(rank, world, port, path, spec, kind="single"):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ch, lc, na = _chain(spec, world, rank, kind)
        np.savez(path % rank, chain=ch, lnp=lc, nacc=na)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("kind,spec", [("single", True), ("single", False), ("tree", True), ("gp", True)])
def test_two_ranks_match_one(kind, spec):
    import torch.multiprocessing as mp
    ref = _chain(True, kind=kind)
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "rank%d.npz")
        mp.spawn(_rank_main, args=(2, port, path, spec, kind), nprocs=2, join=True)
        for r in range(2):
            got = np.load(path % r)
            np.testing.assert_array_equal(got["chain"], ref[0])
            np.testing.assert_array_equal(got["lnp"], ref[1])
            np.testing.assert_array_equal(got["nacc"], ref[2])
