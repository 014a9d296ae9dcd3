"""The fit driver (lfit_python_amd.mcmcfit, mirroring the reference's
mcmcfit.py:51-343): run keys, scatter vectors and D.o.F. on CPU; a short
device run that writes chain_prod.txt on the GPU."""
import os
import shutil

import numpy as np
import pytest

from lfit_python_amd import cvmodel, mcmcfit, sampler

GOLD = os.path.join(os.path.dirname(__file__), "golden", "ref_test_data")
INPUT = os.path.join(GOLD, "mcmc_input.dat")


def test_run_config_of_the_example():
    rc = mcmcfit.read_run_config(INPUT)
    assert (rc["nburn"], rc["nprod"], rc["nwalkers"], rc["nthread"]) == (100, 100, 36, 8)
    assert rc["fit"] == 1 and rc["usePT"] is False and rc["double_burnin"] is False and rc["comp_scat"] is True
    assert (rc["first_scatter"], rc["second_scatter"]) == (0.10, 0.05)


def test_scatter_vectors_and_dof():
    m = cvmodel.construct_model(INPUT)
    names = m.dynasty_par_names
    rc = mcmcfit.read_run_config(INPUT)
    s1, s2 = mcmcfit.scatter_vectors(names, rc)
    # comp_scat factors (mcmcfit.py:210-246): dphi x0.2, ulimb x1e-6, GP params untouched
    assert s1[names.index('dphi_core')] == pytest.approx(0.02)
    assert s1[names.index('ulimb_g')] == pytest.approx(1e-7)
    assert s1[names.index('ln_tau_gp_core')] == pytest.approx(0.10)
    np.testing.assert_allclose(s2, s1 * 0.5)
    rc["comp_scat"] = False
    s1, s2 = mcmcfit.scatter_vectors(names, rc)
    assert s2 is None and np.all(s1 == 0.10)
    n = sum(e.lc.n_data for e in m.search_node_type('Eclipse'))
    assert mcmcfit.degrees_of_freedom(m) == n - 87 - 1


def _small_input(tmp_path, **over):
    text = open(INPUT, encoding="utf-8", errors="replace").read().splitlines()
    keys = dict(useGP="0", complex="0", nwalkers="32", nburn="3", nprod="5", double_burnin="1", comp_scat="1")
    keys.update(over)
    out = []
    for line in text:
        k = line.split("=", 1)[0].strip() if "=" in line else None
        out.append("%s = %s" % (k, keys.pop(k)) if k in keys else line)
    out.append("neclipses = 1")
    out += ["%s = %s" % kv for kv in keys.items()]
    tmp_path.mkdir(parents=True, exist_ok=True)
    (tmp_path / "mcmc_input.dat").write_text("\n".join(out) + "\n")
    shutil.copytree(os.path.join(GOLD, "lightcurves"), tmp_path / "lightcurves")
    return str(tmp_path / "mcmc_input.dat")


@pytest.mark.gpu
def test_short_fit_writes_the_reference_chain_format(tmp_path):
    path = _small_input(tmp_path)
    chain = str(tmp_path / "chain_prod.txt")
    out = mcmcfit.run(path, chain_file=chain, seed=5, chunk=2, log=lambda *a: None)
    assert out["status"] == "ok" and out["npars"] == 14 and out["nwalkers"] == 32
    lines = open(chain).read().splitlines()
    m = cvmodel.construct_model(path)
    assert lines[0] == "walker_no " + " ".join(m.dynasty_par_names) + " ln_prob"
    assert len(lines) == 1 + 5 * 32
    c = sampler.read_chain(chain)
    assert c.shape == (32, 5, 15)
    assert np.all(np.isfinite(c))
    assert 0.0 < out["acceptance"] < 1.0


@pytest.mark.gpu
def test_too_few_walkers_stops_like_the_reference(tmp_path):
    path = _small_input(tmp_path, nwalkers="20")  # < 2 * 14
    assert mcmcfit.run(path, chain_file=str(tmp_path / "c.txt"), log=lambda *a: None)["status"] == "too_few_walkers"
    assert not os.path.exists(tmp_path / "c.txt")
    # the reference's bare exit() is status 0 for this and for a report-only run
    assert mcmcfit.main([path, "--chain", str(tmp_path / "c.txt")]) == 0
    assert mcmcfit.main([_small_input(tmp_path / "nofit", fit="0"), "--chain", str(tmp_path / "c.txt")]) == 0
    assert not os.path.exists(tmp_path / "c.txt")


@pytest.mark.gpu
def test_prior_violation_is_an_error(tmp_path):
    # q fixed outside its prior: the start violates the priors
    path = _small_input(tmp_path, q="0.6 uniform 0.03 0.5 0")
    assert mcmcfit.run(path, chain_file=str(tmp_path / "c.txt"), log=lambda *a: None)["status"] == "prior_violation"
    assert mcmcfit.main([path, "--chain", str(tmp_path / "c.txt")]) == 1


@pytest.mark.gpu
def test_fixed_invalid_parameter_rejects_every_move(tmp_path):
    """A fixed parameter outside its prior makes Node.ln_prior -inf for every
    walker (model.py:439-441): every path (plain ln_prob, the fused half-step,
    the sharded half-step) must score -inf and accept nothing."""
    import torch
    from lfit_python_amd import batch
    path = _small_input(tmp_path, q="0.6 uniform 0.03 0.5 0")
    m = cvmodel.construct_model(path)
    t = batch.compile_tree(m)
    assert t.fixed_invalid
    ev = batch.LnProbEvaluator(t)
    p0 = np.array(m.dynasty_par_vals)
    walk = p0 * (1.0 + 1e-3 * np.random.default_rng(0).standard_normal((32, p0.size)))
    assert np.all(ev(torch.as_tensor(walk, device="cuda")).cpu().numpy() == -np.inf)
    assert np.all(ev.ln_prior(torch.as_tensor(walk, device="cuda")).cpu().numpy() == -np.inf)
    for shard in (False, True):
        S = sampler.EnsembleSampler(32, t.ndim, ev, seed=1)
        S.force_shard = shard
        S.set_state(walk)
        S.run_mcmc(None, 2)
        assert int(S.naccept.sum()) == 0
        assert np.all(S.lnp.cpu().numpy() == -np.inf)
