"""Host logic against fixtures captured from the reference's own Python
(tests/golden/README.md): priors, parameter routing, light-curve loading,
the compiled gather map, and the oracle's batched ln_prob against the
reference tree's ln_prob."""
import json
import os

import numpy as np
import pytest

from lfit_python_amd import batch, cvmodel
from lfit_python_amd.tree import Prior, extract_par_and_key

GOLD = os.path.join(os.path.dirname(__file__), "golden")
INPUT = os.path.join(GOLD, "ref_test_data", "mcmc_input.dat")


def _same(a, b, rtol=1e-13):
    a, b = np.asarray(a, float), np.asarray(b, float)
    assert np.array_equal(np.isfinite(a), np.isfinite(b)), (a, b)
    assert np.array_equal(a[np.isinf(a)], b[np.isinf(b)])
    f = np.isfinite(a)
    np.testing.assert_allclose(a[f], b[f], rtol=rtol, atol=1e-13 if rtol else 0.0)


def test_priors_match_reference(oracle):
    g = json.load(open(os.path.join(GOLD, "priors.json")))
    for case in g["cases"]:
        pr = Prior(case["type"], case["p1"], case["p2"])
        if case["normalise"] is not None:
            assert abs(pr.normalise - case["normalise"]) <= 1e-12 * abs(case["normalise"])
        assert pr.p1 == case["p1_used"]
        _same([pr.ln_prob(v) for v in case["vals"]], case["ln_prob"], rtol=1e-12)
        # the oracle / device formula of the same prior
        code = pr.code
        _same([oracle.prior_lnprob(code, pr.p1, pr.p2, pr.normalise, v) for v in case["vals"]],
              case["ln_prob"], rtol=1e-12)


def test_prior_quirks():
    # log_uniform normaliser integrates the log-density (model.py:77-79)
    assert abs(Prior('log_uniform', 0.001, 0.2).normalise - 0.5139798) < 1e-7
    assert abs(Prior('log_uniform', 0.001, 0.2).ln_prob(0.043) - 3.8121264) < 1e-7
    assert abs(Prior('gauss', 0.284, 0.001).ln_prob(0.284) - 5.9888167) < 1e-7
    assert Prior('gauss', 0.284, 0.001).ln_prob(0.284 + 40 * 0.001) == -np.inf
    assert Prior('uniform', 0.03, 0.5).ln_prob(0.5) == -np.inf          # open interval
    with pytest.raises(AssertionError):
        Prior('beta', 0, 1)


def test_extract_par_and_key():
    assert extract_par_and_key("wdFlux_long_complex_key_label") == ("wdFlux", "long_complex_key_label")
    assert extract_par_and_key("ln_tau_gp_core") == ("ln_tau_gp", "core")
    assert extract_par_and_key("q_core") == ("q", "core")


def test_routing_matches_reference():
    g = json.load(open(os.path.join(GOLD, "routing.json")))
    m = cvmodel.construct_model(INPUT)
    assert type(m).__name__ == g["root"] == "GPLCModel"
    assert m.dynasty_par_names == g["names"]
    assert len(g["names"]) == 87
    _same(m.dynasty_par_vals, g["start"], rtol=0)
    m.dynasty_par_vals = g["vector"]
    leaves = m.leaves()
    assert [l.label for l in leaves] == [e["label"] for e in g["eclipses"]]
    lcs = np.load(os.path.join(GOLD, "lightcurves.npz"))
    for leaf, e in zip(leaves, g["eclipses"]):
        assert leaf.parent.label == e["band"]
        assert leaf.cv_parnames == e["cv_parnames"]
        _same(leaf.cv_parlist, e["cv_parlist"], rtol=0)
        assert leaf.lc.n_data == e["n"]
        for k in ("x", "y", "ye", "w"):
            _same(getattr(leaf.lc, k), lcs["%s_%s" % (k, leaf.label)], rtol=0)
    # yaw/tilt swap: the tree stores yaw before tilt, lfit takes tilt before yaw
    names = leaves[0].node_par_names
    assert names.index('yaw') < names.index('tilt')
    assert leaves[0].cv_parnames.index('tilt') < leaves[0].cv_parnames.index('yaw')


def test_gp_tree_compiles():
    """The shipped example (useGP = 1) compiles: GP hyper-parameters routed
    from the core node, phase-sorted data, the changepoint eclipse range."""
    m = cvmodel.construct_model(INPUT)
    t = batch.compile_tree(m)
    assert t.gp and t.E == 6 and t.ndim == 87
    names = m.dynasty_par_names
    for e in range(t.E):
        assert [names[g] for g in t.gp_gather[e]] == ['ln_ampin_gp_core', 'ln_ampout_gp_core', 'ln_tau_gp_core']
        x = t.x[t.offsets[e]:t.offsets[e + 1]]
        assert np.all(np.diff(x) >= 0)
        assert tuple(t.gp_ecl[e]) == (0, 1)  # phi_start = -0.2, phi_end = 0.3 (CVModel.py:582-590)
    np.testing.assert_array_equal(t.gp_base[:, :3], [[0.1037, 0.0392, 0.0187]] * 6)


def _gp_blocks(oracle, t, e, v, base_dcp):
    """blocks of eclipse e for walker v, as the oracle / kernels form them"""
    p = [v[g] if g >= 0 else t.consts[-1 - g] for g in t.gather[e]]
    q, dphi, rwd, phi0 = p[4], p[5], p[8], p[13]
    B = t.gp_base[e]
    if abs(B[1] - dphi) / dphi > 1.2 or abs(B[0] - q) / q > 1.2 or abs(B[2] - rwd) / rwd > 1.2:
        dcp = oracle.gp_base_dcp(q, dphi, rwd)
    else:
        dcp = base_dcp
    return [[(ec - 1) + dcp + phi0, ec - dcp + phi0] for ec in range(t.gp_ecl[e, 0], t.gp_ecl[e, 1] + 1)]


def test_gp_changepoints_and_kernel_match_reference(oracle):
    """SimpleGPEclipse.calcChangepoints / create_GP of the reference
    (tests/golden/gp_structure.json) against the compiled tree + oracle
    changepoint distance, including the > 120 % recomputation (walkers 5, 6)."""
    g = json.load(open(os.path.join(GOLD, "gp_structure.json")))
    d = np.load(os.path.join(GOLD, "lnprob_gp.npz"))
    m = cvmodel.construct_model(INPUT)
    t = batch.compile_tree(m)
    base_dcp = oracle.gp_base_dcp(*t.gp_base[0, :3])
    seen_recompute = False
    for rec in g["walkers"]:
        v = d["walkers"][rec["walker"]]
        for e, ecl in enumerate(rec["eclipses"]):
            assert ecl["label"] == t.leaf_labels[e]
            cps = _gp_blocks(oracle, t, e, v, base_dcp)
            np.testing.assert_allclose(cps, ecl["changepoints"], rtol=0, atol=1e-11)
            amps = np.exp(v[t.gp_gather[e]])
            terms = ecl["kernel"]
            assert len(terms) == 1 + len(cps)
            np.testing.assert_allclose(terms[0][:2], [amps[0], amps[2]], rtol=1e-14)
            assert terms[0][2] is None
            for term, cp in zip(terms[1:], cps):
                np.testing.assert_allclose(term[:2], [amps[1], amps[2]], rtol=1e-14)
                np.testing.assert_allclose(term[2], cp, rtol=0, atol=1e-11)
        seen_recompute |= rec["walker"] in (5, 6)
    assert seen_recompute


def test_gp_kalman_matches_dense_oracle(oracle):
    """The O(N) state-space likelihood the kernels run (tests/gp_kalman.py)
    equals the dense Cholesky likelihood: ties, empty and edge blocks."""
    from tests.gp_kalman import gp_lnlike_kalman, gp_lnlike_kalman_jordan, gp_lnlike_segments
    rng = np.random.default_rng(7)
    for trial in range(6):
        n = int(rng.integers(2, 120))
        x = np.sort(rng.uniform(-0.2, 0.3, n))
        if trial == 1:
            x[3:6] = x[3]
        r = 0.004 * rng.standard_normal(n)
        ye = rng.uniform(0.002, 0.008, n)
        a1, a2, tau = np.exp(rng.uniform(-12, -7)), np.exp(rng.uniform(-12, -7)), np.exp(rng.uniform(-6.9, -2))
        blocks = [(-0.98, -0.03), (0.02, 0.97)]
        if trial == 2:
            blocks = []
        if trial == 3:
            blocks = [(x[0], x[n // 3]), (x[n // 2], x[-1])]   # closed at data points
        if trial == 4:
            blocks = [(0.5, 0.4)]                               # empty (dist_cp > 1/2)
        dense = oracle.gp_lnlike(x, r, ye, a1, a2, tau, blocks)
        kal = gp_lnlike_kalman(x, r, ye, a1, a2, tau, blocks)
        assert abs(dense - kal) <= 1e-10 * max(1.0, abs(dense)), (trial, dense, kal)
        jor = gp_lnlike_kalman_jordan(x, r, ye, a1, a2, tau, blocks)  # k_gp_like's coordinates
        assert abs(dense - jor) <= 1e-10 * max(1.0, abs(dense)), (trial, dense, jor)
        for K in (1, 3, 8):  # k_gp_like's parallel-in-time form (8 segments), empty segments included
            seg = gp_lnlike_segments(x, r, ye, a1, a2, tau, blocks, K)
            assert abs(dense - seg) <= 1e-10 * max(1.0, abs(dense)), (trial, K, dense, seg)


def test_oracle_gp_lnprob_matches_reference(oracle):
    """The oracle's GP ln_prob (dense GP, changepoint cache rule) against the
    reference GPLCModel tree on the same walkers (tests/golden/lnprob_gp.npz)."""
    d = np.load(os.path.join(GOLD, "lnprob_gp.npz"))
    m = cvmodel.construct_model(INPUT)
    assert m.dynasty_par_names == list(d["names"])
    t = batch.compile_tree(m)
    lnp, lle, _ = oracle.lnprob_batch(d["walkers"], t)
    _same(lnp, d["ln_prob"], rtol=1e-10)
    fin = np.isfinite(d["ln_prior"])
    _same(lle.sum(1)[fin], d["ln_like"][fin], rtol=1e-10)


def _tree_from_golden(tag, tmpdir):
    from tests.helpers import golden_tree
    return golden_tree(tag, tmpdir)


@pytest.mark.parametrize("tag", ["tree", "simple"])
def test_compiled_gather_reproduces_cv_parlists(tag, tmp_path):
    d, m = _tree_from_golden(tag, tmp_path)
    assert m.dynasty_par_names == list(d["names"])
    t = batch.compile_tree(m)
    assert t.ndim == len(d["names"])
    assert t.E == (6 if tag == "tree" else 1)
    for v in d["walkers"][:5]:
        m.dynasty_par_vals = list(v)
        for e, leaf in enumerate(m.leaves()):
            g = t.gather[e, :t.npars[e]]
            got = np.where(g >= 0, v[np.maximum(g, 0)], t.consts[np.maximum(-1 - g, 0)] if len(t.consts) else 0)
            _same(got, leaf.cv_parlist, rtol=0)
    # prior table rows follow the dynasty order
    for k, name in enumerate(t.names):
        par = m[name]
        assert t.prior_type[k] == par.prior.code
        assert t.prior_p1[k] == par.prior.p1 and t.prior_p2[k] == par.prior.p2


def test_fixed_parameters_become_constants(tmp_path):
    d, m = _tree_from_golden("tree", tmp_path)
    m['ulimb_g'].isVar = False
    m['tilt_3'].isVar = False
    t = batch.compile_tree(m)
    assert t.ndim == len(d["names"]) - 2
    assert len(t.consts) == 2 + 1  # ulimb_g feeds both g eclipses, tilt_3 one
    assert 'ulimb_g' not in t.names and 'tilt_3' not in t.names


@pytest.mark.parametrize("tag", ["tree", "simple"])
def test_oracle_lnprob_matches_reference_tree(oracle, tag, tmp_path):
    """The oracle's batched ln_prob (the composition the HIP kernels
    implement) against the reference's own Node.ln_prob on the same walkers
    (reference flux = oracle flux, so this pins priors, Roche priors,
    routing and chi^2 composition)."""
    d, m = _tree_from_golden(tag, tmp_path)
    t = batch.compile_tree(m)
    lnp, lle, _ = oracle.lnprob_batch(d["walkers"], t)
    _same(lnp, d["ln_prob"], rtol=1e-10)
    fin = np.isfinite(d["ln_prior"])
    _same(lle.sum(1)[fin], d["ln_like"][fin], rtol=1e-10)


def test_chain_file_format(tmp_path):
    from lfit_python_amd.sampler import read_chain, write_chain
    rng = np.random.default_rng(1)
    chain = rng.standard_normal((3, 4, 5))
    lnp = rng.standard_normal((3, 4))
    f = tmp_path / "chain_prod.txt"
    names = ["a_core", "b_g", "c_0", "d_0", "e_0"]
    write_chain(str(f), names, chain, lnp)
    lines = f.read_text().splitlines()
    assert lines[0] == "walker_no a_core b_g c_0 d_0 e_0 ln_prob"
    assert lines[1].startswith("   0 ")
    assert len(lines) == 1 + 12
    back = read_chain(str(f))
    np.testing.assert_array_equal(back[:, :, :5], np.transpose(chain, (1, 0, 2)))


def test_oracle_near_round1_rk4_fixture(oracle, tmp_path):
    """A check on the round-2 regeneration of the goldens: the
    simple-BS fixture as made in round 1, when the stream came from 22 RK4
    steps (1e-6 a off in position, 1e-4 in velocity), kept as
    tests/golden/lnprob_simple_rk4.npz.  The table-based oracle must land on
    it within what that stream error moves a chi^2 (measured: <= 0.026 in
    ln_prob, 1e-5 relative), with the same finite pattern: a regeneration
    that broke routing, priors or the flux would miss it by orders more."""
    from tests.helpers import golden_tree
    d, m = golden_tree("simple_rk4", tmp_path)
    t = batch.compile_tree(m)
    lnp, _, _ = oracle.lnprob_batch(d["walkers"], t)
    fin = np.isfinite(d["ln_prob"])
    assert np.array_equal(np.isfinite(lnp), fin)
    assert np.max(np.abs(lnp[fin] - d["ln_prob"][fin]) / np.abs(d["ln_prob"][fin])) < 5e-5
    assert np.max(np.abs(lnp[fin] - d["ln_prob"][fin])) < 0.1
