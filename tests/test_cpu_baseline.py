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


def test_port_refuses_gp_trees(port):
    class T:
        gp = True
    with pytest.raises(ValueError):
        port.lnprob_batch(np.zeros((2, 3)), T())
