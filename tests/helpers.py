"""Shared inputs for the tests (seeded, synthetic)."""
import numpy as np

# eclipse 0 / band g / core of the reference's test_data/mcmc_input.dat:48-86,
# in lfit CV order (tilt before yaw, CVModel.py:384-388)
TRUTH18 = [0.0528, 0.0707, 0.0613, 0.0131, 0.1037, 0.0392, 0.2953, 0.284, 0.0187,
           0.043, 120.0, 0.048, 0.5, 0.001, 1.1342, 4.5971, 72.0006, 5.4]
TRUTH14 = TRUTH18[:14]

# a second, better-constrained eclipse (mcmc_input.dat eclipse 1)
ECL1 = [0.0528, 0.1238, 0.1518, 0.0131, 0.1037, 0.0392, 0.5214, 0.284, 0.0187,
        0.0497, 122.0724, 0.1684, 1.9539, -0.0013, 3.4876, 1.4429, 52.4720, 15.6635]


def random_pars(n, complex_bs=True, seed=0, spread=1.0):
    """n parameter sets scattered around the truth, inside the model domain."""
    rng = np.random.default_rng(seed)
    base = np.array(TRUTH18 if complex_bs else TRUTH14)
    out = []
    while len(out) < n:
        p = base.copy()
        p[0:4] *= 1 + 0.3 * spread * rng.standard_normal(4)
        p[4] = rng.uniform(0.06, 0.4)                       # q
        p[5] = rng.uniform(0.03, 0.06)                      # dphi
        p[6] = rng.uniform(0.25, 0.6)                       # rdisc (xl1 units)
        p[7] = rng.uniform(0.1, 0.5)                        # ulimb
        p[8] = rng.uniform(0.01, 0.03)                      # rwd
        p[9] = p[8] * rng.uniform(0.5, 2.5)                 # scale
        p[10] = rng.uniform(80, 160)                        # az
        p[11] = rng.uniform(0.01, 0.9)                      # fis
        p[12] = rng.uniform(0.1, 1.9)                       # dexp
        p[13] = rng.uniform(-0.005, 0.005)                  # phi0
        if complex_bs:
            p[14] = rng.uniform(0.3, 4.0)
            p[15] = rng.uniform(0.6, 4.5)
            p[16] = rng.uniform(20, 160)
            p[17] = rng.uniform(-40, 40)
        out.append(p)
    return np.array(out)


def phase_grid(n=300, lo=-0.3, hi=0.3):
    x = np.linspace(lo, hi, n)
    w = np.mean(np.diff(x)) * np.ones_like(x) / 2.0
    return x, w


# ---- the reference's sampler call patterns (emcee 2.x surface)
def pattern_run_burnin(sampler, startPos, nSteps, storechain=False):
    """mcmc_utils.run_burnin's use of the sampler (mcmc_utils.py:114-132):
    iterate sample() to the end, keep the last (pos, prob, state)"""
    try:
        for pos, prob, state in sampler.sample(startPos, iterations=nSteps, storechain=storechain):
            pass
    except TypeError:  # emcee 3 spelling
        for pos, prob, state in sampler.sample(startPos, iterations=nSteps, store=storechain):
            pass
    return pos, prob, state


def pattern_run_mcmc_save(sampler, startPos, nSteps, rState, file, col_names=''):
    """mcmc_utils.run_mcmc_save's use of the sampler (mcmc_utils.py:135-164):
    sample() with rstate0 and store=True, one appended row per walker per step"""
    with open(file, "w") as fh:
        fh.write(col_names)
        if col_names:
            fh.write("\n")
    for pos, prob, state in sampler.sample(startPos, iterations=nSteps, rstate0=rState, store=True,
                                           skip_initial_state_check=True):
        for k in range(pos.shape[0]):
            with open(file, "a") as fh:
                fh.write("{0:4d} {1:s} {2:f}\n".format(k, " ".join(map(str, pos[k])), prob[k]))
    return sampler


# ---- golden example trees (tests/golden/lnprob_<tag>.npz hold their input text)
GOLD = __import__("os").path.join(__import__("os").path.dirname(__file__), "golden")


def golden_tree(tag, tmpdir):
    """(fixture, model) of a golden variant of the example input.  The input
    text is written under `tmpdir` (tests never write into tests/golden) with
    its light-curve paths pointed at tests/golden/ref_test_data."""
    import os
    from lfit_python_amd import cvmodel
    d = np.load(os.path.join(GOLD, "lnprob_%s.npz" % tag))
    data = os.path.join(GOLD, "ref_test_data")
    lines = []
    for line in str(d["input"]).splitlines():
        tok = line.split("=", 1)
        key = tok[0].strip()
        if key.startswith("file_") and len(tok) == 2 and not os.path.isabs(tok[1].strip()):
            line = "%s = %s" % (key, os.path.join(data, tok[1].strip()))
        lines.append(line)
    path = os.path.join(str(tmpdir), "mcmc_input_%s.dat" % tag)
    with open(path, "w") as fh:
        fh.write("\n".join(lines) + "\n")
    return d, cvmodel.construct_model(path)
