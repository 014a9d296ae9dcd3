#!/usr/bin/env python3
"""Generate tests/golden/ fixtures from the reference's own Python layers.

Runs ONLY in the build container (it imports /root/reference/model.py and
CVModel.py; nothing of the reference travels).  The reference's third-party
imports are replaced by stand-ins:
  george      kernels / GP -> a recorder of the kernel the reference builds
              (terms, amplitudes, metric, blocks) whose log_likelihood is the
              exact dense GP likelihood (numpy Cholesky): george's HODLR
              solver approximates exactly this
  configobj   ConfigObj(path) -> key = value reader
  lfit        CV(pars).calcFlux(pars, x, w) -> this repo's CPU oracle
  trm.roche   xl1 / findphi / findi / bspot / wdphases -> this repo's CPU oracle
so the fixtures pin the reference's parameter routing, yaw/tilt swap, Prior
quirks, Lightcurve loading/trim, Roche-prior logic and chi^2 / ln_like /
ln_prob composition; the flux arithmetic inside them is the oracle's
(lfit itself is absent: parity of that part is unpinned).

Outputs (JSON / npz, data only):
  tests/golden/priors.json           Prior.ln_prob values and normalisers
  tests/golden/routing.json          dynasty names/order, cv_parlists
  tests/golden/lightcurves.npz       Lightcurve.from_calib + trim arrays
  tests/golden/lnprob_tree.npz       ln_prior / ln_like / ln_prob per walker
                                     (6-eclipse complex tree, useGP = 0)
  tests/golden/lnprob_simple.npz     same for a 1-eclipse simple-BS tree
  tests/golden/lnprob_gp.npz         the shipped example as is (useGP = 1):
                                     ln_prior / ln_like / ln_prob per walker,
                                     each walker on a fresh copy of the model
                                     whose changepoint cache was set by one
                                     ln_like at the start values (what each
                                     emcee pool task receives)
  tests/golden/gp_structure.json     changepoints and kernel terms the
                                     reference builds for a few walkers
"""
import copy
import json
import os
import sys
import tempfile
import types

import numpy as np

REF = "/root/reference"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "tests", "golden")
sys.dont_write_bytecode = True
sys.path.insert(0, ROOT)

from oracle.oracle import Oracle  # noqa: E402

ORC = Oracle()


LAST_GP = {}


class _Kernel:
    """george kernel stand-in: a sum of amp * Matern32(metric) terms, each
    optionally restricted to a block of x (george 0.3: closed [min, max])."""

    def __init__(self, terms):
        self.terms = terms

    def __rmul__(self, a):
        return _Kernel([(float(a) * amp, metric, blk) for amp, metric, blk in self.terms])

    __mul__ = __rmul__

    def __add__(self, other):
        return _Kernel(self.terms + other.terms)


def _matern32(metric, block=None):
    blk = None if block is None else tuple(float(v) for v in np.atleast_2d(block)[0])
    return _Kernel([(1.0, float(metric), blk)])


class _GP:
    def __init__(self, kernel, solver=None):
        self.kernel = kernel
        LAST_GP["kernel"] = kernel.terms

    def compute(self, x, yerr):
        self.x = np.asarray(x, dtype=np.float64)
        self.yerr = np.asarray(yerr, dtype=np.float64)

    def log_likelihood(self, r, quiet=False):
        x = self.x
        d = x[:, None] - x[None, :]
        K = np.diag(self.yerr ** 2)
        for amp, metric, blk in self.kernel.terms:
            u = np.sqrt(3.0 * d * d / metric)
            k = amp * (1.0 + u) * np.exp(-u)
            if blk is not None:
                inb = (x >= blk[0]) & (x <= blk[1])
                k = k * (inb[:, None] & inb[None, :])
            K = K + k
        try:
            L = np.linalg.cholesky(K)
        except np.linalg.LinAlgError:
            if quiet:
                return -np.inf
            raise
        z = np.linalg.solve(L, np.asarray(r, dtype=np.float64))
        ll = -0.5 * (z @ z + 2.0 * np.sum(np.log(np.diag(L))) + len(x) * np.log(2.0 * np.pi))
        return ll if np.isfinite(ll) else -np.inf


def install_standins():
    george = types.ModuleType("george")
    george.kernels = types.SimpleNamespace(Matern32Kernel=_matern32)
    george.GP = _GP
    george.HODLRSolver = object()
    sys.modules["george"] = george

    cfg = types.ModuleType("configobj")

    class ConfigObj(dict):
        def __init__(self, path):
            super().__init__()
            with open(path, encoding="utf-8", errors="replace") as fh:
                for raw in fh:
                    line = raw.split("#", 1)[0].strip()
                    if "=" in line:
                        k, v = line.split("=", 1)
                        self[k.strip()] = v.strip()
    cfg.ConfigObj = ConfigObj
    sys.modules["configobj"] = cfg

    lfit = types.ModuleType("lfit")

    class CV:
        def __init__(self, pars):
            self.pars = list(pars)

        def calcFlux(self, pars, x, w):
            st, (f, ywd, yd, ys, yrs) = ORC.flux(list(pars), np.asarray(x), np.asarray(w), components=True)
            if st:
                raise ValueError("invalid CV parameters (status %d)" % st)
            self.ywd, self.yd, self.ys, self.yrs = ywd, yd, ys, yrs
            return f
    lfit.CV = CV
    sys.modules["lfit"] = lfit

    trm = types.ModuleType("trm")
    roche = types.ModuleType("trm.roche")

    def xl1(q):
        assert q > 0
        return ORC.xl1(q)
    roche.xl1 = xl1
    roche.findphi = ORC.findphi
    roche.findi = ORC.findi
    roche.bspot = ORC.bspot
    roche.wdphases = ORC.wdphases
    trm.roche = roche
    sys.modules["trm"] = trm
    sys.modules["trm.roche"] = roche


def main():
    os.makedirs(OUT, exist_ok=True)
    install_standins()
    sys.path.insert(0, REF)
    import model as refmodel
    import CVModel as refcv
    rng = np.random.default_rng(20261015)

    # ---- priors (model.py:40-113)
    cases = []
    specs = [("uniform", 0.03, 0.5), ("log_uniform", 0.001, 0.2), ("log_uniform", 0.001, 2.0),
             ("gauss", 0.284, 0.001), ("gaussPos", 0.32, 0.03), ("mod_jeff", 0.01, 1.0),
             ("uniform", -90.0, 90.0), ("log_uniform", 1e-40, 1.0)]
    for t, p1, p2 in specs:
        import warnings
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            pr = refmodel.Prior(t, p1, p2)
        vals = [p1, p2, 0.5 * (p1 + p2), p1 + 1e-9, p2 - 1e-9, -1.0, 0.0, 1e-3, 0.043, 0.284,
                0.284 + 40 * 0.001, 0.284 + 37.5 * 0.001, 0.1037, 2.5]
        vals += list(rng.uniform(min(p1, 0.0) - 0.1, p2 + 0.1, 6))
        cases.append({"type": t, "p1": p1, "p2": p2, "normalise": getattr(pr, "normalise", None),
                      "p1_used": pr.p1,
                      "vals": [float(v) for v in vals],
                      "ln_prob": [float(pr.ln_prob(v)) for v in vals]})
    json.dump({"source": "reference model.py Prior", "cases": cases},
              open(os.path.join(OUT, "priors.json"), "w"), indent=1)

    # ---- routing on the shipped example (3 bands x 2 eclipses, complex, GP)
    cwd = os.getcwd()
    os.chdir(os.path.join(REF, "test_data"))
    try:
        m = refcv.construct_model("mcmc_input.dat")
        names = m.dynasty_par_names
        vals0 = list(m.dynasty_par_vals)
        vec = np.asarray(vals0) * (1.0 + 0.01 * rng.standard_normal(len(vals0)))
        m.dynasty_par_vals = list(vec)
        leaves = sorted(m.search_node_type("Eclipse"), key=lambda n: int(n.label))
        routing = {"names": names, "start": vals0, "vector": [float(v) for v in vec],
                   "eclipses": [{"label": e.label, "band": e.parent.label, "cv_parnames": e.cv_parnames,
                                 "cv_parlist": [float(v) for v in e.cv_parlist],
                                 "n": int(e.lc.n_data), "w0": float(e.lc.w[0])} for e in leaves],
                   "root": type(m).__name__}
        lcs = {}
        for e in leaves:
            lcs["x_%s" % e.label] = e.lc.x
            lcs["y_%s" % e.label] = e.lc.y
            lcs["ye_%s" % e.label] = e.lc.ye
            lcs["w_%s" % e.label] = e.lc.w
        np.savez_compressed(os.path.join(OUT, "lightcurves.npz"), **lcs)
    finally:
        os.chdir(cwd)
    json.dump(routing, open(os.path.join(OUT, "routing.json"), "w"), indent=1)

    # ---- ln_prob through the reference tree (useGP = 0), oracle flux
    src = open(os.path.join(REF, "test_data", "mcmc_input.dat"), encoding="utf-8", errors="replace").read()
    for tag, repl in (("tree", {"useGP": "0"}), ("simple", {"useGP": "0", "complex": "0", "neclipses": "1"})):
        text = src
        lines = []
        for line in text.splitlines():
            key = line.split("=", 1)[0].strip() if "=" in line else None
            if key in repl:
                line = "%s = %s" % (key, repl[key])
            lines.append(line)
        if "neclipses" in repl:
            lines.append("neclipses = %s" % repl["neclipses"])
        with tempfile.TemporaryDirectory() as td:
            path = os.path.join(td, "mcmc_input.dat")
            open(path, "w").write("\n".join(lines) + "\n")
            os.symlink(os.path.join(REF, "test_data", "lightcurves"), os.path.join(td, "lightcurves"))
            os.chdir(td)
            try:
                m = refcv.construct_model("mcmc_input.dat")
            finally:
                os.chdir(cwd)
            names = m.dynasty_par_names
            p0 = np.asarray(m.dynasty_par_vals)
            nw = 48 if tag == "tree" else 96
            # a mix of near-truth walkers and wide ones (some invalid)
            walk = p0 * (1.0 + 0.02 * rng.standard_normal((nw, p0.size)))
            walk[nw // 2:] = p0 * (1.0 + 0.3 * rng.standard_normal((nw - nw // 2, p0.size)))
            lp, ll, lprob = [], [], []
            for v in walk:
                m.dynasty_par_vals = list(v)
                pri = m.ln_prior()
                lp.append(pri)
                ll.append(m.ln_like() if np.isfinite(pri) else np.nan)
                lprob.append(m.ln_prob())
            np.savez_compressed(os.path.join(OUT, "lnprob_%s.npz" % tag), names=np.array(names),
                                walkers=walk, ln_prior=np.array(lp), ln_like=np.array(ll),
                                ln_prob=np.array(lprob), input=np.array("\n".join(lines)))
            print(tag, "ndim", len(names), "finite ln_prob", int(np.isfinite(lprob).sum()), "of", nw)
    # ---- the GP example tree as shipped (useGP = 1)
    os.chdir(os.path.join(REF, "test_data"))
    try:
        m = refcv.construct_model("mcmc_input.dat")
    finally:
        os.chdir(cwd)
    names = m.dynasty_par_names
    p0 = np.asarray(m.dynasty_par_vals)
    m.ln_like()  # the sanity evaluation of mcmcfit.py:154: fills the changepoint caches
    nw = 40
    walk = p0 * (1.0 + 0.02 * rng.standard_normal((nw, p0.size)))
    walk[nw // 2:] = p0 * (1.0 + 0.3 * rng.standard_normal((nw - nw // 2, p0.size)))
    iq, idp, irw = names.index("q_core"), names.index("dphi_core"), names.index("rwd_core")
    walk[4, irw] = p0[irw] * 0.4     # > 120 % changes: the changepoints are recomputed
    walk[5, iq] = p0[iq] * 0.4
    walk[6, idp] = p0[idp] * 0.42
    lp, ll, lprob, structs = [], [], [], []
    for i, v in enumerate(walk):
        mc = copy.deepcopy(m)  # what a pool task unpickles
        mc.dynasty_par_vals = list(v)
        pri = mc.ln_prior()
        lp.append(pri)
        ll.append(copy.deepcopy(mc).ln_like() if np.isfinite(pri) else np.nan)
        lprob.append(mc.ln_prob())
        if i < 8 and np.isfinite(pri):
            leaves = sorted(mc.search_node_type("Eclipse"), key=lambda n: int(n.label))
            rec = []
            for leaf in leaves:
                try:
                    cps = [[float(a), float(b)] for a, b in leaf.calcChangepoints()]
                    leaf.create_GP()
                    terms = [[a, mt, list(bk) if bk else None] for a, mt, bk in LAST_GP["kernel"]]
                except Exception as exc:  # noqa: BLE001 - record what the reference raises
                    cps, terms = repr(exc), None
                rec.append({"label": leaf.label, "changepoints": cps, "kernel": terms})
            structs.append({"walker": i, "eclipses": rec})
    np.savez_compressed(os.path.join(OUT, "lnprob_gp.npz"), names=np.array(names), walkers=walk,
                        ln_prior=np.array(lp), ln_like=np.array(ll), ln_prob=np.array(lprob))
    json.dump({"source": "reference CVModel.py SimpleGPEclipse with the george stand-in above",
               "walkers": structs}, open(os.path.join(OUT, "gp_structure.json"), "w"), indent=1)
    print("gp ndim", len(names), "finite ln_prob", int(np.isfinite(lprob).sum()), "of", nw)
    print("wrote", sorted(os.listdir(OUT)))


if __name__ == "__main__":
    main()
