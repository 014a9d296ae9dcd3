#!/usr/bin/env python3
"""Generate tests/golden/ fixtures from the reference's own Python layers.

Runs ONLY in the build container (it imports /root/reference/model.py and
CVModel.py; nothing of the reference travels).  The reference's third-party
imports are replaced by stand-ins:
  george      unused by the non-GP path -> empty module
  configobj   ConfigObj(path) -> key = value reader
  lfit        CV(pars).calcFlux(pars, x, w) -> this repo's CPU oracle
  trm.roche   xl1 / findphi / findi / bspot -> this repo's CPU oracle
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
"""
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


def install_standins():
    george = types.ModuleType("george")
    george.kernels = types.SimpleNamespace(Matern32Kernel=None)
    george.GP = None
    george.HODLRSolver = None
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
    print("wrote", sorted(os.listdir(OUT)))


if __name__ == "__main__":
    main()
