"""Anchor study of the model against the reference's real data (MODEL_SPEC 9).

The reference's example input (test_data/mcmc_input.dat) holds parameters
fitted with the real lfit to its six light curves.  Starting from them, this
runs the device MCMC of this framework (the HIP path) and reports how far the
posterior of this model moves the core parameters q, dphi, rwd, and the
per-eclipse chi^2/N at the start and at the best sample:
  * the chi^2 tree (useGP = 0) of all six eclipses;
  * the reference's own likelihood (useGP = 1, the shipped input).
Prints one JSON document (gpurun_out/anchor_study.json when run on the box).

    python tools/anchor_study.py [--walkers 512] [--burn 3000] [--prod 2000]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
GOLD = os.path.join(ROOT, "tests", "golden")


def load(tag):
    from lfit_python_amd import cvmodel
    src = os.path.join(GOLD, "ref_test_data", "mcmc_input.dat")
    text = open(src, encoding="utf-8", errors="replace").read()
    if tag == "chi2":
        text = text.replace("useGP = 1", "useGP = 0")
    path = os.path.join(GOLD, "ref_test_data", "mcmc_input_anchor_%s.dat" % tag)
    open(path, "w").write(text)
    return cvmodel.construct_model(path)


def study(tag, walkers, burn, prod, seed):
    import torch
    from lfit_python_amd import batch, sampler
    m = load(tag)
    t = batch.compile_tree(m)
    ev = batch.LnProbEvaluator(t, max_walkers=walkers)
    names = m.dynasty_par_names
    p0 = np.array(m.dynasty_par_vals)
    n = np.diff(t.offsets)

    def per_eclipse(p):
        lle = torch.empty((1, t.E), dtype=torch.float64, device="cuda")
        ev(torch.as_tensor(p[None, :], device="cuda"), lnlike_e=lle)
        return lle.cpu().numpy()[0]

    start = per_eclipse(p0)
    lp0 = float(ev(torch.as_tensor(p0[None, :], device="cuda")).cpu().numpy()[0])
    scat = sampler.comp_scatter(names, 0.01)
    init = sampler.initialise_walkers(p0, scat, walkers,
                                      lambda p: ev(torch.as_tensor(p, device="cuda")).cpu().numpy(), seed=seed)
    S = sampler.EnsembleSampler(walkers, t.ndim, ev, seed=seed)
    t0 = time.time()
    pos, lnp, _ = S.run_mcmc(init, burn, storechain=False)
    S.reset()
    S.run_mcmc(None, prod, storechain=True)
    el = time.time() - t0
    ch = S.chain_dev.cpu().numpy().reshape(-1, t.ndim)
    lc = S.lnprob_dev.cpu().numpy().reshape(-1)
    best = ch[np.argmax(lc)]
    out = {"tree": tag, "ndim": t.ndim, "eclipses": t.leaf_labels, "npts": n.tolist(), "walkers": walkers,
           "burn": burn, "prod": prod, "seconds": el, "acceptance": float(np.mean(S.acceptance_fraction)),
           "lnp_start": lp0, "lnp_best": float(lc.max())}
    if not t.gp:
        out["chi2_per_n_start"] = dict(zip(t.leaf_labels, (-2.0 * start / n).round(3).tolist()))
        out["chi2_per_n_best"] = dict(zip(t.leaf_labels, (-2.0 * per_eclipse(best) / n).round(3).tolist()))
    else:
        out["lnlike_start"] = dict(zip(t.leaf_labels, start.round(2).tolist()))
        out["lnlike_best"] = dict(zip(t.leaf_labels, per_eclipse(best).round(2).tolist()))
    pars = {}
    for i, nm in enumerate(names):
        if not (nm.endswith("_core") or nm.endswith("_0")):
            continue
        lo, med, hi = np.percentile(ch[:, i], [16, 50, 84])
        sig = 0.5 * (hi - lo)
        pars[nm] = {"start": float(p0[i]), "median": float(med), "sigma": float(sig), "best": float(best[i]),
                    "shift_sigma": float((med - p0[i]) / sig) if sig > 0 else None,
                    "shift_rel": float((med - p0[i]) / p0[i]) if p0[i] else None}
    out["params"] = pars
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--walkers", type=int, default=512)
    ap.add_argument("--burn", type=int, default=3000)
    ap.add_argument("--prod", type=int, default=2000)
    ap.add_argument("--seed", type=int, default=20261016)
    ap.add_argument("--trees", default="chi2,gp")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "anchor_study.json"))
    args = ap.parse_args()
    res = []
    for tag in args.trees.split(","):
        res.append(study(tag, args.walkers, args.burn, args.prod, args.seed))
        print(json.dumps(res[-1]), flush=True)
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    json.dump(res, open(args.out, "w"), indent=1)


if __name__ == "__main__":
    main()
