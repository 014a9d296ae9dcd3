"""Counted FP64 work per walker-eclipse evaluation (MODEL_SPEC.md section 11).

Builds tools/flop_count/count.cpp (the kernels' device functions compiled for
the host over a counting FP64 type) and runs it on the parameter sets of a
BASELINE config's walker ensemble (the bench's comp_scat ball, resampled to
finite ln_prob with the CPU oracle), then prints the per-evaluation constants
F_setup, F_geom (per element root) and the accumulation terms.

    python tools/flop_count.py [--config 2|3|5] [--walkers 512] [--json out.json]
"""
import argparse
import ctypes
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

HERE = os.path.join(ROOT, "tools", "flop_count")

# direct-form accumulation per element per point per sub-phase (MODEL_SPEC 11.3)
F_ACC_ECL = 3    # overlap |[a,b] n window| (1 sub) + weighted accumulate (1 fma)
F_ACC_DON = 6    # projection dA n.e (1 mul + 2 fma) + max(0, .) accumulate (1 add)
F_POINT = 40     # per point per sub-phase: phase wrap, sincospi, beaming, donor normalisation, chi^2 share
N_ECL, N_DON = 1500, 400
# k_gp_like (lfg.hip), parallel in time: per point, the element pass of its
# segment on a lane quad -- per lane: prediction of its D row, A column and
# c_r 31, gain / innovation / J, eta, c, A, D updates 52, the point's
# transition factors 3 -> 4 x 86; per segment (8 per pair) the 4x4 combine
# in one lane: gap prediction 136, C = I + J Sigma 128, adjugate inverse 144,
# Sigma_post 128, u / ll terms / posterior mean 104, end state 304
F_GP_POINT = 4 * (31 + 52 + 3)
F_GP_SEG, GP_SEG = 944, 8
F_GP_STEP = 150  # one serial Kalman step (unit count gp_kalman_step; the k_gp helper of lfg_gp_lnlike)
U_ROOTS = {"wd": 200, "disc": 500, "spot": 100, "donor": 100}


def build():
    out = os.path.join(tempfile.gettempdir(), "liblfg_flopcount_%d.so" % os.getpid())
    subprocess.run(["g++", "-std=c++20", "-O1", "-fPIC", "-shared", "-I", os.path.join(HERE, "shim"),
                    "-I", os.path.join(ROOT, "lfit_python_amd", "csrc"), "-I", os.path.join(ROOT, "include"),
                    "-o", out, os.path.join(HERE, "count.cpp")], check=True)
    lib = ctypes.CDLL(out)
    lib.lfc_count_pair.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
    lib.lfc_count_prior.restype = ctypes.c_longlong
    lib.lfc_count_prior.argtypes = [ctypes.c_int] + [ctypes.c_double] * 4
    lib.lfc_unit_counts.argtypes = [ctypes.c_void_p]
    return lib


def walkers(config, n, seed=20261015):
    from lfit_python_amd import batch, sampler, synthetic
    from oracle.oracle import Oracle
    o = Oracle()

    def flux_fn(p, x, w, nsub):
        return o.flux(p, x, w, nsub=nsub)[1]
    if config == "gp":
        from lfit_python_amd import cvmodel
        model = cvmodel.construct_model(os.path.join(ROOT, "tests", "golden", "ref_test_data", "mcmc_input.dat"))
    elif config == 3:
        model = synthetic.config_tree(4, 300, flux_fn=flux_fn)
    elif config == 5:
        model = synthetic.config_single(10000, flux_fn=flux_fn, nsub=5)
    else:
        model = synthetic.config_single(300, flux_fn=flux_fn)
    tree = batch.compile_tree(model, nsub=5 if config == 5 else 1)
    p0 = np.array(model.dynasty_par_vals)
    scat = sampler.comp_scatter(model.dynasty_par_names, 0.1)
    init = sampler.initialise_walkers(p0, scat, n, lambda p: o.lnprob_batch(p, tree, nsub=tree.nsub, nthreads=8)[0],
                                      seed=seed)
    return tree, init


def prior_sum_flops(types, chunk=16):
    """Prior.ln_prob sum of a prior lane from the tree's constants
    (lfg_tree.prior_c; lfg.hip prior_lane): per parameter gauss
    (v - p1) c1 and fma(-z/2, z, c0) = 5, plus the running add; log_uniform
    one product multiply, mod_jeff also v + p1; per chunk one log and one sub."""
    per = {0: 6, 1: 6, 2: 1, 3: 2, 4: 3}
    n = len(types)
    return float(sum(per.get(int(t), 1) for t in types) + 2 * ((n + chunk - 1) // chunk))


def cv_pars(tree, walk, e):
    g = tree.gather[e]
    return np.array([[w[k] if k >= 0 else tree.consts[-1 - k] for k in g] for w in walk])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="2", help="2, 3, 5 or gp")
    ap.add_argument("--walkers", type=int, default=512)
    ap.add_argument("--json", default=None)
    ap.add_argument("--like-walkers", type=int, default=None,
                    help="walkers whose k_lnlike work is simulated (default: 64, config 5: 6)")
    args = ap.parse_args()
    args.config = args.config if args.config == "gp" else int(args.config)
    lib = build()
    tree, walk = walkers(args.config, args.walkers)
    rows = []
    for e in range(tree.E):
        for p in cv_pars(tree, walk, e):
            out = np.zeros(32, np.int64)
            rc = lib.lfc_count_pair(p.ctypes.data, int(tree.npars[e]), out.ctypes.data)
            if rc == 0:
                rows.append(out.copy())
    R = np.array(rows, dtype=np.float64)
    m = R.mean(0)
    prior = prior_sum_flops(tree.prior_type)
    unit = np.zeros(8, np.int64)
    lib.lfc_unit_counts(unit.ctypes.data)
    E = tree.E
    f_setup = m[0] + m[2] + (m[4] + prior) / E          # per pair: setup + stream lanes, prior lane shared by E
    step = float(unit[1])  # one tangency_step
    geo = {k: m[6 + i] - (step * m[19 + i] if i < 3 else 0.0) for i, k in enumerate(("wd", "disc", "spot", "donor"))}
    f_geom_total = sum(geo.values())
    n_roots = sum(U_ROOTS.values())
    npts = int(np.max(np.diff(tree.offsets)))
    S = tree.nsub
    f_acc_total = npts * S * (N_ECL * F_ACC_ECL + N_DON * F_ACC_DON + F_POINT)
    # k_lnlike as executed (tools/like_count.py: the sweep and the sub-bin
    # tables on the oracle's element intervals of each pair)
    import like_count
    from oracle.oracle import Oracle
    o = Oracle()
    nlw = args.like_walkers or (6 if args.config == 5 else 64)
    like, like_parts = [], []
    for e in range(E):
        a0, a1 = tree.offsets[e], tree.offsets[e + 1]
        for pars in cv_pars(tree, walk[:nlw], e):
            st, a, b, wg, donor, g16 = o.elements(pars)
            if st != 0:
                continue
            f, parts = like_count.count_pair(tree.x[a0:a1], tree.w[a0:a1], S, a[:1400], b[:1400], a[1400:], b[1400:],
                                             donor, g16[2], pars[13], gp=tree.gp)
            like.append(f)
            like_parts.append(parts)
    f_like = float(np.mean(like))
    npts_mean = float(np.mean(np.diff(tree.offsets)))
    f_gp = (npts_mean * F_GP_POINT + GP_SEG * F_GP_SEG) if tree.gp else 0.0
    like_parts = {k: round(float(np.mean([p[k] for p in like_parts])), 1) for k in like_parts[0]}
    res = {
        "config": args.config, "pairs_counted": int(len(R)), "walkers": int(args.walkers), "E": E,
        "npts": npts, "nsub": S,
        "F_setup": round(f_setup, 1),
        "F_setup_parts": {"setup_lane": round(m[0], 1), "stream_lane": round(m[2], 1),
                          "prior_lane_findphi": round(m[4], 1), "prior_sum": round(prior, 1)},
        "F_geom_per_root": round(f_geom_total / n_roots, 1),
        "F_geom_by_item": {k: round(v / U_ROOTS[k], 1) for k, v in geo.items()},
        "roots_per_pair": n_roots,
        "elements_per_pair": N_ECL + N_DON,
        "F_geom_total": round(f_geom_total, 1),
        "F_acc_ecl": F_ACC_ECL, "F_acc_don": F_ACC_DON, "F_point": F_POINT,
        "F_acc_total": f_acc_total,
        "F_like": round(f_like, 1),
        "F_like_parts": like_parts,
        "like_pairs_simulated": len(like),
        # what each kernel executes per pair on the speculative single-GPU path
        # (bench.py's default): k_elements also forms both candidates' setup
        # for the next half; k_setup runs only off the speculative path
        # (GP trees: the k_lnlike event span also holds k_gp_like, one Kalman
        # step per point)
        "per_kernel": {"k_setup": round(f_setup, 1), "k_elements": round(f_geom_total + 2 * f_setup, 1),
                       "k_lnlike": round(f_like + f_gp, 1)},
        "F_executed_per_pair": round(2 * f_setup + f_geom_total + f_like + f_gp, 1),
        "F_direct_form_equivalent_per_pair": round(f_setup + f_geom_total + f_acc_total, 1),
        "F_total_per_pair": round(f_setup + f_geom_total + f_acc_total, 1),
        "transcendentals_per_pair": round(m[1] + m[3] + m[10] + m[11] + m[12] + m[13] + m[5] / E, 1),
        "newton_steps_per_eclipsed_root": round(m[16] / max(m[14], 1), 2),
        "cone_steps_per_root": round(m[17] / (n_roots - U_ROOTS["donor"]), 2),
        "eclipsed_roots": round(m[14], 1), "fallbacks_per_pair": round(m[15], 3),
        "lockstep_discarded_steps_per_pair": round(m[18], 1),
        "unit_counts": {"cone_point": int(unit[0]), "tangency_step": int(unit[1]), "rk4_step": int(unit[2]),
                        "ray_min_1iter": int(unit[3]), "donor_newton_step": int(unit[4]),
                        "rpot_grad": int(unit[5]), "rotate": int(unit[6]), "gp_kalman_step": int(unit[7])},
    }
    print(json.dumps(res, indent=1))
    if args.json:
        json.dump(res, open(args.json, "w"), indent=1)


if __name__ == "__main__":
    main()
