"""Diagnostic: does the step time depend on where the chain is?

Runs the bench's config-2 sampler (1024 walkers, comp_scat ball) for
`steps` emcee iterations, times every block of `block` steps (synced) and
saves the walkers at a few step counts to gpurun_out/drift_walkers_<k>.npy.

  python tools/chain_drift.py [steps=1000] [block=50]

With `count` as the first argument (and LFG_LIB pointing at a
-DLFG_COUNT_ITERS build) it instead reports the element solver's iteration
counts, per-wave maxima and fallbacks for every saved snapshot.
"""
import ctypes
import glob
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from lfit_python_amd import _native, batch, sampler, synthetic
from lfit_python_amd.lfit import flux_batch

dev = torch.device("cuda", 0)
OUT = os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "gpurun_out")


def flux_fn(p, x, w, nsub):
    f, st = flux_batch(np.asarray(p)[None, :], x, w, nsub=nsub)
    return f[0].cpu().numpy()


model = synthetic.config_single(flux_fn=flux_fn)
tree = batch.compile_tree(model)


def drift(steps, block):
    W = 1024
    ev = batch.LnProbEvaluator(tree, device=dev, max_walkers=W)
    p0 = np.array(model.dynasty_par_vals)
    init = sampler.initialise_walkers(p0, sampler.comp_scatter(model.dynasty_par_names, 0.1), W,
                                      lambda p: ev(torch.as_tensor(p, device=dev)).cpu().numpy(), seed=20261015)
    S = sampler.EnsembleSampler(W, tree.ndim, ev, seed=20261015)
    S.set_state(init)
    save = {0, 100, 200, 500, 1000, 2000, 5000}
    np.save(os.path.join(OUT, "drift_walkers_0.npy"), S.pos.cpu().numpy())
    for _ in range(5):
        S.step()
    done = 0
    while done < steps:
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(block):
            S.step()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        done += block
        lnp = S.lnp.cpu().numpy()
        fin = np.isfinite(lnp)
        print("steps %5d  %.1f us/step  %.2f M evals/s  lnp median %.1f  finite %d  acc %.3f  q sd %.2e"
              % (done, dt / block * 1e6, W * block / dt / 1e6, np.median(lnp[fin]), fin.sum(),
                 float(np.mean(S.acceptance_fraction)), float(S.pos[:, 0].std())), flush=True)
        if done in save:
            np.save(os.path.join(OUT, "drift_walkers_%d.npy" % done), S.pos.cpu().numpy())
    S.close()


def count():
    L = _native.lib()
    L.lfg_diag_iters.argtypes = [ctypes.c_void_p]
    vp = lambda t: ctypes.c_void_p(t.data_ptr())
    files = sorted(glob.glob(os.path.join(OUT, "drift_walkers_*.npy")),
                   key=lambda f: int(f.rsplit("_", 1)[1][:-4]))
    for f in files:
        walk = np.load(f)
        cvp = np.array([walk[:, g] for g in tree.gather[0]]).T  # config 2: every parameter a walker column
        P = torch.as_tensor(cvp, device=dev).contiguous()
        W = P.shape[0]
        st = torch.empty(W, dtype=torch.int32, device=dev)
        ws = torch.empty(L.lfg_workspace_size(W, 1), dtype=torch.uint8, device=dev)
        out = np.zeros(64, dtype=np.uint64)
        L.lfg_diag_iters(out.ctypes.data)  # clear
        L.lfg_elements(vp(P), W, 18, None, None, None, None, None, vp(st), vp(ws), ws.numel(), _native.stream_ptr())
        torch.cuda.synchronize()
        L.lfg_diag_iters(out.ctypes.data)
        print("== %s  status %s" % (os.path.basename(f), np.bincount(st.cpu().numpy(), minlength=6).tolist()))
        for r, name in enumerate(("WD", "disc", "spot")):
            C = out[r * 16:(r + 1) * 16].astype(float)
            n, waves = max(C[7], 1), max(C[9], 1)
            print("  %-5s items %7d  it/item cone %.2f in %.2f out %.2f | wave max cone %.2f in %.2f out %.2f"
                  " | fallback %.5f eclipsed %.3f" % (name, C[7], C[0] / n, C[1] / n, C[2] / n, C[3] / waves,
                                                      C[4] / waves, C[5] / waves, C[6] / n, C[8] / n), flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "count":
        count()
    else:
        drift(int(sys.argv[1]) if len(sys.argv) > 1 else 1000, int(sys.argv[2]) if len(sys.argv) > 2 else 50)
