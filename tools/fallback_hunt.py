"""Diagnostic: which proposals send element solves to the nested fallback?

Runs the bench's config-2 chain on the plain fused half-step (LFG_SPEC=0 is
set here) with a -DLFG_COUNT_ITERS build (LFG_LIB), reads the fallback
records after every half-step and saves the proposal parameter vectors of
the pairs that fell back, with the item, to gpurun_out/fallback_pars.npz.

  LFG_LIB=build/exp/liblfg_count.so python tools/fallback_hunt.py [steps=1000]
"""
import ctypes
import os
import sys
import time

os.environ["LFG_SPEC"] = "0"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from lfit_python_amd import _native, batch, sampler, synthetic
from lfit_python_amd.lfit import flux_batch

dev = torch.device("cuda", 0)
OUT = os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "gpurun_out")
L = _native.lib()
L.lfg_diag_iters.argtypes = [ctypes.c_void_p]


def flux_fn(p, x, w, nsub):
    f, st = flux_batch(np.asarray(p)[None, :], x, w, nsub=nsub)
    return f[0].cpu().numpy()


model = synthetic.config_single(flux_fn=flux_fn)
tree = batch.compile_tree(model)
W = 1024
ev = batch.LnProbEvaluator(tree, device=dev, max_walkers=W)
p0 = np.array(model.dynasty_par_vals)
init = sampler.initialise_walkers(p0, sampler.comp_scatter(model.dynasty_par_names, 0.1), W,
                                  lambda p: ev(torch.as_tensor(p, device=dev)).cpu().numpy(), seed=20261015)
S = sampler.EnsembleSampler(W, tree.ndim, ev, seed=20261015)
S.set_state(init)
buf = np.zeros(64, dtype=np.uint64)
L.lfg_diag_iters(buf.ctypes.data)  # clear
recs, pars, when, nfb = [], [], [], [0]


def hook(pos, lnp, half, a, seed, step, q, zfac, naccept, lnp_new=None, spec=False):
    t0 = time.perf_counter()
    ev.step_half(pos, lnp, half, a, seed, step, q, zfac, naccept, lnp_new=lnp_new)
    L.lfg_diag_iters(buf.ctypes.data)  # syncs, reads, clears
    dt = time.perf_counter() - t0
    n = int(buf[48])
    if n:
        nfb[0] += n
        qh = q.cpu().numpy()
        for k in range(min(n, 15)):
            r = int(buf[49 + k])
            pair, u = r >> 16, r & 0xFFFF
            recs.append((step, half, pair, u))
            pars.append(qh[pair])
            when.append(dt)


S.half_timer = hook
steps = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
for i in range(steps):
    S.step()
    if (i + 1) % 100 == 0:
        print("step %d fallbacks so far %d (records %d)" % (i + 1, nfb[0], len(recs)), flush=True)
np.savez(os.path.join(OUT, "fallback_pars.npz"), recs=np.array(recs), pars=np.array(pars), dt=np.array(when))
for (st, h, p, u), dt in list(zip(recs, when))[:40]:
    print("step %4d half %d pair %4d item %4d  half-step %.2f ms" % (st, h, p, u, dt * 1e3))
S.close()
