"""Diagnostic: why LONG points are not quiet (sub_point_quiet) at config 5.
Needs a build with -DLFG_COUNT_ITERS -DLFG_COUNT_QUIET (tools/build_exp.sh),
loaded with LFG_DIAGNOSTIC=1 LFG_LIB=...

    python tools/quiet_count.py [walkers] [points] [sub-bins]
"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from lfit_python_amd import _native, batch, sampler, synthetic  # noqa: E402
from lfit_python_amd.lfit import flux_batch  # noqa: E402

dev = torch.device("cuda", 0)
W = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
NPTS = int(sys.argv[2]) if len(sys.argv) > 2 else 10000
NSUB = int(sys.argv[3]) if len(sys.argv) > 3 else 5
L = _native.lib()


def flux_fn(pars, x, w, nsub):
    f, st = flux_batch(np.asarray(pars)[None, :], x, w, nsub=nsub, device=dev)
    return f[0].cpu().numpy()


model = synthetic.config_single(npts=NPTS, flux_fn=flux_fn, nsub=NSUB)
tree = batch.compile_tree(model, nsub=NSUB)
ev = batch.LnProbEvaluator(tree, device=dev, max_walkers=W)
p0 = np.array(model.dynasty_par_vals)
init = sampler.initialise_walkers(p0, sampler.comp_scatter(model.dynasty_par_names, 0.1), W,
                                  lambda p: ev(torch.as_tensor(p, device=dev)).cpu().numpy(), seed=5)
S = sampler.EnsembleSampler(W, tree.ndim, ev, seed=5)
S.set_state(init)
S.step()
c = (ctypes.c_ulonglong * 64)()
L.lfg_diag_iters(c)  # clear
for _ in range(3):
    S.step()
torch.cuda.synchronize()
L.lfg_diag_iters(c)
v = np.array(c[56:63], dtype=np.float64)
names = ["points", "zero/NaN width", "wraps", "spot hull", "beaming sign change", "donor entry inside", "quiet"]
for n, x in zip(names, v):
    print("%-22s %12d  (%.1f %%)" % (n, x, 100.0 * x / max(v[0], 1)))
