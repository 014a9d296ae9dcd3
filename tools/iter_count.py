"""Diagnostic: Newton iteration counts of the element solver per region
(build with -DLFG_COUNT_ITERS, load via LFG_LIB).  Walkers: the bench's
comp_scat ball.  Per region: mean iterations per item of the cone search,
ingress and egress tangencies; the per-wave maxima (the cost a wave pays);
fallback and eclipsed fractions."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from lfit_python_amd import _native, batch, sampler, synthetic
from lfit_python_amd.lfit import flux_batch

L = _native.lib()
L.lfg_diag_iters.argtypes = [ctypes.c_void_p]
dev = torch.device("cuda", 0)


def flux_fn(p, x, w, nsub):
    f, st = flux_batch(np.asarray(p)[None, :], x, w, nsub=nsub)
    return f[0].cpu().numpy()


model = synthetic.config_single(flux_fn=flux_fn)
tree = batch.compile_tree(model)
ev = batch.LnProbEvaluator(tree)
p0 = np.array(model.dynasty_par_vals)
init = sampler.initialise_walkers(p0, sampler.comp_scatter(model.dynasty_par_names, 0.1), 512,
                                  lambda p: ev(torch.as_tensor(p, device=dev)).cpu().numpy())
cvp = np.array([init[:, g] for g in tree.gather[0]]).T
P = torch.as_tensor(cvp, device=dev).contiguous()
W = P.shape[0]
st = torch.empty(W, dtype=torch.int32, device=dev)
ws = torch.empty(L.lfg_workspace_size(W, 1), dtype=torch.uint8, device=dev)
out = np.zeros(64, dtype=np.uint64)
L.lfg_diag_iters(out.ctypes.data)  # clear
vp = lambda t: ctypes.c_void_p(t.data_ptr())
L.lfg_elements(vp(P), W, 18, None, None, None, None, None, vp(st), vp(ws), ws.numel(), _native.stream_ptr())
L.lfg_diag_iters(out.ctypes.data)
for r, name in enumerate(("WD", "disc", "spot")):
    C = out[r * 16:(r + 1) * 16].astype(float)
    n, waves = C[7], C[9]
    print("%-5s items %7d  iters/item cone %.2f in %.2f out %.2f | per-wave max cone %.2f in %.2f out %.2f"
          " | fallback %.4f eclipsed %.3f" % (name, n, C[0] / n, C[1] / n, C[2] / n, C[3] / waves, C[4] / waves,
                                              C[5] / waves, C[6] / n, C[8] / n))
    h = C[10:16]
    print("      initial-guess error (rad) <1e-4 %.3f <1e-3 %.3f <1e-2 %.3f <3e-2 %.3f <1e-1 %.3f more %.3f"
          % tuple(h / max(h.sum(), 1)))
print("status", np.bincount(st.cpu().numpy()))
