"""Diagnostic: element-solver iteration counts and fallbacks on the walker
ball of a bench config (build with -DLFG_COUNT_ITERS, load via LFG_LIB).
  LFG_LIB=build/exp/liblfg_count.so python tools/tree_iters.py gp|2|3"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

import bench
from lfit_python_amd import _native, batch, sampler

L = _native.lib()
L.lfg_diag_iters.argtypes = [ctypes.c_void_p]
dev = torch.device("cuda", 0)
args = bench.parse(["--config", sys.argv[1] if len(sys.argv) > 1 else "gp"])


def flux_fn(p, x, w, nsub):
    from lfit_python_amd.lfit import flux_batch
    f, st = flux_batch(np.asarray(p)[None, :], x, w, nsub=nsub)
    return f[0].cpu().numpy()


model = bench.build_model(args, flux_fn)
tree = batch.compile_tree(model, nsub=args.nsub)
ev = batch.LnProbEvaluator(tree, device=dev)
p0 = np.array(model.dynasty_par_vals)
init = sampler.initialise_walkers(p0, sampler.comp_scatter(model.dynasty_par_names, 0.1), 512,
                                  lambda p: ev(torch.as_tensor(p, device=dev)).cpu().numpy(), seed=args.seed)
vp = lambda t: ctypes.c_void_p(t.data_ptr())
for e in range(tree.E):
    g = tree.gather[e]
    npar = int(tree.npars[e])
    cvp = np.array([[w[k] if k >= 0 else tree.consts[-1 - k] for k in g[:npar]] for w in init])
    P = torch.as_tensor(cvp, device=dev).contiguous()
    W = P.shape[0]
    st = torch.empty(W, dtype=torch.int32, device=dev)
    ws = torch.empty(L.lfg_workspace_size(W, 1), dtype=torch.uint8, device=dev)
    out = np.zeros(64, dtype=np.uint64)
    L.lfg_diag_iters(out.ctypes.data)
    L.lfg_elements(vp(P), W, npar, None, None, None, None, None, vp(st), vp(ws), ws.numel(), _native.stream_ptr())
    torch.cuda.synchronize()
    L.lfg_diag_iters(out.ctypes.data)
    print("== eclipse %d (%d pars)  status %s" % (e, npar, np.bincount(st.cpu().numpy(), minlength=6).tolist()))
    for r, name in enumerate(("WD", "disc", "spot")):
        C = out[r * 16:(r + 1) * 16].astype(float)
        n, waves = max(C[7], 1), max(C[9], 1)
        print("  %-5s items %7d  it/item cone %.2f in %.2f out %.2f | wave max cone %.2f in %.2f out %.2f"
              " | fallback %.5f eclipsed %.3f" % (name, C[7], C[0] / n, C[1] / n, C[2] / n, C[3] / waves,
                                                  C[4] / waves, C[5] / waves, C[6] / n, C[8] / n), flush=True)
