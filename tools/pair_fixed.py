"""Diagnostic: ln_prob of one FIXED batch of config-2 walkers (W, default
1024), evaluated repeatedly: the median device time per call (torch events)
and, in a -DLFG_PROFILE_PAIR build, k_pair's per-chunk solve / sink stamps.
The batch does not depend on earlier results, so experiment builds that
change the numbers (tools/build_exp.sh) time the same geometry.

    LFG_PAIR=1 LFG_DIAGNOSTIC=1 LFG_LIB=build/exp/liblfg_<x>.so python tools/pair_fixed.py [W]
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
L = _native.lib()


def flux_fn(pars, x, w, nsub):
    f, st = flux_batch(np.asarray(pars)[None, :], x, w, nsub=nsub, device=dev)
    return f[0].cpu().numpy()


model = synthetic.config_single(npts=300, flux_fn=flux_fn)
tree = batch.compile_tree(model)
ev = batch.LnProbEvaluator(tree, device=dev, max_walkers=W)
# the batch: walkers of a short chain, made once (by the first build a
# session runs: a correct one) and read back by the others
fw = sys.argv[2] if len(sys.argv) > 2 else "gpurun_out/pair_fixed_walkers.npy"
if os.path.exists(fw):
    w0 = np.load(fw)
else:
    p0 = np.array(model.dynasty_par_vals)
    init = sampler.initialise_walkers(p0, sampler.comp_scatter(model.dynasty_par_names, 0.1), W,
                                      lambda p: ev(torch.as_tensor(p, device=dev)).cpu().numpy(), seed=20261015)
    S = sampler.EnsembleSampler(W, tree.ndim, ev, seed=20261015)
    S.set_state(init)
    for _ in range(10):
        S.step()
    w0 = S.pos.cpu().numpy()
    np.save(fw, w0)
walk = torch.as_tensor(w0, device=dev)
for _ in range(5):
    ev(walk)
torch.cuda.synchronize()
ts = []
for _ in range(50):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    lp = ev(walk)
    b.record()
    torch.cuda.synchronize()
    ts.append(a.elapsed_time(b) * 1e3)
print("W %d: ln_prob call median %.2f us (p10 %.2f, p90 %.2f); finite %d" % (
    W, np.median(ts), np.percentile(ts, 10), np.percentile(ts, 90), int(torch.isfinite(lp).sum())))
nb = W
if hasattr(L, "lfg_debug_pair_jobs"):
    t = np.zeros((24, 4096), dtype=np.uint64)
    L.lfg_debug_pair(ctypes.c_void_p(t.ctypes.data))
    t = t[:, :nb].astype(np.float64)
    t0 = t[0]
    for name, k in (("B0", 16), ("B1", 9), ("finish", 15)):
        d = (t[k] - t0) / 100.0
        print("%-8s median %6.2f  p90 %6.2f  max %6.2f us" % (name, np.median(d), np.percentile(d, 90), d.max()))
    print("launch span %.2f us" % ((t[15].max() - t0.min()) / 100.0))
    jb = np.zeros((3, 16, 4096), dtype=np.uint64)
    L.lfg_debug_pair_jobs(ctypes.c_void_p(jb.ctypes.data))
    jb = jb[:, :, :nb].astype(np.float64)
    ssum = ksum = 0.0
    for c in range(15):
        ok = (jb[0, c] > 0) & (jb[1, c] >= jb[0, c]) & (jb[2, c] >= jb[1, c])
        if ok.any():
            sv = np.median((jb[1, c][ok] - jb[0, c][ok]) / 100.0)
            sk = np.median((jb[2, c][ok] - jb[1, c][ok]) / 100.0)
            ssum += sv
            ksum += sk
            print("  chunk %2d  solve %6.2f  sink %6.2f" % (c, sv, sk))
    print("  sum      solve %6.2f  sink %6.2f" % (ssum, ksum))
