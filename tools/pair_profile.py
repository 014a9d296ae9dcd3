"""Diagnostic: phase stamps of k_pair (build with -DLFG_PROFILE_PAIR:
tools/build_exp.sh PAIRPROF -DLFG_PROFILE_PAIR; load with LFG_DIAGNOSTIC=1
LFG_LIB=build/exp/liblfg_PAIRPROF.so).  Runs config-2 chain steps as bench.py
does and prints, for the last launch, each phase's end relative to the
block's start (us, 100 MHz s_memrealtime): the eight waves' element-phase
ends (wave 7: the last chunk + the speculative setup lanes), the barriers,
the sweep + scan, chi^2 and the finish."""
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
NPTS = int(sys.argv[2]) if len(sys.argv) > 2 else 300    # config 5: 1024 10000 5 (the LONG variant)
NSUB = int(sys.argv[3]) if len(sys.argv) > 3 else 1
L = _native.lib()


def flux_fn(pars, x, w, nsub):
    f, st = flux_batch(np.asarray(pars)[None, :], x, w, nsub=nsub, device=dev)
    return f[0].cpu().numpy()


model = synthetic.config_single(npts=NPTS, flux_fn=flux_fn, nsub=NSUB)
tree = batch.compile_tree(model, nsub=NSUB)
LONG = L.lfg_layout(ctypes.byref(batch.LnProbEvaluator(tree, device=dev).ctree)) == 2
ev = batch.LnProbEvaluator(tree, device=dev, max_walkers=W)
p0 = np.array(model.dynasty_par_vals)
init = sampler.initialise_walkers(p0, sampler.comp_scatter(model.dynasty_par_names, 0.1), W,
                                  lambda p: ev(torch.as_tensor(p, device=dev)).cpu().numpy(), seed=20261015)
S = sampler.EnsembleSampler(W, tree.ndim, ev, seed=20261015)
S.set_state(init)
for _ in range(10):
    S.step()
torch.cuda.synchronize()
t = np.zeros((24, 4096), dtype=np.uint64)
assert L.lfg_debug_pair(ctypes.c_void_p(t.ctypes.data)) == 0
nb = W // 2
t = t[:, :nb].astype(np.float64)
t0 = t[0]
span = (t[15].max() - t0.min()) / 100.0
print("blocks %d, launch span %.2f us (first start -> last finish)" % (nb, span))
print("block start spread: %s us" % np.percentile((t0 - t0.min()) / 100.0, [0, 50, 90, 100]).round(2))
rows = [("kernargs, n known", 20), ("partner drawn", 21), ("candidate known", 10), ("own window (phi0)", 11), ("prologue before B0", 19), ("B0 (prologue)", 16)] + [("wave %d elements" % k, 1 + k) for k in range(8)] + [
    ("B1 (phase barrier)", 9)] + ([("LONG tables built", 12), ("LONG points, chi^2", 13), ("finish", 15)] if LONG else [
    ("B2 (items, norms)", 10), ("B3 (cells)", 11), ("scan", 12), ("chi^2", 13), ("finish", 15)])
for name, k in rows:
    if not t[k].any():
        continue
    d = (t[k] - t0) / 100.0
    print("%-22s median %7.2f  p90 %7.2f  max %7.2f us" % (name, np.median(d), np.percentile(d, 90), d.max()))
kind = t[17].astype(int)
for k, nm in ((0, "setup"), (1, "prior"), (2, "stream")):
    m = kind == k
    if m.any():
        pre = (t[16][m] - t0[m]) / 100.0
        spec = (t[1][m] - t[16][m]) / 100.0   # wave 0: its job 0 (the speculative lanes) and the chunks it grabbed
        fin_k = (t[15][m] - t0[m]) / 100.0
        print("spec kind %-6s blocks %3d: B0 median %6.2f | wave 0 after B0 median %6.2f p90 %6.2f max %6.2f"
              " | block finish median %6.2f max %6.2f" % (nm, m.sum(), np.median(pre), np.median(spec),
                                                        np.percentile(spec, 90), spec.max(), np.median(fin_k), fin_k.max()))
fin = (t[15] - t0.min()) / 100.0
print("block finish times from launch start: %s us" % np.percentile(fin, [0, 10, 50, 90, 100]).round(2))
wv = np.zeros((4, 8, 4096), dtype=np.uint64)
if L.lfg_debug_pair_waves(ctypes.c_void_p(wv.ctypes.data)) == 0 and wv.any():
    wv = wv[:, :, :nb].astype(np.float64)
if wv.any() and not LONG:
    b3 = t[11]
    print("sweep per wave from B3 (us): median over blocks of [earliest wave, latest wave]")
    for k, nm in enumerate(("counts", "WD/disc applied", "spot/donor applied", "after B4")):
        d = (wv[k] - b3[None, :]) / 100.0
        print("  %-20s earliest %6.2f  latest %6.2f" % (nm, np.median(d.min(0)), np.median(d.max(0))))
    print("  %-20s %6.2f" % ("scan done (thread 0)", np.median((t[12] - b3) / 100.0)))
jb = np.zeros((3, 16, 4096), dtype=np.uint64)
if hasattr(L, "lfg_debug_pair_jobs") and L.lfg_debug_pair_jobs(ctypes.c_void_p(jb.ctypes.data)) == 0 and jb.any():
    jb = jb[:, :, :nb].astype(np.float64)
    print("element jobs per chunk (us, median over blocks): solve (start -> sink entry), sink (-> end)")
    for c in range(15):
        ok = (jb[0, c] > 0) & (jb[1, c] >= jb[0, c]) & (jb[2, c] >= jb[1, c])
        if ok.any():
            sv = (jb[1, c][ok] - jb[0, c][ok]) / 100.0
            sk = (jb[2, c][ok] - jb[1, c][ok]) / 100.0
            print("  chunk %2d  solve %6.2f  sink %6.2f  (n %d)" % (c, np.median(sv), np.median(sk), ok.sum()))
if LONG:
    lt = np.zeros((8, 4096), dtype=np.uint64)
    try:
        ok = L.lfg_debug_long_tables(ctypes.c_void_p(lt.ctypes.data)) == 0
    except AttributeError:
        ok = False
    if ok and lt.any():
        lt = lt[:, :nb].astype(np.float64)
        prev = t[9]
        for k, nm in enumerate(("(a) hulls", "(b) counts", "(c) cell scans", "(d) scatter", "(e) ranks",
                                "(e) placed", "(f) C per entry, (g) donor fx")):
            d = (lt[k] - prev) / 100.0
            print("LONG table step %-28s median %6.2f  p90 %6.2f us" % (nm, np.median(d), np.percentile(d, 90)))
            prev = lt[k]
if LONG and t[22].any():  # the quiet-point pass (round 6): points in closed form / queued for the sub-bin loop
    qq, qd = t[22].sum(), t[23].sum()
    print("LONG points in closed form %d, queued %d (%.1f %% quiet)" % (qq, qd, 100.0 * qq / max(qq + qd, 1)))
if LONG and wv.any():
    d = (wv[0] - t[12][None, :]) / 100.0
    print("LONG point loop per wave after the tables (us, median over blocks): %s" % np.median(d, axis=1).round(2))
    # s_memtime cycles (~100 MHz-equivalent ticks? printed raw) of the busiest lane per wave
    print("LONG busiest lane's WD/disc cycles per wave (median): %s" % np.median(wv[1], axis=1).round(0))
    print("LONG busiest lane's sub-bin cycles per wave (median): %s" % np.median(wv[2], axis=1).round(0))
    c = wv[3].astype(np.uint64)
    for k, nm in enumerate(("find-walk steps", "window entries", "windows in a hull")):
        print("LONG max lane's %s per wave (median): %s" % (nm, np.median(((c >> np.uint64(16 * k)) & np.uint64(0xffff)).astype(np.float64), axis=1).round(0)))
if len(sys.argv) > 4:  # raw stamps for offline analysis
    np.save(sys.argv[4], t)
