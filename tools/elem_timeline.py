"""Diagnostic: per-wave timeline of k_elements (build with -DLFG_PROFILE_ELEM,
load via LFG_LIB).  Runs a few config-2 chain steps (or --config 3 / gp) on
the device sampler, then reads the last launch's stamps: start / end
(s_memrealtime, 100 MHz) and HW_ID of every one-wave block, and the kind
(0: speculative setup lanes, 1 + k: chunk k of a pair's items).

    LFG_LIB=build/exp/liblfg_ELEMPROF.so python tools/elem_timeline.py [--config 2]
"""
import argparse
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from lfit_python_amd import _native, batch, sampler, synthetic  # noqa: E402
from lfit_python_amd.lfit import flux_batch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="2")
    ap.add_argument("--walkers", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=6)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)

    def flux_fn(p, x, w, nsub):
        f, st = flux_batch(np.asarray(p)[None, :], x, w, nsub=nsub, device=dev)
        return f[0].cpu().numpy()

    model = (synthetic.config_tree(4, 300, flux_fn=flux_fn) if args.config == "3"
             else synthetic.config_single(flux_fn=flux_fn))
    tree = batch.compile_tree(model)
    ev = batch.LnProbEvaluator(tree, device=dev, max_walkers=args.walkers)
    p0 = np.array(model.dynasty_par_vals)
    init = sampler.initialise_walkers(p0, sampler.comp_scatter(model.dynasty_par_names, 0.1), args.walkers,
                                      lambda p: ev(torch.as_tensor(p, device=dev)).cpu().numpy())
    S = sampler.EnsembleSampler(args.walkers, tree.ndim, ev, seed=1)
    S.set_state(init)
    for _ in range(args.steps):
        S.step()
    torch.cuda.synchronize()
    L = _native.lib()
    buf = np.zeros((4, 32768), dtype=np.uint64)
    L.lfg_debug_elem_waves(ctypes.c_void_p(buf.ctypes.data))
    used = buf[1] > 0
    t0 = buf[0][used].astype(np.int64)
    t1 = buf[1][used].astype(np.int64)
    hw = buf[2][used].astype(np.int64)
    kind = buf[3][used].astype(np.int64)
    base = t0.min()
    s, e = (t0 - base) * 10.0 / 1000.0, (t1 - base) * 10.0 / 1000.0  # us
    print("waves %d, kernel span %.1f us (first start -> last end)" % (used.sum(), e.max()))
    for k in sorted(set(kind.tolist())):
        m = kind == k
        d = e[m] - s[m]
        print("kind %2d (%s): waves %5d  start %.1f-%.1f  end %.1f-%.1f  duration median %.2f p90 %.2f max %.2f us"
              % (k, "spec setup" if k == 0 else "chunk %d" % (k - 1), m.sum(), s[m].min(), s[m].max(),
                 e[m].min(), e[m].max(), np.median(d), np.percentile(d, 90), d.max()))
    # concurrency: waves resident per microsecond
    grid = np.arange(0.0, e.max() + 1.0, 1.0)
    conc = [int(np.sum((s <= g) & (e > g))) for g in grid]
    print("resident waves per us:", " ".join(str(c) for c in conc))
    # CU identity: HW_ID cu_id bits 8..11, sh 12, se 13..15 (gfx9 layout); XCC not in it
    cu = (hw >> 8) & 0xF
    se = (hw >> 13) & 0x7
    print("distinct (se, cu) seen:", len(set(zip(se.tolist(), cu.tolist()))))
    last = np.argsort(e)[-10:]
    print("last 10 waves: kind, start, end:", [(int(kind[i]), round(s[i], 1), round(e[i], 1)) for i in last])


if __name__ == "__main__":
    main()
