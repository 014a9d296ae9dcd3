"""Diagnostic: host time per emcee step of the config-2 bench path against
the GPU's.  Runs K steps without a sync and times the host loop (the
launches' enqueue cost, Python included), then the whole region to the sync.
If the host loop takes as long as the region, the steps are host-bound.

    python tools/host_step_probe.py [K]
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from lfit_python_amd import batch, sampler, synthetic  # noqa: E402
from lfit_python_amd.lfit import flux_batch  # noqa: E402

dev = torch.device("cuda", 0)
K = int(sys.argv[1]) if len(sys.argv) > 1 else 200


def flux_fn(pars, x, w, nsub):
    f, st = flux_batch(np.asarray(pars)[None, :], x, w, nsub=nsub, device=dev)
    return f[0].cpu().numpy()


model = synthetic.config_single(npts=300, flux_fn=flux_fn)
tree = batch.compile_tree(model)
W = 1024
ev = batch.LnProbEvaluator(tree, device=dev, max_walkers=W)
p0 = np.array(model.dynasty_par_vals)
init = sampler.initialise_walkers(p0, sampler.comp_scatter(model.dynasty_par_names, 0.1), W,
                                  lambda p: ev(torch.as_tensor(p, device=dev)).cpu().numpy(), seed=1)
S = sampler.EnsembleSampler(W, tree.ndim, ev, seed=1)
S.set_state(init)
for _ in range(10):
    S.step()
torch.cuda.synchronize()
for k in (20, K):
    for rep in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(k):
            S.step()
        th = time.perf_counter() - t0
        torch.cuda.synchronize()
        tt = time.perf_counter() - t0
        print("K %4d: host loop %.1f us/step, region %.1f us/step" % (k, th / k * 1e6, tt / k * 1e6), flush=True)
# host cost of one ln_prob-free step: a half-step call alone, timed in a loop on the host
import cProfile  # noqa: E402
import pstats  # noqa: E402
pr = cProfile.Profile()
pr.enable()
for _ in range(50):
    S.step()
pr.disable()
torch.cuda.synchronize()
pstats.Stats(pr).sort_stats("tottime").print_stats(12)
