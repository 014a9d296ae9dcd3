"""Diagnostic: wall time per emcee iteration, eager vs HIP-graph replay, on
the bench workload (no per-kernel events)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from lfit_python_amd import batch, sampler, synthetic
from lfit_python_amd.lfit import flux_batch

dev = torch.device("cuda", 0)


def flux_fn(p, x, w, nsub):
    f, st = flux_batch(np.asarray(p)[None, :], x, w, nsub=nsub)
    return f[0].cpu().numpy()


model = synthetic.config_single(300, flux_fn=flux_fn)
tree = batch.compile_tree(model)
W = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
ev = batch.LnProbEvaluator(tree, device=dev, max_walkers=W)
p0 = np.array(model.dynasty_par_vals)
init = sampler.initialise_walkers(p0, sampler.comp_scatter(model.dynasty_par_names, 0.1), W,
                                  lambda p: ev(torch.as_tensor(p, device=dev)).cpu().numpy(), seed=1)
for graph in (False, True, False, True):
    S = sampler.EnsembleSampler(W, tree.ndim, ev, seed=1)
    S.set_state(init)
    S.use_graph = graph
    for _ in range(5):
        S.step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    n = 50
    for _ in range(n):
        S.step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / n
    print("graph=%s  %.1f us/iteration  %.3e evals/s" % (graph, dt * 1e6, W / dt), flush=True)
