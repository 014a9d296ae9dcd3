"""Diagnostic: can a second HIP stream hide k_setup-sized work behind the
main stream's kernels?  Main stream A runs lfg_lnprob (k_setup, k_elements,
k_lnlike) on 512 walkers per iteration; stream B runs lfg_lnprior (k_setup +
a tiny combine) on 1024 walkers.  Modes:
  A        A alone
  A+B      B forked after A's previous iteration, A waits for B before its next
           iteration (the pipelined shape: B's work has ~60 us of slack)
  serial   A then B on one stream
Prints us per iteration."""
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


model = synthetic.config_single(flux_fn=flux_fn)
tree = batch.compile_tree(model)
evA = batch.LnProbEvaluator(tree, max_walkers=1024)
evB = batch.LnProbEvaluator(tree, max_walkers=1024)
p0 = np.array(model.dynasty_par_vals)
init = sampler.initialise_walkers(p0, sampler.comp_scatter(model.dynasty_par_names, 0.1), 1024,
                                  lambda p: evA(torch.as_tensor(p, device=dev)).cpu().numpy())
X = torch.as_tensor(init, device=dev)
XA = X[:512].contiguous()
outA = torch.empty(512, dtype=torch.float64, device=dev)
outB = torch.empty(1024, dtype=torch.float64, device=dev)
sA = torch.cuda.current_stream()
sB = torch.cuda.Stream()
N = 200


def run(mode):
    eA = torch.cuda.Event()
    eB = torch.cuda.Event()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(N):
        if mode == "A+B":
            if i:
                sA.wait_event(eB)      # B's previous fork has finished
            eA.record(sA)              # fork point
            with torch.cuda.stream(sB):
                sB.wait_event(eA)
                evB.ln_prior(X, out=outB)
                eB.record(sB)
        evA(XA, out=outA)              # runs beside B
        if mode == "serial":
            evB.ln_prior(X, out=outB)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / N * 1e6


for _ in range(2):
    for mode in ("A", "A+B", "serial"):
        print("%-7s %7.1f us per iteration" % (mode, run(mode)))
