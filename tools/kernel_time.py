"""Diagnostic: repeated lfg_lnprob launches on the bench workload (512
walkers of the comp_scat ball) for rocprofv3 --kernel-trace --stats."""
import os
import sys

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
ev = batch.LnProbEvaluator(tree, max_walkers=512)
p0 = np.array(model.dynasty_par_vals)
cache = os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "gpurun_out", "kernel_time_walkers.npy")
if os.path.exists(cache):  # experiment builds reuse the main build's walkers
    init = np.load(cache)
else:
    init = sampler.initialise_walkers(p0, sampler.comp_scatter(model.dynasty_par_names, 0.1), 512,
                                      lambda p: ev(torch.as_tensor(p, device=dev)).cpu().numpy())
    np.save(cache, init)
x = torch.as_tensor(init, device=dev)
out = torch.empty(512, dtype=torch.float64, device=dev)
for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 30):
    ev(x, out=out)
torch.cuda.synchronize()
print("lnp mean", float(out[torch.isfinite(out)].mean()))
tag = os.path.basename(os.environ.get("LFG_LIB", "main")).replace("liblfg_", "").replace(".so", "")
np.save(os.path.join(os.path.dirname(cache), "kt_lnp_%s.npy" % tag), out.cpu().numpy())
