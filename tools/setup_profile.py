"""Diagnostic: per-lane cycle counts of k_setup (build with -DLFG_PROFILE_SETUP,
load via LFG_LIB).  512 walkers from the bench's comp_scat ball through the
config-2 tree (lfg_lnprob: setup, prior and stream lanes all run); the
counts land in spare geo slots of the evaluator's workspace."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from lfit_python_amd import synthetic, batch, sampler  # noqa: E402
from lfit_python_amd.lfit import flux_batch  # noqa: E402

dev = torch.device('cuda', 0)


def flux_fn(p, x, w, nsub):
    f, st = flux_batch(np.asarray(p)[None, :], x, w, nsub=nsub)
    return f[0].cpu().numpy()


model = synthetic.config_single(flux_fn=flux_fn)
tree = batch.compile_tree(model)
ev = batch.LnProbEvaluator(tree)
p0 = np.array(model.dynasty_par_vals)
init = sampler.initialise_walkers(p0, sampler.comp_scatter(model.dynasty_par_names, 0.1), 512,
                                  lambda p: ev(torch.as_tensor(p, device=dev)).cpu().numpy())
W = init.shape[0]
for _ in range(3):
    ev(torch.as_tensor(init, device=dev))
torch.cuda.synchronize()
import ctypes  # noqa: E402
from lfit_python_amd import _native  # noqa: E402
L = _native.lib()
cyc = np.zeros((11, 4096), dtype=np.uint64)
L.lfg_debug_setup_cycles(ctypes.c_void_p(cyc.ctypes.data))
cyc = cyc[:, :W].astype(np.float64)
names = ['setup: gather', 'setup: roche_init', 'setup: findi', 'setup lane total',
         'stream: gather', 'stream: roche_init', 'stream: bspot (table)', 'stream lane total',
         'prior lane total', None, 'prior: roche_init + findphi90']
for k, name in enumerate(names):
    if name:
        print('%-30s cycles mean %8.0f  max %8.0f' % (name, cyc[k].mean(), cyc[k].max()))
print('shader clock over the prior lanes: %.0f MHz' % (100.0 * cyc[8].sum() / cyc[9].sum()))
