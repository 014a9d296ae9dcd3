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
g = ev._ws[:W * 48 * 8].view(torch.float64).reshape(W, 48).cpu().numpy()
for k, name in [(42, 'setup: gather + roche_init'), (44, 'setup: findi'), (47, 'setup lane'),
                (46, 'stream: roche_init + bspot'), (43, 'stream lane'), (45, 'prior lane')]:
    v = g[:, k]
    print('%-28s cycles mean %9.0f  max %9.0f' % (name, v.mean(), v.max()))
print('shader clock over the prior lanes: %.0f MHz' % (100.0 * g[:, 45].sum() / g[:, 41].sum()))
import ctypes  # noqa: E402
from lfit_python_amd import _native  # noqa: E402
L = _native.lib()
buf = np.zeros((3, 2, 4096), dtype=np.uint64)
L.lfg_debug_setup_stamps(ctypes.c_void_p(buf.ctypes.data))
n = {0: W, 1: W, 2: W}
t0 = min(int(buf[k, 0, :n[k]].min()) for k in n)
for k, name in [(0, 'setup'), (1, 'stream'), (2, 'prior')]:
    st, en = (buf[k, 0, :n[k]].astype(np.int64) - t0) / 100.0, (buf[k, 1, :n[k]].astype(np.int64) - t0) / 100.0
    print('%-7s lanes: start %.2f..%.2f us  end %.2f..%.2f us  (median end %.2f)' % (
        name, st.min(), st.max(), en.min(), en.max(), np.median(en)))
