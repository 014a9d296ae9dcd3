"""Diagnostic: per-phase cycle counts of k_setup (build with -DLFG_PROFILE_SETUP,
load via LFG_LIB).  Walkers from the bench's comp_scat ball."""
import os, sys, ctypes
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from lfit_python_amd import _native, synthetic, batch, sampler
from lfit_python_amd.lfit import flux_batch
L = _native.lib()
dev = torch.device('cuda', 0)
def flux_fn(p, x, w, nsub):
    f, st = flux_batch(np.asarray(p)[None, :], x, w, nsub=nsub); return f[0].cpu().numpy()
model = synthetic.config_single(flux_fn=flux_fn)
tree = batch.compile_tree(model)
ev = batch.LnProbEvaluator(tree)
p0 = np.array(model.dynasty_par_vals)
init = sampler.initialise_walkers(p0, sampler.comp_scatter(model.dynasty_par_names, 0.1), 512,
                                  lambda p: ev(torch.as_tensor(p, device=dev)).cpu().numpy())
# CV parameter sets of those walkers
cvp = np.array([init[:, g] for g in tree.gather[0]]).T
P = torch.as_tensor(cvp, device=dev).contiguous()
W = P.shape[0]
geo = torch.empty((W, 48), dtype=torch.float64, device=dev)
st = torch.empty(W, dtype=torch.int32, device=dev)
ws = torch.empty(L.lfg_workspace_size(W, 1), dtype=torch.uint8, device=dev)
vp = lambda t: ctypes.c_void_p(t.data_ptr())
L.lfg_elements(vp(P), W, 18, None, None, None, None, vp(geo), vp(st), vp(ws), ws.numel(), _native.stream_ptr())
g = geo.cpu().numpy()
for k, name in zip(range(42, 48), ['gather+roche_init', 'stream lane', 'findi', 'findphi90', 'bs_umax',
                                   'setup lane']):
    v = g[:, k]
    print('%-10s cycles mean %9.0f  max %9.0f' % (name, v.mean(), v.max()))
print('status', np.bincount(st.cpu().numpy()))
