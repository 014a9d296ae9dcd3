"""Diagnostic: fraction of elements that take the nested slow path (build with
-DLFG_MARK_FALLBACK, load via LFG_LIB).  Walkers: the bench's ball and a wide
random set."""
import os, sys, ctypes
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from lfit_python_amd import _native
from tests.helpers import random_pars, TRUTH18
L = _native.lib()
def run(P):
    P = torch.as_tensor(P, device='cuda').contiguous(); W = P.shape[0]
    wg = torch.empty((W, 1500), dtype=torch.float64, device='cuda')
    a = torch.empty_like(wg); b = torch.empty_like(wg)
    st = torch.empty(W, dtype=torch.int32, device='cuda')
    ws = torch.empty(L.lfg_workspace_size(W, 1), dtype=torch.uint8, device='cuda')
    vp = lambda t: ctypes.c_void_p(t.data_ptr())
    L.lfg_elements(vp(P), W, 18, vp(a), vp(b), vp(wg), None, None, vp(st), vp(ws), ws.numel(), _native.stream_ptr())
    w = wg.cpu().numpy(); s = st.cpu().numpy(); ok = s == 0
    fb = (w[ok] < 0)
    wave = fb.reshape(ok.sum(), -1)
    print('sets', ok.sum(), 'fallback elements %.4f%%' % (100 * fb.mean()),
          'per region WD/disc/BS %%: %.3f %.3f %.3f' % tuple(100 * fb[:, s0:s1].mean() for s0, s1 in ((0, 400), (400, 1400), (1400, 1500))),
          'eclipsed %.3f' % (a.cpu().numpy()[ok] < b.cpu().numpy()[ok]).mean())
rng = np.random.default_rng(0)
near = np.array(TRUTH18) * (1 + 0.02 * rng.standard_normal((512, 18)))
run(near)
run(random_pars(512, seed=9))
