"""Diagnostic: per-phase cycle stamps of k_lnlike (build with -DLFG_PROFILE_LIKE,
load via LFG_LIB).  Stamps (s_memtime ticks from kernel entry, thread 0 of each
block, first tile, last sub-bin pass): 0 staged, 1 phases + cells,
2 WD/disc sweep (thread 0 only), 3 spot/donor sweep + barrier, 4 scan, 5 tile end."""
import os, sys, ctypes
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from lfit_python_amd import _native
from tests.helpers import random_pars, phase_grid
L = _native.lib()
dev = torch.device('cuda', 0)
W = int(sys.argv[1]) if len(sys.argv) > 1 else 512
NPTS = int(sys.argv[2]) if len(sys.argv) > 2 else 300
NSUB = int(sys.argv[3]) if len(sys.argv) > 3 else 1
pars = torch.as_tensor(random_pars(W, complex_bs=True, seed=1), device=dev).contiguous()
x, w = phase_grid(NPTS)
X = torch.as_tensor(x, device=dev); Wd = torch.as_tensor(w, device=dev)
flux = torch.empty((W, len(x)), dtype=torch.float64, device=dev)
st = torch.empty(W, dtype=torch.int32, device=dev)
ws = torch.empty(L.lfg_workspace_size(W, 1), dtype=torch.uint8, device=dev)
vp = lambda t: ctypes.c_void_p(t.data_ptr())
L.lfg_debug_like_waves(None)
for _ in range(3):
    rc = L.lfg_flux(vp(pars), W, 18, vp(X), vp(Wd), len(x), NSUB, vp(flux), None, vp(st), vp(ws), ws.numel(),
                    _native.stream_ptr())
    assert rc == 0
torch.cuda.synchronize()
import time
t0 = time.perf_counter()
for _ in range(5):
    L.lfg_flux(vp(pars), W, 18, vp(X), vp(Wd), len(x), NSUB, vp(flux), None, vp(st), vp(ws), ws.numel(),
               _native.stream_ptr())
torch.cuda.synchronize()
print('W %d npts %d nsub %d: %.1f us per lfg_flux' % (W, NPTS, NSUB, (time.perf_counter() - t0) / 5 * 1e6))
g = ws[:W * 48 * 8].view(torch.float64).view(W, 48).cpu().numpy()
ok = st.cpu().numpy() == 0
names = ['staged', 'cells', 'sweepWD', 'sweepBD', 'scan', 'end']
prev = np.zeros(ok.sum())
for i, nm in enumerate(names):
    v = g[ok, 41 + i]
    print('%-8s cum mean %8.0f  max %8.0f   delta mean %8.0f' % (nm, v.mean(), v.max(), (v - prev).mean()))
    prev = v

t = g[:, 47] - g[:, 47].min()
print('block start (us, 100 MHz clock): %s' % np.percentile(t / 100.0, [0, 25, 50, 75, 90, 100]).round(2))
hw = g[:, 40].astype(np.int64)
cu = (hw >> 8) & 0xF
sh = (hw >> 12) & 1
se = (hw >> 13) & 0x7
key = se * 32 + sh * 16 + cu
print('distinct (se, sh, cu) slots in use: %d of %d blocks' % (len(np.unique(key)), len(key)))
cyc = np.zeros((8, 4096), dtype=np.uint64)
L.lfg_debug_like_cycles(ctypes.c_void_p(cyc.ctypes.data))
cyc = cyc[:, :W].astype(np.float64)[:, ok]
for k, nm in enumerate(['status known', 'wave sums (before barrier)', 'after the barrier']):
    print('prologue %-28s thread 0 mean %7.0f | last lane mean %7.0f' % (nm, cyc[k].mean(), cyc[4 + k].mean()))

wv = np.zeros((2, 6, 4096), dtype=np.uint64)
L.lfg_debug_like_waves(ctypes.c_void_p(wv.ctypes.data))
wv = wv[:, :, :W].astype(np.float64)[:, :, ok]
print('per-wave stamps (last launch overwrites max only; min is over all launches):')
for i, nm in enumerate(names):
    print('  %-8s first wave mean %8.0f   last wave mean %8.0f   spread %6.0f' % (nm, wv[0, i].mean(), wv[1, i].mean(), (wv[1, i] - wv[0, i]).mean()))
