"""Quick device timing of the lnprob pipeline (development aid)."""
import sys, time, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from tests.helpers import TRUTH18, random_pars, phase_grid
from lfit_python_amd.lfit import flux_batch
from lfit_python_amd.tree import Param, Prior
from lfit_python_amd import batch, cvmodel

def single_eclipse_tree(n=300, seed=1):
    names = cvmodel.ComplexEclipse.cv_parnames
    x, w = phase_grid(n)
    f, st = flux_batch(np.array([TRUTH18]), x, w)
    rng = np.random.default_rng(seed)
    y = f.cpu().numpy()[0] + rng.normal(0, 0.004, n)
    lc = cvmodel.Lightcurve("syn", x, y, 0.004 * np.ones(n), w)
    d = dict(zip(names, TRUTH18))
    P = lambda k, lo, hi: Param(k, d[k], Prior('uniform', lo, hi))
    core = cvmodel.LCModel('core', [P('q', 0.03, 0.5), P('dphi', 0.01, 0.1), P('rwd', 0.001, 0.1)])
    band = cvmodel.Band('g', [P('wdFlux', 0.001, 0.2), P('rsFlux', 0.001, 0.2), P('ulimb', 0.0, 1.0)], parent=core)
    ep = [P('dFlux', 0.001, 0.2), P('sFlux', 0.001, 0.2), P('rdisc', 0.2, 0.7), P('scale', 0.001, 0.2),
          P('az', 50, 175), P('fis', 0.001, 1), P('dexp', 0.001, 2), P('phi0', -0.2, 0.2),
          P('exp1', 0.001, 5), P('exp2', 0.5, 5), P('yaw', -90, 90), P('tilt', 0.001, 180)]
    cvmodel.ComplexEclipse(lc, '0', ep, parent=band)
    return core

core = single_eclipse_tree()
tree = batch.compile_tree(core)
ev = batch.LnProbEvaluator(tree)
p0 = np.array(core.dynasty_par_vals)
for W in [512, 1024, 4096]:
    rng = np.random.default_rng(0)
    walk = p0 * (1 + 1e-3 * rng.standard_normal((W, len(p0))))
    wt = torch.as_tensor(walk, device='cuda')
    out = ev(wt); torch.cuda.synchronize()
    t = time.time(); R = 5
    for _ in range(R): ev(wt)
    torch.cuda.synchronize(); dt = (time.time() - t) / R
    lnp = out.cpu().numpy()
    print(f"W={W}: {dt*1e3:.2f} ms/batch  {W/dt:.3e} evals/s  finite={np.isfinite(lnp).mean():.3f} lnp[0]={lnp[0]:.6f}", flush=True)
