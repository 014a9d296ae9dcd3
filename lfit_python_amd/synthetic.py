"""Synthetic workloads of BASELINE.json's configs.

Parameter values and priors are those of the reference's example input,
test_data/mcmc_input.dat (core :47-49, bands :52-62, eclipses :73-172),
restated here as data so the GPU box (which has no /root/reference) can build
the same trees.  Light curves are synthetic: y = model flux at the truth plus
seeded Gaussian noise of 0.004 (the example data's mean error is 0.0035-0.0067).
"""
import numpy as np

from .cvmodel import Band, ComplexEclipse, LCModel, Lightcurve, SimpleEclipse
from .tree import Param

SEED = 20261015
NOISE = 0.004

CORE = {  # mcmc_input.dat:47-49
    'q': '0.1037 uniform 0.0300 0.5000 1',
    'dphi': '0.0392 uniform 0.0100 0.1000 1',
    'rwd': '0.0187 uniform 0.0010 0.1000 1',
}
BANDS = {  # mcmc_input.dat:52-62
    'g': {'wdFlux': '0.0528 uniform 0.0010 0.2000 1', 'rsFlux': '0.0131 uniform 0.0010 0.2000 1',
          'ulimb': '0.284 gauss 0.284 0.001 1'},
    'KG5': {'wdFlux': '0.0508 uniform 0.0010 0.2000 1', 'rsFlux': '0.0262 uniform 0.0010 0.2000 1',
            'ulimb': '0.284 gauss 0.284 0.001 1'},
    'r': {'wdFlux': '0.0324 uniform 0.0010 0.2000 1', 'rsFlux': '0.0262 uniform 0.0010 0.2000 1',
          'ulimb': '0.284 gauss 0.284 0.001 1'},
}
_EPRI = {'dFlux': 'uniform 0.0010 0.2000', 'sFlux': 'uniform 0.0010 0.2000',
         'rdisc': 'uniform 0.2000 0.7000', 'scale': 'log_uniform 0.0010 0.2000',
         'az': 'uniform 50.0000 175.0000', 'fis': 'uniform 0.0010 1.0000',
         'dexp': 'log_uniform 0.0010 2.0000', 'phi0': 'uniform -0.2000 0.2000',
         'exp1': 'uniform 0.0010 5.0000', 'exp2': 'uniform 0.5000 5.0000',
         'yaw': 'uniform -90.0000 90.0000', 'tilt': 'uniform 0.0010 180.0000'}
_ENAMES = ('dFlux', 'sFlux', 'rdisc', 'scale', 'az', 'fis', 'dexp', 'phi0', 'exp1', 'exp2', 'yaw', 'tilt')
_EVALS = {  # mcmc_input.dat:73-172 (band, values in the order of _ENAMES)
    '0': ('g', (0.0707, 0.0613, 0.2953, 0.0430, 120.0000, 0.0480, 0.5000, 0.0010, 1.1342, 4.5971, 5.4000, 72.0006)),
    '1': ('g', (0.1238, 0.1518, 0.5214, 0.0497, 122.0724, 0.1684, 1.9539, -0.0013, 3.4876, 1.4429, 15.6635, 52.4720)),
    '2': ('KG5', (0.0496, 0.0631, 0.5487, 0.0410, 125.1563, 0.0467, 0.7073, -0.0004, 2.7938, 1.2241, -1.3957, 49.0896)),
    '3': ('KG5', (0.0938, 0.0618, 0.4212, 0.0430, 125.1298, 0.1099, 1.0794, -0.0002, 0.2859, 0.9702, -2.4394, 52.2358)),
    '4': ('r', (0.1267, 0.1084, 0.5954, 0.0487, 99.1185, 0.0317, 1.4333, 0.0004, 2.9879, 1.2802, 22.7125, 138.7462)),
    '5': ('r', (0.0845, 0.0697, 0.5702, 0.0191, 120.9071, 0.0506, 1.7123, -0.0010, 3.0050, 1.3828, 8.6757, 111.5294)),
}


def eclipse_param_strings(label, values=None, complex_bs=True):
    band, vals = _EVALS[label]
    vals = values if values is not None else vals
    names = _ENAMES if complex_bs else _ENAMES[:8]
    d = dict(zip(_ENAMES, vals))
    return band, {n: '%r %s 1' % (float(d[n]), _EPRI[n]) for n in names}


def phase_grid(npts, lo=-0.3, hi=0.3):
    x = np.linspace(lo, hi, npts)
    return x, np.mean(np.diff(x)) * np.ones_like(x) / 2.0


def build_tree(eclipses, npts=300, complex_bs=True, flux_fn=None, seed=SEED, nsub=1):
    """LCModel -> Band -> eclipse tree.  `eclipses` is a list of
    (label, band, {param: 'value prior p1 p2 1'}) leaves.  flux_fn(cv_pars,
    x, w, nsub) -> model flux gives the noiseless synthetic light curve
    (GPU lfit.CV on the box, the oracle in CPU tests)."""
    rng = np.random.default_rng(seed)
    core = LCModel('core', [Param.fromString(k, CORE[k]) for k in LCModel.node_par_names])
    bands = {}
    leaf_cls = ComplexEclipse if complex_bs else SimpleEclipse
    for label, band, pstr in eclipses:
        if band not in bands:
            bands[band] = Band(band, [Param.fromString(k, BANDS[band][k]) for k in Band.node_par_names],
                               parent=core)
        x, w = phase_grid(npts)
        lc = Lightcurve('synthetic_%s' % label, x, np.zeros_like(x), NOISE * np.ones_like(x), w)
        leaf = leaf_cls(lc, label, [Param.fromString(k, pstr[k]) for k in leaf_cls.node_par_names],
                        parent=bands[band])
        leaf.nsub = nsub
    if flux_fn is not None:
        for leaf in core.leaves():
            f = flux_fn(leaf.cv_parlist, leaf.lc.x, leaf.lc.w, nsub)
            leaf.lc.y = f + NOISE * rng.standard_normal(f.shape)
    return core


def config_single(npts=300, complex_bs=True, flux_fn=None, nsub=1, label='0'):
    """Configs 1, 2, 4, 5: one eclipse (band g / eclipse 0 of the example)."""
    band, p = eclipse_param_strings(label, complex_bs=complex_bs)
    return build_tree([(label, band, p)], npts, complex_bs, flux_fn, nsub=nsub)


def config_tree(nper=4, npts=300, flux_fn=None, seed=SEED, nsub=1):
    """Config 3: 3 bands x `nper` eclipses (shared q/dphi/rwd); the two example
    eclipses of each band are reused, jittered by 2 % for the extra copies."""
    rng = np.random.default_rng(seed + 1)
    leaves = []
    by_band = {}
    for lab, (band, vals) in _EVALS.items():
        by_band.setdefault(band, []).append(vals)
    n = 0
    for band in ('g', 'KG5', 'r'):
        for k in range(nper):
            vals = np.array(by_band[band][k % len(by_band[band])], dtype=np.float64)
            if k >= len(by_band[band]):
                vals = vals * (1.0 + 0.02 * rng.standard_normal(vals.shape))
            _, p = eclipse_param_strings('0', values=vals)
            leaves.append((str(n), band, p))
            n += 1
    return build_tree(leaves, npts, True, flux_fn, seed=seed, nsub=nsub)
