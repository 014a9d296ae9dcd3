"""CV eclipse tree: Lightcurve, eclipse leaves, Band and LCModel nodes, and
construct_model() for the reference's mcmc_input.dat format.

Behavioural mirror of the reference's CVModel.py (Lightcurve :20-83,
SimpleEclipse :87-354, ComplexEclipse :357-390, Band :393-415,
LCModel :418-491, construct_model :713-924).  The leaves call this package's
GPU lfit.CV, so the tree can be driven one walker at a time exactly like the
reference; lfit_python_amd.batch compiles the same tree for batched GPU
evaluation of whole ensembles.

The Gaussian-process leaves (SimpleGPEclipse / ComplexGPEclipse,
CVModel.py:517-711) keep the reference's changepoint cache and kernel
construction; their likelihood runs on the GPU (lfit_python_amd.gp).
"""
import os

import numpy as np

from . import gp as georgelike
from . import lfit, roche
from .tree import Node, Param, extract_par_and_key

TINY = -np.inf


def read_config(path):
    """Minimal reader for the configobj `key = value` files the reference
    uses (CVModel.py:729): '#' starts a comment, values keep inner spaces."""
    out = {}
    with open(path, 'r', encoding='utf-8', errors='replace') as fh:
        for raw in fh:
            line = raw.split('#', 1)[0].strip()
            if not line or '=' not in line:
                continue
            key, val = line.split('=', 1)
            out[key.strip()] = val.strip()
    return out


class Lightcurve:
    """phase / flux / error arrays plus exposure half-widths (CVModel.py:20-83)."""

    def __init__(self, name, x, y, ye, w=None):
        self.name = name
        self.fname = None
        x = np.asarray(x, dtype=np.float64)
        if w is None:
            w = np.mean(np.diff(x)) * np.ones_like(x) / 2.
        self.x = x
        self.y = np.asarray(y, dtype=np.float64)
        self.ye = np.asarray(ye, dtype=np.float64)
        self.w = np.asarray(w, dtype=np.float64)

    @property
    def n_data(self):
        return self.x.shape[0]

    @classmethod
    def from_calib(cls, fname, name=None):
        data = None
        for delimiter in (' ', ',', '|'):
            try:
                data = np.loadtxt(fname, delimiter=delimiter, comments='#')
                break
            except ValueError:
                continue
        if data is None:
            data = np.loadtxt(fname, comments='#')
        phase, flux, error = data.T
        keep = ~np.isnan(flux)
        phase, flux, error = phase[keep], flux[keep], error[keep]
        width = np.mean(np.diff(phase)) * np.ones_like(phase) / 2.
        lc = cls(name if name is not None else os.path.split(fname)[1], phase, flux, error, width)
        lc.fname = fname
        return lc

    def trim(self, lo, hi):
        m = (self.x > lo) & (self.x < hi)
        self.x, self.y, self.ye, self.w = self.x[m], self.y[m], self.ye[m], self.w[m]


class SimpleEclipse(Node):
    """One eclipse with the simple (14-parameter) bright spot."""

    node_par_names = ('dFlux', 'sFlux', 'rdisc', 'scale', 'az', 'fis', 'dexp', 'phi0')
    cv_parnames = ['wdFlux', 'dFlux', 'sFlux', 'rsFlux', 'q', 'dphi', 'rdisc', 'ulimb',
                   'rwd', 'scale', 'az', 'fis', 'dexp', 'phi0']
    nsub = 1

    def __init__(self, lightcurve, *args, **kwargs):
        super().__init__(*args, **kwargs)
        if isinstance(lightcurve, Lightcurve):
            self.lc = lightcurve
        elif isinstance(lightcurve, str):
            self.lc = Lightcurve.from_calib(lightcurve)
        else:
            raise TypeError("Argument lightcurve is not a string or Lightcurve! Got {}".format(lightcurve))
        self._cv = None

    @property
    def cv(self):
        if self._cv is None:  # CVModel.py:128, built lazily so no GPU is needed to build trees
            self._cv = lfit.CV(self.cv_parlist, nsub=self.nsub)
        return self._cv

    @property
    def cv_parlist(self):
        d = self.ancestor_param_dict
        return [d[k].currVal for k in self.cv_parnames]

    def calcFlux(self):
        try:
            return self.cv.calcFlux(self.cv_parlist, self.lc.x, self.lc.w)
        except lfit.LfitError:
            return np.nan  # CVModel.py:139-144

    def calcComponents(self):
        flx = self.cv.calcFlux(self.cv_parlist, self.lc.x, self.lc.w)
        return flx, self.cv.ywd, self.cv.ys, self.cv.yrs, self.cv.yd

    def chisq(self):
        flx = self.calcFlux()
        if np.any(np.isnan(flx)):
            return np.inf
        return np.sum(((self.lc.y - flx) / self.lc.ye) ** 2)

    def ln_like(self):
        return -0.5 * self.chisq()

    def ln_prior(self, verbose=False, *args, **kwargs):
        """Roche validity checks of CVModel.py:193-324, then the Param priors."""
        d = self.ancestor_param_dict
        q = d['q'].currVal
        try:
            xl1 = roche.xl1(q)
        except roche.RocheError:
            return TINY
        rdisc_a = d['rdisc'].currVal * xl1
        if rdisc_a > 0.46:
            return TINY
        rwd, scale = d['rwd'].currVal, d['scale'].currVal
        if scale > rwd * 3. or scale < rwd / 3.:
            return TINY
        try:
            x, y, _, _ = roche.bspot(q, rdisc_a)
        except roche.RocheError:
            return TINY
        alpha = np.degrees(np.arctan2(y, x))
        if alpha < 0:
            alpha = 90 - alpha
        tangent = alpha + 90
        az = d['az'].currVal
        if az < max(0, tangent - 80.0) or az > min(178, tangent + 80.0):
            return TINY
        return super().ln_prior(verbose=verbose)


class ComplexEclipse(SimpleEclipse):
    """One eclipse with the complex (18-parameter) bright spot.  The tree
    stores yaw before tilt, lfit takes tilt before yaw (CVModel.py:376-388)."""

    node_par_names = ('dFlux', 'sFlux', 'rdisc', 'scale', 'az', 'fis', 'dexp', 'phi0',
                      'exp1', 'exp2', 'yaw', 'tilt')
    cv_parnames = SimpleEclipse.cv_parnames + ['exp1', 'exp2', 'tilt', 'yaw']


class Band(Node):
    node_par_names = ('wdFlux', 'rsFlux', 'ulimb')

    @property
    def eclipses(self):
        return list(self.search_node_type("Eclipse"))


class LCModel(Node):
    node_par_names = ('q', 'dphi', 'rwd')

    @property
    def eclipses(self):
        return list(self.search_node_type("Eclipse"))

    def ln_prior(self, verbose=False):
        """dphi must stay below findphi(q, 90) - 1e-6 (CVModel.py:440-491)."""
        try:
            maxphi = roche.findphi(self.q.currVal, 90.0)
        except roche.RocheError:
            return TINY
        if self.dphi.currVal > (maxphi - 1e-6):
            return TINY
        return 0.0 + super().ln_prior(verbose=verbose)


class GPLCModel(LCModel):
    node_par_names = LCModel.node_par_names + ('ln_ampin_gp', 'ln_ampout_gp', 'ln_tau_gp')


class SimpleGPEclipse(SimpleEclipse):
    """SimpleEclipse whose likelihood is a GP on its residuals (CVModel.py:517-696)."""

    # changepoint cache (CVModel.py:522-527): filled by the first evaluation
    _olddphi = 9e99
    _oldq = 9e99
    _oldrwd = 9e99
    _dist_cp = 9e99

    def calcChangepoints(self):
        """[[egress, ingress], ...] of the inter-eclipse blocks (CVModel.py:529-601)."""
        d = self.ancestor_param_dict
        dphi, q, rwd, phi0 = d['dphi'], d['q'], d['rwd'], d['phi0']
        dphi_change = np.fabs(self._olddphi - dphi.currVal) / dphi.currVal
        q_change = np.fabs(self._oldq - q.currVal) / q.currVal
        rwd_change = np.fabs(self._oldrwd - rwd.currVal) / rwd.currVal
        if (dphi_change > 1.2) or (q_change > 1.2) or (rwd_change > 1.2):
            inc = roche.findi(q.currVal, dphi.currVal)
            phi3, phi4 = roche.wdphases(q.currVal, inc, rwd.currVal, ntheta=10)
            dist_cp = (dphi.currVal + (phi4 - phi3)) / 2.
            self._dist_cp = dist_cp
            self._oldq = q.currVal
            self._olddphi = dphi.currVal
            self._oldrwd = rwd.currVal
        else:
            dist_cp = self._dist_cp
        min_ecl = int(np.floor(self.lc.x.min()))
        max_ecl = int(np.ceil(self.lc.x.max()))
        eclipses = [e for e in range(min_ecl, max_ecl + 1)
                    if np.logical_and(e > self.lc.x.min(), e < 1 + self.lc.x.max())]
        return [[(e - 1) + dist_cp + phi0.currVal, e - dist_cp + phi0.currVal] for e in eclipses]

    def create_GP(self):
        """george-style GP of CVModel.py:603-648 (lfit_python_amd.gp)."""
        d = self.ancestor_param_dict
        ampin_gp = np.exp(d['ln_ampin_gp'].currVal)
        ampout_gp = np.exp(d['ln_ampout_gp'].currVal)
        tau_gp = np.exp(d['ln_tau_gp'].currVal)
        changepoints = self.calcChangepoints()
        kernel = ampin_gp * georgelike.kernels.Matern32Kernel(tau_gp)
        for gap in changepoints:
            kernel += ampout_gp * georgelike.kernels.Matern32Kernel(tau_gp, block=gap)
        return georgelike.GP(kernel, solver=georgelike.HODLRSolver)

    def ln_like(self):
        residuals = self.lc.y - self.calcFlux()
        if np.any(np.isinf(residuals)) or np.any(np.isnan(residuals)):
            return -np.inf
        gp = self.create_GP()
        gp.compute(self.lc.x, self.lc.ye)
        return gp.log_likelihood(residuals, quiet=True)


class ComplexGPEclipse(SimpleGPEclipse):
    node_par_names = ComplexEclipse.node_par_names
    cv_parnames = ComplexEclipse.cv_parnames


def construct_model(input_file, debug=False, nodata=False, nsub=1):
    """mcmc_input.dat -> model tree (CVModel.py:713-924).  Bands and eclipses
    are discovered in file order; nsub selects exposure sub-binning."""
    cfg = read_config(input_file)
    base = os.path.dirname(os.path.abspath(input_file))
    for key in list(cfg):
        if key in ('ampin_gp', 'ampout_gp', 'tau_gp'):
            raise ValueError("use ln_{0}, not {0}".format(key))
    is_complex = bool(int(cfg['complex']))
    use_gp = bool(int(cfg['useGP']))
    neclipses = int(cfg['neclipses']) if 'neclipses' in cfg else 9999

    root_cls = GPLCModel if use_gp else LCModel
    model = root_cls('core', [Param.fromString(n, cfg[n]) for n in root_cls.node_par_names], DEBUG=debug)

    band_pars = Band.node_par_names
    if use_gp:
        leaf_cls = ComplexGPEclipse if is_complex else SimpleGPEclipse
    else:
        leaf_cls = ComplexEclipse if is_complex else SimpleEclipse
    ecl_pars = leaf_cls.node_par_names

    bands, eclipses = [], []
    with open(input_file, 'r', encoding='utf-8', errors='replace') as fh:
        for line in fh:
            tok = line.strip().split()
            if not tok:
                continue
            key = tok[0]
            if any(key.startswith(p) for p in band_pars):
                _, lab = extract_par_and_key(key)
                if lab not in bands:
                    bands.append(lab)
            if any(key.startswith(p) for p in ecl_pars):
                _, lab = extract_par_and_key(key)
                if lab not in eclipses:
                    eclipses.append(lab)

    for lab in bands:
        Band(lab, [Param.fromString(p, cfg["{}_{}".format(p, lab)]) for p in band_pars], parent=model)

    lo, hi = float(cfg['phi_start']), float(cfg['phi_end'])
    for lab in eclipses[:neclipses]:
        params = [Param.fromString(p, cfg["{}_{}".format(p, lab)]) for p in ecl_pars]
        if nodata:
            x = np.linspace(-0.5, 0.5, 1000)
            lc = Lightcurve("Dummy_Data_{}".format(lab), x, np.zeros_like(x), np.ones_like(x))
        else:
            fname = cfg['file_{}'.format(lab)]
            if not os.path.exists(fname):
                fname = os.path.join(base, fname)
            lc = Lightcurve.from_calib(fname)
            lc.trim(lo, hi)
        band = model.search_Node('Band', cfg['band_{}'.format(lab)])
        leaf = leaf_cls(lc, lab, params, parent=band)
        leaf.nsub = nsub
    model.children = [b for b in model.children if len(b.children)]
    return model
