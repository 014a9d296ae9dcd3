"""Drop-in for the `lfit` module's CV object, backed by the gfx950 kernels.

Mirrors the API the reference uses:
  cv = lfit.CV(pars)                         CVModel.py:128; README.md:45
  flux = cv.calcFlux(pars, phase, width)     CVModel.py:138,154; README.md:63
  flux = cv(pars, phase)                     README.md:48
  cv.ywd, cv.yd, cv.ys, cv.yrs               CVModel.py:155; plot_lc_model.py:135-138
pars are the 14 (simple bright spot) or 18 (complex) CV parameters in lfit's
order (README.md:24-43).  Like lfit, an invalid parameter set raises; the
reference turns that into NaN flux (CVModel.py:137-144).

calcFlux on one parameter set is the scalar convenience path; the batched
entry point `flux_batch` evaluates whole walker ensembles in one launch.
"""
import ctypes

import numpy as np

from . import _native

PARNAMES = ['wdFlux', 'dFlux', 'sFlux', 'rsFlux', 'q', 'dphi', 'rdisc', 'ulimb',
            'rwd', 'scale', 'az', 'fis', 'dexp', 'phi0', 'exp1', 'exp2', 'tilt',
            'yaw']


class LfitError(ValueError):
    """Raised for a parameter set the model cannot evaluate (lfit raises too)."""


def _default_width(x):
    # CVModel.py:29-30 and :64 -- lfit infers the exposure from the data
    if x.shape[0] < 2:
        return np.zeros_like(x)
    return np.mean(np.diff(x)) * np.ones_like(x) / 2.0


def flux_batch(pars, x, width=None, nsub=1, components=False, device=None):
    """Batched lfit.CV.calcFlux.

    pars: [W, P] (P = 14 or 18) array or tensor; x, width: [N] shared phases
    and exposure half-widths.  Returns torch tensors on the device:
    flux [W, N], status [W] int32 and, if components, comps [4, W, N]
    (white dwarf, disc, bright spot, donor).
    """
    import torch
    _native.require_gpu()
    L = _native.lib()
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    P_t = torch.as_tensor(pars, dtype=torch.float64, device=dev)
    if P_t.ndim == 1:
        P_t = P_t[None, :]
    P_t = P_t.contiguous()
    W, P = P_t.shape
    if P not in (14, 18):
        raise ValueError("lfit.CV takes 14 or 18 parameters, got %d" % P)
    x_np = np.ascontiguousarray(np.asarray(x, dtype=np.float64).reshape(-1))
    if width is None:
        width = _default_width(x_np)
    w_np = np.array(np.broadcast_to(np.asarray(width, dtype=np.float64), x_np.shape))
    x_t = torch.as_tensor(x_np, device=dev)
    w_t = torch.as_tensor(np.ascontiguousarray(w_np), device=dev)
    N = x_t.shape[0]
    flux = torch.empty((W, N), dtype=torch.float64, device=dev)
    comps = torch.empty((4, W, N), dtype=torch.float64, device=dev) if components else None
    status = torch.empty(W, dtype=torch.int32, device=dev)
    nbytes = L.lfg_workspace_size(W, 1)
    ws = _native.Workspace.get(nbytes, dev)
    with torch.cuda.device(dev):
        rc = L.lfg_flux(ctypes.c_void_p(P_t.data_ptr()), W, P,
                        ctypes.c_void_p(x_t.data_ptr()), ctypes.c_void_p(w_t.data_ptr()),
                        N, int(nsub), ctypes.c_void_p(flux.data_ptr()),
                        ctypes.c_void_p(comps.data_ptr()) if comps is not None else None,
                        ctypes.c_void_p(status.data_ptr()),
                        ctypes.c_void_p(ws.data_ptr()), ws.numel(), _native.stream_ptr(dev))
    _native.check(rc, "lfg_flux")
    if components:
        return flux, status, comps
    return flux, status


class CV:
    """lfit.CV replacement (one parameter set per call, lfit semantics)."""

    def __init__(self, pars, nsub=1, device=None):
        pars = [float(p) for p in pars]
        if len(pars) not in (14, 18):
            raise LfitError("lfit.CV takes 14 or 18 parameters, got %d" % len(pars))
        self.pars = pars
        self.complex = len(pars) == 18
        self.nsub = int(nsub)
        self.device = device
        self.ywd = self.yd = self.ys = self.yrs = None

    def calcFlux(self, pars, x, width=None):
        pars = [float(p) for p in pars]
        x = np.asarray(x, dtype=np.float64)
        flux, status, comps = flux_batch(np.asarray(pars)[None, :], x, width,
                                         nsub=self.nsub, components=True,
                                         device=self.device)
        st = int(status[0].item())
        if st != 0:
            self.ywd = self.yd = self.ys = self.yrs = None
            raise LfitError("lfit model failed: %s; pars=%r" % (_native.STATUS_TEXT.get(st, st), pars))
        c = comps[:, 0, :].cpu().numpy()
        self.pars = pars
        self.ywd, self.yd, self.ys, self.yrs = c[0], c[1], c[2], c[3]
        return flux[0].cpu().numpy()

    __call__ = calcFlux


# ---------------------------------------------------------------------------
# lfit's component objects (testCV.py:27-49, fitEcl.py:21-24): one
# component each, unit-normalised ("flux at maximum light" = 1), computed at
# a given inclination (CV takes dphi instead and calls findi).  The total of
# lfit.CV is wdFlux*ywd + dFlux*yd + sFlux*ys + rsFlux*yrs of these at
# inc = roche.findi(q, dphi) and phase x - phi0 (testCV.py:65; MODEL_SPEC 5.6).


def lnlike_batch(pars, x, y, ye, width=None, nsub=1, device=None):
    """Batched SimpleEclipse.ln_like (CVModel.py:157-191) of one light curve,
    through lfg_lnlike: -0.5 chi^2 of W parameter sets, fused (no flux array),
    -inf where the model is invalid (chi^2 = inf, CVModel.py:163-171).
    Returns torch tensors on the device: ln_like [W], status [W] int32."""
    import torch
    _native.require_gpu()
    L = _native.lib()
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    P_t = torch.as_tensor(pars, dtype=torch.float64, device=dev)
    if P_t.ndim == 1:
        P_t = P_t[None, :]
    P_t = P_t.contiguous()
    W, P = P_t.shape
    if P not in (14, 18):
        raise ValueError("lfit.CV takes 14 or 18 parameters, got %d" % P)
    x_np = np.ascontiguousarray(np.asarray(x, dtype=np.float64).reshape(-1))
    if width is None:
        width = _default_width(x_np)
    w_np = np.array(np.broadcast_to(np.asarray(width, dtype=np.float64), x_np.shape))
    t = {k: torch.as_tensor(np.ascontiguousarray(v, dtype=np.float64).reshape(-1), device=dev)
         for k, v in (("x", x_np), ("w", w_np), ("y", y), ("ye", ye))}
    N = t["x"].shape[0]
    if t["y"].shape[0] != N or t["ye"].shape[0] != N:
        raise ValueError("x, y and ye must have the same length")
    out = torch.empty(W, dtype=torch.float64, device=dev)
    status = torch.empty(W, dtype=torch.int32, device=dev)
    ws = _native.Workspace.get(L.lfg_workspace_size(W, 1), dev)
    vp = lambda a: ctypes.c_void_p(a.data_ptr())
    with torch.cuda.device(dev):
        rc = L.lfg_lnlike(vp(P_t), W, P, vp(t["x"]), vp(t["w"]), N, int(nsub), vp(t["y"]), vp(t["ye"]), vp(out),
                          vp(status), vp(ws), ws.numel(), _native.stream_ptr(dev))
    _native.check(rc, "lfg_lnlike")
    return out, status

def disc_grid(npts):
    """PyDisc's npts -> (rings, azimuths): 1000 -> 20 x 50 (MODEL_SPEC 5.2,
    5.6); other sizes keep the 2.5 azimuths-per-ring aspect, so the element
    count is rings x azimuths ~ npts."""
    npts = int(npts)
    if npts < 1:
        raise LfitError("PyDisc needs npts >= 1, got %d" % npts)
    nr = max(1, int(round(np.sqrt(npts / 2.5))))
    return nr, max(1, int(round(npts / nr)))


def donor_grid(npts):
    """PyDonor's npts -> (bands, azimuths): 400 -> 20 x 20 (MODEL_SPEC 5.4, 5.6)."""
    npts = int(npts)
    if npts < 1:
        raise LfitError("PyDonor needs npts >= 1, got %d" % npts)
    nt = max(1, int(round(np.sqrt(npts))))
    return nt, max(1, int(round(npts / nt)))


def component_batch(kind, cpars, q, inc, x, width=None, n1=0, n2=0, device=None):
    """Batched component flux (lfg_component, include/lfg.h): kind 0 WD,
    1 disc, 2 bright spot, 3 donor; cpars [W, ncp]; q, inc [W] (degrees);
    x, width [N].  Returns torch tensors (out [W, N], status [W])."""
    import torch
    _native.require_gpu()
    L = _native.lib()
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    q_t = torch.as_tensor(np.atleast_1d(np.asarray(q, dtype=np.float64)), device=dev).contiguous()
    W = q_t.shape[0]
    inc_t = torch.as_tensor(np.broadcast_to(np.asarray(inc, dtype=np.float64), (W,)).copy(), device=dev)
    ncp = {0: 2, 1: 3, 2: 8, 3: 0}[kind]
    if ncp:
        cp_t = torch.as_tensor(np.asarray(cpars, dtype=np.float64).reshape(W, ncp), device=dev).contiguous()
    else:
        cp_t = None
    x_np = np.ascontiguousarray(np.asarray(x, dtype=np.float64).reshape(-1))
    if width is None:
        width = _default_width(x_np)
    w_np = np.array(np.broadcast_to(np.asarray(width, dtype=np.float64), x_np.shape))
    x_t, w_t = torch.as_tensor(x_np, device=dev), torch.as_tensor(w_np, device=dev)
    N = x_t.shape[0]
    out = torch.empty((W, N), dtype=torch.float64, device=dev)
    status = torch.empty(W, dtype=torch.int32, device=dev)
    ws = _native.Workspace.get(L.lfg_component_workspace_size(kind, W, int(n1), int(n2)), dev)
    vp = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None  # noqa: E731
    with torch.cuda.device(dev):
        rc = L.lfg_component(kind, vp(cp_t), ncp, vp(q_t), vp(inc_t), W, int(n1), int(n2), vp(x_t), vp(w_t), N,
                             vp(out), vp(status), vp(ws), ws.numel(), _native.stream_ptr(dev))
    _native.check(rc, "lfg_component")
    return out, status


class _Component:
    kind = -1
    n1 = n2 = 0

    def _cpars(self):
        return []

    def calcFlux(self, q, inc, phi, width=None):
        """Unit-normalised flux of this component at mass ratio q and
        inclination inc (degrees), phases phi (used as given) and exposure
        half-widths width (default mean(diff(phi))/2).  The q given here is
        the one used (lfit's components take it again at every call)."""
        out, st = component_batch(self.kind, np.asarray(self._cpars(), dtype=np.float64)[None, :], [q], [inc],
                                  phi, width, self.n1, self.n2)
        s = int(st[0].item())
        if s != 0:
            raise LfitError("lfit component failed: %s" % _native.STATUS_TEXT.get(s, s))
        return out[0].cpu().numpy()

    __call__ = calcFlux


class PyWhiteDwarf(_Component):
    """lfit.PyWhiteDwarf(rwd, ulimb): rwd in units of xl1 (testCV.py:27
    passes rwd/xl1), linear limb darkening ulimb; 400 tiles (MODEL_SPEC 5.1)."""
    kind = 0

    def __init__(self, rwd, ulimb):
        self.rwd, self.ulimb = float(rwd), float(ulimb)

    def _cpars(self):
        return [self.rwd, self.ulimb]


class PyDisc(_Component):
    """lfit.PyDisc(q, rwd, rdisc, dexp, npts=1000): radii in units of xl1
    (testCV.py:31), r^-dexp surface brightness, npts elements (disc_grid)."""
    kind = 1

    def __init__(self, q, rwd, rdisc, dexp, npts=1000):
        self.q, self.rwd, self.rdisc, self.dexp = float(q), float(rwd), float(rdisc), float(dexp)
        self.n1, self.n2 = disc_grid(npts)
        self.npts = self.n1 * self.n2

    def _cpars(self):
        return [self.rwd, self.rdisc, self.dexp]


class PySpot(_Component):
    """lfit.PySpot(q, rdisc, az, fis, scale, exp1, exp2, tilt, yaw, complex)
    (testCV.py:36-40): rdisc and scale in units of xl1, angles in degrees;
    complex=False is the simple spot (exp1 2, exp2 1, tilt 90, yaw 0;
    MODEL_SPEC 5.3); 100 strip elements."""
    kind = 2

    def __init__(self, q, rdisc, az, fis, scale, exp1=2.0, exp2=1.0, tilt=90.0, yaw=0.0, complex=False, npts=100):
        self.q, self.rdisc, self.az, self.fis, self.scale = (float(v) for v in (q, rdisc, az, fis, scale))
        self.complex = bool(complex)
        if self.complex:
            self.exp1, self.exp2, self.tilt, self.yaw = (float(v) for v in (exp1, exp2, tilt, yaw))
        else:
            self.exp1, self.exp2, self.tilt, self.yaw = 2.0, 1.0, 90.0, 0.0
        self.n1 = int(npts)
        if self.n1 < 1:
            raise LfitError("PySpot needs npts >= 1")

    def _cpars(self):
        return [self.rdisc, self.az, self.fis, self.scale, self.exp1, self.exp2, self.tilt, self.yaw]


class PyDonor(_Component):
    """lfit.PyDonor(q, npts=400) (testCV.py:43): the Roche-lobe-filling
    donor, npts tiles (donor_grid), normalised to quadrature."""
    kind = 3

    def __init__(self, q, npts=400):
        self.q = float(q)
        self.n1, self.n2 = donor_grid(npts)
        self.npts = self.n1 * self.n2
