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
