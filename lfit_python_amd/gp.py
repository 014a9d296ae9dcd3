"""The Gaussian-process likelihood of the reference's GP trees, on the GPU.

Replaces the george objects SimpleGPEclipse builds (CVModel.py:603-696):
  kernel = ampin * kernels.Matern32Kernel(tau)                 CVModel.py:636
  kernel += ampout * kernels.Matern32Kernel(tau, block=gap)    CVModel.py:639-642
  gp = GP(kernel, solver=HODLRSolver)                          CVModel.py:645
  gp.compute(x, ye); gp.log_likelihood(residuals, quiet=True)  CVModel.py:687-691
with the same call shapes.  The likelihood is exact (george's HODLR solver
approximates it) and costs O(N): lfg_gp_lnlike runs a 4-state Kalman filter
over the phase-sorted points (MODEL_SPEC.md section 10).  Only the kernel
family the reference builds is supported: one global Matern-3/2 term plus
Matern-3/2 terms of one common amplitude restricted to blocks, all with the
same metric.
"""
import ctypes

import numpy as np

from . import _native


class _Kernel:
    """A sum of amp * Matern32(metric) terms, each optionally on a block."""

    def __init__(self, terms):
        self.terms = list(terms)

    def __rmul__(self, a):
        return _Kernel([(float(a) * amp, metric, blk) for amp, metric, blk in self.terms])

    __mul__ = __rmul__

    def __add__(self, other):
        return _Kernel(self.terms + other.terms)


class kernels:  # noqa: N801 - mirrors george.kernels
    @staticmethod
    def Matern32Kernel(metric, block=None):  # noqa: N802 - george's name
        """george: k(r^2) = (1 + sqrt(3 r^2)) exp(-sqrt(3 r^2)), r^2 = d^2 / metric;
        with block = (lo, hi), zero unless both points lie in [lo, hi]."""
        blk = None if block is None else tuple(float(v) for v in np.atleast_2d(block)[0])
        return _Kernel([(1.0, float(metric), blk)])


HODLRSolver = None  # accepted and ignored: the solve is exact


def _split(kernel):
    glob = [t for t in kernel.terms if t[2] is None]
    blk = [t for t in kernel.terms if t[2] is not None]
    metrics = {t[1] for t in kernel.terms}
    if len(glob) != 1 or len(metrics) != 1 or len({t[0] for t in blk}) > 1:
        raise NotImplementedError("only ampin*M32(tau) + sum_k ampout*M32(tau, block_k) is supported")
    ampout = blk[0][0] if blk else 0.0
    return glob[0][0], ampout, metrics.pop(), [t[2] for t in blk]


def log_likelihood_batch(x, ye, res, hyp, blocks, device=None):
    """GP log-likelihoods of W residual vectors on the GPU.

    x, ye [N] (any order); res [W, N]; hyp [W, 3] = ampin, ampout, tau;
    blocks [W, nb, 2].  Returns a numpy array [W]."""
    import torch
    _native.require_gpu()
    L = _native.lib()
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    x = np.asarray(x, dtype=np.float64).reshape(-1)
    order = np.argsort(x, kind="stable")  # the filter runs over sorted phases
    res = np.atleast_2d(np.asarray(res, dtype=np.float64))[:, order]
    W, N = res.shape
    hyp = np.ascontiguousarray(np.asarray(hyp, dtype=np.float64).reshape(W, 3))
    blocks = np.asarray(blocks, dtype=np.float64).reshape(W, -1, 2)
    nb = blocks.shape[1]
    t = lambda a: torch.as_tensor(np.ascontiguousarray(a), dtype=torch.float64, device=dev)
    xt, yt, rt, ht = t(x[order]), t(np.asarray(ye, dtype=np.float64).reshape(-1)[order]), t(res), t(hyp)
    bt = t(blocks if nb else np.zeros((W, 1, 2)))
    out = torch.empty(W, dtype=torch.float64, device=dev)
    vp = lambda a: ctypes.c_void_p(a.data_ptr())
    rc = L.lfg_gp_lnlike(vp(xt), vp(yt), vp(rt), W, N, vp(ht), vp(bt), nb, vp(out), _native.stream_ptr(dev))
    _native.check(rc, "lfg_gp_lnlike")
    return out.cpu().numpy()


class GP:
    """george.GP for the kernel of CVModel.py:636-645."""

    def __init__(self, kernel, solver=None, device=None):
        self.kernel = kernel
        self.ampin, self.ampout, self.tau, self.blocks = _split(kernel)
        self.device = device
        self.x = self.ye = None

    def compute(self, x, yerr):
        self.x = np.asarray(x, dtype=np.float64)
        self.ye = np.broadcast_to(np.asarray(yerr, dtype=np.float64), self.x.shape)

    def log_likelihood(self, y, quiet=False):
        if self.x is None:
            raise RuntimeError("call compute(x, yerr) first")
        blocks = np.asarray(self.blocks, dtype=np.float64).reshape(1, -1, 2)
        ll = float(log_likelihood_batch(self.x, self.ye, np.asarray(y)[None, :],
                                        [[self.ampin, self.ampout, self.tau]], blocks, self.device)[0])
        if not np.isfinite(ll) and not quiet:
            raise ValueError("the GP covariance is not positive definite")
        return ll
