"""trm.roche functions used on the reference's hot path, evaluated on the GPU.

    xl1(q)              CVModel.py:222, calcPhysicalParams.py:158
    findphi(q, inc)     CVModel.py:460, testCV.py:25
    findi(q, dphi)      CVModel.py:561, calcPhysicalParams.py:194
    bspot(q, rad)       CVModel.py:288  -> (x, y, vx, vy)
    wdphases(q, inc, r1, ntheta=10)  CVModel.py:564 -> (phi3, phi4)

Geometry follows MODEL_SPEC.md section 4 (separation a = 1, WD at the
origin, donor centre at (1, 0, 0)).  Scalars in, scalars out, like trm.roche;
failures raise RocheError (the reference catches them, CVModel.py:223,309,475).
Array inputs are evaluated in one batched launch.
"""
import ctypes

import numpy as np

from . import _native


class RocheError(ValueError):
    pass


def _run(op, a, b=None):
    import torch
    _native.require_gpu()
    L = _native.lib()
    a_np = np.atleast_1d(np.asarray(a, dtype=np.float64))
    b_np = np.array(np.broadcast_to(np.asarray(b if b is not None else 0.0, dtype=np.float64), a_np.shape))
    dev = torch.device("cuda", torch.cuda.current_device())
    a_t = torch.as_tensor(np.ascontiguousarray(a_np.reshape(-1)), device=dev)
    b_t = torch.as_tensor(np.ascontiguousarray(b_np.reshape(-1)), device=dev)
    n = a_t.shape[0]
    out = torch.empty(n * (4 if op == 3 else 1), dtype=torch.float64, device=dev)
    st = torch.empty(n, dtype=torch.int32, device=dev)
    rc = L.lfg_roche(op, ctypes.c_void_p(a_t.data_ptr()), ctypes.c_void_p(b_t.data_ptr()), n,
                     ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(st.data_ptr()),
                     _native.stream_ptr(dev))
    _native.check(rc, "lfg_roche")
    return out.cpu().numpy(), st.cpu().numpy(), np.ndim(a) == 0 and np.ndim(b) == 0


def _finish(vals, st, scalar, what):
    if scalar:
        if st[0] != 0:
            raise RocheError("%s failed: %s" % (what, _native.STATUS_TEXT.get(int(st[0]), st[0])))
        return float(vals[0])
    return vals


def xl1(q):
    v, st, sc = _run(0, q)
    return _finish(v, st, sc, "xl1")


def findphi(q, inc):
    v, st, sc = _run(1, q, inc)
    return _finish(v, st, sc, "findphi")


def findi(q, dphi):
    v, st, sc = _run(2, q, dphi)
    return _finish(v, st, sc, "findi")


def bspot(q, rad):
    v, st, sc = _run(3, q, rad)
    v = v.reshape(-1, 4)
    if sc:
        if st[0] != 0:
            raise RocheError("bspot failed: the stream does not reach r = %g" % float(rad))
        return tuple(float(t) for t in v[0])
    return v


def wdphases(q, inc, r1, ntheta=10):
    """Third and fourth contact phases of a sphere of radius r1 (units of the
    separation) at the white dwarf (trm.roche.wdphases; MODEL_SPEC 10.2)."""
    import torch
    _native.require_gpu()
    L = _native.lib()
    q_np = np.atleast_1d(np.asarray(q, dtype=np.float64))
    shape = np.broadcast(q_np, np.asarray(inc), np.asarray(r1)).shape
    dev = torch.device("cuda", torch.cuda.current_device())
    t = lambda a: torch.as_tensor(np.array(np.broadcast_to(np.asarray(a, dtype=np.float64), shape)).reshape(-1),
                                  device=dev)
    qt, it, rt = t(q), t(inc), t(r1)
    n = qt.shape[0]
    p3 = torch.empty(n, dtype=torch.float64, device=dev)
    p4 = torch.empty_like(p3)
    st = torch.empty(n, dtype=torch.int32, device=dev)
    vp = lambda a: ctypes.c_void_p(a.data_ptr())
    _native.check(L.lfg_wdphases(vp(qt), vp(it), vp(rt), n, int(ntheta), vp(p3), vp(p4), vp(st),
                                 _native.stream_ptr(dev)), "lfg_wdphases")
    p3, p4, st = p3.cpu().numpy(), p4.cpu().numpy(), st.cpu().numpy()
    if np.ndim(q) == 0 and np.ndim(inc) == 0 and np.ndim(r1) == 0:
        if st[0] != 0:
            raise RocheError("wdphases failed: %s" % _native.STATUS_TEXT.get(int(st[0]), st[0]))
        return float(p3[0]), float(p4[0])
    return p3, p4
