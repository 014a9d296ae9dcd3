"""ctypes wrapper around oracle/liblfg_oracle.so.

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, never by the lfit_python_amd product path.
Parity of the flux arithmetic against the real lfit package is UNPINNED
(SURVEY.md section 8c); this oracle restates MODEL_SPEC.md.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liblfg_oracle.so")

NWD, NDISC, NBS, NDONOR = 400, 1000, 100, 400
NEL = NWD + NDISC + NBS

_dp = ctypes.POINTER(ctypes.c_double)
_ip = ctypes.POINTER(ctypes.c_int)


def build(march="x86-64-v2", out=None):
    """Compile the oracle with gcc.  Returns the path of the shared object."""
    out = out or LIB_PATH
    src = os.path.join(HERE, "lfg_oracle.c")
    cmd = ["gcc", "-O3", "-march=%s" % march, "-fopenmp", "-fPIC", "-std=c11",
           "-shared", "-o", out, src, "-lm"]
    subprocess.run(cmd, check=True)
    return out


def _f(a):
    a = np.ascontiguousarray(a, dtype=np.float64)
    return a, a.ctypes.data_as(_dp)


def _i(a):
    a = np.ascontiguousarray(a, dtype=np.int32)
    return a, a.ctypes.data_as(_ip)


class Oracle:
    def __init__(self, path=None):
        path = path or LIB_PATH
        if not os.path.exists(path):
            build(out=path)
        lib = ctypes.CDLL(path)
        lib.lfo_xl1.restype = ctypes.c_double
        lib.lfo_xl1.argtypes = [ctypes.c_double]
        lib.lfo_findphi.argtypes = [ctypes.c_double, ctypes.c_double, _dp]
        lib.lfo_findi.argtypes = [ctypes.c_double, ctypes.c_double, _dp]
        lib.lfo_bspot.argtypes = [ctypes.c_double, ctypes.c_double, _dp]
        lib.lfo_flux.argtypes = [_dp, ctypes.c_int, _dp, _dp, ctypes.c_int,
                                 ctypes.c_int, _dp, _dp, _dp, _dp, _dp]
        lib.lfo_elements.argtypes = [_dp, ctypes.c_int, _dp, _dp, _dp, _dp, _dp]
        lib.lfo_prior_lnprob.restype = ctypes.c_double
        lib.lfo_prior_lnprob.argtypes = [ctypes.c_int] + [ctypes.c_double] * 4
        lib.lfo_lnprob_batch.argtypes = [
            _dp, ctypes.c_int, ctypes.c_int, ctypes.c_int, _ip, _ip, _dp,
            _ip, _dp, _dp, _dp, _dp, ctypes.c_int, _ip, _dp, _dp, _dp,
            _dp, _dp, ctypes.c_int]
        lib.lfo_lnprob_batch_gp.argtypes = [
            _dp, ctypes.c_int, ctypes.c_int, ctypes.c_int, _ip, _ip, _dp,
            _ip, _dp, _dp, _dp, _dp, ctypes.c_int, _ip, _dp, _dp, _dp,
            _ip, _dp, _ip, _dp, _dp, ctypes.c_int]
        lib.lfo_wdphases.argtypes = [ctypes.c_double, ctypes.c_double, ctypes.c_double, ctypes.c_int, _dp, _dp]
        lib.lfo_gp_lnlike.restype = ctypes.c_double
        lib.lfo_gp_lnlike.argtypes = [_dp, _dp, _dp, ctypes.c_int, ctypes.c_double, ctypes.c_double,
                                      ctypes.c_double, _dp, ctypes.c_int]
        lib.lfo_gp_base_dcp.argtypes = [ctypes.c_double, ctypes.c_double, ctypes.c_double, _dp]
        lib.lfo_component.argtypes = [ctypes.c_int, _dp, ctypes.c_double, ctypes.c_double, ctypes.c_int,
                                      ctypes.c_int, _dp, _dp, ctypes.c_int, _dp]
        self.lib = lib

    # roche -----------------------------------------------------------------
    def xl1(self, q):
        return self.lib.lfo_xl1(float(q))

    def findphi(self, q, inc):
        out = ctypes.c_double()
        st = self.lib.lfo_findphi(float(q), float(inc), ctypes.byref(out))
        if st:
            raise ValueError("findphi failed (status %d)" % st)
        return out.value

    def findi(self, q, dphi):
        out = ctypes.c_double()
        st = self.lib.lfo_findi(float(q), float(dphi), ctypes.byref(out))
        if st:
            raise ValueError("findi failed (status %d)" % st)
        return out.value

    def bspot(self, q, rad):
        out = np.zeros(4)
        st = self.lib.lfo_bspot(float(q), float(rad), out.ctypes.data_as(_dp))
        if st:
            raise ValueError("bspot failed (status %d)" % st)
        return tuple(out)

    def wdphases(self, q, inc, r1, ntheta=10):
        p3, p4 = ctypes.c_double(), ctypes.c_double()
        st = self.lib.lfo_wdphases(float(q), float(inc), float(r1), int(ntheta), ctypes.byref(p3), ctypes.byref(p4))
        if st:
            raise ValueError("wdphases failed (status %d)" % st)
        return p3.value, p4.value

    # GP --------------------------------------------------------------------
    def gp_lnlike(self, x, r, ye, ampin, ampout, tau, blocks):
        x, xp = _f(x)
        r, rp = _f(r)
        ye, yp = _f(ye)
        b, bp = _f(np.asarray(blocks, dtype=np.float64).reshape(-1, 2) if len(blocks) else np.zeros((1, 2)))
        return self.lib.lfo_gp_lnlike(xp, rp, yp, x.shape[0], float(ampin), float(ampout), float(tau), bp,
                                      len(blocks))

    def gp_base_dcp(self, q, dphi, rwd):
        out = ctypes.c_double()
        st = self.lib.lfo_gp_base_dcp(float(q), float(dphi), float(rwd), ctypes.byref(out))
        if st:
            raise ValueError("changepoints failed (status %d)" % st)
        return out.value

    # CV --------------------------------------------------------------------
    def flux(self, pars, x, w=None, nsub=1, components=False):
        pars, pp = _f(pars)
        x, xp = _f(x)
        n = x.shape[0]
        if w is None:
            w = np.mean(np.diff(x)) * np.ones_like(x) / 2.0
        w, wp = _f(w)
        out = [np.empty(n) for _ in range(5)]
        ptrs = [o.ctypes.data_as(_dp) for o in out]
        st = self.lib.lfo_flux(pp, len(pars), xp, wp, n, int(nsub), *ptrs)
        if components:
            return st, out
        return st, out[0]

    def component(self, kind, cp, q, inc, x, w=None, n1=0, n2=0):
        """lfo_component: one unit-normalised component (MODEL_SPEC 5.6)."""
        cp, cpp = _f(cp if len(cp) else [0.0])
        x, xp = _f(x)
        w_, wp = _f(w) if w is not None else (None, None)
        out = np.empty(x.shape[0])
        st = self.lib.lfo_component(int(kind), cpp, float(q), float(inc), int(n1), int(n2), xp, wp, x.shape[0],
                                    out.ctypes.data_as(_dp))
        return st, out

    def elements(self, pars):
        pars, pp = _f(pars)
        a, b, wg = np.empty(NEL), np.empty(NEL), np.empty(NEL)
        donor = np.empty((NDONOR, 3))
        geo = np.empty(16)
        st = self.lib.lfo_elements(pp, len(pars), a.ctypes.data_as(_dp),
                                   b.ctypes.data_as(_dp), wg.ctypes.data_as(_dp),
                                   donor.ctypes.data_as(_dp), geo.ctypes.data_as(_dp))
        return st, a, b, wg, donor, geo

    def prior_lnprob(self, ptype, p1, p2, norm, v):
        return self.lib.lfo_prior_lnprob(int(ptype), float(p1), float(p2),
                                         float(norm), float(v))

    def lnprob_batch(self, walkers, tree, nsub=1, nthreads=0):
        """tree: lfit_python_amd.batch.CompiledTree (plain numpy fields)."""
        walkers, wp = _f(walkers)
        W, ndim = walkers.shape
        keep = []

        def F(a):
            a, p = _f(a)
            keep.append(a)
            return p

        def I(a):
            a, p = _i(a)
            keep.append(a)
            return p

        lnp = np.empty(W)
        lle = np.empty((W, tree.E))
        gp = getattr(tree, "gp", False)
        used = self.lib.lfo_lnprob_batch_gp(
            wp, W, ndim, tree.E, I(tree.gather.reshape(-1)), I(tree.npars),
            F(tree.consts if len(tree.consts) else np.zeros(1)),
            I(tree.offsets), F(tree.x), F(tree.y), F(tree.ye), F(tree.w),
            int(nsub), I(tree.prior_type), F(tree.prior_p1), F(tree.prior_p2),
            F(tree.prior_norm),
            I(tree.gp_gather.reshape(-1)) if gp else None,
            F(tree.gp_base[:, :3].reshape(-1)) if gp else None,
            I(tree.gp_ecl.reshape(-1)) if gp else None,
            lnp.ctypes.data_as(_dp), lle.ctypes.data_as(_dp), int(nthreads))
        if getattr(tree, "fixed_invalid", False):  # an invalid fixed parameter: Node.ln_prior = -inf
            lnp[:] = -np.inf
        return lnp, lle, used
