"""The GPU path's algorithm on CPU cores (cpu_baseline/lfg_cpu.cpp): a fair
CPU baseline for bench.py, beside the oracle.  Not a product path: nothing
in lfit_python_amd loads it.

    build(out=None, march="native") -> path of liblfg_cpu.so
    CpuPort(path).lnprob_batch(walkers, tree, nthreads=0) -> (lnp, threads)
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
LIB_PATH = os.path.join(HERE, "liblfg_cpu.so")
_dp = ctypes.POINTER(ctypes.c_double)
_ip = ctypes.POINTER(ctypes.c_int)


def build(out=None, march="x86-64-v3"):
    out = out or LIB_PATH
    cmd = ["g++", "-O3", "-march=%s" % march, "-fopenmp", "-std=c++17", "-fPIC", "-shared",
           "-I", HERE, "-I", os.path.join(HERE, "shim"), "-I", os.path.join(ROOT, "lfit_python_amd", "csrc"),
           "-I", os.path.join(ROOT, "include"), "-o", out, os.path.join(HERE, "lfg_cpu.cpp")]
    subprocess.run(cmd, check=True)
    return out


class CpuPort:
    def __init__(self, path=None):
        self.lib = ctypes.CDLL(path or LIB_PATH)
        f = self.lib.lfc_lnprob_batch
        f.restype = ctypes.c_int
        f.argtypes = [_dp, ctypes.c_int, ctypes.c_int, ctypes.c_int, _ip, _ip, _dp, _ip, _dp, _dp, _dp, _dp,
                      ctypes.c_int, _ip, _dp, _dp, _dp, ctypes.c_int, _dp, ctypes.c_int]
        for name in ("lfg_cpu_flux", "lfg_cpu_lnlike", "lfg_cpu_lnprob"):
            getattr(self.lib, name).restype = ctypes.c_int
        self.lib.lfg_cpu_flux.argtypes = [_dp, ctypes.c_int, ctypes.c_int, _dp, _dp, ctypes.c_int, ctypes.c_int,
                                          _dp, _ip, ctypes.c_int]
        self.lib.lfg_cpu_lnlike.argtypes = [_dp, ctypes.c_int, ctypes.c_int, _dp, _dp, ctypes.c_int, ctypes.c_int,
                                            _dp, _dp, _dp, _ip, ctypes.c_int]
        g = self.lib.lfc_lnprob_batch_gp
        g.restype = ctypes.c_int
        g.argtypes = [_dp, ctypes.c_int, ctypes.c_int, ctypes.c_int, _ip, _ip, _dp, _ip, _dp, _dp, _dp, _dp,
                      ctypes.c_int, _ip, _dp, _dp, _dp, ctypes.c_int, _ip, _dp, _ip, _dp, ctypes.c_int]

    def lnprob_batch(self, walkers, tree, nthreads=0):
        """ln_prob of walkers [W, ndim] of a compiled tree
        (lfit_python_amd.batch.CompiledTree), chi^2 or GP."""
        keep = []

        def F(a):
            a = np.ascontiguousarray(a, dtype=np.float64)
            keep.append(a)
            return a.ctypes.data_as(_dp)

        def I(a):
            a = np.ascontiguousarray(a, dtype=np.int32)
            keep.append(a)
            return a.ctypes.data_as(_ip)
        w = np.ascontiguousarray(walkers, dtype=np.float64)
        W, ndim = w.shape
        lnp = np.empty(W)
        gp = bool(getattr(tree, "gp", False))
        used = self.lib.lfc_lnprob_batch_gp(
            F(w), W, ndim, tree.E, I(tree.gather.reshape(-1)), I(tree.npars),
            F(tree.consts if len(tree.consts) else np.zeros(1)), I(tree.offsets), F(tree.x), F(tree.y), F(tree.ye),
            F(tree.w), int(tree.nsub), I(tree.prior_type), F(tree.prior_p1), F(tree.prior_p2), F(tree.prior_norm),
            int(tree.roche_priors), I(tree.gp_gather.reshape(-1)) if gp else None,
            F(tree.gp_base.reshape(-1)) if gp else None, I(tree.gp_ecl.reshape(-1)) if gp else None,
            lnp.ctypes.data_as(_dp), int(nthreads))
        if getattr(tree, "fixed_invalid", False):
            lnp[:] = -np.inf
        return lnp, used

    # ---- the lfg_cpu_* twins (cpu_baseline/lfg_cpu.h) of lfg_flux,
    # lfg_lnlike and lfg_lnprob: host arrays, the same argument meaning
    def flux(self, pars, x, w, nsub=1, nthreads=0):
        """lfg_cpu_flux: (flux [W, N], status [W])"""
        pars = np.ascontiguousarray(np.atleast_2d(pars), dtype=np.float64)
        x = np.ascontiguousarray(x, dtype=np.float64)
        w = None if w is None else np.ascontiguousarray(w, dtype=np.float64)
        W, P = pars.shape
        flux = np.empty((W, x.size))
        st = np.empty(W, dtype=np.int32)
        rc = self.lib.lfg_cpu_flux(pars.ctypes.data_as(_dp), W, P, x.ctypes.data_as(_dp),
                                   None if w is None else w.ctypes.data_as(_dp), x.size, int(nsub),
                                   flux.ctypes.data_as(_dp), st.ctypes.data_as(_ip), int(nthreads))
        if rc != 0:
            raise ValueError("lfg_cpu_flux: code %d" % rc)
        return flux, st

    def lnlike(self, pars, x, w, y, ye, nsub=1, nthreads=0):
        """lfg_cpu_lnlike: (ln_like [W], status [W])"""
        pars = np.ascontiguousarray(np.atleast_2d(pars), dtype=np.float64)
        arr = [np.ascontiguousarray(a, dtype=np.float64) for a in (x, y, ye)]
        w = None if w is None else np.ascontiguousarray(w, dtype=np.float64)
        W, P = pars.shape
        out = np.empty(W)
        st = np.empty(W, dtype=np.int32)
        rc = self.lib.lfg_cpu_lnlike(pars.ctypes.data_as(_dp), W, P, arr[0].ctypes.data_as(_dp),
                                     None if w is None else w.ctypes.data_as(_dp), arr[0].size, int(nsub),
                                     arr[1].ctypes.data_as(_dp), arr[2].ctypes.data_as(_dp), out.ctypes.data_as(_dp),
                                     st.ctypes.data_as(_ip), int(nthreads))
        if rc != 0:
            raise ValueError("lfg_cpu_lnlike: code %d" % rc)
        return out, st

    def lnprob(self, walkers, tree, nthreads=0):
        """lfg_cpu_lnprob through a struct lfg_tree of host arrays"""
        from lfit_python_amd import _native
        keep = []

        def F(a):
            a = np.ascontiguousarray(a, dtype=np.float64)
            keep.append(a)
            return ctypes.c_void_p(a.ctypes.data)

        def I(a):
            a = np.ascontiguousarray(a, dtype=np.int32)
            keep.append(a)
            return ctypes.c_void_p(a.ctypes.data)
        gp = bool(tree.gp)
        T = _native.LfgTree(tree.E, tree.ndim, tree.nsub, tree.max_n, I(tree.gather.reshape(-1)), I(tree.npars),
                            F(tree.consts if len(tree.consts) else np.zeros(1)), I(tree.offsets), F(tree.x),
                            F(tree.y), F(tree.ye), F(tree.w), I(tree.prior_type), F(tree.prior_p1), F(tree.prior_p2),
                            F(tree.prior_norm), int(tree.roche_priors), int(gp),
                            I(tree.gp_gather.reshape(-1)) if gp else None, F(tree.gp_base.reshape(-1)) if gp else None,
                            I(tree.gp_ecl.reshape(-1)) if gp else None, int(tree.fixed_invalid), None)
        w = np.ascontiguousarray(walkers, dtype=np.float64)
        lnp = np.empty(w.shape[0])
        self.lib.lfg_cpu_lnprob.argtypes = [_dp, ctypes.c_int, ctypes.POINTER(_native.LfgTree), _dp, ctypes.c_int]
        rc = self.lib.lfg_cpu_lnprob(w.ctypes.data_as(_dp), w.shape[0], ctypes.byref(T), lnp.ctypes.data_as(_dp),
                                     int(nthreads))
        if rc != 0:
            raise ValueError("lfg_cpu_lnprob: code %d" % rc)
        return lnp
