"""Diagnostic (CPU): the tangency Newton's stopping rule (TH_LAST, T_LAST of
lfg_device.hpp) against ln_prob parity with the oracle and the Newton steps
a k_elements wave runs (the max over its 64 lanes), on the host build of the
GPU algorithm (cpu_baseline/lfg_cpu.cpp -DLFC_COUNT).

    python tools/tol_study.py [--walkers 256] [--config 2|3|5] th:t[:pth:pt][+DEFINE...] ...
"""
import argparse
import ctypes
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

from cpu_baseline import cpu  # noqa: E402
from lfit_python_amd import batch, sampler, synthetic  # noqa: E402
from oracle.oracle import Oracle  # noqa: E402


def build(th, t, out, extra=()):
    cmd = ["g++", "-O3", "-march=native", "-fopenmp", "-std=c++17", "-fPIC", "-shared", "-DLFC_COUNT",
           "-DLFG_TH_LAST=%s" % th, "-DLFG_T_LAST=%s" % t] + list(extra) + [
           "-I", os.path.join(ROOT, "cpu_baseline", "shim"), "-I", os.path.join(ROOT, "lfit_python_amd", "csrc"),
           "-I", os.path.join(ROOT, "include"), "-o", out, os.path.join(ROOT, "cpu_baseline", "lfg_cpu.cpp")]
    subprocess.run(cmd, check=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--walkers", type=int, default=256)
    ap.add_argument("--config", default="2")
    ap.add_argument("variants", nargs="+", help="the first is the reference for the interval errors")
    a = ap.parse_args()
    O = Oracle()
    f = lambda p, x, w, nsub: O.flux(p, x, w, nsub=nsub)[1]  # noqa: E731
    nsub = 5 if a.config == "5" else 1
    m = (synthetic.config_tree(4, 300, flux_fn=f) if a.config == "3" else
         synthetic.config_single(2000 if a.config == "5" else 300, flux_fn=f, nsub=nsub))
    t = batch.compile_tree(m, nsub=nsub)
    p0 = np.array(m.dynasty_par_vals)
    walk = sampler.initialise_walkers(p0, sampler.comp_scatter(m.dynasty_par_names, 0.1), a.walkers,
                                      lambda p: O.lnprob_batch(p, t, nsub=nsub)[0], seed=3)
    ref, _, _ = O.lnprob_batch(walk, t, nsub=nsub)
    fin = np.isfinite(ref)
    print("walkers %d finite %d" % (len(walk), fin.sum()))
    base = None
    for v in a.variants:
        spec, *flags = v.split("+")
        th, tt = spec.split(":")[:2]
        extra = ["-DLFG_NEWTON_PRED", "-DLFG_PRED_TH=%s" % spec.split(":")[2], "-DLFG_PRED_T=%s" % spec.split(":")[3]] \
            if spec.count(":") == 3 else []
        extra += ["-D" + f for f in flags]
        out = "/tmp/tol/liblfc_%s.so" % v.replace(":", "_").replace("+", "_")
        build(th, tt, out, extra)
        P = cpu.CpuPort(out)
        t0 = time.perf_counter()
        got, _ = P.lnprob_batch(walk, t)
        dt = time.perf_counter() - t0
        c = (ctypes.c_ulonglong * 28)()
        P.lib.lfc_counts(c)
        hist = np.array(c[4:]).reshape(3, 8)
        hist = "  ".join("%s %s" % (r, np.round(h / max(h.sum(), 1), 3)[1:7]) for r, h in zip(("wd", "disc", "spot"), hist))
        assert np.array_equal(np.isfinite(got), fin)
        ab = np.zeros(64 * 800 * 2)
        P.lib.lfc_dump(ab.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), ctypes.c_long(0))  # clear
        P.lnprob_batch(walk[:64], t, nthreads=1)
        n = P.lib.lfc_dump(ab.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), ctypes.c_long(ab.size))
        ab = ab[:n]
        if base is None:
            base = ab
        d = np.abs(ab - base)
        ecl = np.repeat(base[0::2] < base[1::2], 2)
        dab = "interval err (phase) max %.1e p99.9 %.1e" % (d[ecl].max(), np.percentile(d[ecl], 99.9))
        err = np.abs(got[fin] - ref[fin]) / np.abs(ref[fin])
        print("%-24s lnp err max %.1e med %.1e | steps/lane %.3f  wave-max %.3f"
              "  | %s\n    lane steps 1..6: %s" % (v, err.max(), np.median(err), c[1] / c[0], c[3] / c[2], dab, hist))


if __name__ == "__main__":
    main()
