"""Diagnostic (CPU): initial-guess error of the tangency solve (MODEL_SPEC
4.3) for WD and disc elements: the calibrated-sphere guess of
element_interval_fast, and the sphere guess corrected by the gradient of
(exact - sphere) contact phase at the WD centre.  Exact contacts by the
envelope Newton (lfg_device.hpp tangency_step) run to 1e-15.
python tools/guess_study.py"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle.oracle import Oracle

O = Oracle()
q, dphi = 0.1037, 0.0392
if len(sys.argv) > 2:
    q, dphi = float(sys.argv[1]), float(sys.argv[2])
inc = O.findi(q, dphi)
s, c = np.sin(np.radians(inc)), np.cos(np.radians(inc))
xl1 = O.xl1(q)
cA = 2 / (1 + q); cB = q * cA; mu = q / (1 + q)


def pot(x, y, z):
    return -cA / np.sqrt(x * x + y * y + z * z) - cB / np.sqrt((x - 1) ** 2 + y * y + z * z) - (x - mu) ** 2 - y * y


pl1 = pot(xl1, 0, 0)
sce = s * np.cos(np.pi * dphi)
Rcal = np.sqrt(1 - sce * sce)


def cone_point(P, th, t):
    Px, Py, Pz = P
    ex, ey = s * np.cos(th), -s * np.sin(th)
    x, y, z = Px + t * ex, Py + t * ey, Pz + t * c
    r1s = x * x + y * y + z * z; ir1 = 1 / np.sqrt(r1s); ir1s = ir1 * ir1
    dx = x - 1; r2s = dx * dx + y * y + z * z; ir2 = 1 / np.sqrt(r2s); ir2s = ir2 * ir2
    i1 = cA * ir1s * ir1; i2 = cB * ir2s * ir2; i12 = i1 + i2; xm = x - mu
    phi = -cA * ir1 - cB * ir2 - xm * xm - y * y
    gx = i1 * x + i2 * dx - 2 * xm; gy = (i12 - 2) * y; gz = i12 * z
    p1 = x * ex + y * ey + z * c; p2 = p1 - ex; q1 = x * ey - y * ex; q2 = q1 - ey
    k1 = 3 * i1 * ir1s; k2 = 3 * i2 * ir2s; s2 = ex * ex + ey * ey
    F2 = gx * ex + gy * ey + gz * c; gth = gx * ey - gy * ex
    eHe = i12 - k1 * p1 * p1 - k2 * p2 * p2 - 2 * s2; etHe = -k1 * p1 * q1 - k2 * p2 * q2
    return phi, gth, F2, eHe, etHe


def solve(P, th, t, n=40, tol=1e-15):
    for it in range(n):
        phi, gth, F2, eHe, etHe = cone_point(P, th, t)
        F1 = phi - pl1; J11 = t * gth; J21 = t * etHe + gth; J22 = eHe
        dt0 = -F2 / J22
        F1m = F1 - F2 * F2 / (2 * J22)
        dth = -F1m / (J11 + J21 * dt0)
        dth = min(max(dth, -0.05), 0.05)
        dt = dt0 - (J21 / J22) * dth
        th += dth; t += dt
        if abs(dth) <= tol and abs(dt) <= 1e-12:
            return th, t, it + 1
    return th, t, -1


def sphere(P):
    ux, uy, uz = 1 - P[0], -P[1], -P[2]
    uxy2 = ux * ux + uy * uy; uu = uxy2 + uz * uz; uxy = np.sqrt(uxy2)
    ce = (np.sqrt(max(uu - Rcal * Rcal, 0)) - c * uz) / uxy / s
    thc = np.arctan2(-uy, ux); de = np.arccos(ce)
    ti, to = thc - de, thc + de
    t_i = s * (ux * np.cos(ti) - uy * np.sin(ti)) + uz * c
    t_o = s * (ux * np.cos(to) - uy * np.sin(to)) + uz * c
    return (ti, t_i), (to, t_o)


def exact(P):
    (ti, tti), (to, tto) = sphere(P)
    a = solve(P, ti, tti)
    b = solve(P, to, tto)
    assert a[2] > 0 and b[2] > 0, P
    return np.array([a[0], b[0]]), np.array([ti, to]), np.array([a[1], b[1]]), np.array([tti, tto])


def steps(P, th, t):
    # the kernel's rule: stop after the step once |dth| <= 3e-8 and |dt| <= 1e-5
    for it in range(16):
        phi, gth, F2, eHe, etHe = cone_point(P, th, t)
        F1 = phi - pl1; J11 = t * gth; J21 = t * etHe + gth; J22 = eHe
        dt0 = -F2 / J22
        F1m = F1 - F2 * F2 / (2 * J22)
        dth = -F1m / (J11 + J21 * dt0)
        dth = min(max(dth, -0.05), 0.05)
        dt = dt0 - (J21 / J22) * dth
        th += dth; t += dt
        if abs(dth) <= 3e-8 and abs(dt) <= 1e-5:
            return it + 1, th
    return 99, th


# gradient of (exact - sphere) at the WD centre
h = 1e-5
g = np.zeros((2, 3))
gt = np.zeros((2, 3))
for k in range(3):
    e = np.zeros(3); e[k] = h
    xp, sp, tp, tsp = exact(e); xm_, sm, tm, tsm = exact(-e)
    g[:, k] = ((xp - sp) - (xm_ - sm)) / (2 * h)
    gt[:, k] = ((tp - tsp) - (tm - tsm)) / (2 * h)
x0, s0, t0x, t0s = exact(np.zeros(3))
dt0c = t0x - t0s  # t offset of the sphere guess at the WD centre
print('q %.4f dphi %.4f inc %.3f  d(exact - sphere)/dP at the WD centre: in %s out %s' % (q, dphi, inc, g[0].round(4), g[1].round(4)))

rwd = 0.0187 * xl1
rdisc = 0.2953 * xl1
rng = np.random.default_rng(1)
pts = {'WD': [], 'disc': []}
for _ in range(300):  # WD surface, the observer-facing hemisphere
    v = rng.standard_normal(3); v /= np.linalg.norm(v)
    if v @ np.array([s, 0, c]) < 0: v = -v
    pts['WD'].append(rwd * v)
for r in np.linspace(rwd, rdisc, 20):
    for al in np.linspace(0.03, np.pi - 0.03, 25):
        pts['disc'].append(np.array([r * np.cos(al), r * np.sin(al), 0.0]))
for name, P in pts.items():
    es, ec, ets, etc_, ns, nc = [], [], [], [], [], []
    for p in P:
        x, sg, tx, ts = exact(p)
        es.append(np.abs(sg - x).max())
        ec.append(np.abs(sg + g @ p - x).max())
        ets.append(np.abs(ts - tx).max())
        tc = ts + dt0c + gt @ p
        etc_.append(np.abs(tc - tx).max())
        ns.append(max(steps(p, sg[0], ts[0])[0], steps(p, sg[1], ts[1])[0]))
        gc = sg + g @ p
        nc.append(max(steps(p, gc[0], tc[0])[0], steps(p, gc[1], tc[1])[0]))
    es, ec = np.array(es), np.array(ec)
    for lab, e in (('sphere', es), ('sphere + grad', ec)):
        print('%-5s %-14s guess err  median %.1e  p90 %.1e  max %.1e  frac<1e-4 %.2f' % (
            name, lab, np.median(e), np.percentile(e, 90), e.max(), (e < 1e-4).mean()))
    print('%-5s t guess err: sphere median %.1e max %.1e | corrected median %.1e max %.1e' % (
        name, np.median(ets), np.max(ets), np.median(etc_), np.max(etc_)))
    print('%-5s steps (max of in/out): sphere %s | corrected %s' % (
        name, np.bincount(ns).tolist(), np.bincount(nc).tolist()))
