"""Generate lfit_python_amd/csrc/lfg_stream_table.h: the converged ballistic
stream of MODEL_SPEC 4.5 as piecewise tensor Chebyshev series.

bspot(q, r) (trm.roche.bspot, CVModel.py:288) is the state where the stream
from L1 first reaches radius r.  For each q the stream leaves the L1 unstable
manifold at the second-order start point of MODEL_SPEC 4.5 (radius r0(q)) and
falls to periastron (radius rmin(q)).  In the variables

    xi = ln q,    s = sqrt((r - rmin(q)) / (r0(q) - rmin(q)))

the crossing state is analytic (s absorbs the square-root turn at
periastron), so it is tabulated as Chebyshev series on patches of
(xi, s): NQ equal patches in xi, graded patches in s (denser near
periastron, s -> 0, and toward the start, s -> 1, where the exponential
departure from L1 puts a singularity just past s = 1).  Outputs per patch:
phi = atan2(y, x) of the crossing point (x = r cos phi, y = r sin phi), vx,
vy.  ln rmin(q) is a 1-D series per xi patch.

The same patches in xi also carry xl1(q) (the start of roche_init's Newton
solve) and findphi(q, 90 deg) (the LCModel dphi prior, CVModel.py:452-473),
from an independent solve in the orbital plane (findphi90 below).

Reference solution: scipy DOP853 at rtol 2.3e-14 / atol 1e-16 with a step cap,
the crossing located by Brent's method on its dense output.  The table
reproduces it to ~1e-13 in position and ~5e-12 in velocity (printed at the
end; tests/test_stream_table.py re-checks it).

Run in the build container only (scipy); the header is committed.
    python tools/gen_stream_table.py [out.h]
"""
import os
import sys
import time

import numpy as np
from numpy.polynomial import chebyshev as C
from scipy.integrate import solve_ivp
from scipy.optimize import brentq, minimize_scalar

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "lfit_python_amd", "csrc", "lfg_stream_table.h")

Q_LO, Q_HI = 0.002, 5.0
NQ, DQ = 10, 9
SB = [0.0, 0.1, 0.2, 0.4, 0.65, 0.8, float(np.sqrt(0.8)), float(np.sqrt(0.9)), 0.975, 0.99, 0.997, 1.0]
DS = 12
DR = 12
DELTA = 1e-2  # MODEL_SPEC 4.5 / 7: manifold start offset


def xl1(q):
    """MODEL_SPEC 4.1 (Newton to machine precision)."""
    cA, cB, mu = 2.0 / (1.0 + q), 2.0 * q / (1.0 + q), q / (1.0 + q)
    x = 1.0 - (mu / 3.0) ** (1.0 / 3.0)
    for _ in range(100):
        f = cA / x ** 2 - cB / (1.0 - x) ** 2 - 2.0 * (x - mu)
        df = -2.0 * cA / x ** 3 - 2.0 * cB / (1.0 - x) ** 3 - 2.0
        dx = f / df
        x -= dx
        if abs(dx) < 1e-16:
            break
    return x


def start(q):
    """MODEL_SPEC 4.5: second-order point of the L1 unstable manifold."""
    x1 = xl1(q)
    m1, m2 = 1.0 / (1.0 + q), q / (1.0 + q)
    Rs = 1.0 - x1
    K = m1 / x1 ** 3 + m2 / Rs ** 3
    Uxx, Uyy = -2.0 * K - 1.0, K - 1.0
    L = 0.5 * ((K - 2.0) + np.sqrt((K - 2.0) ** 2 + 4.0 * (2.0 * K + 1.0) * (K - 1.0)))
    lam = np.sqrt(L)
    A = -1.0
    B = (L - 2.0 * K - 1.0) / (2.0 * lam) * A
    nrm = np.hypot(A, B)
    v = np.array([A / nrm, B / nrm, lam * A / nrm, lam * B / nrm])
    Uxxx = 6.0 * m1 / x1 ** 4 - 6.0 * m2 / Rs ** 4
    Uxyy = -0.5 * Uxxx
    N2x = -0.5 * (Uxxx * v[0] ** 2 + Uxyy * v[1] ** 2)
    N2y = -Uxyy * v[0] * v[1]
    a11, a22 = Uxx + 4.0 * L, Uyy + 4.0 * L
    det = a11 * a22 + 16.0 * L
    w0 = (N2x * a22 + 4.0 * lam * N2y) / det
    w1 = (a11 * N2y - 4.0 * lam * N2x) / det
    w = np.array([w0, w1, 2.0 * lam * w0, 2.0 * lam * w1])
    return np.array([x1, 0.0, 0.0, 0.0]) + DELTA * v + DELTA ** 2 * w


def rhs(t, s, q):
    m1, m2, mu = 1.0 / (1.0 + q), q / (1.0 + q), q / (1.0 + q)
    x, y, vx, vy = s
    r1 = np.hypot(x, y)
    r2 = np.hypot(x - 1.0, y)
    Ux = m1 * x / r1 ** 3 + m2 * (x - 1.0) / r2 ** 3 - (x - mu)
    Uy = m1 * y / r1 ** 3 + m2 * y / r2 ** 3 - y
    return [vx, vy, -Ux + 2.0 * vy, -Uy - 2.0 * vx]


class Stream:
    """Converged stream of one q: dense solution up to periastron."""

    def __init__(self, q):
        s0 = start(q)

        def peri(t, s, q):
            return s[0] * s[2] + s[1] * s[3]
        peri.terminal = True
        peri.direction = 1
        sol = solve_ivp(rhs, (0.0, 50.0), s0, method="DOP853", rtol=2.3e-14, atol=1e-16,
                        max_step=0.005, dense_output=True, args=(q,), events=peri)
        self.sol = sol
        self.tp = sol.t_events[0][0]
        sp = sol.sol(self.tp)
        self.rmin = float(np.hypot(sp[0], sp[1]))
        self.r0 = float(np.hypot(s0[0], s0[1]))

    def at_radius(self, rad):
        if rad <= self.rmin:
            return self.sol.sol(self.tp)
        if rad >= self.r0:
            return self.sol.sol(0.0)
        t = brentq(lambda t: np.hypot(*self.sol.sol(t)[:2]) - rad, 0.0, self.tp, xtol=1e-16, rtol=1e-15)
        return self.sol.sol(t)

    def at_s(self, s):
        return self.at_radius(self.rmin + (self.r0 - self.rmin) * s * s)


def rpot2(q, x, y):
    """Phi in the orbital plane (MODEL_SPEC 2)."""
    cA, cB, mu = 2.0 / (1.0 + q), 2.0 * q / (1.0 + q), q / (1.0 + q)
    return -cA / np.hypot(x, y) - cB / np.hypot(x - 1.0, y) - (x - mu) ** 2 - y ** 2


def findphi90(q):
    """MODEL_SPEC 4.4 at i = 90 deg: the line of sight from the WD centre at
    orbital angle theta lies in the orbital plane; g(theta) = min over the
    ray of Phi - Phi(L1) (the minimum, hence g, converged by Brent in t and
    Newton on dPhi/dt), and the WD-centre egress is the root of g."""
    x1 = xl1(q)
    pl1 = rpot2(q, x1, 0.0)
    Rs = 1.0 - x1

    def g(th):
        ex, ey = np.cos(th), -np.sin(th)
        tc = ex  # closest approach of the ray to the donor centre D = (1, 0)
        f = lambda t: rpot2(q, t * ex, t * ey)
        lo, hi = max(0.0, tc - Rs), tc + Rs
        r = minimize_scalar(f, bounds=(lo, hi), method="bounded", options={"xatol": 1e-12})
        t = r.x
        for _ in range(3):  # Newton on dPhi/dt (central differences of the analytic Phi)
            h = 1e-5
            d1 = (f(t + h) - f(t - h)) / (2 * h)
            d2 = (f(t + h) - 2 * f(t) + f(t - h)) / (h * h)
            t -= d1 / d2
        return f(t) - pl1
    thmax = np.arcsin(Rs)  # the ray leaves the donor's sphere
    th = brentq(g, 0.0, thmax * (1.0 - 1e-12), xtol=1e-16, rtol=1e-15)
    return th / np.pi


def cheb_nodes(n):
    return np.cos(np.pi * (np.arange(n) + 0.5) / n)


def outputs(state):
    x, y, vx, vy = state
    return np.array([np.arctan2(y, x), vx, vy])


def build():
    lqb = np.linspace(np.log(Q_LO), np.log(Q_HI), NQ + 1)
    NS = len(SB) - 1
    coef = np.zeros((NQ, NS, 3, DQ + 1, DS + 1))
    rmc = np.zeros((NQ, DR + 1))
    q1d = np.zeros((2, NQ, DR + 1))  # xl1(q), findphi(q, 90 deg)
    for iq in range(NQ):
        xr = cheb_nodes(DR + 1)
        qr = np.exp(lqb[iq] + (lqb[iq + 1] - lqb[iq]) * (xr + 1.0) / 2.0)
        rmc[iq] = C.chebfit(xr, np.log([Stream(q).rmin for q in qr]), DR)
        q1d[0, iq] = C.chebfit(xr, [xl1(q) for q in qr], DR)
        q1d[1, iq] = C.chebfit(xr, [findphi90(q) for q in qr], DR)
        xq = cheb_nodes(DQ + 1)
        qs = np.exp(lqb[iq] + (lqb[iq + 1] - lqb[iq]) * (xq + 1.0) / 2.0)
        streams = [Stream(q) for q in qs]
        for js in range(NS):
            xs = cheb_nodes(DS + 1)
            ss = SB[js] + (SB[js + 1] - SB[js]) * (xs + 1.0) / 2.0
            V = np.array([[outputs(st.at_s(s)) for s in ss] for st in streams])  # [DQ+1][DS+1][3]
            for k in range(3):
                # phi: keep one branch across the patch (no 2 pi jumps)
                vk = np.unwrap(V[:, :, k], axis=1) if k == 0 else V[:, :, k]
                c1 = np.array([C.chebfit(xs, vk[a], DS) for a in range(DQ + 1)])
                coef[iq, js, k] = np.array([C.chebfit(xq, c1[:, b], DQ) for b in range(DS + 1)]).T
    return lqb, coef, rmc, q1d


def evaluate(lqb, coef, rmc, q, s):
    iq = min(NQ - 1, int((np.log(q) - lqb[0]) / (lqb[1] - lqb[0])))
    xq = 2.0 * (np.log(q) - lqb[iq]) / (lqb[iq + 1] - lqb[iq]) - 1.0
    js = min(max(int(np.searchsorted(SB, s)) - 1, 0), len(SB) - 2)
    xs = 2.0 * (s - SB[js]) / (SB[js + 1] - SB[js]) - 1.0
    return np.array([C.chebval2d(xq, xs, coef[iq, js, k]) for k in range(3)]), np.exp(C.chebval(xq, rmc[iq]))


def check(lqb, coef, rmc, q1d, ntraj=40, seed=7):
    rng = np.random.default_rng(seed)
    err = np.zeros(5)
    for _ in range(ntraj):
        q = float(np.exp(rng.uniform(np.log(Q_LO), np.log(Q_HI))))
        st = Stream(q)
        for s in rng.uniform(0.0, SB[-1], 6):
            v, rmin = evaluate(lqb, coef, rmc, q, s)
            ref = st.at_s(s)
            rad = st.rmin + (st.r0 - st.rmin) * s * s
            err[0] = max(err[0], abs(rad * np.cos(v[0]) - ref[0]), abs(rad * np.sin(v[0]) - ref[1]))
            err[1] = max(err[1], abs(v[1] - ref[2]), abs(v[2] - ref[3]))
            err[2] = max(err[2], abs(rmin - st.rmin))
        iq = min(NQ - 1, int((np.log(q) - lqb[0]) / (lqb[1] - lqb[0])))
        xq = 2.0 * (np.log(q) - lqb[iq]) / (lqb[iq + 1] - lqb[iq]) - 1.0
        err[3] = max(err[3], abs(C.chebval(xq, q1d[0, iq]) - xl1(q)))
        err[4] = max(err[4], abs(C.chebval(xq, q1d[1, iq]) - findphi90(q)))
    return err


def write(path, lqb, coef, rmc, q1d, err):
    lines = [
        "// lfg_stream_table.h -- GENERATED by tools/gen_stream_table.py; do not edit.",
        "// The converged ballistic stream of MODEL_SPEC 4.5 (trm.roche.bspot,",
        "// CVModel.py:288) as piecewise tensor Chebyshev series in xi = ln q and",
        "// s = sqrt((r - rmin(q)) / (r0(q) - rmin(q))).  Plain C initialisers: the",
        "// HIP kernels and the CPU oracle declare their own arrays from them.",
        "// Check against the DOP853 reference (max abs): position %.1e, velocity %.1e," % (err[0], err[1]),
        "// rmin %.1e; xl1 %.1e, findphi(q, 90) %.1e." % (err[2], err[3], err[4]),
        "#pragma once",
        "#define LFG_ST_QLO %r" % Q_LO,
        "#define LFG_ST_QHI %r" % Q_HI,
        "#define LFG_ST_NQ %d" % NQ,
        "#define LFG_ST_DQ %d" % DQ,
        "#define LFG_ST_NS %d" % (len(SB) - 1),
        "#define LFG_ST_DS %d" % DS,
        "#define LFG_ST_DR %d" % DR,
        "#define LFG_ST_LQLO %r" % float(lqb[0]),
        "#define LFG_ST_LQW %r" % float(lqb[1] - lqb[0]),
        "#define LFG_ST_STOP %r" % SB[-1],
        "// patch edges in s",
        "#define LFG_ST_SB { %s }" % ", ".join(repr(float(v)) for v in SB),
        "// ln rmin: [NQ][DR + 1] Chebyshev coefficients in the patch's xi",
        "#define LFG_ST_RMIN { %s }" % ", ".join(repr(float(v)) for v in rmc.ravel()),
        "// xl1(q) (MODEL_SPEC 4.1; the Newton start of roche_init) and findphi(q, 90 deg)",
        "// (MODEL_SPEC 4.4; the LCModel dphi prior): [NQ][DR + 1] each, as LFG_ST_RMIN",
        "#define LFG_ST_XL1 { %s }" % ", ".join(repr(float(v)) for v in q1d[0].ravel()),
        "#define LFG_ST_PHI90 { %s }" % ", ".join(repr(float(v)) for v in q1d[1].ravel()),
        "// [NQ][NS][3: phi, vx, vy][DQ + 1][DS + 1]: c[i][j] multiplies T_i(xi') T_j(s')",
        "#define LFG_ST_COEF { \\",
    ]
    flat = coef.ravel()
    per = (DQ + 1) * (DS + 1)
    for k in range(0, flat.size, per):
        lines.append("    " + ", ".join(repr(float(v)) for v in flat[k:k + per]) + ", \\")
    lines.append("}")
    with open(path, "w") as fh:
        fh.write("\n".join(lines) + "\n")


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else OUT
    t0 = time.time()
    lqb, coef, rmc, q1d = build()
    err = check(lqb, coef, rmc, q1d)
    print("built in %.1f s; max abs error vs DOP853: position %.2e velocity %.2e rmin %.2e; "
          "xl1 %.2e findphi90 %.2e" % (time.time() - t0, err[0], err[1], err[2], err[3], err[4]))
    write(out, lqb, coef, rmc, q1d, err)
    print("wrote", out)


if __name__ == "__main__":
    main()
