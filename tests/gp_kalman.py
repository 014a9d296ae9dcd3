"""Test helper: the O(N) state-space form of the GP likelihood that the HIP
kernels evaluate (MODEL_SPEC 10.4), restated in plain Python loops so the
CPU suite can check the recursion against the dense Cholesky oracle before
any GPU runs it.

A Matern-3/2 process with variance a and scale l = sqrt(tau) (george's
metric tau) is the stationary solution of a 2-state linear SDE; between
sorted points spaced d it moves by
    Phi(d) = e^{-u} [[1 + u, d], [-lam^2 d, 1 - u]],  u = lam d, lam = sqrt(3/tau)
with stationary covariance Pinf = a diag(1, lam^2).  The kernel of
CVModel.py:636-645 is one global process (ampin) plus, inside each
changepoint block, an independent process (ampout) that starts stationary
at the block's first point.  A 4-state Kalman filter over the sorted points
gives the exact log-likelihood.  Covariances are carried as D = P - Pinf so
that the prediction is D <- Phi D Phi^T (no cancellation in Q = Pinf -
Phi Pinf Phi^T).
"""
import math

import numpy as np


def block_of(x, blocks):
    """index of the closed block [lo, hi] holding x, or -1"""
    for k, (lo, hi) in enumerate(blocks):
        if lo <= x <= hi:
            return k
    return -1


def gp_lnlike_kalman(x, r, ye, ampin, ampout, tau, blocks):
    x, r, ye = (np.asarray(v, dtype=np.float64) for v in (x, r, ye))
    assert np.all(np.diff(x) >= 0), "points must be sorted by phase"
    lam = math.sqrt(3.0 / tau)
    m = np.zeros(4)                    # g, g', h, h'
    D = np.zeros((4, 4))               # P - blockdiag(ampin Pinf1, ampout Pinf1)
    pinf = np.diag([ampin, ampin * lam * lam, ampout, ampout * lam * lam])
    ll = 0.0
    prev_blk = -1
    for i in range(len(x)):
        if i > 0:
            d = x[i] - x[i - 1]
            u = lam * d
            e = math.exp(-u)
            F2 = e * np.array([[1.0 + u, d], [-lam * u, 1.0 - u]])
            F = np.zeros((4, 4))
            F[:2, :2] = F2
            F[2:, 2:] = F2
            m = F @ m
            D = F @ D @ F.T
        blk = block_of(x[i], blocks)
        if blk >= 0 and blk != prev_blk:  # a new block: its process starts stationary
            m[2:] = 0.0
            D[2:, :] = 0.0
            D[:, 2:] = 0.0
        prev_blk = blk
        H = np.array([1.0, 0.0, 1.0 if blk >= 0 else 0.0, 0.0])
        P = D + pinf
        k = P @ H
        S = H @ k + ye[i] * ye[i]
        v = r[i] - H @ m
        ll += v * v / S + math.log(S)
        m = m + k * (v / S)
        D = D - np.outer(k, k) / S
    return -0.5 * (ll + len(x) * math.log(2.0 * math.pi))


def gp_lnlike_kalman_jordan(x, r, ye, ampin, ampout, tau, blocks):
    """The same filter in the coordinates k_gp_like runs it in (MODEL_SPEC
    10.4): with K = [[lam, 1], [-lam^2, -lam]] (K^2 = 0) Phi(d) = e^{-u}
    (I + d K); z = (x0, lam x0 + x1) makes it e^{-u} [[1, d], [0, 1]].  The
    observation is still z0; Pinf = a [[1, lam], [lam, 2 lam^2]]."""
    x, r, ye = (np.asarray(v, dtype=np.float64) for v in (x, r, ye))
    assert np.all(np.diff(x) >= 0), "points must be sorted by phase"
    lam = math.sqrt(3.0 / tau)
    p1 = np.array([[1.0, lam], [lam, 2.0 * lam * lam]])
    pinf = np.zeros((4, 4))
    pinf[:2, :2] = ampin * p1
    pinf[2:, 2:] = ampout * p1
    m = np.zeros(4)
    D = np.zeros((4, 4))
    ll = 0.0
    prev_blk = -1
    for i in range(len(x)):
        if i > 0:
            d = x[i] - x[i - 1]
            e = math.exp(-lam * d)
            F = np.zeros((4, 4))
            F[:2, :2] = F[2:, 2:] = e * np.array([[1.0, d], [0.0, 1.0]])
            m = F @ m
            D = F @ D @ F.T
        blk = block_of(x[i], blocks)
        if blk >= 0 and blk != prev_blk:
            m[2:] = 0.0
            D[2:, :] = 0.0
            D[:, 2:] = 0.0
        prev_blk = blk
        H = np.array([1.0, 0.0, 1.0 if blk >= 0 else 0.0, 0.0])
        k = (D + pinf) @ H
        S = H @ k + ye[i] * ye[i]
        v = r[i] - H @ m
        ll += v * v / S + math.log(S)
        m = m + k * (v / S)
        D = D - np.outer(k, k) / S
    return -0.5 * (ll + len(x) * math.log(2.0 * math.pi))


def gp_lnlike_segments(x, r, ye, ampin, ampout, tau, blocks, K=4):
    """Parallel-in-time form of the same likelihood (k_gp_like's): the points
    are cut into K segments.  Each segment runs the filter conditioned on an
    unknown state x_s (the prior state at its first point): the state mean is
    affine in it (A x_s + c), the covariance starts at 0, and the segment's
    data contribute exp(-1/2 x_s^T J x_s + eta^T x_s - kappa / 2) with J =
    sum hA^T hA / S, eta = sum hA^T v~ / S, kappa = sum (v~^2 / S + log S).
    A sequential pass over the segments then integrates x_s against its
    prior N(mu, Sigma) and carries the filtered end state to the next
    segment.  Jordan coordinates as gp_lnlike_kalman_jordan."""
    x, r, ye = (np.asarray(v, dtype=np.float64) for v in (x, r, ye))
    n = len(x)
    lam = math.sqrt(3.0 / tau)
    p1 = np.array([[1.0, lam], [lam, 2.0 * lam * lam]])
    pinf = np.zeros((4, 4))
    pinf[:2, :2] = ampin * p1
    pinf[2:, 2:] = ampout * p1
    blk = [block_of(v, blocks) for v in x]
    fresh = [blk[i] >= 0 and blk[i] != (blk[i - 1] if i else -1) for i in range(n)]

    def trans(d):
        e = math.exp(-lam * d)
        F = np.zeros((4, 4))
        F[:2, :2] = F[2:, 2:] = e * np.array([[1.0, d], [0.0, 1.0]])
        return F

    keep = np.diag([1.0, 1.0, 0.0, 0.0])
    bounds = [(n * s) // K for s in range(K + 1)]
    elems = []
    for s in range(K):
        i0, i1 = bounds[s], bounds[s + 1]
        A, c, D = np.eye(4), np.zeros(4), -pinf.copy()
        J, eta, kap = np.zeros((4, 4)), np.zeros(4), 0.0
        for i in range(i0, i1):
            if i > i0:
                F = trans(x[i] - x[i - 1])
                A, c, D = F @ A, F @ c, F @ D @ F.T
                if fresh[i]:  # the new block's process: independent of x_s, stationary
                    A, c = keep @ A, keep @ c
                    D = keep @ D @ keep
            H = np.array([1.0, 0.0, 1.0 if blk[i] >= 0 else 0.0, 0.0])
            k = (D + pinf) @ H
            S = H @ k + ye[i] * ye[i]
            hA = H @ A
            vt = r[i] - H @ c
            J += np.outer(hA, hA) / S
            eta += hA * vt / S
            kap += vt * vt / S + math.log(S)
            c = c + k * vt / S
            A = A - np.outer(k, hA) / S
            D = D - np.outer(k, k) / S
        elems.append((A, c, D + pinf, J, eta, kap, i1 - i0))
    ll = 0.0
    mu, Sig = np.zeros(4), pinf.copy()
    for s, (A, c, Pend, J, eta, kap, ns) in enumerate(elems):
        if s > 0:
            i = bounds[s]
            F = trans(x[i] - x[i - 1])
            mu = F @ mu
            Sig = F @ (Sig - pinf) @ F.T + pinf
            if fresh[i]:
                mu = keep @ mu
                Sig = keep @ Sig @ keep + (np.eye(4) - keep) @ pinf
        L = np.linalg.cholesky(Sig)
        B = np.eye(4) + L.T @ J @ L
        M = np.linalg.cholesky(B)
        logdet = 2.0 * np.sum(np.log(np.diag(M)))
        Spost = L @ np.linalg.solve(B, L.T)
        u = eta - J @ mu
        ll += -0.5 * logdet + eta @ mu - 0.5 * mu @ J @ mu + 0.5 * u @ Spost @ u - 0.5 * kap
        mpost = mu + Spost @ u
        mu, Sig = A @ mpost + c, A @ Spost @ A.T + Pend
    return ll - 0.5 * n * math.log(2.0 * math.pi)
