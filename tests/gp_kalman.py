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
