"""Counted FP64 work of k_lnlike per walker-eclipse pair (MODEL_SPEC.md 11.2).

k_lnlike is restated here block phase by block phase (lfit_python_amd/csrc/
lfg.hip, k_lnlike<MODE, SUB>) as counts of the FP64 operations each thread
executes, with MODEL_SPEC 11's rules: add, sub, mul 1; fma 2; div, sqrt,
rcp 1; each transcendental 1 (sincospi = sin + cos = 2); compares,
selects, min / max, conversions, integer and fixed-point (int64) work 0.
The data-dependent counts (eclipsed elements, windows an element only
partly covers, tiles the elements reach, breakpoints met by the sub-bin
lookups) come from simulating the kernel's own decisions on the oracle's
element intervals of the pair (they equal the GPU's to ~1e-13).

Per pair:
  F_like = F_pro + F_tab                      (once per pair)
         + sum over tiles [512 F_thr + m F_pt + F_wdd + F_sd]
         + sum over points F_sub               (SUB: nsub > 1)
with the constants below (C_*), one per code block, cited to the kernel.
"""
import math

import numpy as np

LIKE_THREADS = 512
NWD, NDISC, NBS, NDONOR = 400, 1000, 100, 400
NI = (NWD + NDISC + LIKE_THREADS - 1) // LIKE_THREADS  # sweep slots per thread
TCELLS = 256

# ---- once per pair (prologue, lfg.hip k_lnlike before the tile loop)
C_RING = 4          # wd_ring_weight: fma(kWdA, 1 - ul, kWdB * ul), 10 lanes
C_DONOR_NORM = 5    # dn = max(-s vy + c vz, 0) (3), vs = |vx| + |vy| + |vz| (2), 400 lanes
C_WAVESUM = 6       # one DPP wave sum: 6 adds per lane
C_TWD = 5           # twd = 2 pi ((1 - ul) / 2 + ul / 3), every thread
C_SWN = 2           # swn = wring x (1 / twd or 1 / td), 30 lanes
C_FINISH = 16       # lane 0: chi^2 total over 8 waves (8), -1/2 (1), ln_prob and the Metropolis test (4), draw (3)


def prologue():
    return (10 * C_RING + NDONOR * C_DONOR_NORM + LIKE_THREADS * 3 * C_WAVESUM + 64 * 3 * C_WAVESUM + 2
            + LIKE_THREADS * C_TWD + 30 * C_SWN + C_FINISH)


# ---- per tile, every thread
C_PHASE = 3         # ph0 = x - phi0 (1), phc = wrap_phase (2)
C_PINDEX = 2        # phase_index: span (1), NC / span (1)
C_CHI_WAVE = 7      # chi wave sum (6) + the running per-wave sum (1)
C_SCAN_CONV = 3     # fw, fd, eb: double(r) x 2^-61 (the R3..5 conversions are 0)
C_FLUX1 = 24        # S = 1 per thread: sincospi(2 ph) (1 + 2), e0, e1 (2), D (7), beam (9), sbs, srs (3)
# ---- per tile, every point of the tile
C_WINDOW = 4        # put_window: lo, hi, iw = 1 / (2 hw) (1 + 1)
C_HULL = 2          # phc +- wk against the WD/disc hull (multi-tile / SUB only)
C_CELLS = 4         # build_cells: two ci() of (x - t0) ginv
C_POINT = 15        # flux of the point from its components (11) and its chi^2 term (4)
# ---- the WD/disc sweep of a tile the elements reach (wdd)
C_QUERIES = 2 * NI * 2  # count_lt_multi: 2 NI cell_of = (x - t0) ginv
C_WHOLE = 1         # to_fx(wn) of a whole-covered run
C_PART0 = 1         # a partial window: ov = min(b, hi) - max(a, lo)
C_PART1 = 3         # ... and ov > 0: wn ov iw (2) + to_fx (1)
# ---- S = 1: the spot (window mode) and donor (point mode) sweeps
C_SD_THR = 4        # two phase_index (XW, XP), every thread
C_SPOT_W = 1        # wB = sbw x itb, 100 lanes
C_SPOT_RUNS = 4     # element_runs: two count_below (2 each)
C_DON_HW = 1        # 0.5 - hw of the z-mirrored tiles (200 lanes)
C_DON_Q = 6         # three to_fx(v ivs)
C_DON_ARC = 2       # lo, hi
C_DON_WRAP = 1      # the wrapped interval's end
C_DON_SEARCH = 4    # count_below x 2 per interval
# ---- SUB: the breakpoint tables (once per pair) and the sub-bin lookups
C_TAB_THR = 4       # dginv, sginv
C_TAB_PT0 = 2       # a0 = x - phi0, hp = w / S
C_TAB_SUB = 5       # a sub-bin centre: (2j + 1) hp, a0 - wp, +, wrap (2)
C_TAB_DON = 3       # lane_breakpoints' arc (lo, hi, 0.5 - hw of mirrored tiles) x 2 calls + donor_q (3)
C_TCELL = 2         # tcell: (x - t0) ginv
C_SUBPT = 2 + 4     # h = wk / S, 1 / (2 h); the point's sums: / bden (1), x FX_INV VN[3] / VN[2] (3)
C_SUBJ = 5 + 2 + 2 + 6 + 8 + 3       # centre (5), window lo / hi (2), e0 e1 (2), D (3 fma), beam (8), sbs (3)
C_FRESH = 2 + 6     # a fresh lookup: tcell (2) + sincospi2 (2 muls + 4)
C_STEP = 6          # a carried sub-bin: the cursor's compare (0) + the rotation (6)
C_DQ = 3            # donor_q of a counted entry
C_SPOT_IN = 3       # a sub-bin window inside the spot hull: E = C FX_INV + corr / (2 h) (fma)
C_SPOT_INIT = 2     # the spot cursor's start: tcell (2) ...
C_SPOT_C = 1        # ... and each counted entry of the cell: wn = sbw itb
C_SPOT_CORR = 4     # an entry inside the window: wn (1), overlap (1), fma (2)


def wrap(ph):
    return ph - np.floor(ph + 0.5)


def count_pair(x, w, nsub, a, b, sa, sb, donor, inc_deg, phi0, gp=False):
    """Counted FP64 FLOPs of k_lnlike for one pair.  x, w: the eclipse's
    points (kernel order); a, b: the 1400 WD/disc intervals (oracle order;
    the mirror of each unique item is among them); sa, sb: the 100 spot
    intervals; donor [400, 3]: the tile vectors."""
    n, S = len(x), int(nsub)
    sub = S > 1
    T = -(-n // LIKE_THREADS)
    hull = sub or n > LIKE_TILE_N
    ecl = a < b
    ea, eb = a[ecl], b[ecl]
    wa, wb = (ea.min(), eb.max()) if ecl.any() else (np.inf, -np.inf)
    secl = sa < sb
    ssa, ssb = sa[secl], sb[secl]
    s_, c_ = math.sin(math.radians(inc_deg)), math.cos(math.radians(inc_deg))
    vx, vy, vz = donor[:, 0], donor[:, 1], donor[:, 2]
    srho = s_ * np.hypot(vx, vy)
    with np.errstate(divide="ignore", invalid="ignore"):
        kap = np.where(srho > 0, -c_ * vz / srho, np.where(c_ * vz > 0, -2.0, 2.0))
    cen = -np.arctan2(vy, vx) / (2 * math.pi)
    hw = np.arccos(np.clip(kap, -1.0, 1.0)) / (2 * math.pi)
    ph_all = wrap(x - phi0)
    hw_all = w if w is not None else np.zeros(n)

    f = prologue()
    parts = {"prologue": f, "tables": 0.0, "tiles_thread": 0.0, "tiles_point": 0.0, "wd_disc": 0.0,
             "spot_donor": 0.0, "subbins": 0.0}
    if sub:  # table build (lfg.hip k_lnlike, `if (TAB)`)
        ft = LIKE_THREADS * C_TAB_THR + n * (C_TAB_PT0 + C_TAB_SUB * S)
        alive = hw > 0
        ft += int(alive.sum()) * (C_TAB_DON + 2 * 2 * C_TCELL) + int(secl.sum()) * (2 + 2 * 2 * C_TCELL)
        parts["tables"] = ft
        f += ft
    for t in range(T):
        sl = slice(t * LIKE_THREADS, min(n, (t + 1) * LIKE_THREADS))
        ph, h = ph_all[sl], hw_all[sl]
        m = len(ph)
        lo, hi = ph - h, ph + h
        thr = C_PHASE + C_PINDEX + C_CHI_WAVE + (0 if sub else C_PINDEX)
        pt = C_WINDOW + C_CELLS + (C_HULL if hull else 0) + (0 if sub else C_CELLS) + C_POINT
        parts["tiles_thread"] += LIKE_THREADS * thr
        parts["tiles_point"] += m * pt
        f += LIKE_THREADS * thr + m * pt
        wdd = (not hull) or bool(np.any((hi >= wa) & (lo <= wb)))
        if wdd:  # the WD/disc sweep over the tile's windows
            fw = LIKE_THREADS * (C_PINDEX + C_QUERIES)
            for aa, bb in zip(ea, eb):
                P2, P4 = np.searchsorted(lo, aa, "left"), np.searchsorted(lo, bb, "left")
                P1, P3 = np.searchsorted(hi, aa, "right"), np.searchsorted(hi, bb, "right")
                if P2 < P3:
                    fw += C_WHOLE
                    rng = list(range(P1, P2)) + list(range(P3, P4))
                else:
                    rng = range(P1, P4)
                for p in rng:
                    ov = min(bb, hi[p]) - max(aa, lo[p])
                    fw += C_PART0 + (C_PART1 if ov > 0 else 0)
            parts["wd_disc"] += fw
            f += fw
        if not sub:  # S = 1: spot / donor sweeps, the scan, the flux per thread
            fs = LIKE_THREADS * (C_SD_THR + C_SCAN_CONV + C_FLUX1) + NBS * C_SPOT_W
            for aa, bb in zip(ssa, ssb):
                fs += C_SPOT_RUNS
                P2, P4 = np.searchsorted(lo, aa, "left"), np.searchsorted(lo, bb, "left")
                P1, P3 = np.searchsorted(hi, aa, "right"), np.searchsorted(hi, bb, "right")
                if P2 < P3:
                    fs += C_WHOLE
                    rng = list(range(P1, P2)) + list(range(P3, P4))
                else:
                    rng = range(P1, P4)
                for p in rng:
                    ov = min(bb, hi[p]) - max(aa, lo[p])
                    fs += C_PART0 + (C_PART1 if ov > 0 else 0)
            fs += 200 * C_DON_HW
            for c0, h0 in zip(cen, hw):
                if not h0 > 0:
                    continue
                fs += C_DON_Q
                if h0 < 0.5:
                    fs += C_DON_ARC
                    two = (c0 - h0 < -0.5) or (c0 + h0 > 0.5)
                    fs += (C_DON_WRAP + 2 * C_DON_SEARCH) if two else C_DON_SEARCH
                else:
                    fs += C_DON_SEARCH
            parts["spot_donor"] += fs
            f += fs
        else:
            f += LIKE_THREADS * C_SCAN_CONV
            parts["spot_donor"] += LIKE_THREADS * C_SCAN_CONV
    if sub:  # the sub-bin lookups of every point (sub_point)
        f += _subbins(ph_all, hw_all, S, cen, hw, ssa, ssb, parts)
    if gp:  # k_lnlike<2>: e^{-lam dx} and the block of each point (5), a residual instead of chi^2 (1 - 4)
        f += n * (5 + 1 - 4)
    parts = {k: float(v) for k, v in parts.items()}
    return float(f), parts


LIKE_TILE_N = LIKE_THREADS


def _subbins(ph_all, hw_all, S, cen, hw, ssa, ssb, parts):
    """sub_point over every point: cell-table lookups as the kernel makes
    them (the donor cells span every sub-bin centre of the pair)"""
    n = len(ph_all)
    cs = np.array([[wrap(ph_all[p] - hw_all[p] + (2 * j + 1) * hw_all[p] / S) for j in range(S)] for p in range(n)])
    t0, t1 = cs.min(), cs.max()
    ginv = TCELLS / (t1 - t0) if t1 > t0 else 0.0
    # donor breakpoints inside the cells' range, by kind (start counted for
    # th > pos, end for th >= pos), as lane_breakpoints forms them
    bps, kinds = [], []
    for c0, h0 in zip(cen, hw):
        if not h0 > 0 or h0 >= 0.5:
            continue
        lo, hi = c0 - h0, c0 + h0
        if lo < -0.5:
            sp, ep = lo + 1.0, hi
        elif hi > 0.5:
            sp, ep = lo, hi - 1.0
        else:
            sp, ep = lo, hi
        if t0 <= sp < t1:
            bps.append(sp); kinds.append(0)
        if t0 < ep <= t1:
            bps.append(ep); kinds.append(1)
    bps, kinds = np.array(bps), np.array(kinds)

    def cell(v):
        u = (v - t0) * ginv
        return np.where(u <= 0, 0, np.where(u >= TCELLS - 1, TCELLS - 1, np.floor(u))).astype(int)
    bcell = cell(bps) if len(bps) else np.zeros(0, int)
    # spot: the hull and its cells
    sa_min, sb_max = (ssa.min(), ssb.max()) if len(ssa) else (np.inf, -np.inf)
    sginv = TCELLS / (sb_max - sa_min) if sb_max > sa_min else 0.0
    spos = np.concatenate([ssa, ssb]) if len(ssa) else np.zeros(0)
    sfrom_a = np.concatenate([np.ones(len(ssa), bool), np.zeros(len(ssb), bool)])
    ssa2 = np.concatenate([ssa, ssa]) if len(ssa) else np.zeros(0)

    def scell(v):
        u = (v - sa_min) * sginv
        return np.where(u <= 0, 0, np.where(u >= TCELLS - 1, TCELLS - 1, np.floor(u))).astype(int)
    scl = scell(spos) if len(spos) else np.zeros(0, int)
    order = np.argsort(spos, kind="stable") if len(spos) else np.zeros(0, int)
    spos_s = spos[order] if len(spos) else spos
    f = 0.0
    for p in range(n):
        f += C_SUBPT
        h = hw_all[p] / S
        prev = None
        sv = False
        for j in range(S):
            th = cs[p, j]
            f += C_SUBJ
            if prev is None or not th >= prev:
                sv = False
                g = cell(np.array([th]))[0]
                sel = bcell == g
                cnt = int(np.sum(np.where(kinds[sel] == 1, bps[sel] <= th, bps[sel] < th)))
                f += C_FRESH + C_DQ * cnt
            else:
                sel = (bps >= prev) & (bps <= th)
                cnt = int(np.sum(np.where(kinds == 1, (bps > prev) & (bps <= th), (bps >= prev) & (bps < th))))
                f += C_STEP + C_DQ * cnt
            prev = th
            lo, hi = th - h, th + h
            inside = (hi > sa_min and lo < sb_max) and h > 0 and len(spos)
            if inside:  # the spot cursor (sub_point)
                f += C_SPOT_IN
                if not sv:
                    g0 = scell(np.array([lo]))[0]
                    f += C_SPOT_INIT + C_SPOT_C * int(np.sum(spos[scl == g0] <= lo))
                sv = True
                f += C_SPOT_CORR * int(np.searchsorted(spos_s, hi, "right") - np.searchsorted(spos_s, lo, "right"))
            else:
                sv = False
    parts["subbins"] += f
    return f
