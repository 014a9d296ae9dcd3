// lfg_device.hpp -- gfx950 device functions for the CV eclipse light-curve
// model (MODEL_SPEC.md).  FP64 throughout.  Each function carries the
// MODEL_SPEC section it implements; the CPU oracle (oracle/lfg_oracle.c) is an
// independent restatement of the same spec used only to check these.
//
// Reference behaviour replaced: lfit.CV.calcFlux (CVModel.py:138) and the
// trm.roche primitives xl1/findphi/findi/bspot (CVModel.py:222,288,460,561).
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>

#include "lfg_stream_table.h"

namespace lfg {

constexpr double PI = 3.14159265358979323846;
constexpr double TWO_PI = 6.28318530717958647693;
constexpr double DEG = PI / 180.0;
constexpr double LN2 = 0.69314718055994530942;

// MODEL_SPEC.md section 7
constexpr double RAY_TOL = 1e-13;
constexpr int RAY_MAXIT = 100;
constexpr double TH_TOL = 1e-13;
constexpr int ROOT_MAXIT = 100;
// 1-D safeguarded Newton (L1, donor radius, stream crossing) stops after a
// Newton step of at most ROOT_LAST: convergence is quadratic, so the error
// left is ~ROOT_LAST^2.  (A tolerance near machine precision stalls on
// rounding noise and falls back to bisection for tens of iterations.)
constexpr double ROOT_LAST = 1e-9;
constexpr int MIN_MAXIT = 100;
constexpr double BS_TAIL = 16.0;
constexpr double STREAM_DELTA = 1e-2;
// outside the stream table: RK4 with dt = min(0.15, 0.15 r^1.5) / 32
// (converged to ~1e-12 a)
constexpr double STREAM_KAPPA_FINE = 0.15 / 32.0;
constexpr double STREAM_DTMAX_FINE = 0.15 / 32.0;
constexpr int STREAM_MAXSTEP_FINE = 128000;
constexpr double DISC_MAX_A = 0.46;  // CVModel.py:217
constexpr double AZ_SLOPE = 80.0;    // CVModel.py:282
constexpr double DPHI_TOL = 1e-6;    // CVModel.py:452

constexpr int NWD_RINGS = 10;
constexpr int NWD = 400;
constexpr int NDISC_R = 20;
constexpr int NDISC_AZ = 50;
constexpr int NDISC = 1000;
constexpr int NBS = 100;
constexpr int NDONOR_T = 20;
constexpr int NDONOR_P = 20;
constexpr int NDONOR = 400;
constexpr int NEL = NWD + NDISC + NBS;      // eclipsable elements
constexpr int NALL = NEL + NDONOR;          // + donor tiles

enum Status { ST_OK = 0, ST_BAD_Q = 1, ST_BAD_DPHI = 2, ST_BAD_GEOMETRY = 3,
              ST_BAD_STREAM = 4, ST_BAD_ARGS = 5 };

// geometry record written by the setup kernel, one per (walker, eclipse)
enum Geo {
    G_Q, G_CA, G_CB, G_MU, G_XL1, G_PL1, G_RS, G_RS2,
    G_S, G_C, G_INC, G_RWD, G_RDISC, G_REFF, G_ULIMB, G_DEXP,
    G_BSX, G_BSY, G_BSVX, G_BSVY, G_L, G_UPK, G_UMAX, G_LNPK,
    G_EXP1, G_EXP2, G_CAZ, G_SAZ, G_NB0, G_NB1, G_NB2, G_BDEN,
    G_FIS, G_PHI0, G_WDF, G_DF, G_SF, G_RSF, G_RPRIOR, G_RCAL,
    G_RPRIOR_BS,  // bright-spot part of the eclipse Roche prior (stream lanes)
    G_GP_AIN, G_GP_AOUT, G_GP_LAM, G_GP_DCP, G_GP_OK,  // GP likelihood (MODEL_SPEC 10)
    G_GP_DPHI, G_GP_RWD,  // a changepoint distance pending (G_GP_OK = 2): the walker's dphi, rwd for k_gp_dcp
    G_COUNT
};
static_assert(G_COUNT <= 48, "LFG_NGEO");

struct Roche {
    double q, cA, cB, mu, xl1, pl1, Rs, Rs2;
};

// 1/sqrt(x) for finite x > 0: v_rsq_f64 and one third-order correction (the
// ocml form without its zero/infinity select, which adds a dependent level;
// a lone stream wave is bound by dependent FP64 latency, ~30 cycles a level)
__device__ __forceinline__ double rsqrt_pos(double x)
{
    const double y = __builtin_amdgcn_rsq(x);
    const double e = fma(-x * y, y, 1.0);
    return fma(y * e, fma(e, 0.375, 0.5), y);
}

// 1/x for finite x != 0: v_rcp_f64 and one Newton correction (the IEEE
// quotient's div_scale/div_fmas/div_fixup sequence is ~10 issue slots; a
// Newton step only needs its length to a few ulp -- the root it converges to
// is fixed by F = 0, not by the step; on the serial setup chains every IEEE
// quotient is ~7 dependent levels more than this)
__device__ __forceinline__ double rcp_fast(double x)
{
    const double y = __builtin_amdgcn_rcp(x);
    return fma(y, fma(-x, y, 1.0), y);
}

// 1/x for a Newton step's length only (the step's direction and size need a
// few digits: the root is fixed by F = 0, and a relative error e in the
// step leaves e |dth| after it, ~1e-7 x 3e-8 at the last step): the raw
// v_rcp_f64.
__device__ __forceinline__ double rcp_step(double x)
{
    return __builtin_amdgcn_rcp(x);
}

__device__ __forceinline__ double rpot(const Roche& R, double x, double y, double z)
{
    const double dx = x - 1.0;
    const double xc = x - R.mu;
    return -R.cA * rsqrt(x * x + y * y + z * z) - R.cB * rsqrt(dx * dx + y * y + z * z)
           - xc * xc - y * y;
}

// Phi and grad Phi at one point, sharing the two rsqrt
__device__ __forceinline__ double rpot_grad(const Roche& R, double x, double y, double z, double& gx, double& gy,
                                            double& gz)
{
    const double ir1 = rsqrt(x * x + y * y + z * z);
    const double dx = x - 1.0;
    const double ir2 = rsqrt(dx * dx + y * y + z * z);
    const double i1 = R.cA * ir1 * ir1 * ir1, i2 = R.cB * ir2 * ir2 * ir2;
    const double xc = x - R.mu;
    gx = i1 * x + i2 * dx - 2.0 * xc;
    gy = (i1 + i2 - 2.0) * y;
    gz = (i1 + i2) * z;
    return -R.cA * ir1 - R.cB * ir2 - xc * xc - y * y;
}

__device__ __forceinline__ void rgrad(const Roche& R, double x, double y, double z,
                                      double& gx, double& gy, double& gz)
{
    const double ir1 = rsqrt(x * x + y * y + z * z);
    const double i1 = R.cA * ir1 * ir1 * ir1;
    const double dx = x - 1.0;
    const double ir2 = rsqrt(dx * dx + y * y + z * z);
    const double i2 = R.cB * ir2 * ir2 * ir2;
    gx = i1 * x + i2 * dx - 2.0 * (x - R.mu);
    gy = (i1 + i2 - 2.0) * y;
    gz = (i1 + i2) * z;
}

// Patch of ln q in the q series of lfg_stream_table.h (tools/gen_stream_table.py):
// iq < 0 when q lies outside [LFG_ST_QLO, LFG_ST_QHI]
struct QPatch {
    int iq;
    double xq;
};

__constant__ const double kStXl1[LFG_ST_NQ * (LFG_ST_DR + 1)] = LFG_ST_XL1;
__constant__ const double kStPhi90[LFG_ST_NQ * (LFG_ST_DR + 1)] = LFG_ST_PHI90;

// Clenshaw sum of c[0..n-1] T_k(x)
template <int N>
__device__ __forceinline__ double clenshaw(const double* c, double x)
{
    const double x2 = x + x;
    double b1 = 0.0, b2 = 0.0;
#pragma unroll
    for (int k = N - 1; k >= 1; --k) {
        const double t = fma(x2, b1, c[k] - b2);
        b2 = b1;
        b1 = t;
    }
    return fma(x, b1, c[0] - b2);
}

__device__ inline QPatch q_patch(double q)
{
    if (!(q >= LFG_ST_QLO && q <= LFG_ST_QHI)) return QPatch{-1, 0.0};
    const double fq = (log(q) - LFG_ST_LQLO) * (1.0 / LFG_ST_LQW);
    const int iq = min(max(int(fq), 0), LFG_ST_NQ - 1);
    return QPatch{iq, 2.0 * (fq - iq) - 1.0};
}

// a 1-D q series of the table (LFG_ST_XL1, LFG_ST_PHI90, LFG_ST_RMIN layout)
__device__ __forceinline__ double q_series(const double* tab, const QPatch& p)
{
    return clenshaw<LFG_ST_DR + 1>(tab + p.iq * (LFG_ST_DR + 1), p.xq);
}

// MODEL_SPEC 4.1: L1 point, safeguarded Newton on dPhi/dx (monotone on (0,1)),
// from x0: the q series of xl1 (within ~1e-16: one Newton step confirms it)
// or 1 - (mu/3)^(1/3)
__device__ inline double xl1_solve(double q, double x0)
{
    const double i1q = rcp_fast(1.0 + q);
    const double cA = 2.0 * i1q, cB = q * cA, mu = q * i1q;
    double lo = 0.0, hi = 1.0;
    double x = (x0 > 0.0 && x0 < 1.0) ? x0 : 1.0 - cbrt(mu * (1.0 / 3.0));
    for (int it = 0; it < 200; ++it) {
        const double omx = 1.0 - x;
        const double ix = rcp_fast(x), io = rcp_fast(omx);
        const double f = cA * ix * ix - cB * io * io - 2.0 * (x - mu);
        const double df = -2.0 * cA * ix * ix * ix - 2.0 * cB * io * io * io - 2.0;
        if (f > 0.0) lo = x; else hi = x;
        const double step = f * rcp_fast(df);
        if (fabs(step) <= ROOT_LAST) { x -= step; break; }  // converged: last Newton step
        double xn = x - step;
        if (!(xn > lo && xn < hi)) xn = 0.5 * (lo + hi);
        x = xn;
    }
    return x;
}

// qp (nullable) receives q's table patch for later lookups (bspot)
__device__ inline int roche_init(Roche& R, double q, QPatch* qp = nullptr)
{
    if (!(q > 0.0) || !isfinite(q)) return ST_BAD_Q;
    R.q = q;
    const double i1q = rcp_fast(1.0 + q);
    R.cA = 2.0 * i1q;
    R.cB = q * R.cA;
    R.mu = q * i1q;
    const QPatch p = q_patch(q);
    if (qp) *qp = p;
    R.xl1 = xl1_solve(q, p.iq >= 0 ? q_series(kStXl1, p) : -1.0);
    R.pl1 = rpot(R, R.xl1, 0.0, 0.0);
    R.Rs = 1.0 - R.xl1;
    R.Rs2 = R.Rs * R.Rs;
    return ST_OK;
}

__device__ inline double eggleton(double q)
{
    const double q3 = cbrt(q), q23 = q3 * q3;
    return 0.49 * q23 / (0.6 * q23 + log(1.0 + q3));
}

// MODEL_SPEC 4.2: minimum of Phi along P + t e over the chord of the sphere
// |X - D| <= Rs.  Uses X.e = P.e + t (|e| = 1) so each Newton iteration
// needs two rsqrt and one division.
__device__ inline bool ray_min(const Roche& R, double Px, double Py, double Pz,
                               double ex, double ey, double ez, double& tw, double& fmin)
{
    const double ux = 1.0 - Px, uy = -Py, uz = -Pz;
    const double tc = ux * ex + uy * ey + uz * ez;
    const double b2 = ux * ux + uy * uy + uz * uz - tc * tc;
    if (b2 >= R.Rs2) return false;
    const double h = sqrt(R.Rs2 - b2);
    double lo = tc - h, hi = tc + h;
    if (hi <= 0.0) return false;
    lo = fmax(lo, 0.0);
    double t = tw;
    if (!(t > lo && t < hi)) t = (tc > lo && tc < hi) ? tc : 0.5 * (lo + hi);
    const double Pe = Px * ex + Py * ey + Pz * ez;
    const double exy2 = 2.0 * (ex * ex + ey * ey);
    for (int it = 0; it < RAY_MAXIT; ++it) {
        const double x = fma(t, ex, Px), y = fma(t, ey, Py), z = fma(t, ez, Pz);
        const double r1s = x * x + y * y + z * z;
        const double ir1 = rsqrt(r1s);
        const double ir1s = ir1 * ir1;
        const double i1 = R.cA * ir1s * ir1;
        const double dx = x - 1.0;
        const double ir2 = rsqrt(dx * dx + y * y + z * z);
        const double ir2s = ir2 * ir2;
        const double i2 = R.cB * ir2s * ir2;
        const double p1 = Pe + t;
        const double p2 = p1 - ex;
        const double f1 = i1 * p1 + i2 * p2 - 2.0 * ((x - R.mu) * ex + y * ey);
        const double f2 = i1 * (1.0 - 3.0 * p1 * p1 * ir1s) + i2 * (1.0 - 3.0 * p2 * p2 * ir2s) - exy2;
        if (f1 > 0.0) hi = t; else lo = t;
        double tn = (f2 > 0.0) ? t - f1 / f2 : 0.5 * (lo + hi);
        if (!(tn > lo && tn < hi)) tn = 0.5 * (lo + hi);
        const double d = tn - t;
        t = tn;
        if (fabs(d) <= RAY_TOL) break;
    }
    tw = t;
    fmin = rpot(R, fma(t, ex, Px), fma(t, ey, Py), fma(t, ez, Pz));
    return true;
}

// g(theta) = min Phi - Phi_L1 along the line of sight at orbital angle theta
// (MODEL_SPEC 4.3); dg by the envelope theorem.  Miss: g = +1, dg = 0.
__device__ inline bool g_eval(const Roche& R, double Px, double Py, double Pz,
                              double s, double c, double th, double& tw,
                              double& g, double& dg)
{
    double sn, cs;
    sincos(th, &sn, &cs);
    const double ex = s * cs, ey = -s * sn;
    double fm;
    if (!ray_min(R, Px, Py, Pz, ex, ey, c, tw, fm)) {
        g = 1.0;
        dg = 0.0;
        return false;
    }
    double gx, gy, gz;
    rgrad(R, fma(tw, ex, Px), fma(tw, ey, Py), fma(tw, c, Pz), gx, gy, gz);
    g = fm - R.pl1;
    dg = tw * (gx * (-s * sn) + gy * (-s * cs));
    return true;
}

__device__ inline double theta_root(const Roche& R, double Px, double Py, double Pz,
                                    double s, double c, double lo, double hi, bool pos_lo,
                                    double th, double& tw)
{
    if (!(th > lo && th < hi)) th = 0.5 * (lo + hi);
    for (int it = 0; it < ROOT_MAXIT; ++it) {
        double g, dg;
        g_eval(R, Px, Py, Pz, s, c, th, tw, g, dg);
        if ((g > 0.0) == pos_lo) lo = th; else hi = th;
        double tn = (dg != 0.0) ? th - g / dg : 0.5 * (lo + hi);
        if (!(tn > lo && tn < hi)) tn = 0.5 * (lo + hi);
        const double d = tn - th;
        th = tn;
        if (fabs(d) <= TH_TOL) break;
    }
    return th;
}

// MODEL_SPEC 4.3: eclipse interval [a, b] (phase units) of the point P.
// Returns false (a = 1, b = -1) when P is never eclipsed.
__device__ inline bool element_interval(const Roche& R, double Px, double Py, double Pz,
                                        double s, double c, double Reff, double& a, double& b)
{
    a = 1.0;
    b = -1.0;
    const double ux = 1.0 - Px, uy = -Py, uz = -Pz;
    const double uxy = sqrt(ux * ux + uy * uy);
    const double uu = ux * ux + uy * uy + uz * uz;
    if (uu <= R.Rs2 || uxy <= 0.0 || s <= 0.0) return false;
    const double thc = atan2(-uy, ux);
    const double cosD = (sqrt(uu - R.Rs2) - c * uz) / (s * uxy);
    if (!(cosD < 1.0)) return false;  // never eclipsed (or non-finite geometry: no Newton on NaN)
    const double Dm = (cosD <= -1.0) ? PI : acos(cosD);
    const double lo = thc - Dm, hi = thc + Dm;

    double tw = -1.0, g, dg;
    bool chord = g_eval(R, Px, Py, Pz, s, c, thc, tw, g, dg);
    if (!chord) return false;
    double thi = thc;
    if (!(g < 0.0)) {
        bool found = false, have = false;
        double th = thc, pth = 0.0, pdg = 0.0, mlo = lo, mhi = hi;
        for (int it = 0; it < MIN_MAXIT; ++it) {
            if (chord) {
                if (g < 0.0) { found = true; thi = th; break; }
                if (dg > 0.0) mhi = th; else mlo = th;
            } else {
                if (th < thc) mlo = th; else mhi = th;
            }
            double tn = (chord && have && dg != pdg) ? th - dg * (th - pth) / (dg - pdg)
                                                     : 0.5 * (mlo + mhi);
            if (!(tn > mlo && tn < mhi)) tn = 0.5 * (mlo + mhi);
            if (fabs(tn - th) <= TH_TOL) break;
            if (chord) { pth = th; pdg = dg; have = true; }
            th = tn;
            chord = g_eval(R, Px, Py, Pz, s, c, th, tw, g, dg);
        }
        if (!found) return false;
    }
    double de;
    const double ce = (sqrt(fmax(uu - Reff * Reff, 0.0)) - c * uz) / (s * uxy);
    de = (ce > -1.0 && ce < 1.0) ? acos(ce) : 0.5 * Dm;
    double twi = tw, two = tw;
    const double thin = theta_root(R, Px, Py, Pz, s, c, lo, thi, true, thc - de, twi);
    const double thout = theta_root(R, Px, Py, Pz, s, c, thi, hi, false, thc + de, two);
    a = thin * (1.0 / TWO_PI);
    b = thout * (1.0 / TWO_PI);
    return true;
}

// ---------------------------------------------------------------------------
// Fast path for element_interval (same converged answer, ~10x less work).
// The contact phases are the tangencies of the line of sight with the lobe
// surface: F1 = Phi(X) - Phi_L1 = 0 and F2 = grad Phi(X).e = 0 at
// X = P + t e(theta), solved by 2-D Newton in (theta, t).  With
// e_theta = de/dtheta = (e_y, -e_x, 0) the Jacobian needs only scalars:
//   J11 = t grad.e_th, J12 = F2, J21 = t e_th.H.e + grad.e_th, J22 = e.H.e
// Existence is decided by Newton minimisation of Phi over the cone of lines
// of sight (theta, t), which stops as soon as a point inside the lobe is seen.
// Anything not cleanly converged falls back to the nested solver above.
struct ConePt {
    double phi, gth, F2, eHe, etHe, ethHeth, gtt, dX2;
};

// direction given by (cos theta, sin theta): no trig inside the Newton loops
__device__ __forceinline__ void cone_point(const Roche& R, double Px, double Py, double Pz, double s,
                                           double c, double cs, double sn, double t, ConePt& o)
{
    const double ex = s * cs, ey = -s * sn;
    const double x = fma(t, ex, Px), y = fma(t, ey, Py), z = fma(t, c, Pz);
    const double r1s = x * x + y * y + z * z;
    const double ir1 = rsqrt_pos(r1s), ir1s = ir1 * ir1;
    const double dx = x - 1.0;
    const double r2s = dx * dx + y * y + z * z;
    const double ir2 = rsqrt_pos(r2s), ir2s = ir2 * ir2;
    const double i1 = R.cA * ir1s * ir1, i2 = R.cB * ir2s * ir2, i12 = i1 + i2;
    const double xm = x - R.mu;
    o.phi = -R.cA * ir1 - R.cB * ir2 - xm * xm - y * y;
    const double gx = i1 * x + i2 * dx - 2.0 * xm;
    const double gy = (i12 - 2.0) * y;
    const double gz = i12 * z;
    const double p1 = x * ex + y * ey + z * c, p2 = p1 - ex;
    const double q1 = x * ey - y * ex, q2 = q1 - ey;
    const double k1 = 3.0 * i1 * ir1s, k2 = 3.0 * i2 * ir2s;
    const double s2 = ex * ex + ey * ey;
    o.F2 = gx * ex + gy * ey + gz * c;
    o.gth = gx * ey - gy * ex;
    o.eHe = i12 - k1 * p1 * p1 - k2 * p2 * p2 - 2.0 * s2;
    o.etHe = -k1 * p1 * q1 - k2 * p2 * q2;
    o.ethHeth = i12 * s2 - k1 * q1 * q1 - k2 * q2 * q2 - 2.0 * s2;
    o.gtt = -(gx * ex + gy * ey);
    o.dX2 = r2s;
}

// rotate (cs, sn) by d, |d| <= 0.05: Taylor series, error < 1e-20
__device__ __forceinline__ void rotate(double& cs, double& sn, double d)
{
    const double d2 = d * d;
    const double sd = d * (1.0 - d2 * (1.0 / 6.0) * (1.0 - d2 * (1.0 / 20.0) * (1.0 - d2 * (1.0 / 42.0) *
                                                                              (1.0 - d2 * (1.0 / 72.0)))));
    const double cd = 1.0 - d2 * 0.5 * (1.0 - d2 * (1.0 / 12.0) * (1.0 - d2 * (1.0 / 30.0) *
                                                                    (1.0 - d2 * (1.0 / 56.0) * (1.0 - d2 * (1.0 / 90.0)))));
    const double c2 = cs * cd - sn * sd;
    sn = fma(sn, cd, cs * sd);
    cs = c2;
}

// 2-D Newton for one contact phase.  Tan holds the running angle th, its
// cosine and sine (advanced by rotation), the distance t along the line of
// sight and the state: 0 running, 1 converged to a tangency of the right kind
// (ingress: g falling with theta), -1 failed.
//
// Each step is Newton on the envelope g(th) = min_t Phi - Phi_L1 evaluated
// at one point: t moves to the ray's minimum of Phi (dt0 = -F2 / J22), which
// lowers F1 by F2^2 / (2 J22), and th takes the Newton step of that corrected
// F1 with the envelope slope J11 + J21 dt0; t then follows th along the
// valley (dt = dt0 - J21 / J22 dth).  In the joint 2-D step a t error leaks
// into th at first order, here only at second order.
// The first step is Halley's on the envelope (g'' = F1_thth - F1_tht^2 /
// F1_tt, the Schur complement; F1_thth = t^2 e_th.H.e_th + t grad.e_thth):
// from the sphere guesses (1e-3..1e-2 rad off) it lands ~1e-7..1e-5 off, so
// most contacts stop after a second, Newton, step.  t starts at the ray's
// minimum of Phi to first order (element_interval_fast), not at the closest
// approach to D (~1e-2 off): with t that far off the second step's |dt| kept
// a third step in play (tools/tol_study.py: k_elements' wave-max steps per
// lane 4.27 -> 3.43 at config 2, interval errors < 3e-12 in phase).
// Stop once |dth| <= TH_LAST (th error ~TH_LAST^2 after a Newton step) and
// |dt| <= T_LAST (t errors reach th at second order): ~1e-12 rad (MODEL_SPEC 7).
#ifndef LFG_TH_LAST
#define LFG_TH_LAST 1e-6
#endif
#ifndef LFG_T_LAST
#define LFG_T_LAST 3e-5
#endif
constexpr double TH_LAST = LFG_TH_LAST;
constexpr double T_LAST = LFG_T_LAST;

struct Tan {
    double th, cs, sn, t;
    int st;
};

// one branch-free step (two solves can run interleaved in one lane);
// HALLEY: the curvature-corrected first step
template <bool HALLEY = false>
__device__ __forceinline__ void tangency_step(const Roche& R, double Px, double Py, double Pz, double s, double c,
                                              bool ingress, Tan& T)
{
    ConePt o;
    cone_point(R, Px, Py, Pz, s, c, T.cs, T.sn, T.t, o);
    const double F1 = o.phi - R.pl1;
    const double J11 = T.t * o.gth;
    const double J21 = T.t * o.etHe + o.gth, J22 = o.eHe;
    const double iJ22 = rcp_step(J22);
    const double dt0 = -o.F2 * iJ22;
    const double F1m = fma(0.5 * o.F2, dt0, F1);  // F1 - F2^2 / (2 J22)
    const double den = fma(J21, dt0, J11);
    const bool bad = !(J22 != 0.0) || !(den != 0.0);
    const double iden = rcp_step(den);
    double dth = -F1m * iden;
    if (HALLEY) {  // dth / (1 + dth g'' / (2 g')); plain Newton where that factor is far from 1
        const double g2 = fma(T.t, fma(T.t, o.ethHeth, o.gtt), -J21 * J21 * iJ22);
        const double h = 0.5 * dth * g2 * iden;
        if (fabs(h) < 0.5) dth = dth * rcp_step(1.0 + h);
    }
    dth = fmin(fmax(dth, -0.05), 0.05);
    const double dt = fma(-J21 * iJ22, dth, dt0);
    T.th += dth;
    T.t += dt;
    const bool conv = fabs(dth) <= TH_LAST && fabs(dt) <= T_LAST;
    const bool good = J22 > 0.0 && ((J11 < 0.0) == ingress) && T.t > 0.0 && o.dX2 < R.Rs2;
    rotate(T.cs, T.sn, dth);
    T.st = bad ? -1 : (conv ? (good ? 1 : -1) : 0);
}

// one contact phase on its own; false unless cleanly converged
__device__ inline bool tangency(const Roche& R, double Px, double Py, double Pz, double s, double c,
                                bool ingress, double& th, double cs, double sn, double& t, int* nit = nullptr)
{
    Tan T{th, cs, sn, t, 0};
    for (int it = 0; it < 16 && T.st == 0; ++it) {
        if (nit) ++*nit;  // diagnostic builds only
        tangency_step(R, Px, Py, Pz, s, c, ingress, T);
    }
    th = T.th;
    t = T.t;
    return T.st == 1;
}

// ingress and egress in lockstep: two independent dependency chains per lane
__device__ inline void tangency_pair(const Roche& R, double Px, double Py, double Pz, double s, double c, Tan& A,
                                     Tan& B, int* nit = nullptr)
{
    tangency_step<true>(R, Px, Py, Pz, s, c, true, A);  // both start running: no lockstep copies
    tangency_step<true>(R, Px, Py, Pz, s, c, false, B);
    if (nit) { nit[0] += 1; nit[1] += 1; }  // diagnostic builds only
    if (A.st != 0 && B.st != 0) return;
    for (int it = 1; it < 16; ++it) {
        Tan A2 = A, B2 = B;
        tangency_step(R, Px, Py, Pz, s, c, true, A2);
        tangency_step(R, Px, Py, Pz, s, c, false, B2);
        if (nit) { nit[0] += (A.st == 0); nit[1] += (B.st == 0); }  // diagnostic builds only
        if (A.st == 0) A = A2;
        if (B.st == 0) B = B2;
        if (A.st != 0 && B.st != 0) break;
    }
}

// 0: not eclipsed, 1: eclipsed, -1: undecided (use the nested solver)
__device__ inline int cone_exists(const Roche& R, double Px, double Py, double Pz, double s, double c,
                                  double cs, double sn, double t, int* nit = nullptr)
{
    for (int it = 0; it < 16; ++it) {
        if (nit) ++*nit;
        ConePt o;
        cone_point(R, Px, Py, Pz, s, c, cs, sn, t, o);
        if (o.phi < R.pl1) return (o.dX2 < R.Rs2) ? 1 : -1;
        const double Gth = t * o.gth, Gt = o.F2;
        const double Htt = o.eHe, Hht = o.gth + t * o.etHe, Hhh = t * t * o.ethHeth + t * o.gtt;
        const double det = Hhh * Htt - Hht * Hht;
        if (!(Hhh > 0.0 && Htt > 0.0 && det > 0.0)) return -1;
        const double idet = rcp_fast(det);
        double dth = -(Htt * Gth - Hht * Gt) * idet;
        double dt = -(Hhh * Gt - Hht * Gth) * idet;
        const double big = fmax(fabs(dth), fabs(dt));
        if (big > 0.05) {  // trust region: shorten the step, keep its direction
            dth *= 0.05 / big;
            dt *= 0.05 / big;
        }
        t += dt;
        if (fabs(dth) <= 1e-12 && fabs(dt) <= 1e-12) return 0;
        rotate(cs, sn, dth);
    }
    return -1;
}

// element_interval with the fast path; Rcal = sphere radius reproducing the
// WD-centre contact (initial guesses only).  Trig: one atan2 and one acos.
__device__ inline bool element_interval_fast(const Roche& R, double Px, double Py, double Pz, double s,
                                             double c, double Rcal, double Reff, double& a, double& b,
                                             bool* fallback = nullptr, int* nit = nullptr, double* guess = nullptr)
{
    // nit (diagnostic builds): iterations of the cone search, ingress and egress
    const double ux = 1.0 - Px, uy = -Py, uz = -Pz;
    const double uxy2 = ux * ux + uy * uy;
    const double uu = uxy2 + uz * uz;
    if (uu > R.Rs2 && uxy2 > 0.0 && s > 0.0) {
        const double iuxy = rsqrt(uxy2), uxy = uxy2 * iuxy;
        const double cosD = (sqrt(uu - R.Rs2) - c * uz) * iuxy / s;
        if (!(cosD < 1.0)) { a = 1.0; b = -1.0; return false; }  // (non-finite geometry included)
        // theta_c = atan2(-uy, ux): closest approach of the line of sight to D
        const double cc = ux * iuxy, sc = -uy * iuxy;
        const double tc = s * uxy + uz * c;
        // the closest approach to D inside the lobe decides at once (one
        // potential, no gradient or Hessian); otherwise the cone search
        int ex;
        {
            const double ex0 = s * cc, ey0 = -s * sc;
            const double x = fma(tc, ex0, Px), y = fma(tc, ey0, Py), z = fma(tc, c, Pz);
            const double dx = x - 1.0, xm = x - R.mu;
            const double r2s = dx * dx + y * y + z * z;
            const double phi = -R.cA * rsqrt_pos(x * x + y * y + z * z) - R.cB * rsqrt_pos(r2s) - xm * xm - y * y;
            if (phi < R.pl1 && r2s < R.Rs2) {
                ex = 1;
                if (nit) ++nit[0];  // diagnostic builds: one cone step
            } else {
                ex = cone_exists(R, Px, Py, Pz, s, c, cc, sc, tc, nit);
            }
        }
        if (ex == 0) { a = 1.0; b = -1.0; return false; }
        if (ex == 1) {
            const double ce = (sqrt(fmax(uu - Rcal * Rcal, 0.0)) - c * uz) * iuxy / s;
            if (ce > -1.0 && ce < 1.0) {
                const double se = sqrt(1.0 - ce * ce);
                const double thc = atan2(-uy, ux), de = acos(ce);
                // cos/sin of thc -+ de; t at closest approach to D along each ray
                double ci = cc * ce + sc * se, si = sc * ce - cc * se;
                double co = cc * ce - sc * se, so = sc * ce + cc * se;
                Tan In{thc - de, ci, si, s * (ux * ci - uy * si) + uz * c, 0};
                Tan Out{thc + de, co, so, s * (ux * co - uy * so) + uz * c, 0};
                if (guess) { guess[0] = In.th; guess[1] = Out.th; }  // diagnostic builds only
                // t at the ray's minimum of Phi, one Newton step from the
                // closest approach X_c to D: there the donor's own term has
                // no slope along e, so e.grad Phi = e.grad(-cA/r1 - (x-mu)^2
                // - y^2), and e.H.e = cB/d^3 + the WD's and the centrifugal
                // parts, with d = Rcal (the guess rays graze that sphere)
                {
                    const double icb = R.cB / (Rcal * Rcal * Rcal) - 2.0 * s * s;
                    for (Tan* T : {&In, &Out}) {
                        const double ex = s * T->cs, ey = -s * T->sn;
                        const double x = fma(T->t, ex, Px), y = fma(T->t, ey, Py), z = fma(T->t, c, Pz);
                        const double ir1 = rsqrt_pos(x * x + y * y + z * z), ir1s = ir1 * ir1;
                        const double eX = x * ex + y * ey + z * c;
                        const double i1 = R.cA * ir1s * ir1;
                        const double slope = fma(i1, eX, -2.0 * fma(x - R.mu, ex, y * ey));
                        const double curv = fma(i1, fma(-3.0 * eX * eX, ir1s, 1.0), icb);
                        T->t -= slope * rcp_fast(curv);
                    }
                }
                tangency_pair(R, Px, Py, Pz, s, c, In, Out, nit ? nit + 1 : nullptr);
                // both contacts within Dm of thc (where the ray meets the
                // donor's sphere), tested as cos(th - thc) > cos Dm with the
                // rotated cosines: no acos; the steps are clamped to 0.05 rad
                // and the solve is short, so |th - thc| stays far below pi
                const double cin = In.cs * cc + In.sn * sc, cout = Out.cs * cc + Out.sn * sc;
                if (In.st == 1 && Out.st == 1 && In.th < Out.th && cin > cosD && cout > cosD) {
                    a = In.th * (1.0 / TWO_PI);
                    b = Out.th * (1.0 / TWO_PI);
                    return true;
                }
            }
        }
    }
    if (fallback) *fallback = true;
    return element_interval(R, Px, Py, Pz, s, c, Reff, a, b);
}

// findphi / findi with the same 2-D tangency Newton, nested solver fallback
__device__ inline int findphi(const Roche& R, double inc_deg, double& dphi);

__device__ inline int findphi_fast(const Roche& R, double inc_deg, double& dphi)
{
    double s, c;
    sincos(inc_deg * DEG, &s, &c);
    const double cosD = sqrt(1.0 - R.Rs2) / s;
    if (s > 0.0 && cosD < 1.0) {
        const double Dm = acos(cosD);
        const double R0 = eggleton(R.q);
        const double c0 = sqrt(1.0 - R0 * R0) / s;
        double th = (c0 < 1.0) ? acos(c0) : 0.5 * Dm;
        double sn, cs;
        sincos(th, &sn, &cs);
        double t = s * cs;
        if (tangency(R, 0.0, 0.0, 0.0, s, c, false, th, cs, sn, t) && th > 0.0 && th < Dm) {
            dphi = th / PI;
            return ST_OK;
        }
    }
    return findphi(R, inc_deg, dphi);
}

// MODEL_SPEC 4.4: full phase width of the WD-centre eclipse
__device__ inline int findphi(const Roche& R, double inc_deg, double& dphi)
{
    const double i = inc_deg * DEG;
    double s, c;
    sincos(i, &s, &c);
    dphi = 0.0;
    const double cosD = sqrt(1.0 - R.Rs2) / s;
    if (!(s > 0.0) || cosD >= 1.0) return ST_BAD_DPHI;
    const double Dm = acos(cosD);
    double tw = -1.0, g, dg;
    g_eval(R, 0.0, 0.0, 0.0, s, c, 0.0, tw, g, dg);
    if (!(g < 0.0)) return ST_BAD_DPHI;
    const double th = theta_root(R, 0.0, 0.0, 0.0, s, c, 0.0, Dm, false, 0.5 * Dm, tw);
    dphi = th / PI;
    return ST_OK;
}

__device__ inline bool h_eval(const Roche& R, double cth, double sth, double c,
                              double& tw, double& h, double& dh)
{
    const double s = sqrt(1.0 - c * c);
    const double ex = s * cth, ey = -s * sth;
    double fm;
    if (!ray_min(R, 0.0, 0.0, 0.0, ex, ey, c, tw, fm)) { h = 1.0; dh = 0.0; return false; }
    double gx, gy, gz;
    rgrad(R, tw * ex, tw * ey, tw * c, gx, gy, gz);
    h = fm - R.pl1;
    const double r = c / s;
    dh = tw * (gx * (-r * cth) + gy * (r * sth) + gz);
    return true;
}

// MODEL_SPEC 4.4: inclination (deg) whose WD-centre eclipse has width dphi
__device__ inline int findi(const Roche& R, double dphi, double& inc_deg)
{
    if (!(dphi > 0.0) || !(dphi < 0.5)) return ST_BAD_DPHI;
    const double the = PI * dphi;
    double sth, cth;
    sincos(the, &sth, &cth);
    if (!(cth > 0.0)) return ST_BAD_DPHI;
    const double smin = sqrt(1.0 - R.Rs2) / cth;
    if (smin >= 1.0) return ST_BAD_DPHI;
    const double cmax = sqrt(1.0 - smin * smin);
    double tw = -1.0, h, dh;
    h_eval(R, cth, sth, 0.0, tw, h, dh);
    if (!(h < 0.0)) return ST_BAD_DPHI;
    double lo = 0.0, hi = cmax, c = 0.5 * cmax;
    for (int it = 0; it < ROOT_MAXIT; ++it) {
        h_eval(R, cth, sth, c, tw, h, dh);
        if (h > 0.0) hi = c; else lo = c;
        double cn = (dh != 0.0) ? c - h / dh : 0.5 * (lo + hi);
        if (!(cn > lo && cn < hi)) cn = 0.5 * (lo + hi);
        const double d = cn - c;
        c = cn;
        if (fabs(d) <= TH_TOL) break;
    }
    inc_deg = acos(c) / DEG;
    return ST_OK;
}

__device__ inline int findi_fast(const Roche& R, double dphi, double& inc_deg)
{
    if (dphi > 0.0 && dphi < 0.5) {
        double sth, cth;
        sincos(PI * dphi, &sth, &cth);
        const double smin = sqrt(1.0 - R.Rs2) / cth;
        if (cth > 0.0 && smin < 1.0) {
            const double cmax = sqrt(1.0 - smin * smin);
            const double R0 = eggleton(R.q);
            double s0 = fmin(sqrt(1.0 - R0 * R0) / cth, 0.9999);
            double c = sqrt(1.0 - s0 * s0), t = s0 * cth;
            for (int it = 0; it < 20; ++it) {
                const double s = sqrt(1.0 - c * c);
                const double ex = s * cth, ey = -s * sth;
                const double x = t * ex, y = t * ey, z = t * c;
                const double r1s = x * x + y * y + z * z;
                const double ir1 = rsqrt_pos(r1s), ir1s = ir1 * ir1;
                const double dx = x - 1.0;
                const double r2s = dx * dx + y * y + z * z;
                const double ir2 = rsqrt_pos(r2s), ir2s = ir2 * ir2;
                const double i1 = R.cA * ir1s * ir1, i2 = R.cB * ir2s * ir2, i12 = i1 + i2;
                const double xm = x - R.mu;
                const double phi = -R.cA * ir1 - R.cB * ir2 - xm * xm - y * y;
                const double gx = i1 * x + i2 * dx - 2.0 * xm, gy = (i12 - 2.0) * y, gz = i12 * z;
                const double p1 = t, p2 = t - ex;
                const double k1 = 3.0 * i1 * ir1s, k2 = 3.0 * i2 * ir2s;
                const double r = c * rcp_fast(s);
                const double ecx = -r * cth, ecy = r * sth;
                const double F1 = phi - R.pl1, F2 = gx * ex + gy * ey + gz * c;
                const double gec = gx * ecx + gy * ecy + gz;
                const double J11 = t * gec, J12 = F2;
                const double J21 = t * (k2 * p2 * ecx - 2.0 * (ecx * ex + ecy * ey)) + gec;
                const double J22 = i12 - k1 * p1 * p1 - k2 * p2 * p2 - 2.0 * (ex * ex + ey * ey);
                const double det = J11 * J22 - J12 * J21;
                if (!(det != 0.0)) break;
                const double idet = rcp_fast(det);
                double dc = -(F1 * J22 - F2 * J12) * idet;
                const double dt = -(J11 * F2 - J21 * F1) * idet;
                dc = fmin(fmax(dc, -0.05), 0.05);
                c += dc;
                t += dt;
                if (fmax(fabs(dc), fabs(dt)) <= TH_LAST) {
                    if (J22 > 0.0 && J11 > 0.0 && c >= 0.0 && c < cmax && t > 0.0 && r2s < R.Rs2) {
                        inc_deg = acos(c) / DEG;
                        return ST_OK;
                    }
                    break;
                }
                if (!(c > -0.5 && c < 0.99)) break;
            }
        }
    }
    return findi(R, dphi, inc_deg);
}

// MODEL_SPEC 4.5: ballistic stream from L1 to radius rad (trm.roche.bspot)
struct StreamState { double x, y, vx, vy; };

__device__ __forceinline__ StreamState stream_deriv(const Roche& R, const StreamState& s)
{
    const double m1 = 0.5 * R.cA, m2 = 0.5 * R.cB;
    const double ir1 = rsqrt_pos(s.x * s.x + s.y * s.y);
    const double i1 = m1 * ir1 * ir1 * ir1;
    const double dx = s.x - 1.0;
    const double ir2 = rsqrt_pos(dx * dx + s.y * s.y);
    const double i2 = m2 * ir2 * ir2 * ir2;
    const double Ux = i1 * s.x + i2 * dx - (s.x - R.mu);
    const double Uy = (i1 + i2 - 1.0) * s.y;
    return StreamState{s.vx, s.vy, -Ux + 2.0 * s.vy, -Uy - 2.0 * s.vx};
}

__device__ __forceinline__ StreamState axpy(const StreamState& s, double a, const StreamState& k)
{
    return StreamState{fma(a, k.x, s.x), fma(a, k.y, s.y), fma(a, k.vx, s.vx), fma(a, k.vy, s.vy)};
}

__device__ inline void hermite(const StreamState& s0, const StreamState& s1, double dt, double idt,
                               double tau, double out[4])
{
    const double t2 = tau * tau, t3 = t2 * tau;
    const double h00 = 2.0 * t3 - 3.0 * t2 + 1.0, h10 = t3 - 2.0 * t2 + tau;
    const double h01 = -2.0 * t3 + 3.0 * t2, h11 = t3 - t2;
    const double d00 = 6.0 * t2 - 6.0 * tau, d10 = 3.0 * t2 - 4.0 * tau + 1.0;
    const double d01 = -6.0 * t2 + 6.0 * tau, d11 = 3.0 * t2 - 2.0 * tau;
    out[0] = h00 * s0.x + h10 * dt * s0.vx + h01 * s1.x + h11 * dt * s1.vx;
    out[1] = h00 * s0.y + h10 * dt * s0.vy + h01 * s1.y + h11 * dt * s1.vy;
    out[2] = fma(d00 * s0.x + d01 * s1.x, idt, d10 * s0.vx + d11 * s1.vx);
    out[3] = fma(d00 * s0.y + d01 * s1.y, idt, d10 * s0.vy + d11 * s1.vy);
}

// second-order point of the L1 unstable manifold (MODEL_SPEC 4.5)
__device__ inline StreamState stream_start(const Roche& R)
{
    const double x1 = R.xl1;
    const double m1 = 0.5 * R.cA, m2 = 0.5 * R.cB;
    const double ix1 = rcp_fast(x1), irs = rcp_fast(R.Rs);
    const double K = m1 * ix1 * ix1 * ix1 + m2 * irs * irs * irs;
    const double Uxx = -2.0 * K - 1.0, Uyy = K - 1.0;
    const double L = 0.5 * ((K - 2.0) + sqrt((K - 2.0) * (K - 2.0) + 4.0 * (2.0 * K + 1.0) * (K - 1.0)));
    const double lam = sqrt(L);
    const double B = -(L - 2.0 * K - 1.0) * (0.5 * rcp_fast(lam));
    const double inrm = rsqrt(1.0 + B * B);
    const double v0 = -inrm, v1 = B * inrm;
    const double Uxxx = 6.0 * m1 * ix1 * ix1 * ix1 * ix1 - 6.0 * m2 * irs * irs * irs * irs;
    const double Uxyy = -0.5 * Uxxx;
    const double N2x = -0.5 * (Uxxx * v0 * v0 + Uxyy * v1 * v1);
    const double N2y = -Uxyy * v0 * v1;
    const double a11 = Uxx + 4.0 * L, a22 = Uyy + 4.0 * L;
    const double idet = rcp_fast(a11 * a22 + 16.0 * L);
    const double w0 = (N2x * a22 + 4.0 * lam * N2y) * idet;
    const double w1 = (a11 * N2y - 4.0 * lam * N2x) * idet;
    const double d = STREAM_DELTA, d2 = d * d;
    return StreamState{x1 + d * v0 + d2 * w0, d * v1 + d2 * w1, d * lam * v0 + d2 * 2.0 * lam * w0,
                       d * lam * v1 + d2 * 2.0 * lam * w1};
}

// The converged stream outside the table's domain (MODEL_SPEC 4.5): RK4 with
// step dt = min(STREAM_DTMAX_FINE, STREAM_KAPPA_FINE r^(3/2)) (~1e-12 a from
// the DOP853 reference) and the crossing on the cubic Hermite interpolant of
// the last step.  Slow (~700 steps); the prior ranges never reach it.
__device__ inline int bspot_rk4(const Roche& R, double rad, double out[4])
{
    // the loop tests squared radii: the exit branch waits on one fma level,
    // not on a sqrt (~5 dependent levels); r itself only sets the next dt,
    // which runs beside k1
    StreamState s = stream_start(R);
    double r2c = s.x * s.x + s.y * s.y;
    const double rad2 = rad * rad;
    if (!(rad2 < r2c)) return ST_BAD_STREAM;  // the stream starts inside rad (as the table path)
    for (int n = 0; n < STREAM_MAXSTEP_FINE; ++n) {
        // r^(3/2) = r2 (r2 (r2)^(-1/2))^(-1/2): two v_rsq steps
        const double r32 = r2c * rsqrt_pos(r2c * rsqrt_pos(r2c));
        const double dt = fmin(STREAM_KAPPA_FINE * r32, STREAM_DTMAX_FINE);
        const StreamState k1 = stream_deriv(R, s);
        const StreamState k2 = stream_deriv(R, axpy(s, 0.5 * dt, k1));
        const StreamState k3 = stream_deriv(R, axpy(s, 0.5 * dt, k2));
        const StreamState k4 = stream_deriv(R, axpy(s, dt, k3));
        const double h6 = dt * (1.0 / 6.0);
        StreamState sn{s.x + h6 * (k1.x + 2.0 * k2.x + 2.0 * k3.x + k4.x),
                       s.y + h6 * (k1.y + 2.0 * k2.y + 2.0 * k3.y + k4.y),
                       s.vx + h6 * (k1.vx + 2.0 * k2.vx + 2.0 * k3.vx + k4.vx),
                       s.vy + h6 * (k1.vy + 2.0 * k2.vy + 2.0 * k3.vy + k4.vy)};
        const double rn2 = sn.x * sn.x + sn.y * sn.y;
        if (rn2 < rad2) {  // Hermite crossing, safeguarded Newton on |H|^2 - rad^2
            const double r2 = rad2;
            const double f0 = r2c - r2, f1 = rn2 - r2;
            const double idt = rcp_fast(dt);
            double lo = 0.0, hi = 1.0, tau = f0 * rcp_fast(f0 - f1), p[4];
            for (int it = 0; it < 100; ++it) {
                hermite(s, sn, dt, idt, tau, p);
                const double f = p[0] * p[0] + p[1] * p[1] - r2;
                const double df = 2.0 * dt * (p[0] * p[2] + p[1] * p[3]);
                if (f > 0.0) lo = tau; else hi = tau;
                const double step = (df != 0.0) ? f * rcp_fast(df) : 0.0;
                if (df != 0.0 && fabs(step) <= ROOT_LAST) { tau -= step; break; }  // last Newton step
                double tn = (df != 0.0) ? tau - step : 0.5 * (lo + hi);
                if (!(tn > lo && tn < hi)) tn = 0.5 * (lo + hi);
                tau = tn;
            }
            hermite(s, sn, dt, idt, tau, out);
            return ST_OK;
        }
        if (rn2 > r2c && n > 0) return ST_BAD_STREAM;
        s = sn;
        r2c = rn2;
    }
    return ST_BAD_STREAM;
}

// The converged stream as piecewise tensor Chebyshev series (MODEL_SPEC 4.5,
// lfg_stream_table.h from tools/gen_stream_table.py): patch (iq, js) of
// xi = ln q and s = sqrt((r - rmin) / (r0 - rmin)) holds phi, vx, vy.
__constant__ const double kStRmin[LFG_ST_NQ * (LFG_ST_DR + 1)] = LFG_ST_RMIN;
__constant__ const double kStCoef[LFG_ST_NQ * LFG_ST_NS * 3 * (LFG_ST_DQ + 1) * (LFG_ST_DS + 1)] = LFG_ST_COEF;
constexpr double kStSb[LFG_ST_NS + 1] = LFG_ST_SB;
constexpr int ST_PATCH = (LFG_ST_DQ + 1) * (LFG_ST_DS + 1);

// one output of a patch: sum_i T_i(xq) sum_j c[i][j] T_j(xs); the DQ + 1 inner
// sums are independent chains (13 levels), then one 10-level chain
__device__ __forceinline__ double st_patch(const double* c, double xq, double xs)
{
    double a[LFG_ST_DQ + 1];
#pragma unroll
    for (int i = 0; i <= LFG_ST_DQ; ++i) a[i] = clenshaw<LFG_ST_DS + 1>(c + i * (LFG_ST_DS + 1), xs);
    return clenshaw<LFG_ST_DQ + 1>(a, xq);
}

// MODEL_SPEC 4.5: bspot(q, rad) -> (x, y, vx, vy) of the converged stream
// (trm.roche.bspot).  VEL = false leaves out[2..3] unset: the hot path
// needs the impact point only.
template <bool VEL = true>
__device__ inline int bspot(const Roche& R, double rad, double out[4], const QPatch* qp = nullptr)
{
    if (!(rad > 0.0) || !(rad < R.xl1)) return ST_BAD_STREAM;
    const QPatch p = qp ? *qp : q_patch(R.q);
    if (p.iq < 0) return bspot_rk4(R, rad, out);
    const int iq = p.iq;
    const double xq = p.xq;
    const StreamState s0 = stream_start(R);
    const double r0 = sqrt(s0.x * s0.x + s0.y * s0.y);
    const double rmin = exp(q_series(kStRmin, p));
    if (!(rad > rmin) || !(rad < r0)) return ST_BAD_STREAM;  // misses the disc / starts inside rad
    const double s = sqrt((rad - rmin) / (r0 - rmin));
    if (!(s <= LFG_ST_STOP)) return bspot_rk4(R, rad, out);
    int js = 0;
#pragma unroll
    for (int k = 1; k < LFG_ST_NS; ++k) js += (s >= kStSb[k]) ? 1 : 0;
    double lo = kStSb[0], w = kStSb[1] - kStSb[0];
#pragma unroll
    for (int k = 1; k < LFG_ST_NS; ++k)
        if (js == k) { lo = kStSb[k]; w = kStSb[k + 1] - kStSb[k]; }
    const double xs = 2.0 * (s - lo) / w - 1.0;
#ifdef LFG_ABL_STTAB  // (diagnostic builds) every lane reads patch 0: the table's share of the traffic
    const double* c = kStCoef + 0 * size_t(iq * LFG_ST_NS + js);
#else
    const double* c = kStCoef + size_t(iq * LFG_ST_NS + js) * 3 * ST_PATCH;
#endif
    double sp, cp;
    sincos(st_patch(c, xq, xs), &sp, &cp);
    out[0] = rad * cp;
    out[1] = rad * sp;
    if (VEL) {
        out[2] = st_patch(c + ST_PATCH, xq, xs);
        out[3] = st_patch(c + 2 * ST_PATCH, xq, xs);
    }
    return ST_OK;
}

// MODEL_SPEC 5.3: end of the bright-spot strip, F(u) = BS_TAIL below the peak
// (in v = u^b: G(v) = v - (a/b) ln v - C is convex increasing past its
// minimum, so Newton from the right converges monotonically; one log per step)
__device__ inline double bs_umax(double a, double b, double lnpk)
{
    const double k = a / b, C = BS_TAIL - lnpk;
    double v = fmax(2.0 * k, C + k * log(C + 2.0 * k) + 1.0);
    for (int it = 0; it < 200 && v - k * log(v) - C <= 0.0; ++it) v *= 2.0;
    for (int it = 0; it < ROOT_MAXIT; ++it) {
        const double G = v - k * log(v) - C;
        const double dv = G * v * rcp_fast(v - k);  // G / (1 - k / v)
        v -= dv;
        if (fabs(dv) <= ROOT_LAST * v) break;  // quadratic: the error left is ~1e-18 v
    }
    return exp(log(v) / b);
}

// MODEL_SPEC 10.2: trm.roche.wdphases(q, iangle, r1, ntheta) (CVModel.py:564):
// third and fourth contact phases of a sphere of radius r1 at the WD, from
// ntheta points on the limb circle perpendicular to the line of sight at the
// WD-centre egress phase; the nested solver (as the oracle) for each point
__device__ inline int wdphases(const Roche& R, double inc_deg, double r1, int ntheta, double& ph3, double& ph4)
{
    if (!(r1 > 0.0) || ntheta < 1) return ST_BAD_GEOMETRY;
    double dphi;
    int st = findphi_fast(R, inc_deg, dphi);
    if (st != ST_OK) return st;
    double s, c, sth, cth;
    sincos(inc_deg * DEG, &s, &c);
    sincos(PI * dphi, &sth, &cth);
    const double Reff = eggleton(R.q);
    double lo = INFINITY, hi = -INFINITY;
    for (int k = 0; k < ntheta; ++k) {
        double sp, cp;
        sincos(TWO_PI * k / ntheta, &sp, &cp);
        double a, b;
        if (element_interval(R, r1 * (cp * sth - sp * c * cth), r1 * (cp * cth + sp * c * sth), r1 * (sp * s), s, c,
                             Reff, a, b)) {
            lo = fmin(lo, b);
            hi = fmax(hi, b);
        }
    }
    if (!(lo <= hi)) return ST_BAD_DPHI;
    ph3 = lo;
    ph4 = hi;
    return ST_OK;
}

// MODEL_SPEC 10.4: the GP log-likelihood of CVModel.py:636-691 as a 4-state
// Kalman filter over phase-sorted points (tests/gp_kalman.py restates it in
// numpy).  State (g, g', h, h'): the global Matern-3/2 process (variance
// ampin) and the process of the current changepoint block (ampout), which
// starts stationary at the block's first point; both share
//   Phi(d) = e^{-u} [[1 + u, d], [-lam^2 d, 1 - u]],  u = lam d,
//   lam = sqrt(3 / tau) (george's metric tau), Pinf = a diag(1, lam^2).
// Covariances are carried as D = P - Pinf, so prediction is D <- Phi D Phi^T.
struct GPFilter {
    double lam, ain, aout;
    double m0, m1, m2, m3;
    double d00, d01, d11, d22, d23, d33, d02, d03, d12, d13;  // g-g, h-h, g-h blocks of D
    double xp, ll;
    int bp, n;
    bool bad;

    __device__ void init(double ampin, double ampout, double tau)
    {
        lam = sqrt(3.0 / tau);
        ain = ampin;
        aout = ampout;
        m0 = m1 = m2 = m3 = 0.0;
        d00 = d01 = d11 = d22 = d23 = d33 = d02 = d03 = d12 = d13 = 0.0;
        xp = 0.0;
        ll = 0.0;
        bp = -1;
        n = 0;
        bad = !(tau > 0.0) || !(ampin >= 0.0) || !(ampout >= 0.0);
    }

    // one point: phase x (sorted), error ye, residual r, changepoint block blk (-1: none)
    __device__ void step(double x, double ye, double r, int blk)
    {
        if (n > 0) {
            const double d = x - xp;
            const double u = lam * d, e = exp(-u);
            const double f00 = e * (1.0 + u), f01 = e * d, f10 = -e * lam * u, f11 = e * (1.0 - u);
            double t0 = f00 * m0 + f01 * m1;
            m1 = f10 * m0 + f11 * m1;
            m0 = t0;
            t0 = f00 * m2 + f01 * m3;
            m3 = f10 * m2 + f11 * m3;
            m2 = t0;
            sym(f00, f01, f10, f11, d00, d01, d11);
            sym(f00, f01, f10, f11, d22, d23, d33);
            const double t00 = f00 * d02 + f01 * d12, t01 = f00 * d03 + f01 * d13;
            const double t10 = f10 * d02 + f11 * d12, t11 = f10 * d03 + f11 * d13;
            d02 = t00 * f00 + t01 * f01;
            d03 = t00 * f10 + t01 * f11;
            d12 = t10 * f00 + t11 * f01;
            d13 = t10 * f10 + t11 * f11;
            bad = bad || !(d >= 0.0);
        }
        xp = x;
        ++n;
        if (blk >= 0 && blk != bp) {  // a new block: its process starts stationary, independent
            m2 = m3 = 0.0;
            d22 = d23 = d33 = d02 = d03 = d12 = d13 = 0.0;
        }
        bp = blk;
        const double a = (blk >= 0) ? 1.0 : 0.0;
        const double k0 = (d00 + ain) + a * d02, k1 = d01 + a * d12;
        const double k2 = d02 + a * (d22 + aout), k3 = d03 + a * d23;
        const double S = fma(a, k2, k0) + ye * ye;
        const double v = r - fma(a, m2, m0);
        const double iS = 1.0 / S;
        bad = bad || !(S > 0.0) || !isfinite(v);
        ll += v * v * iS + log(S);
        const double g = v * iS;
        m0 = fma(k0, g, m0);
        m1 = fma(k1, g, m1);
        m2 = fma(k2, g, m2);
        m3 = fma(k3, g, m3);
        d00 -= k0 * k0 * iS; d01 -= k0 * k1 * iS; d11 -= k1 * k1 * iS;
        d22 -= k2 * k2 * iS; d23 -= k2 * k3 * iS; d33 -= k3 * k3 * iS;
        d02 -= k0 * k2 * iS; d03 -= k0 * k3 * iS; d12 -= k1 * k2 * iS; d13 -= k1 * k3 * iS;
    }

    __device__ double lnlike() const
    {
        const double v = -0.5 * (ll + n * 1.8378770664093454836);  // log(2 pi)
        return (bad || !isfinite(v)) ? -INFINITY : v;
    }

    __device__ static void sym(double f00, double f01, double f10, double f11, double& a, double& b, double& c)
    {
        const double t00 = f00 * a + f01 * b, t01 = f00 * b + f01 * c;
        const double t10 = f10 * a + f11 * b, t11 = f10 * b + f11 * c;
        a = t00 * f00 + t01 * f01;
        b = t00 * f10 + t01 * f11;
        c = t10 * f10 + t11 * f11;
    }
};

// CVModel.py:582-599: changepoint block k of eclipse number ec is
// [(ec - 1) + dcp + phi0, (ec - dcp) + phi0], closed as george tests blocks;
// returns the block index of x in [e0, e1], or -1
__device__ __forceinline__ int gp_block(double x, int e0, int e1, double dcp, double phi0)
{
    int blk = -1;
    for (int ec = e0; ec <= e1; ++ec) {
        const double lo = (double(ec - 1) + dcp) + phi0, hi = (double(ec) - dcp) + phi0;
        if (x >= lo && x <= hi) blk = ec - e0;
    }
    return blk;
}

// Prior.ln_prob, model.py:83-113 (gauss through log(pdf), as scipy does)
__device__ inline double prior_lnprob(int type, double p1, double p2, double norm, double v)
{
    switch (type) {
    case 0:
    case 1: {
        if (type == 1 && v <= 0.0) return -INFINITY;
        const double z = (v - p1) / p2;
        const double pdf = exp(-z * z / 2.0) / sqrt(2.0 * PI) / p2;
        return (pdf > 0.0) ? log(pdf) : -INFINITY;
    }
    case 2: return (v > p1 && v < p2) ? log(1.0 / fabs(p1 - p2)) : -INFINITY;
    case 3: return (v > p1 && v < p2) ? log(1.0 / norm / v) : -INFINITY;
    case 4: return (v > 0.0 && v < p2) ? log(1.0 / norm / (v + p1)) : -INFINITY;
    }
    return -INFINITY;
}

// ln of the smallest positive double (a denormal): below it scipy's pdf is
// 0 and log(pdf) -inf (model.py:85-89)
constexpr double PDF_LN_MIN = -745.1332191019412;

}  // namespace lfg
