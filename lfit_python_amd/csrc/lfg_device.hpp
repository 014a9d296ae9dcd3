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

namespace lfg {

constexpr double PI = 3.14159265358979323846;
constexpr double TWO_PI = 6.28318530717958647693;
constexpr double DEG = PI / 180.0;

// MODEL_SPEC.md section 7
constexpr double RAY_TOL = 1e-13;
constexpr int RAY_MAXIT = 100;
constexpr double TH_TOL = 1e-13;
constexpr int ROOT_MAXIT = 100;
constexpr int MIN_MAXIT = 100;
constexpr double BS_TAIL = 16.0;
constexpr double STREAM_DELTA = 1e-5;
constexpr double STREAM_KAPPA = 0.1;
constexpr double STREAM_DTMAX = 0.1;
constexpr int STREAM_MAXSTEP = 4000;
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
    G_FIS, G_PHI0, G_WDF, G_DF, G_SF, G_RSF, G_RPRIOR,
    G_COUNT
};
static_assert(G_COUNT <= 48, "LFG_NGEO");

struct Roche {
    double q, cA, cB, mu, xl1, pl1, Rs, Rs2;
};

__device__ __forceinline__ double rpot(const Roche& R, double x, double y, double z)
{
    const double dx = x - 1.0;
    const double xc = x - R.mu;
    return -R.cA * rsqrt(x * x + y * y + z * z) - R.cB * rsqrt(dx * dx + y * y + z * z)
           - xc * xc - y * y;
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

// MODEL_SPEC 4.1: L1 point, safeguarded Newton on dPhi/dx (monotone on (0,1))
__device__ inline double xl1_solve(double q)
{
    const double cA = 2.0 / (1.0 + q), cB = q * cA, mu = q / (1.0 + q);
    double lo = 0.0, hi = 1.0;
    double x = 1.0 - cbrt(q / (3.0 * (1.0 + q)));
    for (int it = 0; it < 200; ++it) {
        const double omx = 1.0 - x;
        const double ix = 1.0 / x, io = 1.0 / omx;
        const double f = cA * ix * ix - cB * io * io - 2.0 * (x - mu);
        const double df = -2.0 * cA * ix * ix * ix - 2.0 * cB * io * io * io - 2.0;
        if (f > 0.0) lo = x; else hi = x;
        double xn = x - f / df;
        if (!(xn > lo && xn < hi)) xn = 0.5 * (lo + hi);
        const double d = xn - x;
        x = xn;
        if (fabs(d) <= 1e-15) break;
    }
    return x;
}

__device__ inline int roche_init(Roche& R, double q)
{
    if (!(q > 0.0) || !isfinite(q)) return ST_BAD_Q;
    R.q = q;
    R.cA = 2.0 / (1.0 + q);
    R.cB = q * R.cA;
    R.mu = q / (1.0 + q);
    R.xl1 = xl1_solve(q);
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
    if (cosD >= 1.0) return false;
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

// MODEL_SPEC 4.5: ballistic stream from L1 to radius rad (trm.roche.bspot)
struct StreamState { double x, y, vx, vy; };

__device__ __forceinline__ StreamState stream_deriv(const Roche& R, const StreamState& s)
{
    const double m1 = 0.5 * R.cA, m2 = 0.5 * R.cB;
    const double ir1 = rsqrt(s.x * s.x + s.y * s.y);
    const double i1 = m1 * ir1 * ir1 * ir1;
    const double dx = s.x - 1.0;
    const double ir2 = rsqrt(dx * dx + s.y * s.y);
    const double i2 = m2 * ir2 * ir2 * ir2;
    const double Ux = i1 * s.x + i2 * dx - (s.x - R.mu);
    const double Uy = (i1 + i2 - 1.0) * s.y;
    return StreamState{s.vx, s.vy, -Ux + 2.0 * s.vy, -Uy - 2.0 * s.vx};
}

__device__ __forceinline__ StreamState axpy(const StreamState& s, double a, const StreamState& k)
{
    return StreamState{fma(a, k.x, s.x), fma(a, k.y, s.y), fma(a, k.vx, s.vx), fma(a, k.vy, s.vy)};
}

__device__ inline void hermite(const StreamState& s0, const StreamState& s1, double dt,
                               double tau, double out[4])
{
    const double t2 = tau * tau, t3 = t2 * tau;
    const double h00 = 2.0 * t3 - 3.0 * t2 + 1.0, h10 = t3 - 2.0 * t2 + tau;
    const double h01 = -2.0 * t3 + 3.0 * t2, h11 = t3 - t2;
    const double d00 = 6.0 * t2 - 6.0 * tau, d10 = 3.0 * t2 - 4.0 * tau + 1.0;
    const double d01 = -6.0 * t2 + 6.0 * tau, d11 = 3.0 * t2 - 2.0 * tau;
    out[0] = h00 * s0.x + h10 * dt * s0.vx + h01 * s1.x + h11 * dt * s1.vx;
    out[1] = h00 * s0.y + h10 * dt * s0.vy + h01 * s1.y + h11 * dt * s1.vy;
    out[2] = (d00 * s0.x + d01 * s1.x) / dt + d10 * s0.vx + d11 * s1.vx;
    out[3] = (d00 * s0.y + d01 * s1.y) / dt + d10 * s0.vy + d11 * s1.vy;
}

__device__ inline int bspot(const Roche& R, double rad, double out[4])
{
    if (!(rad > 0.0) || !(rad < R.xl1)) return ST_BAD_STREAM;
    const double q = R.q, x1 = R.xl1;
    const double K = 1.0 / ((1.0 + q) * x1 * x1 * x1) + q / ((1.0 + q) * R.Rs2 * R.Rs);
    const double L = 0.5 * ((K - 2.0) + sqrt((K - 2.0) * (K - 2.0) + 4.0 * (2.0 * K + 1.0) * (K - 1.0)));
    const double lam = sqrt(L);
    const double A = -1.0, B = (L - 2.0 * K - 1.0) / (2.0 * lam) * A;
    const double nrm = sqrt(A * A + B * B);
    StreamState s{x1 + STREAM_DELTA * A / nrm, STREAM_DELTA * B / nrm,
                  STREAM_DELTA * lam * A / nrm, STREAM_DELTA * lam * B / nrm};
    double r = sqrt(s.x * s.x + s.y * s.y);
    for (int n = 0; n < STREAM_MAXSTEP; ++n) {
        const double dt = fmin(STREAM_KAPPA * r * sqrt(r), STREAM_DTMAX);
        const StreamState k1 = stream_deriv(R, s);
        const StreamState k2 = stream_deriv(R, axpy(s, 0.5 * dt, k1));
        const StreamState k3 = stream_deriv(R, axpy(s, 0.5 * dt, k2));
        const StreamState k4 = stream_deriv(R, axpy(s, dt, k3));
        const double h6 = dt / 6.0;
        StreamState sn{s.x + h6 * (k1.x + 2.0 * k2.x + 2.0 * k3.x + k4.x),
                       s.y + h6 * (k1.y + 2.0 * k2.y + 2.0 * k3.y + k4.y),
                       s.vx + h6 * (k1.vx + 2.0 * k2.vx + 2.0 * k3.vx + k4.vx),
                       s.vy + h6 * (k1.vy + 2.0 * k2.vy + 2.0 * k3.vy + k4.vy)};
        const double rn = sqrt(sn.x * sn.x + sn.y * sn.y);
        if (rn < rad) {
            double lo = 0.0, hi = 1.0, p[4];
            for (int it = 0; it < 60; ++it) {
                const double m = 0.5 * (lo + hi);
                hermite(s, sn, dt, m, p);
                if (sqrt(p[0] * p[0] + p[1] * p[1]) > rad) lo = m; else hi = m;
            }
            hermite(s, sn, dt, 0.5 * (lo + hi), out);
            return ST_OK;
        }
        if (rn > r && n > 0) return ST_BAD_STREAM;
        s = sn;
        r = rn;
    }
    return ST_BAD_STREAM;
}

// MODEL_SPEC 5.3: end of the bright-spot strip, F(u) = BS_TAIL below the peak
__device__ inline double bs_umax(double a, double b, double lnpk)
{
    const double upk = pow(a / b, 1.0 / b);
    double lo = upk, hi = 2.0 * upk + 1.0;
    for (int k = 0; k < 200; ++k) {
        if (a * log(hi) - pow(hi, b) - lnpk + BS_TAIL < 0.0) break;
        lo = hi;
        hi *= 2.0;
    }
    double u = 0.5 * (lo + hi);
    for (int it = 0; it < ROOT_MAXIT; ++it) {
        const double ub = pow(u, b);
        const double F = a * log(u) - ub - lnpk + BS_TAIL;
        const double dF = (a - b * ub) / u;
        if (F > 0.0) lo = u; else hi = u;
        double un = (dF != 0.0) ? u - F / dF : 0.5 * (lo + hi);
        if (!(un > lo && un < hi)) un = 0.5 * (lo + hi);
        const double d = un - u;
        u = un;
        if (fabs(d) <= 1e-14 * u) break;
    }
    return u;
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

}  // namespace lfg
