// lfg_cpu.cpp -- the MI355X path's algorithm run on the host: a CPU baseline
// for bench.py (kind "port-fast"), not a product path and not the oracle.
//
// The oracle (oracle/lfg_oracle.c) restates MODEL_SPEC with the nested
// eclipse solver and the direct element x point sum: the slow, independent
// form.  This file runs what the GPU runs, on CPU cores: the device functions
// of lfit_python_amd/csrc/lfg_device.hpp compiled for the host (stream table,
// L1 and findi solves, the envelope-Newton tangency solver with its nested
// fallback, mirror symmetry), then the interval sweep of k_lnlike over the
// sorted exposure windows (each element's covered run into a difference
// array, partial windows directly, O((N S + N_el) log N) per walker), one
// walker per OpenMP thread at a time.  Chi^2 trees only (the GP likelihood
// is left to the oracle).  Sums are in FP64 in a fixed order; results match
// the oracle and the GPU to ~1e-12 (tests/test_cpu_baseline.py).
#include <omp.h>
#include <stdint.h>
#include <stdlib.h>

#include <algorithm>
#include <cmath>
#include <vector>

#include "lfg.h"
#include "lfg_cpu.h"
#include "lfg_device.hpp"
#include "lfg_tables.hpp"

using namespace lfg;

namespace {

constexpr int U_WD = NWD / 2, U_DISC = NDISC / 2, U_DON = NDONOR / 4;

// the pair's geometry (k_setup's record)
struct Pair {
    Roche R;
    double s, c, rwd_a, rdisc_a, reff, rcal, ulimb, dexp, L, upk, umax, lnpk, exp1, exp2;
    double bsx, bsy, caz, saz, nb0, nb1, nb2, bden, fis, phi0, wdf, df, sf, rsf;
    double inc;  // degrees (findi)
};

int wd_ring_of(int u)
{
    int ir = int(std::sqrt(u * 0.5));
    if (2 * (ir + 1) * (ir + 1) <= u) ++ir;
    if (2 * ir * ir > u) --ir;
    return ir;
}

double disc_boundary(int i, const Pair& G)
{
    const double r = G.rwd_a + i * ((G.rdisc_a - G.rwd_a) / NDISC_R);
    const double ex = 2.0 - G.dexp;
    return (std::fabs(ex) < 1e-10) ? std::log(r) : std::pow(r, ex) / ex;
}

// k_setup's setup lane and stream lane for one (walker, eclipse): status and
// the eclipse's Roche prior (CVModel.py:193-324), MODEL_SPEC 6 order
int setup_pair(const double* pin, int np, Pair& G, double& rprior)
{
    double p[18];
    bool finite = (np == 14 || np == 18);
    for (int k = 0; k < 18; ++k) {
        p[k] = k < np ? pin[k] : 0.0;
        finite = finite && std::isfinite(p[k]);
    }
    if (np == 14) { p[14] = 2.0; p[15] = 1.0; p[16] = 90.0; p[17] = 0.0; }
    rprior = 0.0;
    if (!finite) { rprior = -INFINITY; return ST_BAD_ARGS; }
    QPatch qp;
    int st = roche_init(G.R, p[4], &qp);
    if (st != ST_OK) { rprior = -INFINITY; return st; }
    const Roche& R = G.R;
    if (p[6] * R.xl1 > DISC_MAX_A) rprior = -INFINITY;
    if (p[9] > p[8] * 3.0 || p[9] < p[8] / 3.0) rprior = -INFINITY;
    double inc = 0.0;
    st = findi_fast(R, p[5], inc);
    G.rwd_a = p[8] * R.xl1;
    G.rdisc_a = p[6] * R.xl1;
    if (st == ST_OK && (!(G.rwd_a > 0.0) || !(G.rdisc_a > G.rwd_a) || !(G.rdisc_a < R.xl1))) st = ST_BAD_GEOMETRY;
    if (st == ST_OK && (!(p[9] > 0.0) || !(p[14] > 0.0) || !(p[15] > 0.0))) st = ST_BAD_GEOMETRY;
    // stream lane: impact point, azimuth prior, strip profile
    double bs[4] = {0.0, 0.0, 0.0, 0.0};
    int bst = (std::isfinite(p[6]) && std::isfinite(p[10])) ? bspot<false>(R, G.rdisc_a, bs, &qp) : ST_BAD_ARGS;
    if (bst != ST_OK) {
        rprior = -INFINITY;
    } else {
        double alpha = std::atan2(bs[1], bs[0]) / DEG;
        if (alpha < 0.0) alpha = 90.0 - alpha;
        const double tangent = alpha + 90.0;
        if (p[10] < std::fmax(0.0, tangent - AZ_SLOPE) || p[10] > std::fmin(178.0, tangent + AZ_SLOPE)) rprior = -INFINITY;
    }
    if (st != ST_OK) return st;
    if (bst != ST_OK) return bst;
    const double a1 = p[14], a2 = p[15];
    G.upk = std::pow(a1 / a2, 1.0 / a2);
    G.lnpk = a1 * std::log(G.upk) - std::pow(G.upk, a2);
    G.umax = bs_umax(a1, a2, G.lnpk);
    if (!(std::isfinite(G.upk) && std::isfinite(G.lnpk) && std::isfinite(G.umax))) return ST_BAD_GEOMETRY;
    G.exp1 = a1;
    G.exp2 = a2;
    G.bsx = bs[0];
    G.bsy = bs[1];
    G.s = std::sin(inc * DEG);
    G.c = std::cos(inc * DEG);
    const double tilt = p[16] * DEG, psi = (p[10] - 90.0 + p[17]) * DEG;
    const double st_ = std::sin(tilt), ct_ = std::cos(tilt);
    G.nb0 = st_ * std::cos(psi);
    G.nb1 = st_ * std::sin(psi);
    G.nb2 = ct_;
    G.caz = std::cos(p[10] * DEG);
    G.saz = std::sin(p[10] * DEG);
    G.bden = p[11] + (1.0 - p[11]) * std::fmax(std::fabs(st_) * G.s + ct_ * G.c, 0.0);
    G.fis = p[11];
    G.phi0 = p[13];
    G.ulimb = p[7];
    G.dexp = p[12];
    G.L = p[9] * R.xl1;
    G.reff = eggleton(R.q);
    const double sce = G.s * std::cos(PI * p[5]);
    G.rcal = std::sqrt(1.0 - sce * sce);
    G.wdf = p[0]; G.df = p[1]; G.sf = p[2]; G.rsf = p[3];
    G.inc = inc;
    return ST_OK;
}

// the 1400 WD/disc intervals (each unique item and its mirror) with their
// weights normalised by the component totals, the 100 spot intervals and
// weights (normalised), and the 400 donor tile vectors with visibility arcs
struct Tables {
    double a[NWD + NDISC], b[NWD + NDISC], w[NWD + NDISC];
    int wd[NWD + NDISC];  // 1: WD element, 0: disc
    double sa[NBS], sb[NBS], sw[NBS];
    double dv[NDONOR][3], dcen[NDONOR], dhw[NDONOR];
    double dnorm;  // donor flux at quadrature
};

#ifdef LFC_COUNT  // diagnostic build: Newton steps per lane and per 64-lane chunk (k_elements' waves)
static unsigned long long g_cnt[4 + 3 * 8];  // lanes, sum of lane steps, chunks, sum of chunk maxima; per region (WD, disc, spot) histogram of lane steps
extern "C" void lfc_counts(unsigned long long* o) { for (int i = 0; i < 4 + 24; ++i) o[i] = g_cnt[i]; }
static unsigned long long g_ucost[U_WD + U_DISC + NBS];  // per unique item: sum of lane steps over pairs
extern "C" void lfc_ucost(unsigned long long* o) { for (int i = 0; i < U_WD + U_DISC + NBS; ++i) { o[i] = g_ucost[i]; g_ucost[i] = 0; } }
static void count_pair(const int* cost, int n)
{
    unsigned long long ls = 0, cm = 0, nc = 0;
    for (int k = 0; k < n; k += 64) {
        int m = 0;
        for (int i = k; i < std::min(n, k + 64); ++i) {
            m = std::max(m, cost[i]);
            ls += cost[i];
            const int reg = i < U_WD ? 0 : (i < U_WD + U_DISC ? 1 : 2);
#pragma omp atomic
            g_ucost[i] += cost[i];
#pragma omp atomic
            g_cnt[4 + reg * 8 + std::min(cost[i], 7)] += 1;
        }
        cm += m; ++nc;
    }
#pragma omp atomic
    g_cnt[0] += n;
#pragma omp atomic
    g_cnt[1] += ls;
#pragma omp atomic
    g_cnt[2] += nc;
#pragma omp atomic
    g_cnt[3] += cm;
}
#define LFC_NIT int nit[3] = {0, 0, 0}; bool fb = false; double gs[2] = {0.0, 0.0};
#define LFC_NITARGS , &fb, nit, gs
#if LFC_COST_MODE == 1  // FP32 lockstep steps only (LFG_F32_FIRST counts them x 1000 in nit[0])
#define LFC_COST(v) cost[v] = nit[0] / 1000
#elif LFC_COST_MODE == 2  // everything else
#define LFC_COST(v) cost[v] = nit[0] % 1000 + std::max(nit[1], nit[2]) + (fb ? 30 : 0)
#else
#define LFC_COST(v) cost[v] = nit[0] + std::max(nit[1], nit[2]) + (fb ? 30 : 0)
#endif
// element intervals in solve order (run with one thread to compare variants)
static std::vector<double> g_ab;
extern "C" long lfc_dump(double* o, long n)
{
    const long m = std::min<long>(n, long(g_ab.size()));
    for (long i = 0; i < m; ++i) o[i] = g_ab[i];
    g_ab.clear();
    return m;
}
#define LFC_AB(a, b) do { _Pragma("omp critical") { g_ab.push_back(a); g_ab.push_back(b); g_gs.push_back(gs[0]); g_gs.push_back(gs[1]); } } while (0)
static std::vector<double> g_gs;  // the initial guesses (rad) of the same solves
extern "C" long lfc_dump_guess(double* o, long n)
{
    const long m = std::min<long>(n, long(g_gs.size()));
    for (long i = 0; i < m; ++i) o[i] = g_gs[i];
    g_gs.clear();
    return m;
}
#else
#define LFC_NIT
#define LFC_NITARGS
#define LFC_COST(v)
#define LFC_AB(a, b)
#endif

void elements(const Pair& G, Tables& T)
{
#ifdef LFC_COUNT
    int cost[U_WD + U_DISC + NBS] = {0};
#endif
    const Roche& R = G.R;
    const double s = G.s, c = G.c;
    const double twd = TWO_PI * ((1.0 - G.ulimb) * 0.5 + G.ulimb / 3.0);
    const double td = TWO_PI * (disc_boundary(NDISC_R, G) - disc_boundary(0, G));
    int k = 0;
    for (int u = 0; u < U_WD + U_DISC; ++u) {
        double Px, Py, Pz, wgt;
        bool isw = u < U_WD;
        if (isw) {
            const int ir = wd_ring_of(u);
            const double rc = kWdRc[ir], mu0 = kWdMu0[ir], cp = kWdCos[u], sp = kWdSin[u];
            Px = G.rwd_a * (-rc * sp * c + mu0 * s);
            Py = G.rwd_a * (rc * cp);
            Pz = G.rwd_a * (rc * sp * s + mu0 * c);
            wgt = std::fma(kWdA[ir], 1.0 - G.ulimb, kWdB[ir] * G.ulimb) / twd;
        } else {
            const int uu = u - U_WD, ir = uu / (NDISC_AZ / 2), j = uu - ir * (NDISC_AZ / 2);
            const double rc = G.rwd_a + (ir + 0.5) * ((G.rdisc_a - G.rwd_a) / NDISC_R);
            Px = rc * kDiscCos[j];
            Py = rc * kDiscSin[j];
            Pz = 0.0;
            wgt = (TWO_PI / NDISC_AZ) * (disc_boundary(ir + 1, G) - disc_boundary(ir, G)) / td;
        }
        double a, b;
        LFC_NIT
        element_interval_fast(R, Px, Py, Pz, s, c, G.rcal, G.reff, a, b LFC_NITARGS);
        LFC_COST(u);
        LFC_AB(a, b);
        T.a[k] = a; T.b[k] = b; T.w[k] = wgt; T.wd[k] = isw; ++k;
        const bool ecl = a < b;  // the mirror image's interval (MODEL_SPEC 7)
        T.a[k] = ecl ? -b : 1.0; T.b[k] = ecl ? -a : -1.0; T.w[k] = wgt; T.wd[k] = isw; ++k;
    }
    double tot = 0.0;
    for (int j = 0; j < NBS; ++j) {
        const double uk = (j + 0.5) * (G.umax / NBS);
        T.sw[j] = std::exp(G.exp1 * std::log(uk) - std::pow(uk, G.exp2) - G.lnpk);
        tot += T.sw[j];
        const double off = G.L * (uk - G.upk);
        LFC_NIT
        element_interval_fast(R, std::fma(off, G.caz, G.bsx), std::fma(off, G.saz, G.bsy), 0.0, s, c, G.rcal, G.reff,
                              T.sa[j], T.sb[j] LFC_NITARGS);
        LFC_COST(U_WD + U_DISC + j);
        LFC_AB(T.sa[j], T.sb[j]);
    }
#ifdef LFC_COUNT
    count_pair(cost, U_WD + U_DISC + NBS);
#endif
    for (int j = 0; j < NBS; ++j) T.sw[j] /= tot;
    double dn = 0.0;
    for (int uu = 0; uu < U_DON; ++uu) {
        const int it = uu / (NDONOR_P / 4), ip = uu - it * (NDONOR_P / 4);
        const double dx = -kDonCt[it], dy = kDonSt[it] * kDonCp[ip], dz = kDonSt[it] * kDonSp[ip];
        double lo = 0.0, hi = R.Rs, r = G.reff, gx, gy, gz;
        if (!(r > lo && r < hi)) r = 0.5 * hi;
        for (int itr = 0; itr < ROOT_MAXIT; ++itr) {
            const double f = rpot_grad(R, std::fma(r, dx, 1.0), r * dy, r * dz, gx, gy, gz) - R.pl1;
            const double df = gx * dx + gy * dy + gz * dz;
            if (f > 0.0) hi = r; else lo = r;
            if (df > 0.0 && std::fabs(f / df) <= ROOT_LAST) { r -= f / df; break; }
            double rn = (df > 0.0) ? r - f / df : 0.5 * (lo + hi);
            if (!(rn > lo && rn < hi)) rn = 0.5 * (lo + hi);
            r = rn;
        }
        rgrad(R, std::fma(r, dx, 1.0), r * dy, r * dz, gx, gy, gz);
        const double ig = 1.0 / std::sqrt(gx * gx + gy * gy + gz * gz);
        const double nx = gx * ig, ny = gy * ig, nz = gz * ig;
        const double dA = r * r * kDonOmega[it] / (nx * dx + ny * dy + nz * dz);
        const double vx = dA * nx, vy = dA * ny, vz = dA * nz;
        const double srho = s * std::sqrt(vx * vx + vy * vy);
        const double kap = (srho > 0.0) ? -c * vz / srho : (c * vz > 0.0 ? -2.0 : 2.0);
        const double cen = -std::atan2(vy, vx) / TWO_PI, hw = std::acos(std::fmin(std::fmax(kap, -1.0), 1.0)) / TWO_PI;
        for (int mr = 0; mr < 4; ++mr) {  // mirror images (vx, +-vy, +-vz)
            const int t = 4 * uu + mr;
            T.dv[t][0] = vx;
            T.dv[t][1] = (mr & 1) ? -vy : vy;
            T.dv[t][2] = (mr & 2) ? -vz : vz;
            T.dcen[t] = (mr & 1) ? -cen : cen;
            T.dhw[t] = (mr & 2) ? 0.5 - hw : hw;
            dn += std::fmax(-s * T.dv[t][1] + c * T.dv[t][2], 0.0);
        }
    }
    T.dnorm = dn;
}

double wrap_phase(double ph) { return ph - std::floor(ph + 0.5); }

// sorted windows [lo, hi] (1 / width iw): add wn x covered fraction of
// [a, b] to acc (difference array d for whole-covered runs, partial
// windows directly); zero-width windows are points, a < ph < b
void sweep_window(const double* lo, const double* hi, const double* iw, int m, double a, double b, double wn,
                  double* d, double* direct)
{
    const int P2 = int(std::lower_bound(lo, lo + m, a) - lo);   // #{lo < a}
    const int P4 = int(std::lower_bound(lo, lo + m, b) - lo);   // #{lo < b}
    const int P1 = int(std::upper_bound(hi, hi + m, a) - hi);   // #{hi <= a}
    const int P3 = int(std::upper_bound(hi, hi + m, b) - hi);   // #{hi <= b}
    int e0 = P4, s1 = P4;
    if (P2 < P3) {
        d[P2] += wn;
        d[P3] -= wn;
        e0 = P2;
        s1 = P3;
    }
    for (int r = 0; r < 2; ++r)
        for (int p = r ? s1 : P1; p < (r ? P4 : e0); ++p) {
            if (hi[p] > lo[p]) {
                const double ov = std::fmin(b, hi[p]) - std::fmax(a, lo[p]);
                if (ov > 0.0) direct[p] += wn * ov * iw[p];
            } else if (a < lo[p] && lo[p] < b) {
                direct[p] += wn;
            }
        }
}

// point mode: add v (3-vector) to the phases ph (sorted) strictly inside (x1, x2)
void sweep_points(const double* ph, int m, double x1, double x2, const double* v, std::vector<double>& d3)
{
    const int P = int(std::upper_bound(ph, ph + m, x1) - ph), Q = int(std::lower_bound(ph, ph + m, x2) - ph);
    if (P < Q)
        for (int k = 0; k < 3; ++k) {
            d3[3 * P + k] += v[k];
            d3[3 * Q + k] -= v[k];
        }
}

// chi^2 of one pair against its light curve (k_lnlike restated on the host)
double chisq(const Pair& G, const Tables& T, const double* x, const double* w, const double* y, const double* ye, int n,
             int S, std::vector<double>& buf, double* fout = nullptr)
{
    // point windows, and the sub-bin windows / centres (flattened, sorted when
    // the windows are)
    const int ns = n * S;
    buf.assign(size_t(9) * n + size_t(10) * ns + 8, 0.0);
    double* lo = buf.data();
    double* hi = lo + n;
    double* iw = hi + n;
    double* dw = iw + n;       // WD difference array [n + 1]
    double* dd = dw + n + 1;   // disc
    double* xw = dd + n + 1;   // WD direct
    double* xd = xw + n;       // disc direct
    double* slo = xd + n + 1;  // sub-bin windows
    double* shi = slo + ns;
    double* siw = shi + ns;
    double* sph = siw + ns;
    double* ds = sph + ns;      // spot difference array [ns + 1]
    double* xs = ds + ns + 1;   // spot direct
    bool sorted = true;
    for (int p = 0; p < n; ++p) {
        const double ph = wrap_phase(x[p] - G.phi0), h = (w && !(w[p] < 0.0)) ? w[p] : 0.0;  // MODEL_SPEC 3
        lo[p] = ph - h;
        hi[p] = ph + h;
        iw[p] = 1.0 / (2.0 * h);
        sorted = sorted && h >= 0.0 && (p == 0 || (lo[p] >= lo[p - 1] && hi[p] >= hi[p - 1]));
        const double hs = h / S;
        for (int j = 0; j < S; ++j) {
            const int q = p * S + j;
            sph[q] = wrap_phase(ph - h + (2 * j + 1) * hs);
            slo[q] = sph[q] - hs;
            shi[q] = sph[q] + hs;
            siw[q] = 1.0 / (2.0 * hs);
            sorted = sorted && (q == 0 || (slo[q] >= slo[q - 1] && shi[q] >= shi[q - 1] && sph[q] >= sph[q - 1]));
        }
    }
    std::vector<double> d3(size_t(3) * (ns + 1), 0.0);
    std::vector<double> eb(ns, 0.0), V(size_t(3) * ns, 0.0);
    std::vector<double> fw(n, 0.0), fd(n, 0.0);
    if (sorted) {
        for (int k = 0; k < NWD + NDISC; ++k)
            if (T.a[k] < T.b[k]) sweep_window(lo, hi, iw, n, T.a[k], T.b[k], T.w[k], T.wd[k] ? dw : dd, T.wd[k] ? xw : xd);
        for (int k = 0; k < NBS; ++k)
            if (T.sa[k] < T.sb[k]) sweep_window(slo, shi, siw, ns, T.sa[k], T.sb[k], T.sw[k], ds, xs);
        for (int t = 0; t < NDONOR; ++t) {
            const double cen = T.dcen[t], hwd = T.dhw[t];
            if (!(hwd > 0.0)) continue;
            if (hwd >= 0.5) { sweep_points(sph, ns, -INFINITY, INFINITY, T.dv[t], d3); continue; }
            const double l = cen - hwd, h = cen + hwd;
            if (l < -0.5) {
                sweep_points(sph, ns, -INFINITY, h, T.dv[t], d3);
                sweep_points(sph, ns, l + 1.0, INFINITY, T.dv[t], d3);
            } else if (h > 0.5) {
                sweep_points(sph, ns, -INFINITY, h - 1.0, T.dv[t], d3);
                sweep_points(sph, ns, l, INFINITY, T.dv[t], d3);
            } else {
                sweep_points(sph, ns, l, h, T.dv[t], d3);
            }
        }
        double aw = 0.0, ad = 0.0, as = 0.0, av[3] = {0.0, 0.0, 0.0};
        for (int p = 0; p < n; ++p) {
            aw += dw[p];
            ad += dd[p];
            fw[p] = aw + xw[p];
            fd[p] = ad + xd[p];
        }
        for (int q = 0; q < ns; ++q) {
            as += ds[q];
            eb[q] = as + xs[q];
            for (int k = 0; k < 3; ++k) {
                av[k] += d3[3 * q + k];
                V[3 * q + k] = av[k];
            }
        }
    } else {  // unsorted windows: every element against each point
        for (int p = 0; p < n; ++p)
            for (int k = 0; k < NWD + NDISC; ++k) {
                if (!(T.a[k] < T.b[k])) continue;
                double cov;
                if (hi[p] > lo[p]) cov = std::fmax(std::fmin(T.b[k], hi[p]) - std::fmax(T.a[k], lo[p]), 0.0) * iw[p];
                else cov = (T.a[k] < lo[p] && lo[p] < T.b[k]) ? 1.0 : 0.0;
                (T.wd[k] ? fw[p] : fd[p]) += T.w[k] * cov;
            }
        for (int q = 0; q < ns; ++q) {
            for (int k = 0; k < NBS; ++k) {
                if (!(T.sa[k] < T.sb[k])) continue;
                double cov;
                if (shi[q] > slo[q]) cov = std::fmax(std::fmin(T.sb[k], shi[q]) - std::fmax(T.sa[k], slo[q]), 0.0) * siw[q];
                else cov = (T.sa[k] < sph[q] && sph[q] < T.sb[k]) ? 1.0 : 0.0;
                eb[q] += T.sw[k] * cov;
            }
            const double e0 = G.s * std::cos(TWO_PI * sph[q]), e1 = -G.s * std::sin(TWO_PI * sph[q]);
            for (int t = 0; t < NDONOR; ++t)
                if (T.dv[t][0] * e0 + T.dv[t][1] * e1 + T.dv[t][2] * G.c > 0.0)
                    for (int k = 0; k < 3; ++k) V[3 * q + k] += T.dv[t][k];
        }
    }
    double chi = 0.0;
    for (int p = 0; p < n; ++p) {
        double sbs = 0.0, srs = 0.0;
        for (int j = 0; j < S; ++j) {
            const int q = p * S + j;
            const double e0 = G.s * std::cos(TWO_PI * sph[q]), e1 = -G.s * std::sin(TWO_PI * sph[q]);
            const double D = e0 * V[3 * q] + e1 * V[3 * q + 1] + G.c * V[3 * q + 2];
            double beam = 0.0;
            if (G.bden > 0.0) beam = (G.fis + (1.0 - G.fis) * std::fmax(G.nb0 * e0 + G.nb1 * e1 + G.nb2 * G.c, 0.0)) / G.bden;
            sbs += beam * (1.0 - eb[q]);
            srs += D / T.dnorm;
        }
        const double f = G.wdf * (1.0 - fw[p]) + G.df * (1.0 - fd[p]) + G.sf * sbs / S + G.rsf * srs / S;
        if (fout) {  // GP trees: the model flux, the residuals are the caller's
            fout[p] = f;
            continue;
        }
        if (std::isnan(f)) return INFINITY;
        const double r = (y[p] - f) / ye[p];
        chi += r * r;
    }
    return chi;
}

// SimpleGPEclipse.calcChangepoints when the cache rule trips (k_gp_dcp):
// dist_cp = (dphi + phi4 - phi3) / 2, phi3 / phi4 the extreme egress phases
// of ten limb points of a sphere of radius rwd (units of x_L1, as the
// reference passes it) at the WD-centre egress phase; NaN when none is
// eclipsed or a solve fails
double gp_dcp(const Pair& G, double dphi, double rwd)
{
    const Roche& R = G.R;
    double dphi_c;
    if (!(rwd > 0.0) || findphi_fast(R, G.inc, dphi_c) != ST_OK) return NAN;
    const double sth = std::sin(PI * dphi_c), cth = std::cos(PI * dphi_c);
    double lo = INFINITY, hi = -INFINITY;
    for (int k = 0; k < 10; ++k) {
        const double sp = std::sin(TWO_PI * k / 10), cp = std::cos(TWO_PI * k / 10);
        double a, b;
        if (element_interval(R, rwd * (cp * sth - sp * G.c * cth), rwd * (cp * cth + sp * G.c * sth), rwd * (sp * G.s),
                             G.s, G.c, eggleton(R.q), a, b)) {
            lo = std::fmin(lo, b);
            hi = std::fmax(hi, b);
        }
    }
    return lo <= hi ? (dphi + (hi - lo)) / 2.0 : NAN;
}

// the GP ln_like of one pair (SimpleGPEclipse.ln_like, CVModel.py:650-696)
double gp_lnlike(const Pair& G, const Tables& T, const double* v, const double* consts, const double* pin, int e,
                 const int* gp_gather, const double* gp_base, const int* gp_ecl, const double* x, const double* w,
                 const double* y, const double* ye, int n, int S, std::vector<double>& buf, std::vector<double>& res)
{
    auto par = [&](int g) { return g >= 0 ? v[g] : consts[-1 - g]; };
    const int* gg = gp_gather + 3 * e;
    const double ain = std::exp(par(gg[0])), aout = std::exp(par(gg[1])), tau = std::exp(par(gg[2]));
    if (!(tau > 0.0 && std::isfinite(ain) && std::isfinite(aout))) return -INFINITY;
    const double* B = gp_base + 4 * e;
    const double q = G.R.q, dphi = pin[5], rwd = pin[8];
    const bool pend = std::fabs(B[1] - dphi) / dphi > 1.2 || std::fabs(B[0] - q) / q > 1.2 ||
                      std::fabs(B[2] - rwd) / rwd > 1.2;
    const double dcp = pend ? gp_dcp(G, dphi, rwd) : B[3];
    if (!std::isfinite(dcp)) return -INFINITY;
    res.resize(n > 0 ? n : 1);
    chisq(G, T, x, w, y, ye, n, S, buf, res.data());
    GPFilter F;
    F.init(ain, aout, tau);
    for (int p = 0; p < n; ++p) {
        const double r = y[p] - res[p];
        if (!std::isfinite(r)) return -INFINITY;
        F.step(x[p], ye[p], r, gp_block(x[p], gp_ecl[2 * e], gp_ecl[2 * e + 1], dcp, G.phi0));
    }
    return F.lnlike();
}

}  // namespace

extern "C" {

// ln_prob of W walkers of a compiled chi^2 tree (the oracle's
// lfo_lnprob_batch arguments); returns the threads used
int lfc_lnprob_batch_gp(const double* walkers, int W, int ndim, int E, const int* gather, const int* npars,
                        const double* consts, const int* off, const double* x, const double* y, const double* ye,
                        const double* w, int nsub, const int* prior_type, const double* prior_p1,
                        const double* prior_p2, const double* prior_norm, int roche_priors, const int* gp_gather,
                        const double* gp_base, const int* gp_ecl, double* lnp, int nthreads);

int lfc_lnprob_batch(const double* walkers, int W, int ndim, int E, const int* gather, const int* npars,
                     const double* consts, const int* off, const double* x, const double* y, const double* ye,
                     const double* w, int nsub, const int* prior_type, const double* prior_p1, const double* prior_p2,
                     const double* prior_norm, int roche_priors, double* lnp, int nthreads)
{
    return lfc_lnprob_batch_gp(walkers, W, ndim, E, gather, npars, consts, off, x, y, ye, w, nsub, prior_type,
                               prior_p1, prior_p2, prior_norm, roche_priors, nullptr, nullptr, nullptr, lnp, nthreads);
}

// the same with a GP likelihood per eclipse (gp_gather [E][3]: ln_ampin,
// ln_ampout, ln_tau; gp_base [E][4]: the changepoint cache q, dphi, rwd,
// dist_cp; gp_ecl [E][2]: first and last eclipse number); all null: chi^2
int lfc_lnprob_batch_gp(const double* walkers, int W, int ndim, int E, const int* gather, const int* npars,
                        const double* consts, const int* off, const double* x, const double* y, const double* ye,
                        const double* w, int nsub, const int* prior_type, const double* prior_p1,
                        const double* prior_p2, const double* prior_norm, int roche_priors, const int* gp_gather,
                        const double* gp_base, const int* gp_ecl, double* lnp, int nthreads)
{
    if (nthreads <= 0) nthreads = omp_get_max_threads();
    // a changepoint cache the host never filled (dist_cp NaN): findi +
    // wdphases at the cache's q, dphi, rwd (as the evaluator does)
    std::vector<double> base;
    if (gp_gather) {
        base.assign(gp_base, gp_base + 4 * E);
        for (int e = 0; e < E; ++e) {
            double* B = &base[4 * e];
            if (std::isfinite(B[3])) continue;
            Pair G{};
            double inc;
            if (roche_init(G.R, B[0]) != ST_OK || findi_fast(G.R, B[1], inc) != ST_OK) continue;
            G.inc = inc;
            G.s = std::sin(inc * DEG);
            G.c = std::cos(inc * DEG);
            B[3] = gp_dcp(G, B[1], B[2]);
        }
        gp_base = base.data();
    }
    int used = 1;
#pragma omp parallel num_threads(nthreads)
    {
#pragma omp single
        used = omp_get_num_threads();
        std::vector<double> buf, res;
        std::vector<Pair> pairs(E);
        std::vector<double> pins(size_t(18) * E);
        std::vector<int> status(E);
        Tables* T = new Tables;
#pragma omp for schedule(dynamic, 1)
        for (int iw = 0; iw < W; ++iw) {
            const double* v = walkers + size_t(iw) * ndim;
            double lp = 0.0;
            auto par = [&](int g) { return g >= 0 ? v[g] : consts[-1 - g]; };
            if (roche_priors) {  // LCModel.ln_prior: dphi <= findphi(q, 90) - 1e-6 (CVModel.py:452-473)
                Roche R;
                double maxphi = -INFINITY;
                if (roche_init(R, par(gather[4])) == ST_OK && findphi_fast(R, 90.0, maxphi) != ST_OK) maxphi = -INFINITY;
                if (!(par(gather[5]) <= maxphi - DPHI_TOL)) lp = -INFINITY;
            }
            for (int d = 0; d < ndim && lp > -INFINITY; ++d)
                lp += lfg::prior_lnprob(prior_type[d], prior_p1[d], prior_p2[d], prior_norm[d], v[d]);  // Prior.ln_prob (model.py:83-113)
            double pin[18];
            for (int e = 0; e < E && lp > -INFINITY; ++e) {
                for (int k = 0; k < npars[e]; ++k) pin[k] = par(gather[e * 18 + k]);
                std::copy(pin, pin + 18, pins.begin() + 18 * e);
                double rp;
                status[e] = setup_pair(pin, npars[e], pairs[e], rp);
                if (roche_priors) lp += rp;
            }
            double ll = 0.0;
            for (int e = 0; e < E && lp > -INFINITY; ++e) {
                if (status[e] != ST_OK) { ll = -INFINITY; break; }
                elements(pairs[e], *T);
                const int n = off[e + 1] - off[e];
                if (gp_gather)
                    ll += gp_lnlike(pairs[e], *T, v, consts, &pins[18 * e], e, gp_gather, gp_base, gp_ecl, x + off[e],
                                    w ? w + off[e] : nullptr, y + off[e], ye + off[e], n, nsub, buf, res);
                else
                    ll += -0.5 * chisq(pairs[e], *T, x + off[e], w ? w + off[e] : nullptr, y + off[e], ye + off[e], n,
                                       nsub, buf);
            }
            lnp[iw] = lp > -INFINITY ? lp + ll : -INFINITY;
        }
        delete T;
    }
    return used;
}

}  // extern "C"

// per parameter set: setup, elements, then f(pair, tables) -> its outputs
template <typename F>
static int per_set(const double* pars, int W, int P, int* status, int nthreads, F f)
{
    if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel num_threads(nthreads)
    {
        std::vector<double> buf;
        Tables* T = new Tables;
#pragma omp for schedule(dynamic, 1)
        for (int i = 0; i < W; ++i) {
            Pair G{};
            double rp;
            const int st = setup_pair(pars + size_t(i) * P, P, G, rp);
            if (status) status[i] = st;
            if (st == ST_OK) elements(G, *T);
            f(i, st, G, *T, buf);
        }
        delete T;
    }
    return LFG_OK;
}

extern "C" {

// ---- the lfg_cpu_* twins of include/lfg.h's entry points (lfg_cpu.h):
// host pointers, the same argument meaning and status codes
int lfg_cpu_flux(const double* pars, int W, int P, const double* x, const double* w, int N, int nsub, double* flux,
                 int* status, int nthreads)
{
    if (W <= 0 || N < 0 || nsub < 1 || (P != 14 && P != 18) || !pars || !flux || (N > 0 && !x)) return LFG_E_ARGS;
    return per_set(pars, W, P, status, nthreads,
                   [&](int i, int st, const Pair& G, const Tables& T, std::vector<double>& buf) {
                       double* f = flux + size_t(i) * N;
                       if (st != ST_OK) { std::fill(f, f + N, NAN); return; }
                       chisq(G, T, x, w, nullptr, nullptr, N, nsub, buf, f);
                   });
}

int lfg_cpu_lnlike(const double* pars, int W, int P, const double* x, const double* w, int N, int nsub,
                   const double* y, const double* ye, double* lnlike, int* status, int nthreads)
{
    if (W <= 0 || N < 0 || nsub < 1 || (P != 14 && P != 18) || !pars || !lnlike || (N > 0 && (!x || !y || !ye)))
        return LFG_E_ARGS;
    return per_set(pars, W, P, status, nthreads,
                   [&](int i, int st, const Pair& G, const Tables& T, std::vector<double>& buf) {
                       lnlike[i] = (st != ST_OK) ? -INFINITY : -0.5 * chisq(G, T, x, w, y, ye, N, nsub, buf);
                   });
}

int lfg_cpu_lnprob(const double* walkers, int W, const lfg_tree* T, double* lnp, int nthreads)
{
    if (W <= 0 || !T || T->E <= 0 || T->ndim <= 0 || !walkers || !lnp) return LFG_E_ARGS;
    lfc_lnprob_batch_gp(walkers, W, T->ndim, T->E, T->gather, T->npars, T->consts, T->off, T->x, T->y, T->ye, T->w,
                        T->nsub, T->prior_type, T->prior_p1, T->prior_p2, T->prior_norm, T->roche_priors,
                        T->gp ? T->gp_gather : nullptr, T->gp ? T->gp_base : nullptr, T->gp ? T->gp_ecl : nullptr, lnp,
                        nthreads);
    if (T->fixed_invalid)
        for (int i = 0; i < W; ++i) lnp[i] = -INFINITY;
    return LFG_OK;
}

}  // extern "C"
