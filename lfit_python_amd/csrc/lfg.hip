// lfg.hip -- MI355X (gfx950) kernels and the C ABI of liblfg_hip.so.
//
// Pipeline for one batch of walkers (one emcee half-step):
//   k_setup     one lane per (walker, eclipse): parameter gather, L1, findi,
//               bright-spot stream, strip/beam frame, eclipse Roche priors;
//               extra lanes per walker: LCModel dphi prior + Prior.ln_prob sum
//   k_elements  one lane per (walker, eclipse, element): eclipse interval of
//               every WD / disc / bright-spot element, donor surface tiles
//   k_lnlike    one workgroup per (walker, eclipse): element tables staged in
//               LDS, lanes stride the phase axis (coalesced), exposure
//               integration, fused chi^2 with a wavefront/LDS reduction
//   k_combine   one lane per walker: ln_prob = ln_prior + sum_e ln_like_e
// Replaces, per walker, mcmcfit.ln_prob (mcmcfit.py:37-41) -> Node.ln_prob
// (model.py:476-498) -> lfit.CV.calcFlux (CVModel.py:138).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lfg.h"
#include "lfg_device.hpp"
#include "lfg_tables.hpp"

using namespace lfg;

namespace {

constexpr int SETUP_BLOCK = 64;
constexpr int ELEM_BLOCK = 256;

__device__ const int kIdentityGather[18] = {0, 1, 2, 3, 4, 5, 6, 7, 8,
                                            9, 10, 11, 12, 13, 14, 15, 16, 17};

struct Ws {
    double* geo;
    int* status;
    double2* ab;    // [pairs][NEL] eclipse intervals (a, b)
    double* donor;  // [pairs][NDONOR/4][3] symmetry-unique donor tiles
    double* prior;
    double* lle;
    size_t total;
};

inline size_t align256(size_t v) { return (v + 255) & ~size_t(255); }

Ws carve(void* base, int W, int E)
{
    const size_t pairs = size_t(W) * size_t(E);
    Ws ws{};
    char* p = static_cast<char*>(base);
    size_t off = 0;
    auto take = [&](size_t bytes) { char* r = p ? p + off : nullptr; off += align256(bytes); return r; };
    ws.geo = reinterpret_cast<double*>(take(pairs * LFG_NGEO * sizeof(double)));
    ws.status = reinterpret_cast<int*>(take(pairs * sizeof(int)));
    ws.ab = reinterpret_cast<double2*>(take(pairs * NEL * sizeof(double2)));
    ws.donor = reinterpret_cast<double*>(take(pairs * (NDONOR / 4) * 3 * sizeof(double)));
    ws.prior = reinterpret_cast<double*>(take(size_t(W) * sizeof(double)));
    ws.lle = reinterpret_cast<double*>(take(pairs * sizeof(double)));
    ws.total = off;
    return ws;
}

// ---------------------------------------------------------------- k_setup
struct SetupArgs {
    const double* walkers;
    int W, ndim, E, P;
    const int* gather;  // nullptr -> identity
    const int* npars;   // nullptr -> P
    const double* consts;
    const int* prior_type;
    const double* prior_p1;
    const double* prior_p2;
    const double* prior_norm;
    int roche_priors;
    double* geo;
    int* status;
    double* prior;
};

__device__ inline double gather_par(const SetupArgs& A, int w, int g)
{
    return g >= 0 ? A.walkers[size_t(w) * A.ndim + g] : A.consts[-1 - g];
}

__global__ __launch_bounds__(SETUP_BLOCK) void k_setup(SetupArgs A)
{
    const int t = blockIdx.x * SETUP_BLOCK + threadIdx.x;
    const int npairs = A.W * A.E;
    if (t >= npairs + A.W) return;
    const int* gat = A.gather ? A.gather : kIdentityGather;

    if (t >= npairs) {
        // per-walker lane: LCModel.ln_prior dphi check (CVModel.py:452-473)
        // and Node.ln_prior over the variable parameters (model.py:439-449)
        const int w = t - npairs;
        double lp = 0.0;
        if (A.roche_priors) {
            const double q = gather_par(A, w, gat[4]);
            const double dphi = gather_par(A, w, gat[5]);
            Roche R;
            double maxphi;
            if (roche_init(R, q) != ST_OK || findphi_fast(R, 90.0, maxphi) != ST_OK) lp = -INFINITY;
            else if (dphi > maxphi - DPHI_TOL) lp = -INFINITY;
        }
        if (A.prior_type) {
            const double* v = A.walkers + size_t(w) * A.ndim;
            for (int d = 0; d < A.ndim && isfinite(lp); ++d)
                lp += prior_lnprob(A.prior_type[d], A.prior_p1[d], A.prior_p2[d], A.prior_norm[d], v[d]);
        }
        A.prior[w] = lp;
        return;
    }

    const int w = t / A.E, e = t - (t / A.E) * A.E;
    const int np = A.npars ? A.npars[e] : A.P;
    double p[18];
    bool finite = (np == 14 || np == 18);
    for (int k = 0; k < 18; ++k) {
        p[k] = (k < np) ? gather_par(A, w, gat[e * 18 + k]) : 0.0;
        finite = finite && isfinite(p[k]);
    }
    if (np == 14) { p[14] = 2.0; p[15] = 1.0; p[16] = 90.0; p[17] = 0.0; }  // MODEL_SPEC 5.3
    double* G = A.geo + size_t(t) * LFG_NGEO;
    int st = ST_OK;
    double rprior = 0.0;
    Roche R;
    if (!finite) st = ST_BAD_ARGS;
    else st = roche_init(R, p[4]);

#ifdef LFG_PROFILE_SETUP
    // diagnostic build only: phase cycle counts into spare geo slots
    unsigned long long tp0 = __builtin_amdgcn_s_memtime(), tp1 = tp0, tp2 = tp0, tp3 = tp0;
#define LFG_STAMP(v) (v) = __builtin_amdgcn_s_memtime()
#else
#define LFG_STAMP(v)
#endif
    double bs[4] = {0.0, 0.0, 0.0, 0.0};
    int bst = ST_BAD_STREAM;
    LFG_STAMP(tp1);
    if (st == ST_OK) {
        const double rdisc_a = p[6] * R.xl1;
        bst = bspot(R, rdisc_a, bs);
        LFG_STAMP(tp2);
        // SimpleEclipse.ln_prior Roche checks (CVModel.py:215-316)
        if (rdisc_a > DISC_MAX_A) rprior = -INFINITY;
        const double rwd = p[8], scale = p[9];
        if (scale > rwd * 3.0 || scale < rwd / 3.0) rprior = -INFINITY;
        if (bst != ST_OK) rprior = -INFINITY;
        else {
            double alpha = atan2(bs[1], bs[0]) / DEG;
            if (alpha < 0.0) alpha = 90.0 - alpha;
            const double tangent = alpha + 90.0;
            const double minaz = fmax(0.0, tangent - AZ_SLOPE), maxaz = fmin(178.0, tangent + AZ_SLOPE);
            if (p[10] < minaz || p[10] > maxaz) rprior = -INFINITY;
        }
    } else {
        rprior = -INFINITY;
    }

    double inc = 0.0;
    if (st == ST_OK) st = findi_fast(R, p[5], inc);
    LFG_STAMP(tp3);
#ifdef LFG_PROFILE_SETUP
    {
        double mp;
        const unsigned long long ta = __builtin_amdgcn_s_memtime();
        findphi_fast(R, 90.0, mp);
        const unsigned long long tb = __builtin_amdgcn_s_memtime();
        const double um = bs_umax(p[14], p[15], p[14] * log(pow(p[14] / p[15], 1.0 / p[15])) - p[14] / p[15]);
        const unsigned long long tc2 = __builtin_amdgcn_s_memtime();
        G[42] = double(tp1 - tp0);
        G[43] = double(tp2 - tp1);
        G[44] = double(tp3 - tp2);
        G[45] = double(tb - ta);
        G[46] = double(tc2 - tb) + 0.0 * um;
    }
#endif
    const double rwd_a = p[8] * R.xl1, rdisc_a = p[6] * R.xl1;
    if (st == ST_OK && (!(rwd_a > 0.0) || !(rdisc_a > rwd_a) || !(rdisc_a < R.xl1))) st = ST_BAD_GEOMETRY;
    if (st == ST_OK && (!(p[9] > 0.0) || !(p[14] > 0.0) || !(p[15] > 0.0))) st = ST_BAD_GEOMETRY;
    if (st == ST_OK && bst != ST_OK) st = bst;

    A.status[t] = st;
    G[G_RPRIOR] = A.roche_priors ? rprior : 0.0;
    if (st != ST_OK) return;

    double s, c;
    sincos(inc * DEG, &s, &c);
    const double a1 = p[14], a2 = p[15];
    const double upk = pow(a1 / a2, 1.0 / a2);
    const double lnpk = a1 * log(upk) - pow(upk, a2);
    const double tilt = p[16] * DEG, psi = (p[10] - 90.0 + p[17]) * DEG;
    double st_, ct_, sp_, cp_;
    sincos(tilt, &st_, &ct_);
    sincos(psi, &sp_, &cp_);
    const double nmax = fabs(st_) * s + ct_ * c;
    double saz, caz;
    sincos(p[10] * DEG, &saz, &caz);

    G[G_Q] = R.q; G[G_CA] = R.cA; G[G_CB] = R.cB; G[G_MU] = R.mu;
    G[G_XL1] = R.xl1; G[G_PL1] = R.pl1; G[G_RS] = R.Rs; G[G_RS2] = R.Rs2;
    G[G_S] = s; G[G_C] = c; G[G_INC] = inc;
    G[G_RWD] = rwd_a; G[G_RDISC] = rdisc_a; G[G_REFF] = eggleton(R.q);
    G[G_ULIMB] = p[7]; G[G_DEXP] = p[12];
    G[G_BSX] = bs[0]; G[G_BSY] = bs[1]; G[G_BSVX] = bs[2]; G[G_BSVY] = bs[3];
    G[G_L] = p[9] * R.xl1; G[G_UPK] = upk; G[G_UMAX] = bs_umax(a1, a2, lnpk); G[G_LNPK] = lnpk;
    G[G_EXP1] = a1; G[G_EXP2] = a2; G[G_CAZ] = caz; G[G_SAZ] = saz;
    G[G_NB0] = st_ * cp_; G[G_NB1] = st_ * sp_; G[G_NB2] = ct_;
    G[G_BDEN] = p[11] + (1.0 - p[11]) * fmax(nmax, 0.0);
    G[G_FIS] = p[11]; G[G_PHI0] = p[13];
    G[G_WDF] = p[0]; G[G_DF] = p[1]; G[G_SF] = p[2]; G[G_RSF] = p[3];
    const double sce = s * cos(PI * p[5]);
    G[G_RCAL] = sqrt(1.0 - sce * sce);
}

// ------------------------------------------------------------- k_elements
// One lane per symmetry-unique element.  The WD/disc grids are mirror
// symmetric under y -> -y and the donor grid under y -> -y and z -> -z; the
// Roche potential shares those symmetries, so a mirrored element's eclipse
// interval is [-b, -a] and a mirrored tile's vector has y (and/or z) negated.
// Unique items per (walker, eclipse): WD 200, disc 500, spot 100, donor 100.
// Output: eclipse intervals as (a, b) pairs and the 100 unique donor tile
// vectors; weights depend on ring only and are formed in k_lnlike.
constexpr int U_WD = NWD / 2, U_DISC = NDISC / 2, U_BS = NBS, U_DON = NDONOR / 4;
constexpr int NUNIQ = U_WD + U_DISC + U_BS + U_DON;

__device__ __forceinline__ int wd_ring_of(int u)  // ring of unique WD tile u (ring ir starts at 2 ir^2)
{
    int ir = int(sqrt(u * 0.5));
    if (2 * (ir + 1) * (ir + 1) <= u) ++ir;
    if (2 * ir * ir > u) --ir;
    return ir;
}

__global__ __launch_bounds__(ELEM_BLOCK) void k_elements(const double* __restrict__ geo,
                                                         const int* __restrict__ status, int npairs,
                                                         double2* __restrict__ AB, double* __restrict__ DON)
{
    const long t = long(blockIdx.x) * ELEM_BLOCK + threadIdx.x;
    const int pair = int(t / NUNIQ);
    const int u = int(t - long(pair) * NUNIQ);
    if (pair >= npairs) return;
    if (status[pair] != ST_OK) return;
    const double* G = geo + size_t(pair) * LFG_NGEO;
    const Roche R{G[G_Q], G[G_CA], G[G_CB], G[G_MU], G[G_XL1], G[G_PL1], G[G_RS], G[G_RS2]};
    const double s = G[G_S], c = G[G_C];

    if (u >= U_WD + U_DISC + U_BS) {  // donor tile (MODEL_SPEC 5.4), phi' in (0, pi/2)
        const int uu = u - (U_WD + U_DISC + U_BS);
        const int it = uu / (NDONOR_P / 4), ip = uu - it * (NDONOR_P / 4);
        const double stc = kDonSt[it], ctc = kDonCt[it];
        const double dx = -ctc, dy = stc * kDonCp[ip], dz = stc * kDonSp[ip];
        double lo = 0.0, hi = R.Rs, r = G[G_REFF];
        if (!(r > lo && r < hi)) r = 0.5 * hi;
        double gx, gy, gz;
        for (int itr = 0; itr < ROOT_MAXIT; ++itr) {
            const double X0 = fma(r, dx, 1.0), X1 = r * dy, X2 = r * dz;
            const double f = rpot(R, X0, X1, X2) - R.pl1;
            rgrad(R, X0, X1, X2, gx, gy, gz);
            const double df = gx * dx + gy * dy + gz * dz;
            if (f > 0.0) hi = r; else lo = r;
            double rn = (df > 0.0) ? r - f / df : 0.5 * (lo + hi);
            if (!(rn > lo && rn < hi)) rn = 0.5 * (lo + hi);
            const double d = rn - r;
            r = rn;
            if (fabs(d) <= 1e-15) break;
        }
        rgrad(R, fma(r, dx, 1.0), r * dy, r * dz, gx, gy, gz);
        const double ig = rsqrt(gx * gx + gy * gy + gz * gz);
        const double nx = gx * ig, ny = gy * ig, nz = gz * ig;
        const double dA = r * r * kDonOmega[it] / (nx * dx + ny * dy + nz * dz);
        double* D = DON + (size_t(pair) * U_DON + uu) * 3;
        D[0] = dA * nx;
        D[1] = dA * ny;
        D[2] = dA * nz;
        return;
    }

    double Px, Py, Pz;
    int k, km;
    if (u < U_WD) {  // white dwarf tile (MODEL_SPEC 5.1), cos(psi) > 0 half
        const int ir = wd_ring_of(u);
        const int nk = 4 * (2 * ir + 1), q4 = nk / 4, jj = u - 2 * ir * ir;
        const int j = (jj < q4) ? jj : jj - q4 + 3 * q4;
        const int jm = (j < nk / 2) ? nk / 2 - 1 - j : 3 * nk / 2 - 1 - j;
        k = 4 * ir * ir + j;
        km = 4 * ir * ir + jm;
        const double rc = kWdRc[ir], mu0 = kWdMu0[ir];
        const double cp = kWdCos[u], sp = kWdSin[u];
        const double rw = G[G_RWD];
        Px = rw * (-rc * sp * c + mu0 * s);
        Py = rw * (rc * cp);
        Pz = rw * (rc * sp * s + mu0 * c);
    } else if (u < U_WD + U_DISC) {  // disc (MODEL_SPEC 5.2), alpha in (0, pi)
        const int uu = u - U_WD;
        const int ir = uu / (NDISC_AZ / 2), j = uu - ir * (NDISC_AZ / 2);
        k = NWD + ir * NDISC_AZ + j;
        km = NWD + ir * NDISC_AZ + NDISC_AZ - 1 - j;
        const double rin = G[G_RWD];
        const double rc = rin + (ir + 0.5) * ((G[G_RDISC] - rin) / NDISC_R);
        Px = rc * kDiscCos[j];
        Py = rc * kDiscSin[j];
        Pz = 0.0;
    } else {  // bright-spot strip (MODEL_SPEC 5.3): no mirror partner
        const int j = u - U_WD - U_DISC;
        k = km = NWD + NDISC + j;
        const double uk = (j + 0.5) * (G[G_UMAX] / NBS);
        const double off = G[G_L] * (uk - G[G_UPK]);
        Px = fma(off, G[G_CAZ], G[G_BSX]);
        Py = fma(off, G[G_SAZ], G[G_BSY]);
        Pz = 0.0;
    }
    double a, b;
#ifdef LFG_MARK_FALLBACK
    bool fb = false;  // diagnostic build: NaN-tagged b marks a slow-path element
    element_interval_fast(R, Px, Py, Pz, s, c, G[G_RCAL], G[G_REFF], a, b, &fb);
    if (fb) a = -a - 10.0;
#else
    element_interval_fast(R, Px, Py, Pz, s, c, G[G_RCAL], G[G_REFF], a, b);
#endif
    const size_t o = size_t(pair) * NEL;
    AB[o + k] = make_double2(a, b);
    if (km != k) {
        const bool ecl = a < b;
        AB[o + km] = ecl ? make_double2(-b, -a) : make_double2(1.0, -1.0);
    }
}

// element weights (MODEL_SPEC 5.1-5.3): per WD ring, per disc ring, per spot element
__device__ inline double wd_ring_weight(int ir, double ul) { return fma(kWdA[ir], 1.0 - ul, kWdB[ir] * ul); }

// radial integral of r^(1 - dexp) dr over the disc annuli (MODEL_SPEC 5.2):
// the boundary term P(r) = r^ex / ex, or ln r when ex = 2 - dexp vanishes
__device__ inline double disc_boundary(int i, const double* G)
{
    const double rin = G[G_RWD];
    const double r = rin + i * ((G[G_RDISC] - rin) / NDISC_R);
    const double ex = 2.0 - G[G_DEXP];
    return (fabs(ex) < 1e-10) ? log(r) : pow(r, ex) / ex;
}

__device__ inline double disc_ring_weight(int ir, const double* G)
{
    return (TWO_PI / NDISC_AZ) * (disc_boundary(ir + 1, G) - disc_boundary(ir, G));
}

__device__ inline double bs_weight(int j, const double* G)
{
    const double uk = (j + 0.5) * (G[G_UMAX] / NBS);
    return exp(G[G_EXP1] * log(uk) - pow(uk, G[G_EXP2]) - G[G_LNPK]);
}

// test/inspection only: per-element weights and the full 400-tile donor
__global__ void k_expand(const double* __restrict__ geo, const int* __restrict__ status, int npairs,
                         const double2* __restrict__ AB, const double* __restrict__ DON, double* __restrict__ A,
                         double* __restrict__ B, double* __restrict__ WG, double* __restrict__ DFULL)
{
    const long t = long(blockIdx.x) * blockDim.x + threadIdx.x;
    const int pair = int(t / NEL), k = int(t - long(pair) * NEL);
    if (pair >= npairs || status[pair] != ST_OK) return;
    const double* G = geo + size_t(pair) * LFG_NGEO;
    const double2 ab = AB[size_t(pair) * NEL + k];
    if (A) A[size_t(pair) * NEL + k] = ab.x;
    if (B) B[size_t(pair) * NEL + k] = ab.y;
    double w;
    if (k < NWD) {
        int ir = int(sqrt(k * 0.25));
        if (4 * (ir + 1) * (ir + 1) <= k) ++ir;
        if (4 * ir * ir > k) --ir;
        w = wd_ring_weight(ir, G[G_ULIMB]);
    } else if (k < NWD + NDISC) {
        w = disc_ring_weight((k - NWD) / NDISC_AZ, G);
    } else {
        w = bs_weight(k - NWD - NDISC, G);
    }
    if (WG) WG[size_t(pair) * NEL + k] = w;
    if (DFULL && k < U_DON) {
        const int it = k / (NDONOR_P / 4), ip = k - it * (NDONOR_P / 4);
        const double* v = DON + (size_t(pair) * U_DON + k) * 3;
        const int base = it * NDONOR_P;
        const int ks[4] = {base + ip, base + NDONOR_P - 1 - ip, base + NDONOR_P / 2 - 1 - ip,
                           base + NDONOR_P / 2 + ip};
        const double sy[4] = {1.0, 1.0, -1.0, -1.0}, sz[4] = {1.0, -1.0, 1.0, -1.0};
        double* D = DFULL + size_t(pair) * NDONOR * 3;
        for (int m = 0; m < 4; ++m) {
            D[3 * ks[m]] = v[0];
            D[3 * ks[m] + 1] = sy[m] * v[1];
            D[3 * ks[m] + 2] = sz[m] * v[2];
        }
    }
}

// --------------------------------------------------------------- k_lnlike
__device__ __forceinline__ double wave_sum(double v)
{
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

struct LikeArgs {
    const double* geo;
    const int* status;
    const double2* AB;
    const double* DON;
    int E;
    const int* off;  // nullptr: every pair uses x[0..N)
    int N;
    const double* x;
    const double* y;
    const double* ye;
    const double* w;
    int nsub;
    double* flux;   // nullable, [pairs][N]
    double* comps;  // nullable, [4][pairs][N]
    double* lle;    // nullable, [pairs]
    int npairs;
};

// element groups with their own [min a, max b] window: 10 WD rings, 20 disc
// rings, 5 spot blocks of 20 -- a point only scans the groups it overlaps
constexpr int NG_WD = NWD_RINGS, NG_DISC = NDISC_R, NG_BS = 5, NGROUP = NG_WD + NG_DISC + NG_BS;

__device__ __forceinline__ int group_start(int g)
{
    return g < NG_WD ? 4 * g * g : (g < NG_WD + NG_DISC ? NWD + (g - NG_WD) * NDISC_AZ
                                                       : NWD + NDISC + (g - NG_WD - NG_DISC) * (NBS / NG_BS));
}

__device__ __forceinline__ double ov1(double2 e, double lo, double hi)
{
    return fmax(fmin(e.y, hi) - fmax(e.x, lo), 0.0);
}

// sum over k in [k0, k1) of |[a_k, b_k] n [lo, hi]|; four independent chains
// keep four 128-bit LDS reads in flight
__device__ __forceinline__ double overlap_sum(const double2* __restrict__ ab, int k0, int k1, double lo,
                                              double hi)
{
    double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
    int k = k0;
#pragma unroll 1
    for (; k + 3 < k1; k += 4) {
        const double2 e0 = ab[k], e1 = ab[k + 1], e2 = ab[k + 2], e3 = ab[k + 3];
        s0 += ov1(e0, lo, hi);
        s1 += ov1(e1, lo, hi);
        s2 += ov1(e2, lo, hi);
        s3 += ov1(e3, lo, hi);
    }
#pragma unroll 1
    for (; k < k1; ++k) s0 += ov1(ab[k], lo, hi);
    return (s0 + s1) + (s2 + s3);
}

// weighted variant for the spot strip (per-element weights wt[k - k0])
__device__ __forceinline__ double overlap_wsum(const double2* __restrict__ ab, const double* __restrict__ wt,
                                               int k0, int k1, double lo, double hi)
{
    double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
    int k = k0;
#pragma unroll 1
    for (; k + 3 < k1; k += 4) {
        const double2 e0 = ab[k], e1 = ab[k + 1], e2 = ab[k + 2], e3 = ab[k + 3];
        const int i = k - k0;
        s0 = fma(wt[i], ov1(e0, lo, hi), s0);
        s1 = fma(wt[i + 1], ov1(e1, lo, hi), s1);
        s2 = fma(wt[i + 2], ov1(e2, lo, hi), s2);
        s3 = fma(wt[i + 3], ov1(e3, lo, hi), s3);
    }
#pragma unroll 1
    for (; k < k1; ++k) s0 = fma(wt[k - k0], ov1(ab[k], lo, hi), s0);
    return (s0 + s1) + (s2 + s3);
}

// bit g set when group g's eclipse window meets [lo, hi]
__device__ __forceinline__ unsigned long long group_mask(const double2* __restrict__ gb, int g0, int g1, double lo,
                                                         double hi)
{
    unsigned long long m = 0;
#pragma unroll 5
    for (int g = g0; g < g1; ++g) {
        const double2 b = gb[g];
        m |= (hi >= b.x && lo <= b.y) ? (1ull << g) : 0ull;
    }
    return m;
}

__device__ __forceinline__ double inside_count(const double2* __restrict__ ab, const double* wt, int k0, int k1,
                                               double ph)
{
    double s = 0.0;
    for (int k = k0; k < k1; ++k) s += (ph > ab[k].x && ph < ab[k].y) ? (wt ? wt[k - k0] : 1.0) : 0.0;
    return s;
}

// ---- sweep over a phase-sorted tile of points (MODEL_SPEC 6.1 restated) ----
// With lo_p = phase_p - w_p and hi_p = phase_p + w_p both non-decreasing in p,
// the points an element [a, b] overlaps form the contiguous range [P1, P4),
// and those it covers whole form [P2, P3):
//   P1 = #{hi <= a}, P2 = #{lo < a}, P3 = #{hi <= b}, P4 = #{lo < b}.
// Covered points gain the element's normalised weight through a difference
// array; the (few) partly covered points gain w |[a,b] n [lo,hi]| / (hi - lo)
// directly.  Contributions are 2^-61 fixed point in int64 so that LDS atomics
// sum them exactly and the result is independent of summation order.
constexpr int LIKE_THREADS = 256;
constexpr int LIKE_TILE = 2 * LIKE_THREADS;  // points per sweep tile
constexpr double FX_SCALE = 2305843009213693952.0;  // 2^61
constexpr double FX_INV = 1.0 / FX_SCALE;

__device__ __forceinline__ void count4(const double* __restrict__ lo, const double* __restrict__ hi, int m,
                                       double a, double b, int& P1, int& P2, int& P3, int& P4)
{
    // branch-free lower bounds; the trip count depends on m only (wave-uniform)
    int b1 = 0, b2 = 0, b3 = 0, b4 = 0, len = m;
    while (len > 1) {
        const int half = len >> 1;
        b1 += (hi[b1 + half - 1] <= a) ? half : 0;
        b2 += (lo[b2 + half - 1] < a) ? half : 0;
        b3 += (hi[b3 + half - 1] <= b) ? half : 0;
        b4 += (lo[b4 + half - 1] < b) ? half : 0;
        len -= half;
    }
    P1 = b1 + (hi[b1] <= a);
    P2 = b2 + (lo[b2] < a);
    P3 = b3 + (hi[b3] <= b);
    P4 = b4 + (lo[b4] < b);
}

__device__ __forceinline__ void fx_add(unsigned long long* acc, int p, long long q)
{
    atomicAdd(acc + p, static_cast<unsigned long long>(q));
}

__device__ __forceinline__ long long wave_scan_incl(long long v, int lane)
{
    for (int off = 1; off < 64; off <<= 1) {
        const long long u = __shfl_up(v, off, 64);
        if (lane >= off) v += u;
    }
    return v;
}

template <bool CHI>
__global__ __launch_bounds__(LIKE_THREADS) void k_lnlike(LikeArgs L)
{
    __shared__ double2 sab[NEL];
    __shared__ double sbw[NBS];
    __shared__ double swr[NG_WD + NG_DISC];
    __shared__ double sdb[NDISC_R + 1];
    __shared__ double2 sgb[NGROUP];
    __shared__ double2 sdxy[U_DON];
    __shared__ double sdz[U_DON];
    __shared__ double slo[LIKE_TILE], shi[LIKE_TILE];
    __shared__ unsigned long long sacc[2][LIKE_TILE + 1];
    __shared__ long long sscan[2][LIKE_THREADS / 64];
    __shared__ double red[4][LIKE_THREADS / 64];

    constexpr int nt = LIKE_THREADS, nw = LIKE_THREADS / 64;
    const int pair = blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int e = pair % L.E;
    const int o0 = L.off ? L.off[e] : 0;
    const int n = L.off ? L.off[e + 1] - o0 : L.N;
    const int st = L.status[pair];
    if (st != ST_OK) {
        for (int p = tid; p < n; p += nt) {
            if (L.flux) L.flux[size_t(pair) * n + p] = NAN;
            if (L.comps)
                for (int m = 0; m < 4; ++m) L.comps[(size_t(m) * L.npairs + pair) * n + p] = NAN;
        }
        if (CHI && tid == 0) L.lle[pair] = -INFINITY;
        return;
    }
    const double* G = L.geo + size_t(pair) * LFG_NGEO;
    const double s = G[G_S], c = G[G_C];

    // stage: intervals, spot weights, disc annulus boundaries, donor quads
    const double2* ABp = L.AB + size_t(pair) * NEL;
    for (int k = tid; k < NEL; k += nt) sab[k] = ABp[k];
    double tb = 0.0, dn = 0.0;
    for (int i = tid; i < NBS + NDISC_R + 1 + NG_WD; i += nt) {
        if (i < NBS) {
            const double w = bs_weight(i, G);
            sbw[i] = w;
            tb += w;
        } else if (i < NBS + NDISC_R + 1) {
            sdb[i - NBS] = disc_boundary(i - NBS, G);
        } else {
            swr[i - NBS - NDISC_R - 1] = wd_ring_weight(i - NBS - NDISC_R - 1, G[G_ULIMB]);
        }
    }
    const double* Dp = L.DON + size_t(pair) * U_DON * 3;
    for (int q = tid; q < U_DON; q += nt) {
        const double vx = Dp[3 * q], vy = Dp[3 * q + 1], vz = Dp[3 * q + 2];
        sdxy[q] = make_double2(vx, vy);
        const double zc = vz * c;
        sdz[q] = zc;
        // donor normalisation at quadrature (theta = pi/2): X = +-vz c, Y = vy s
        const double ay = fabs(vy * s);
        dn += fmax(zc + ay, 0.0) + fmax(zc - ay, 0.0) + fmax(-zc + ay, 0.0) + fmax(-zc - ay, 0.0);
    }
    tb = wave_sum(tb);
    dn = wave_sum(dn);
    if (lane == 0) { red[0][wv] = tb; red[1][wv] = dn; }
    __syncthreads();
    if (tid < NDISC_R) swr[NG_WD + tid] = (TWO_PI / NDISC_AZ) * (sdb[tid + 1] - sdb[tid]);
    for (int g = wv; g < NGROUP; g += nw) {  // eclipse window of each group, one wave per group
        const int k0 = group_start(g), k1 = group_start(g + 1);
        double lo = INFINITY, hi = -INFINITY;
        for (int k = k0 + lane; k < k1; k += 64) {
            const double2 ab = sab[k];
            if (ab.x < ab.y) { lo = fmin(lo, ab.x); hi = fmax(hi, ab.y); }
        }
        for (int sh = 32; sh > 0; sh >>= 1) {
            lo = fmin(lo, __shfl_xor(lo, sh, 64));
            hi = fmax(hi, __shfl_xor(hi, sh, 64));
        }
        if (lane == 0) sgb[g] = make_double2(lo, hi);
    }
    // totals telescope: WD 2 pi [F(1) - F(0)], disc 2 pi [P(rdisc) - P(rin)]
    const double ul = G[G_ULIMB];
    const double twd = TWO_PI * ((1.0 - ul) * 0.5 + ul / 3.0);
    const double td = TWO_PI * (sdb[NDISC_R] - sdb[0]);
    tb = dn = 0.0;
    for (int i = 0; i < nw; ++i) { tb += red[0][i]; dn += red[1][i]; }
    __syncthreads();
    const double iwd = 1.0 / twd, id = 1.0 / td;

    const double wdF = G[G_WDF], dF = G[G_DF], sF = G[G_SF], rsF = G[G_RSF];
    const double phi0 = G[G_PHI0], fis = G[G_FIS], bden = G[G_BDEN];
    const double nb0 = G[G_NB0], nb1 = G[G_NB1], nb2 = G[G_NB2];
    const int S = L.nsub;
    double chi = 0.0;
    for (int t0 = 0; t0 < n; t0 += LIKE_TILE) {
        const int m = min(LIKE_TILE, n - t0);
        // tile phases; the sweep needs lo, hi non-decreasing and widths > 0
        int bad = 0;
        for (int i = tid; i < m; i += nt) {
            const int p = o0 + t0 + i;
            const double wk = L.w ? L.w[p] : 0.0;
            const double ph0 = L.x[p] - phi0;
            const double phc = ph0 - floor(ph0 + 0.5);
            slo[i] = phc - wk;
            shi[i] = phc + wk;
            bad |= !(wk > 0.0);
            sacc[0][i] = 0ull;
            sacc[1][i] = 0ull;
        }
        __syncthreads();
        for (int i = tid + 1; i < m; i += nt) bad |= (slo[i] < slo[i - 1]) || (shi[i] < shi[i - 1]);
        const bool sweep = !__syncthreads_or(bad);
        if (sweep) {
            const double tlo = slo[0], thi = shi[m - 1];
            for (int k = tid; k < NWD + NDISC; k += nt) {
                const double2 ab = sab[k];
                if (!(ab.x < ab.y) || ab.y <= tlo || ab.x >= thi) continue;
                int comp, ring;
                if (k < NWD) {
                    ring = int(sqrt(k * 0.25));
                    if (4 * (ring + 1) * (ring + 1) <= k) ++ring;
                    if (4 * ring * ring > k) --ring;
                    comp = 0;
                } else {
                    ring = NG_WD + (k - NWD) / NDISC_AZ;
                    comp = 1;
                }
                const double wn = swr[ring] * (comp ? id : iwd);
                int P1, P2, P3, P4;
                count4(slo, shi, m, ab.x, ab.y, P1, P2, P3, P4);
                unsigned long long* acc = sacc[comp];
                int e0 = P4, s1 = P4;  // partial ranges [P1, e0) and [s1, P4)
                if (P2 < P3) {
                    const long long q = llrint(wn * FX_SCALE);
                    fx_add(acc, P2, q);
                    fx_add(acc, P3, -q);
                    e0 = P2;
                    s1 = P3;
                }
                for (int r = 0; r < 2; ++r) {
                    const int pe = r ? P4 : e0;
                    for (int p = r ? s1 : P1; p < pe; ++p) {
                        const double lo = slo[p], hi = shi[p];
                        const double ov = fmin(ab.y, hi) - fmax(ab.x, lo);
                        if (ov > 0.0) {
                            const long long q = llrint(wn * (ov / (hi - lo)) * FX_SCALE);
                            fx_add(acc, p, q);
                            fx_add(acc, p + 1, -q);
                        }
                    }
                }
            }
            __syncthreads();
            // inclusive scan of both difference arrays (2 entries per thread)
            long long v0[2], v1[2];
            for (int j = 0; j < 2; ++j) {
                const int i = 2 * tid + j;
                v0[j] = (i < m) ? static_cast<long long>(sacc[0][i]) : 0;
                v1[j] = (i < m) ? static_cast<long long>(sacc[1][i]) : 0;
            }
            v0[1] += v0[0];
            v1[1] += v1[0];
            const long long w0 = wave_scan_incl(v0[1], lane), w1 = wave_scan_incl(v1[1], lane);
            if (lane == 63) { sscan[0][wv] = w0; sscan[1][wv] = w1; }
            __syncthreads();
            long long b0 = w0 - v0[1], b1 = w1 - v1[1];
            for (int i = 0; i < wv; ++i) { b0 += sscan[0][i]; b1 += sscan[1][i]; }
            if (2 * tid < m) { sacc[0][2 * tid] = b0 + v0[0]; sacc[1][2 * tid] = b1 + v1[0]; }
            if (2 * tid + 1 < m) { sacc[0][2 * tid + 1] = b0 + v0[1]; sacc[1][2 * tid + 1] = b1 + v1[1]; }
            __syncthreads();
        }
        for (int i = tid; i < m; i += nt) {
            const int p = o0 + t0 + i;
            const double lo = slo[i], hi = shi[i];
            const double wk = L.w ? L.w[p] : 0.0;
            const double phc = 0.5 * (lo + hi);
            double fwd, fdd;  // eclipsed fractions of WD and disc
            if (sweep) {
                fwd = double(static_cast<long long>(sacc[0][i])) * FX_INV;
                fdd = double(static_cast<long long>(sacc[1][i])) * FX_INV;
            } else {  // unsorted points or zero widths: scan the overlapping rings
                double ewd = 0.0, ed = 0.0;
                for (unsigned long long msk = group_mask(sgb, 0, NG_WD + NG_DISC, lo, hi); msk; msk &= msk - 1) {
                    const int g = __builtin_ctzll(msk);
                    const int k0 = group_start(g), k1 = group_start(g + 1);
                    const double ov = (wk > 0.0) ? overlap_sum(sab, k0, k1, lo, hi)
                                                 : inside_count(sab, nullptr, k0, k1, phc);
                    if (g < NG_WD) ewd = fma(swr[g], ov, ewd); else ed = fma(swr[g], ov, ed);
                }
                if (wk > 0.0) {
                    ewd /= 2.0 * wk;
                    ed /= 2.0 * wk;
                }
                fwd = ewd * iwd;
                fdd = ed * id;
            }
            const double fw = wdF * (1.0 - fwd);
            const double fd = dF * (1.0 - fdd);
            const double ph0 = L.x[p] - phi0;
            const double h = wk / S;
            double sbs = 0.0, srs = 0.0;
#pragma unroll 1
            for (int j = 0; j < S; ++j) {
                double ph = ph0 - wk + (2 * j + 1) * h;
                ph -= floor(ph + 0.5);
                double sn, cs;
                sincospi(2.0 * ph, &sn, &cs);  // |2 ph| <= 1: cheap exact reduction
                const double e0 = s * cs, e1 = -s * sn;
                double beam = 0.0;
                if (bden > 0.0) beam = (fis + (1.0 - fis) * fmax(nb0 * e0 + nb1 * e1 + nb2 * c, 0.0)) / bden;
                double eb = 0.0;
                const double l2 = ph - h, h2 = ph + h;
                for (unsigned long long msk = group_mask(sgb, NG_WD + NG_DISC, NGROUP, l2, h2); msk;
                     msk &= msk - 1) {
                    const int g = __builtin_ctzll(msk);
                    const int k0 = group_start(g), k1 = group_start(g + 1);
                    const double* wt = sbw + (k0 - NWD - NDISC);
                    eb += (h > 0.0) ? overlap_wsum(sab, wt, k0, k1, l2, h2) : inside_count(sab, wt, k0, k1, ph);
                }
                if (h > 0.0) eb /= 2.0 * h;
                sbs += beam * (1.0 - eb / tb);
                // donor: 100 quads of mirror tiles (vx, +-vy, +-vz); for A = vx e0 +- vz c and
                // Y = |vy e1|: max(A + Y, 0) + max(A - Y, 0) = max(A + max(Y, A), 0)
                double d0 = 0.0, d1 = 0.0;
#pragma unroll 4
                for (int q = 0; q < U_DON; ++q) {
                    const double2 v = sdxy[q];
                    const double z = sdz[q];
                    const double y = fabs(v.y * e1);
                    const double A1 = fma(v.x, e0, z), A2 = fma(v.x, e0, -z);
                    d0 += fmax(A1 + fmax(y, A1), 0.0);
                    d1 += fmax(A2 + fmax(y, A2), 0.0);
                }
                srs += (d0 + d1) / dn;
            }
            const double fb = sF * sbs / S, fr = rsF * srs / S;
            const double f = fw + fd + fb + fr;
            if (L.flux) L.flux[size_t(pair) * n + t0 + i] = f;
            if (L.comps) {
                L.comps[(size_t(0) * L.npairs + pair) * n + t0 + i] = fw;
                L.comps[(size_t(1) * L.npairs + pair) * n + t0 + i] = fd;
                L.comps[(size_t(2) * L.npairs + pair) * n + t0 + i] = fb;
                L.comps[(size_t(3) * L.npairs + pair) * n + t0 + i] = fr;
            }
            if (CHI) {
                const double r = (L.y[p] - f) / L.ye[p];
                chi += isnan(f) ? INFINITY : r * r;
            }
        }
        __syncthreads();  // tile buffers are rewritten by the next tile
    }
    if (CHI) {
        chi = wave_sum(chi);
        if (lane == 0) red[2][wv] = chi;
        __syncthreads();
        if (tid == 0) {
            double tot = 0.0;
            for (int i = 0; i < nw; ++i) tot += red[2][i];
            L.lle[pair] = -0.5 * tot;
        }
    }
}

// -------------------------------------------------------------- k_combine
__global__ void k_combine(int W, int E, const double* __restrict__ prior, const double* __restrict__ geo,
                          double* __restrict__ lle, double* __restrict__ lnp)
{
    const int w = blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= W) return;
    double lp = prior[w];
    for (int e = 0; e < E; ++e) lp += geo[(size_t(w) * E + e) * LFG_NGEO + G_RPRIOR];
    if (!isfinite(lp)) {
        for (int e = 0; e < E; ++e) lle[size_t(w) * E + e] = -INFINITY;
        lnp[w] = -INFINITY;
        return;
    }
    double ll = 0.0;
    for (int e = 0; e < E; ++e) ll += lle[size_t(w) * E + e];
    lnp[w] = lp + ll;
}

// ------------------------------------------------------- stretch-move sampler
// Philox4x32-10 (Salmon et al. 2011), counter = (walker, step lo, step hi,
// half | purpose), key = seed.  Stateless: any rank reproduces any draw.
__device__ inline uint4 philox(uint4 c, uint2 k)
{
    for (int r = 0; r < 10; ++r) {
        const unsigned lo0 = c.x * 0xD2511F53u, hi0 = __umulhi(c.x, 0xD2511F53u);
        const unsigned lo1 = c.z * 0xCD9E8D57u, hi1 = __umulhi(c.z, 0xCD9E8D57u);
        c = make_uint4(hi1 ^ c.y ^ k.x, lo1, hi0 ^ c.w ^ k.y, lo0);
        k.x += 0x9E3779B9u;
        k.y += 0xBB67AE85u;
    }
    return c;
}

__device__ inline double u53(unsigned a, unsigned b)  // uniform on [0, 1)
{
    return double((static_cast<unsigned long long>(a >> 5) << 26) | (b >> 6)) * (1.0 / 9007199254740992.0);
}

__device__ inline uint4 draw(unsigned long long seed, unsigned long long step, int half, int purpose, int i)
{
    return philox(make_uint4(unsigned(i), unsigned(step), unsigned(step >> 32), unsigned(half * 2 + purpose)),
                  make_uint2(unsigned(seed), unsigned(seed >> 32)));
}

// emcee StretchMove.get_proposal: z = ((a-1) u + 1)^2 / a,
// q = c_j - (c_j - s) z = c_j + z (s - c_j), factor = (ndim - 1) ln z
__global__ void k_propose(const double* __restrict__ pos, int W, int ndim, int half, double a,
                          unsigned long long seed, unsigned long long step, double* __restrict__ q,
                          double* __restrict__ zfac)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const int ns = W / 2;
    if (i >= ns) return;
    const uint4 r = draw(seed, step, half, 0, i);
    const double u = u53(r.x, r.y);
    const double zr = (a - 1.0) * u + 1.0;
    const double z = zr * zr / a;
    const int j = int(__umulhi(r.z, unsigned(ns)));  // partner in the other half
    const double* s = pos + size_t(half * ns + i) * ndim;
    const double* cj = pos + size_t((1 - half) * ns + j) * ndim;
    double* out = q + size_t(i) * ndim;
    for (int d = 0; d < ndim; ++d) out[d] = cj[d] - (cj[d] - s[d]) * z;
    zfac[i] = (ndim - 1.0) * log(z);
}

// Metropolis acceptance: accept if ln u < factor + lnp_new - lnp_old
__global__ void k_accept(double* __restrict__ pos, double* __restrict__ lnp, int W, int ndim, int half,
                         const double* __restrict__ q, const double* __restrict__ zfac,
                         const double* __restrict__ lnp_new, unsigned long long seed, unsigned long long step,
                         int* __restrict__ naccept)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const int ns = W / 2;
    if (i >= ns) return;
    const int w = half * ns + i;
    const uint4 r = draw(seed, step, half, 1, i);
    const double lu = log(u53(r.x, r.y));
    const double diff = zfac[i] + lnp_new[i] - lnp[w];
    if (lu < diff) {
        double* p = pos + size_t(w) * ndim;
        const double* qi = q + size_t(i) * ndim;
        for (int d = 0; d < ndim; ++d) p[d] = qi[d];
        lnp[w] = lnp_new[i];
        if (naccept) naccept[w] += 1;
    }
}

// ---------------------------------------------------------------- k_roche
__global__ void k_roche(int op, const double* __restrict__ a, const double* __restrict__ b, int n,
                        double* __restrict__ out, int* __restrict__ status)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    Roche R;
    int st = roche_init(R, a[i]);
    if (op == 0) {
        out[i] = (st == ST_OK) ? R.xl1 : NAN;
    } else if (op == 1) {
        double v = NAN;
        if (st == ST_OK) st = findphi(R, b[i], v);
        out[i] = (st == ST_OK) ? v : NAN;
    } else if (op == 2) {
        double v = NAN;
        if (st == ST_OK) st = findi(R, b[i], v);
        out[i] = (st == ST_OK) ? v : NAN;
    } else {
        double v[4] = {NAN, NAN, NAN, NAN};
        if (st == ST_OK) st = bspot(R, b[i], v);
        if (st != ST_OK) v[0] = v[1] = v[2] = v[3] = NAN;
        for (int m = 0; m < 4; ++m) out[4 * size_t(i) + m] = v[m];
    }
    status[i] = st;
}

inline int launch_ok() { return hipGetLastError() == hipSuccess ? LFG_OK : LFG_E_LAUNCH; }

int run_front(const SetupArgs& S, const Ws& ws, hipStream_t st)
{
    const int npairs = S.W * S.E;
    const int nlanes = npairs + S.W;
    hipLaunchKernelGGL(k_setup, dim3((nlanes + SETUP_BLOCK - 1) / SETUP_BLOCK), dim3(SETUP_BLOCK), 0, st, S);
    if (launch_ok() != LFG_OK) return LFG_E_LAUNCH;
    const long nthreads = long(npairs) * NUNIQ;
    hipLaunchKernelGGL(k_elements, dim3(unsigned((nthreads + ELEM_BLOCK - 1) / ELEM_BLOCK)), dim3(ELEM_BLOCK), 0,
                       st, ws.geo, ws.status, npairs, ws.ab, ws.donor);
    return launch_ok();
}

}  // namespace

extern "C" {

size_t lfg_workspace_size(int W, int E)
{
    if (W <= 0 || E <= 0) return 0;
    return carve(nullptr, W, E).total;
}

int lfg_flux(const double* pars, int W, int P, const double* x, const double* w, int N, int nsub,
             double* flux, double* comps, int* status, void* wsp, size_t ws_bytes, void* stream)
{
    if (W <= 0 || N < 0 || nsub < 1 || (P != 14 && P != 18) || !pars || (!x && N > 0)) return LFG_E_ARGS;
    Ws ws = carve(wsp, W, 1);
    if (!wsp || ws_bytes < ws.total) return LFG_E_WORKSPACE;
    hipStream_t st = static_cast<hipStream_t>(stream);
    SetupArgs S{pars, W, P, 1, P, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, 0,
                ws.geo, ws.status, ws.prior};
    int rc = run_front(S, ws, st);
    if (rc) return rc;
    if (N > 0) {
        LikeArgs L{ws.geo, ws.status, ws.ab, ws.donor, 1, nullptr, N, x, nullptr, nullptr, w,
                   nsub, flux, comps, nullptr, W};
        hipLaunchKernelGGL(k_lnlike<false>, dim3(W), dim3(LIKE_THREADS), 0, st, L);
        if ((rc = launch_ok())) return rc;
    }
    if (status && hipMemcpyAsync(status, ws.status, sizeof(int) * W, hipMemcpyDeviceToDevice, st) != hipSuccess)
        return LFG_E_LAUNCH;
    return LFG_OK;
}

static int lnprob_impl(const double* walkers, int W, const lfg_tree* T, double* lnp, double* lnlike_e, void* wsp,
                       size_t ws_bytes, void* stream, void* const* ev)
{
    if (W <= 0 || !T || T->E <= 0 || T->ndim <= 0 || T->nsub < 1 || !walkers || !lnp) return LFG_E_ARGS;
    Ws ws = carve(wsp, W, T->E);
    if (!wsp || ws_bytes < ws.total) return LFG_E_WORKSPACE;
    hipStream_t st = static_cast<hipStream_t>(stream);
    auto mark = [&](int i) {
        if (ev && ev[i]) (void)hipEventRecord(static_cast<hipEvent_t>(ev[i]), st);
    };
    SetupArgs S{walkers, W, T->ndim, T->E, 18, T->gather, T->npars, T->consts, T->prior_type, T->prior_p1,
                T->prior_p2, T->prior_norm, T->roche_priors, ws.geo, ws.status, ws.prior};
    const int npairs = W * T->E;
    const int nlanes = npairs + W;
    mark(0);
    hipLaunchKernelGGL(k_setup, dim3((nlanes + SETUP_BLOCK - 1) / SETUP_BLOCK), dim3(SETUP_BLOCK), 0, st, S);
    int rc = launch_ok();
    if (rc) return rc;
    mark(1);
    const long nthreads = long(npairs) * NUNIQ;
    hipLaunchKernelGGL(k_elements, dim3(unsigned((nthreads + ELEM_BLOCK - 1) / ELEM_BLOCK)), dim3(ELEM_BLOCK), 0,
                       st, ws.geo, ws.status, npairs, ws.ab, ws.donor);
    if ((rc = launch_ok())) return rc;
    mark(2);
    double* lle = lnlike_e ? lnlike_e : ws.lle;
    LikeArgs L{ws.geo, ws.status, ws.ab, ws.donor, T->E, T->off, T->max_n, T->x, T->y, T->ye,
               T->w, T->nsub, nullptr, nullptr, lle, npairs};
    hipLaunchKernelGGL(k_lnlike<true>, dim3(npairs), dim3(LIKE_THREADS), 0, st, L);
    if ((rc = launch_ok())) return rc;
    mark(3);
    hipLaunchKernelGGL(k_combine, dim3((W + 255) / 256), dim3(256), 0, st, W, T->E, ws.prior, ws.geo, lle, lnp);
    rc = launch_ok();
    mark(4);
    return rc;
}

int lfg_lnprob(const double* walkers, int W, const lfg_tree* T, double* lnp, double* lnlike_e, void* wsp,
               size_t ws_bytes, void* stream)
{
    return lnprob_impl(walkers, W, T, lnp, lnlike_e, wsp, ws_bytes, stream, nullptr);
}

int lfg_lnprob_timed(const double* walkers, int W, const lfg_tree* T, double* lnp, double* lnlike_e, void* wsp,
                     size_t ws_bytes, void* stream, void* const* ev)
{
    return lnprob_impl(walkers, W, T, lnp, lnlike_e, wsp, ws_bytes, stream, ev);
}

int lfg_stretch_propose(const double* pos, int W, int ndim, int half, double a, unsigned long long seed,
                        unsigned long long step, double* q, double* zfac, void* stream)
{
    if (W < 4 || (W & 1) || ndim <= 0 || (half != 0 && half != 1) || !(a > 1.0) || !pos || !q || !zfac)
        return LFG_E_ARGS;
    const int ns = W / 2;
    hipLaunchKernelGGL(k_propose, dim3((ns + 63) / 64), dim3(64), 0, static_cast<hipStream_t>(stream), pos, W,
                       ndim, half, a, seed, step, q, zfac);
    return launch_ok();
}

int lfg_stretch_accept(double* pos, double* lnp, int W, int ndim, int half, const double* q, const double* zfac,
                       const double* lnp_new, unsigned long long seed, unsigned long long step, int* naccept,
                       void* stream)
{
    if (W < 4 || (W & 1) || ndim <= 0 || (half != 0 && half != 1) || !pos || !lnp || !q || !zfac || !lnp_new)
        return LFG_E_ARGS;
    const int ns = W / 2;
    hipLaunchKernelGGL(k_accept, dim3((ns + 63) / 64), dim3(64), 0, static_cast<hipStream_t>(stream), pos, lnp,
                       W, ndim, half, q, zfac, lnp_new, seed, step, naccept);
    return launch_ok();
}

int lfg_event_create(void** ev)
{
    if (!ev) return LFG_E_ARGS;
    hipEvent_t e;
    if (hipEventCreate(&e) != hipSuccess) return LFG_E_LAUNCH;
    *ev = static_cast<void*>(e);
    return LFG_OK;
}

int lfg_event_destroy(void* ev)
{
    return hipEventDestroy(static_cast<hipEvent_t>(ev)) == hipSuccess ? LFG_OK : LFG_E_LAUNCH;
}

int lfg_event_elapsed_ms(void* start, void* stop, float* ms)
{
    if (!ms) return LFG_E_ARGS;
    return hipEventElapsedTime(ms, static_cast<hipEvent_t>(start), static_cast<hipEvent_t>(stop)) == hipSuccess
               ? LFG_OK
               : LFG_E_LAUNCH;
}

int lfg_elements(const double* pars, int W, int P, double* a, double* b, double* wgt, double* donor,
                 double* geo, int* status, void* wsp, size_t ws_bytes, void* stream)
{
    if (W <= 0 || (P != 14 && P != 18) || !pars) return LFG_E_ARGS;
    Ws ws = carve(wsp, W, 1);
    if (!wsp || ws_bytes < ws.total) return LFG_E_WORKSPACE;
    hipStream_t st = static_cast<hipStream_t>(stream);
    SetupArgs S{pars, W, P, 1, P, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, 0,
                ws.geo, ws.status, ws.prior};
    int rc = run_front(S, ws, st);
    if (rc) return rc;
    if (a || b || wgt || donor) {
        const long nt = long(W) * NEL;
        hipLaunchKernelGGL(k_expand, dim3(unsigned((nt + 255) / 256)), dim3(256), 0, st, ws.geo, ws.status, W, ws.ab,
                           ws.donor, a, b, wgt, donor);
        if ((rc = launch_ok())) return rc;
    }
    bool ok = true;
    if (geo)
        ok &= hipMemcpyAsync(geo, ws.geo, size_t(W) * LFG_NGEO * sizeof(double), hipMemcpyDeviceToDevice, st) ==
              hipSuccess;
    if (status) ok &= hipMemcpyAsync(status, ws.status, sizeof(int) * W, hipMemcpyDeviceToDevice, st) == hipSuccess;
    return ok ? LFG_OK : LFG_E_LAUNCH;
}

int lfg_roche(int op, const double* a, const double* b, int n, double* out, int* status, void* stream)
{
    if (op < 0 || op > 3 || n < 0 || !a || !out || !status || (op > 0 && !b)) return LFG_E_ARGS;
    if (n == 0) return LFG_OK;
    hipLaunchKernelGGL(k_roche, dim3((n + 63) / 64), dim3(64), 0, static_cast<hipStream_t>(stream), op, a, b, n,
                       out, status);
    return launch_ok();
}

const char* lfg_version(void) { return "lfg 0.1.0 gfx950 fp64"; }

}  // extern "C"
