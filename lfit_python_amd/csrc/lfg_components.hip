// lfg_components.hip -- lfit's component objects on gfx950: the unit-
// normalised flux of ONE component (white dwarf, disc, bright spot or donor)
// at a given inclination, on a caller-chosen grid (MODEL_SPEC 5.6).
// Replaces lfit.PyWhiteDwarf / PyDisc / PySpot / PyDonor(...).calcFlux(q,
// inc, phi, width) (testCV.py:27-49, fitEcl.py:21-24).
//
// Not the sampler's hot path (that is lfg.hip's fused CV pipeline, with
// compile-time grids and mirror symmetry); this path takes any grid size, so
// it solves every element directly and accumulates element x point directly:
//   k_comp_setup     one lane per set: Roche geometry, findphi for the
//                    tangency guess, the stream and strip frame (spot)
//   k_comp_elements  one lane per (set, element): position, weight and
//                    eclipse interval (the same solver as k_elements), or the
//                    donor tile vector
//   k_comp_flux      one 256-lane block per set: the set's elements staged
//                    through LDS in tiles, lanes stride the phase axis
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lfg.h"
#include "lfg_device.hpp"

using namespace lfg;

namespace {

enum CompGeo {
    C_Q, C_CA, C_CB, C_MU, C_XL1, C_PL1, C_RS, C_RS2,
    C_S, C_C, C_RCAL, C_REFF,
    C_P0, C_P1, C_P2,                       // WD: rwd_a, ulimb; disc: rin, rout, ex
    C_BSX, C_BSY, C_L, C_UPK, C_UMAX, C_LNPK, C_E1, C_E2, C_CAZ, C_SAZ,
    C_NB0, C_NB1, C_NB2, C_BDEN, C_FIS,
    C_COUNT
};
constexpr int CGEO = 32;
static_assert(C_COUNT <= CGEO, "component geometry record");

constexpr int COMP_BLOCK = 256;
constexpr int COMP_TILE = 512;  // elements staged per LDS tile

inline size_t align256(size_t v) { return (v + 255) & ~size_t(255); }

int comp_nel(int kind, int n1, int n2)
{
    switch (kind) {
    case 0: return NWD;
    case 1: return n1 * n2;
    case 2: return n1;
    case 3: return n1 * n2;
    }
    return 0;
}

struct CompWs {
    double* geo;     // [W][CGEO]
    int* status;     // [W]
    double* e3;      // [W][nel][3]: a, b, weight (eclipsed components) or the donor tile vector
    size_t total;
};

CompWs comp_carve(void* base, int W, int nel)
{
    CompWs ws{};
    char* p = static_cast<char*>(base);
    size_t off = 0;
    auto take = [&](size_t bytes) { char* r = p ? p + off : nullptr; off += align256(bytes); return r; };
    ws.geo = reinterpret_cast<double*>(take(size_t(W) * CGEO * sizeof(double)));
    ws.status = reinterpret_cast<int*>(take(size_t(W) * sizeof(int)));
    ws.e3 = reinterpret_cast<double*>(take(size_t(W) * size_t(nel) * 3 * sizeof(double)));
    ws.total = off;
    return ws;
}

__global__ __launch_bounds__(64) void k_comp_setup(int kind, const double* __restrict__ cp, int ncp,
                                                   const double* __restrict__ qv, const double* __restrict__ incv,
                                                   int W, int n1, double* __restrict__ geo, int* __restrict__ status)
{
    const int i = blockIdx.x * 64 + threadIdx.x;
    if (i >= W) return;
    const double* p = cp + size_t(i) * ncp;
    double* G = geo + size_t(i) * CGEO;
    const double inc = incv[i];
    Roche R;
    int st = roche_init(R, qv[i]);
    bool fin = isfinite(inc);
    for (int k = 0; k < ncp; ++k) fin = fin && isfinite(p[k]);
    if (st == ST_OK && (!fin || !(inc > 0.0 && inc <= 90.0))) st = ST_BAD_ARGS;
    double s = 0.0, c = 0.0;
    if (st == ST_OK) {
        sincos(inc * DEG, &s, &c);
        // tangency guesses (element_interval_fast): the sphere reproducing
        // the WD-centre contact at this inclination, else the Eggleton radius
        double dphi, rcal = eggleton(R.q);
        if (findphi_fast(R, inc, dphi) == ST_OK) {
            const double sce = s * cos(PI * dphi);
            rcal = sqrt(1.0 - sce * sce);
        }
        G[C_RCAL] = rcal;
        G[C_REFF] = eggleton(R.q);
    }
    if (st == ST_OK && kind == 0) {  // rwd/xl1, ulimb
        G[C_P0] = p[0] * R.xl1;
        G[C_P1] = p[1];
        if (!(G[C_P0] > 0.0) || !(G[C_P0] < R.xl1)) st = ST_BAD_GEOMETRY;
    } else if (st == ST_OK && kind == 1) {  // rwd/xl1, rdisc/xl1, dexp
        G[C_P0] = p[0] * R.xl1;
        G[C_P1] = p[1] * R.xl1;
        G[C_P2] = 2.0 - p[2];
        if (!(G[C_P0] > 0.0) || !(G[C_P1] > G[C_P0]) || !(G[C_P1] < R.xl1)) st = ST_BAD_GEOMETRY;
    } else if (st == ST_OK && kind == 2) {  // rdisc/xl1, az, fis, scale/xl1, exp1, exp2, tilt, yaw
        const double rd = p[0] * R.xl1, az = p[1], fis = p[2], a1 = p[4], a2 = p[5];
        if (!(rd > 0.0) || !(rd < R.xl1) || !(p[3] > 0.0) || !(a1 > 0.0) || !(a2 > 0.0)) st = ST_BAD_GEOMETRY;
        double bs[4];
        if (st == ST_OK) st = bspot(R, rd, bs);
        if (st == ST_OK) {
            const double upk = pow(a1 / a2, 1.0 / a2);
            const double lnpk = a1 * log(upk) - pow(upk, a2);
            double stl, ctl, sps, cps, saz, caz;
            sincos(p[6] * DEG, &stl, &ctl);
            sincos((az - 90.0 + p[7]) * DEG, &sps, &cps);
            sincos(az * DEG, &saz, &caz);
            G[C_BSX] = bs[0]; G[C_BSY] = bs[1];
            G[C_L] = p[3] * R.xl1; G[C_UPK] = upk; G[C_LNPK] = lnpk; G[C_UMAX] = bs_umax(a1, a2, lnpk);
            G[C_E1] = a1; G[C_E2] = a2; G[C_CAZ] = caz; G[C_SAZ] = saz;
            G[C_NB0] = stl * cps; G[C_NB1] = stl * sps; G[C_NB2] = ctl;
            G[C_BDEN] = fis + (1.0 - fis) * fmax(fabs(stl) * s + ctl * c, 0.0);
            G[C_FIS] = fis;
        }
    }
    if (st == ST_OK) {
        G[C_Q] = R.q; G[C_CA] = R.cA; G[C_CB] = R.cB; G[C_MU] = R.mu;
        G[C_XL1] = R.xl1; G[C_PL1] = R.pl1; G[C_RS] = R.Rs; G[C_RS2] = R.Rs2;
        G[C_S] = s; G[C_C] = c;
    }
    status[i] = st;
    (void)n1;
}

__global__ __launch_bounds__(64) void k_comp_elements(int kind, int W, int n1, int n2, int nel,
                                                      const double* __restrict__ geo, const int* __restrict__ status,
                                                      double* __restrict__ e3)
{
    const long t = long(blockIdx.x) * 64 + threadIdx.x;
    if (t >= long(W) * nel) return;
    const int set = int(t / nel), k = int(t - long(set) * nel);
    if (status[set] != ST_OK) return;
    const double* G = geo + size_t(set) * CGEO;
    const Roche R{G[C_Q], G[C_CA], G[C_CB], G[C_MU], G[C_XL1], G[C_PL1], G[C_RS], G[C_RS2]};
    const double s = G[C_S], c = G[C_C];
    double* o = e3 + size_t(t) * 3;
    double Px, Py, Pz = 0.0, wgt;
    if (kind == 3) {  // donor tile (MODEL_SPEC 5.4), band it, azimuth ip
        const int it = k / n2, ip = k - it * n2;
        const double t0 = PI * it / n1, t1 = PI * (it + 1) / n1;
        double stc, ctc, sph, cph;
        sincos(0.5 * (t0 + t1), &stc, &ctc);
        sincos(TWO_PI * (ip + 0.5) / n2, &sph, &cph);
        const double dOm = (cos(t0) - cos(t1)) * (TWO_PI / n2);
        const double dx = -ctc, dy = stc * cph, dz = stc * sph;
        double lo = 0.0, hi = R.Rs, r = G[C_REFF];
        if (!(r > lo && r < hi)) r = 0.5 * hi;
        double gx, gy, gz;
        for (int itr = 0; itr < ROOT_MAXIT; ++itr) {
            const double f = rpot_grad(R, fma(r, dx, 1.0), r * dy, r * dz, gx, gy, gz) - R.pl1;
            const double df = gx * dx + gy * dy + gz * dz;
            if (f > 0.0) hi = r; else lo = r;
            if (df > 0.0 && fabs(f / df) <= ROOT_LAST) { r -= f / df; break; }
            double rn = (df > 0.0) ? r - f / df : 0.5 * (lo + hi);
            if (!(rn > lo && rn < hi)) rn = 0.5 * (lo + hi);
            r = rn;
        }
        rgrad(R, fma(r, dx, 1.0), r * dy, r * dz, gx, gy, gz);
        const double ig = 1.0 / sqrt(gx * gx + gy * gy + gz * gz);
        const double nx = gx * ig, ny = gy * ig, nz = gz * ig;
        const double dA = r * r * dOm / (nx * dx + ny * dy + nz * dz);
        o[0] = dA * nx;
        o[1] = dA * ny;
        o[2] = dA * nz;
        return;
    }
    if (kind == 0) {  // WD tile (MODEL_SPEC 5.1): ring ir holds tiles 4 ir^2 .. 4 (ir + 1)^2
        int ir = int(sqrt(k * 0.25));
        if (4 * (ir + 1) * (ir + 1) <= k) ++ir;
        if (4 * ir * ir > k) --ir;
        const int nk = 4 * (2 * ir + 1), j = k - 4 * ir * ir;
        const double r0 = double(ir) / NWD_RINGS, r1 = double(ir + 1) / NWD_RINGS, u = G[C_P1];
        const double F0 = (1.0 - u) * 0.5 * r0 * r0 - u * pow(1.0 - r0 * r0, 1.5) / 3.0;
        const double F1 = (1.0 - u) * 0.5 * r1 * r1 - u * pow(1.0 - r1 * r1, 1.5) / 3.0;
        wgt = (TWO_PI / nk) * (F1 - F0);
        const double rc = sqrt(0.5 * (r0 * r0 + r1 * r1)), mu0 = sqrt(1.0 - rc * rc);
        double sp, cpp;
        sincos(TWO_PI * (j + 0.5) / nk, &sp, &cpp);
        const double rw = G[C_P0];
        Px = rw * (-rc * sp * c + mu0 * s);
        Py = rw * (rc * cpp);
        Pz = rw * (rc * sp * s + mu0 * c);
    } else if (kind == 1) {  // disc element (MODEL_SPEC 5.2): ring ir of n1, azimuth j of n2
        const int ir = k / n2, j = k - ir * n2;
        const double rin = G[C_P0], dr = (G[C_P1] - rin) / n1, ex = G[C_P2];
        const double r0 = rin + ir * dr, r1 = rin + (ir + 1) * dr, rc = 0.5 * (r0 + r1);
        const double I = (fabs(ex) < 1e-10) ? log(r1 / r0) : (pow(r1, ex) - pow(r0, ex)) / ex;
        wgt = (TWO_PI / n2) * I;
        double sa, ca;
        sincos(TWO_PI * (j + 0.5) / n2, &sa, &ca);
        Px = rc * ca;
        Py = rc * sa;
    } else {  // bright-spot strip element (MODEL_SPEC 5.3)
        const double uk = (k + 0.5) * (G[C_UMAX] / n1);
        wgt = exp(G[C_E1] * log(uk) - pow(uk, G[C_E2]) - G[C_LNPK]);
        const double off = G[C_L] * (uk - G[C_UPK]);
        Px = fma(off, G[C_CAZ], G[C_BSX]);
        Py = fma(off, G[C_SAZ], G[C_BSY]);
    }
    double a, b;
    element_interval_fast(R, Px, Py, Pz, s, c, G[C_RCAL], G[C_REFF], a, b);
    o[0] = a;
    o[1] = b;
    o[2] = wgt;
}

__device__ __forceinline__ double block_sum(double v, double* red)
{
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    __syncthreads();
    if (lane == 0) red[wv] = v;
    __syncthreads();
    double t = 0.0;
    for (int i = 0; i < COMP_BLOCK / 64; ++i) t += red[i];
    return t;
}

__global__ __launch_bounds__(COMP_BLOCK) void k_comp_flux(int kind, int nel, const double* __restrict__ geo,
                                                          const int* __restrict__ status,
                                                          const double* __restrict__ e3, const double* __restrict__ x,
                                                          const double* __restrict__ w, int N, double* __restrict__ out)
{
    __shared__ double se[COMP_TILE * 3];
    __shared__ double red[COMP_BLOCK / 64];
    const int set = blockIdx.x, tid = threadIdx.x;
    const double* G = geo + size_t(set) * CGEO;
    const double* E = e3 + size_t(set) * nel * 3;
    double* o = out + size_t(set) * N;
    if (status[set] != ST_OK) {
        for (int p = tid; p < N; p += COMP_BLOCK) o[p] = NAN;
        return;
    }
    const double s = G[C_S], c = G[C_C];
    // normalisation: total weight, or the donor's projected area at quadrature
    double tot = 0.0;
    for (int k = tid; k < nel; k += COMP_BLOCK)
        tot += (kind == 3) ? fmax(-s * E[3 * k + 1] + c * E[3 * k + 2], 0.0) : E[3 * k + 2];
    tot = block_sum(tot, red);
    for (int p0 = 0; p0 < N; p0 += COMP_BLOCK) {
        const int p = p0 + tid;
        double ph = 0.0, h = 0.0;
        if (p < N) {
            ph = x[p];
            h = w ? w[p] : 0.0;
        }
        ph -= floor(ph + 0.5);
        double sn, cs;
        sincospi(2.0 * ph, &sn, &cs);
        const double e0 = s * cs, e1 = -s * sn;
        const double lo = ph - h, hi = ph + h;
        double acc = 0.0;
        for (int k0 = 0; k0 < nel; k0 += COMP_TILE) {
            const int m = min(COMP_TILE, nel - k0);
            __syncthreads();
            for (int i = tid; i < 3 * m; i += COMP_BLOCK) se[i] = E[3 * k0 + i];
            __syncthreads();
            if (kind == 3) {
                for (int j = 0; j < m; ++j)
                    acc += fmax(se[3 * j] * e0 + se[3 * j + 1] * e1 + se[3 * j + 2] * c, 0.0);
            } else if (h > 0.0) {  // exact overlap of the window with the eclipse interval
                for (int j = 0; j < m; ++j)
                    acc += se[3 * j + 2] * fmax(fmin(se[3 * j + 1], hi) - fmax(se[3 * j], lo), 0.0);
            } else {
                for (int j = 0; j < m; ++j)
                    acc += (ph > se[3 * j] && ph < se[3 * j + 1]) ? se[3 * j + 2] : 0.0;
            }
        }
        if (p >= N) continue;
        double f;
        if (kind == 3) {
            f = acc / tot;
        } else {
            const double ecl = (h > 0.0) ? acc / (2.0 * h) : acc;  // eclipsed weight
            f = (tot - ecl) / tot;
            if (kind == 2) {
                const double bden = G[C_BDEN], fis = G[C_FIS];
                const double beam = (bden > 0.0)
                    ? (fis + (1.0 - fis) * fmax(G[C_NB0] * e0 + G[C_NB1] * e1 + G[C_NB2] * c, 0.0)) / bden
                    : 0.0;
                f *= beam;
            }
        }
        o[p] = f;
    }
}

inline int launch_ok() { return hipGetLastError() == hipSuccess ? LFG_OK : LFG_E_LAUNCH; }

}  // namespace

extern "C" {

size_t lfg_component_workspace_size(int kind, int W, int n1, int n2)
{
    const int nel = comp_nel(kind, n1, n2);
    if (W <= 0 || nel <= 0) return 0;
    return comp_carve(nullptr, W, nel).total;
}

int lfg_component(int kind, const double* cpars, int ncp, const double* q, const double* inc, int W, int n1, int n2,
                  const double* x, const double* w, int N, double* out, int* status, void* wsp, size_t ws_bytes,
                  void* stream)
{
    static const int kNcp[4] = {2, 3, 8, 0};
    if (kind < 0 || kind > 3 || W <= 0 || N < 0 || !q || !inc || !out || !status || (N > 0 && !x)) return LFG_E_ARGS;
    if (ncp != kNcp[kind] || (ncp > 0 && !cpars)) return LFG_E_ARGS;
    if ((kind == 1 || kind == 3) && (n1 < 1 || n2 < 1)) return LFG_E_ARGS;
    if (kind == 2 && n1 < 1) return LFG_E_ARGS;
    const int nel = comp_nel(kind, n1, n2);
    CompWs ws = comp_carve(wsp, W, nel);
    if (!wsp || ws_bytes < ws.total) return LFG_E_WORKSPACE;
    hipStream_t st = static_cast<hipStream_t>(stream);
    hipLaunchKernelGGL(k_comp_setup, dim3((W + 63) / 64), dim3(64), 0, st, kind, cpars, ncp, q, inc, W, n1, ws.geo,
                       ws.status);
    int rc = launch_ok();
    if (rc) return rc;
    const long nt = long(W) * nel;
    hipLaunchKernelGGL(k_comp_elements, dim3(unsigned((nt + 63) / 64)), dim3(64), 0, st, kind, W, n1, n2, nel, ws.geo,
                       ws.status, ws.e3);
    if ((rc = launch_ok())) return rc;
    if (N > 0) {
        hipLaunchKernelGGL(k_comp_flux, dim3(W), dim3(COMP_BLOCK), 0, st, kind, nel, ws.geo, ws.status, ws.e3, x, w,
                           N, out);
        if ((rc = launch_ok())) return rc;
    }
    if (hipMemcpyAsync(status, ws.status, sizeof(int) * W, hipMemcpyDeviceToDevice, st) != hipSuccess)
        return LFG_E_LAUNCH;
    return LFG_OK;
}

}  // extern "C"
