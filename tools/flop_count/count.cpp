// count.cpp -- FP64 operation counts of the MI355X path's algorithm, per
// walker-eclipse evaluation (MODEL_SPEC.md section 11).  The device functions
// of lfit_python_amd/csrc/lfg_device.hpp are compiled for the host over the
// counting type of flop.hpp (`double` -> F64), and the lane bodies of k_setup
// and k_elements (lfg.hip) are restated around them, so the counts are those
// of the kernels' own arithmetic, iteration by iteration, on given parameter
// sets.  Built and driven by tools/flop_count.py; tooling only.
#include <algorithm>

#include "flop.hpp"
#define double F64
#include "lfg_device.hpp"
#include "lfg_tables.hpp"
#undef double

using namespace lfg;

namespace {

FlopCtr snap() { return g_ctr; }
long long since(const FlopCtr& a) { return g_ctr.flops() - a.flops(); }
long long trans_since(const FlopCtr& a) { return g_ctr.trans - a.trans; }

int wd_ring_of(int u)
{
    int ir = int(std::sqrt(u * 0.5));
    if (2 * (ir + 1) * (ir + 1) <= u) ++ir;
    if (2 * ir * ir > u) --ir;
    return ir;
}

constexpr int U_WD = NWD / 2, U_DISC = NDISC / 2, U_BS = NBS, U_DON = NDONOR / 4;

}  // namespace

extern "C" {

// out[0..]: see COUNT_FIELDS in tools/flop_count.py
int lfc_count_pair(const double* pin, int np, long long* out)
{
    for (int i = 0; i < 32; ++i) out[i] = 0;
    F64 p[18];
    for (int k = 0; k < 18; ++k) p[k] = F64(k < np ? pin[k] : 0.0);
    if (np == 14) { p[14] = 2.0; p[15] = 1.0; p[16] = 90.0; p[17] = 0.0; }

    // ---- k_setup setup lane (lfg.hip k_setup, pair part)
    FlopCtr c0 = snap();
    Roche R;
    if (roche_init(R, p[4]) != ST_OK) return 1;
    F64 inc;
    if (findi_fast(R, p[5], inc) != ST_OK) return 2;
    {
        F64 s, c;
        sincos(inc * DEG, &s, &c);
        const F64 tilt = p[16] * DEG, psi = (p[10] - 90.0 + p[17]) * DEG;
        F64 st_, ct_, sp_, cp_, saz, caz;
        sincos(tilt, &st_, &ct_);
        sincos(psi, &sp_, &cp_);
        const F64 nmax = fabs(st_) * s + ct_ * c;
        sincos(p[10] * DEG, &saz, &caz);
        const F64 bden = p[11] + (1.0 - p[11]) * fmax(nmax, 0.0);
        const F64 sce = s * cos(PI * p[5]);
        const F64 rcal = sqrt(1.0 - sce * sce);
        const F64 reff = eggleton(R.q);
        const F64 nb0 = st_ * cp_, nb1 = st_ * sp_;
        (void)bden; (void)rcal; (void)reff; (void)nb0; (void)nb1;
    }
    out[0] = since(c0);
    out[1] = trans_since(c0);

    // ---- k_setup stream lane: the stream table (MODEL_SPEC 4.5), the
    // azimuth prior's angle and the strip shape (MODEL_SPEC 5.3)
    c0 = snap();
    Roche Rb;
    QPatch qp;
    roche_init(Rb, p[4], &qp);
    F64 bs[4];
    if (bspot<false>(Rb, p[6] * Rb.xl1, bs, &qp) != ST_OK) return 3;
    {
        F64 alpha = atan2(bs[1], bs[0]) / DEG;
        const F64 a1 = p[14], a2 = p[15];
        const F64 upk = pow(a1 / a2, 1.0 / a2);
        const F64 lnpk = a1 * log(upk) - pow(upk, a2);
        const F64 umax = bs_umax(a1, a2, lnpk);
        (void)alpha; (void)umax;
    }
    out[2] = since(c0);
    out[3] = trans_since(c0);

    // ---- k_setup prior lane: the LCModel dphi prior from the findphi(q, 90)
    // series (Prior sums are counted per parameter by the caller)
    c0 = snap();
    {
        const QPatch pq = q_patch(p[4]);
        F64 maxphi = pq.iq >= 0 ? q_series(kStPhi90, pq) : F64(0.0);
        if (pq.iq < 0) {
            Roche Rp;
            roche_init(Rp, p[4]);
            findphi_fast(Rp, 90.0, maxphi);
        }
        const F64 lim = maxphi - DPHI_TOL;
        (void)lim;
    }
    out[4] = since(c0);
    out[5] = trans_since(c0);

    // ---- k_elements: geometry shared by the items
    F64 s, c;
    sincos(inc * DEG, &s, &c);
    const F64 rwd_a = p[8] * R.xl1, rdisc_a = p[6] * R.xl1;
    const F64 sce = s * cos(PI * p[5]);
    const F64 rcal = sqrt(1.0 - sce * sce), reff = eggleton(R.q);
    const F64 a1 = p[14], a2 = p[15];
    const F64 upk = pow(a1 / a2, 1.0 / a2);
    const F64 lnpk = a1 * log(upk) - pow(upk, a2);
    const F64 umax = bs_umax(a1, a2, lnpk);
    F64 saz, caz;
    sincos(p[10] * DEG, &saz, &caz);
    const F64 L = p[9] * R.xl1;

    // out[6..9]: WD, disc, spot, donor FLOPs summed over the unique items;
    // out[10..13] their transcendental counts; out[14..16] items eclipsed,
    // fallbacks to the nested solver, Newton steps (ingress + egress);
    // out[17] cone-search steps
    auto item = [&](F64 Px, F64 Py, F64 Pz, int slot) {
        FlopCtr a = snap();
        F64 ea, eb;
        bool fb = false;
        int nit[3] = {0, 0, 0};
        const bool ecl = element_interval_fast(R, Px, Py, Pz, s, c, rcal, reff, ea, eb, &fb, nit);
        out[6 + slot] += since(a);
        out[10 + slot] += trans_since(a);
        out[14] += ecl ? 1 : 0;
        out[15] += fb ? 1 : 0;
        out[16] += nit[1] + nit[2];
        out[17] += nit[0];
        // tangency_pair steps both sides in lockstep until both have
        // converged: the steps of an already converged side are discarded
        // work of the implementation, not of the algorithm (taken off below)
        if (nit[1] + nit[2] > 0) out[18] += 2 * (nit[1] > nit[2] ? nit[1] : nit[2]) - (nit[1] + nit[2]);
        out[19 + slot] += (nit[1] + nit[2] > 0) ? 2 * (nit[1] > nit[2] ? nit[1] : nit[2]) - (nit[1] + nit[2]) : 0;
    };
    for (int u = 0; u < U_WD; ++u) {  // k_elements WD item
        const int ir = wd_ring_of(u);
        const F64 rc = kWdRc[ir], mu0 = kWdMu0[ir], cp = kWdCos[u], sp = kWdSin[u];
        FlopCtr a = snap();
        const F64 Px = rwd_a * (-rc * sp * c + mu0 * s), Py = rwd_a * (rc * cp), Pz = rwd_a * (rc * sp * s + mu0 * c);
        out[6] += since(a);
        item(Px, Py, Pz, 0);
    }
    for (int uu = 0; uu < U_DISC; ++uu) {  // disc item
        const int ir = uu / (NDISC_AZ / 2), j = uu - ir * (NDISC_AZ / 2);
        FlopCtr a = snap();
        const F64 rc = rwd_a + (ir + 0.5) * ((rdisc_a - rwd_a) / NDISC_R);
        const F64 Px = rc * kDiscCos[j], Py = rc * kDiscSin[j];
        if (j == 0) {  // ring weight: two boundary terms
            const F64 ex = 2.0 - p[12];
            const F64 r0 = rwd_a + ir * ((rdisc_a - rwd_a) / NDISC_R), r1 = rwd_a + (ir + 1) * ((rdisc_a - rwd_a) / NDISC_R);
            const F64 w = (TWO_PI / NDISC_AZ) * (pow(r1, ex) / ex - pow(r0, ex) / ex);
            (void)w;
        }
        out[7] += since(a);
        out[11] += trans_since(a);
        item(Px, Py, F64(0.0), 1);
    }
    for (int j = 0; j < U_BS; ++j) {  // spot item
        FlopCtr a = snap();
        const F64 uk = (j + 0.5) * (umax / NBS);
        const F64 w = exp(a1 * log(uk) - pow(uk, a2) - lnpk);
        const F64 off = L * (uk - upk);
        const F64 Px = fma(off, caz, bs[0]), Py = fma(off, saz, bs[1]);
        (void)w;
        out[8] += since(a);
        out[12] += trans_since(a);
        item(Px, Py, F64(0.0), 2);
    }
    for (int uu = 0; uu < U_DON; ++uu) {  // donor tile: radius root, normal, area, visibility arc
        FlopCtr a = snap();
        const int it = uu / (NDONOR_P / 4), ip = uu - it * (NDONOR_P / 4);
        const F64 stc = kDonSt[it], ctc = kDonCt[it];
        const F64 dx = -ctc, dy = stc * kDonCp[ip], dz = stc * kDonSp[ip];
        F64 lo = 0.0, hi = R.Rs, r = reff;
        if (!(r > lo && r < hi)) r = 0.5 * hi;
        F64 gx, gy, gz;
        for (int itr = 0; itr < ROOT_MAXIT; ++itr) {
            const F64 X0 = fma(r, dx, 1.0), X1 = r * dy, X2 = r * dz;
            const F64 f = rpot_grad(R, X0, X1, X2, gx, gy, gz) - R.pl1;
            const F64 df = gx * dx + gy * dy + gz * dz;
            if (f > 0.0) hi = r; else lo = r;
            if (df > 0.0 && fabs(f / df) <= ROOT_LAST) { r -= f / df; break; }
            F64 rn = (df > 0.0) ? r - f / df : 0.5 * (lo + hi);
            if (!(rn > lo && rn < hi)) rn = 0.5 * (lo + hi);
            r = rn;
        }
        rgrad(R, fma(r, dx, 1.0), r * dy, r * dz, gx, gy, gz);
        const F64 ig = rsqrt(gx * gx + gy * gy + gz * gz);
        const F64 nx = gx * ig, ny = gy * ig, nz = gz * ig;
        const F64 dA = r * r * kDonOmega[it] / (nx * dx + ny * dy + nz * dz);
        const F64 vx = dA * nx, vy = dA * ny, vz = dA * nz;
        const F64 srho = s * sqrt(vx * vx + vy * vy);
        const F64 kap = (srho > 0.0) ? -c * vz / srho : F64(2.0);
        const F64 cen = -atan2(vy, vx) * (1.0 / TWO_PI);
        const F64 hw = acos(fmin(fmax(kap, -1.0), 1.0)) * (1.0 / TWO_PI);
        (void)cen; (void)hw;
        out[9] += since(a);
        out[13] += trans_since(a);
    }
    return 0;
}

// static counts of single building blocks (one call each), for the tables
// of MODEL_SPEC 11: out[0] cone_point, [1] tangency_step, [2] one RK4 step
// of the stream, [3] one ray_min Newton iteration (nested solver), [4] one
// donor-radius Newton step, [5] rpot_grad, [6] rotate
void lfc_unit_counts(long long* out)
{
    Roche R;
    roche_init(R, F64(0.1037));
    FlopCtr a = snap();
    ConePt o;
    cone_point(R, 0.01, 0.02, 0.0, 0.99, 0.1, 0.9, 0.43, 0.8, o);
    out[0] = since(a);
    a = snap();
    Tan T{0.3, 0.95, 0.3, 0.8, 0};
    tangency_step(R, 0.01, 0.02, 0.0, 0.99, 0.1, true, T);
    out[1] = since(a);
    a = snap();
    StreamState s0{0.7, 0.01, -0.1, 0.05};
    const F64 dt = 0.01;
    const StreamState k1 = stream_deriv(R, s0);
    const StreamState k2 = stream_deriv(R, axpy(s0, 0.5 * dt, k1));
    const StreamState k3 = stream_deriv(R, axpy(s0, 0.5 * dt, k2));
    const StreamState k4 = stream_deriv(R, axpy(s0, dt, k3));
    const F64 h6 = dt / 6.0;
    StreamState sn{s0.x + h6 * (k1.x + 2.0 * k2.x + 2.0 * k3.x + k4.x), s0.y + h6 * (k1.y + 2.0 * k2.y + 2.0 * k3.y + k4.y),
                   s0.vx + h6 * (k1.vx + 2.0 * k2.vx + 2.0 * k3.vx + k4.vx),
                   s0.vy + h6 * (k1.vy + 2.0 * k2.vy + 2.0 * k3.vy + k4.vy)};
    (void)sn;
    out[2] = since(a);
    a = snap();
    F64 tw = 0.9, fm;
    // one Newton iteration: ray_min with a pre-converged t runs exactly one
    ray_min(R, 0.01, 0.02, 0.0, 0.99, -0.1, 0.1, tw, fm);
    out[3] = since(a);
    a = snap();
    {
        F64 gx, gy, gz;
        const F64 r = 0.2, dx = -0.9, dy = 0.3, dz = 0.3;
        const F64 f = rpot_grad(R, fma(r, dx, 1.0), r * dy, r * dz, gx, gy, gz) - R.pl1;
        const F64 df = gx * dx + gy * dy + gz * dz;
        const F64 rn = r - f / df;
        (void)rn;
    }
    out[4] = since(a);
    a = snap();
    {
        F64 gx, gy, gz;
        rpot_grad(R, 0.7, 0.1, 0.1, gx, gy, gz);
    }
    out[5] = since(a);
    a = snap();
    F64 cs = 0.9, sn2 = 0.43;
    rotate(cs, sn2, 0.01);
    out[6] = since(a);
    // one Kalman step of the GP likelihood (MODEL_SPEC 10.4), inside a block
    GPFilter gpf;
    gpf.init(1e-4, 2e-4, 0.01);
    gpf.step(0.0, 0.004, 0.001, 0);
    a = snap();
    gpf.step(0.001, 0.004, 0.002, 0);
    out[7] = since(a);
}

}  // extern "C"

extern "C" long long lfc_count_prior(int type, double p1, double p2, double norm, double v)
{
    FlopCtr a = snap();
    const F64 r = prior_lnprob(type, F64(p1), F64(p2), F64(norm), F64(v));
    (void)r;
    return since(a);
}
