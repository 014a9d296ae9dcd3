// fbdebug.cpp -- why does an element leave the fast path?  Restates
// element_interval_fast (lfg_device.hpp) step by step over the host build of
// the device functions (count.cpp's recipe) and reports, for every item of a
// pair that falls back, which test sent it there.  Tooling only
// (tools/fallback_debug.py).
#include <algorithm>
#include <cstdio>

#include "flop.hpp"
#define double F64
#include "lfg_device.hpp"
#include "lfg_tables.hpp"
#undef double

using namespace lfg;

namespace {
constexpr int U_WD = NWD / 2, U_DISC = NDISC / 2, U_BS = NBS;

// reason codes: 1 cone undecided, 2 contact guess outside (-1, 1),
// 3 ingress not converged/wrong kind, 4 egress, 5 order, 6 range (cin/cout)
int why(const Roche& R, F64 Px, F64 Py, F64 Pz, F64 s, F64 c, F64 Rcal, double* info)
{
    const F64 ux = 1.0 - Px, uy = -Py, uz = -Pz;
    const F64 uxy2 = ux * ux + uy * uy, uu = uxy2 + uz * uz;
    if (!(uu > R.Rs2 && uxy2 > 0.0 && s > 0.0)) return 7;
    const F64 iuxy = rsqrt(uxy2), uxy = uxy2 * iuxy;
    const F64 cosD = (sqrt(uu - R.Rs2) - c * uz) * iuxy / s;
    if (cosD >= 1.0) return 0;
    const F64 cc = ux * iuxy, sc = -uy * iuxy, tc = s * uxy + uz * c;
    int ex = cone_exists(R, Px, Py, Pz, s, c, cc, sc, tc);
    {
        const F64 ex0 = s * cc, ey0 = -s * sc;
        const F64 x = fma(tc, ex0, Px), y = fma(tc, ey0, Py), z = fma(tc, c, Pz);
        const F64 dx = x - 1.0, xm = x - R.mu;
        const F64 r2s = dx * dx + y * y + z * z;
        const F64 phi = -R.cA * rsqrt_pos(x * x + y * y + z * z) - R.cB * rsqrt_pos(r2s) - xm * xm - y * y;
        if (phi < R.pl1 && r2s < R.Rs2) ex = 1;
    }
    info[0] = ex;
    if (ex == 0) return 0;
    if (ex == -1) return 1;
    const F64 ce = (sqrt(fmax(uu - Rcal * Rcal, 0.0)) - c * uz) * iuxy / s;
    info[1] = ce.v;
    if (!(ce > -1.0 && ce < 1.0)) return 2;
    const F64 se = sqrt(1.0 - ce * ce);
    const F64 thc = atan2(-uy, ux), de = acos(ce);
    F64 ci = cc * ce + sc * se, si = sc * ce - cc * se;
    F64 co = cc * ce - sc * se, so = sc * ce + cc * se;
    Tan In{thc - de, ci, si, s * (ux * ci - uy * si) + uz * c, 0};
    Tan Out{thc + de, co, so, s * (ux * co - uy * so) + uz * c, 0};
    int nit[2] = {0, 0};
    tangency_pair(R, Px, Py, Pz, s, c, In, Out, nit);
    info[2] = In.st; info[3] = Out.st; info[4] = nit[0]; info[5] = nit[1];
    info[6] = In.th.v; info[7] = Out.th.v; info[8] = thc.v; info[9] = de.v;
    const F64 cin = In.cs * cc + In.sn * sc, cout = Out.cs * cc + Out.sn * sc;
    info[10] = cin.v; info[11] = cout.v; info[12] = cosD.v;
    if (In.st != 1) return 3;
    if (Out.st != 1) return 4;
    if (!(In.th < Out.th)) return 5;
    if (!(cin > cosD && cout > cosD)) return 6;
    return 0;
}
}  // namespace

extern "C" {

// p: 18 cv parameters; prints the fallback items of the pair; returns their count
int fbd_pair(const double* pin, int verbose)
{
    F64 p[18];
    for (int k = 0; k < 18; ++k) p[k] = F64(pin[k]);
    Roche R;
    if (roche_init(R, p[4]) != ST_OK) return -1;
    F64 inc;
    if (findi_fast(R, p[5], inc) != ST_OK) return -2;
    Roche Rb;
    QPatch qp;
    roche_init(Rb, p[4], &qp);
    F64 bs[4];
    if (bspot<false>(Rb, p[6] * Rb.xl1, bs, &qp) != ST_OK) return -3;
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
    int nfb = 0;
    auto item = [&](F64 Px, F64 Py, F64 Pz, int u) {
        F64 ea, eb;
        bool fb = false;
        element_interval_fast(R, Px, Py, Pz, s, c, rcal, reff, ea, eb, &fb);
        if (!fb) return;
        ++nfb;
        double info[13] = {0};
        const int w = why(R, Px, Py, Pz, s, c, rcal, info);
        if (verbose)
            std::printf("  item %4d P (%.5f %.5f %.5f) why %d ex %g ce %.4f st %g/%g it %g/%g th %.5f/%.5f thc %.5f "
                        "de %.5f cin %.5f cout %.5f cosD %.5f -> nested [%.6f, %.6f]\n",
                        u, Px.v, Py.v, Pz.v, w, info[0], info[1], info[2], info[3], info[4], info[5], info[6],
                        info[7], info[8], info[9], info[10], info[11], info[12], ea.v, eb.v);
    };
    for (int u = 0; u < U_WD; ++u) {
        const int ir = int(std::sqrt(u * 0.5)) + 0;
        int r = ir;
        if (2 * (r + 1) * (r + 1) <= u) ++r;
        if (2 * r * r > u) --r;
        const F64 rc = kWdRc[r], mu0 = kWdMu0[r], cp = kWdCos[u], sp = kWdSin[u];
        item(rwd_a * (-rc * sp * c + mu0 * s), rwd_a * (rc * cp), rwd_a * (rc * sp * s + mu0 * c), u);
    }
    for (int uu = 0; uu < U_DISC; ++uu) {
        const int ir = uu / (NDISC_AZ / 2), j = uu - ir * (NDISC_AZ / 2);
        const F64 rc = rwd_a + (ir + 0.5) * ((rdisc_a - rwd_a) / NDISC_R);
        item(rc * kDiscCos[j], rc * kDiscSin[j], F64(0.0), U_WD + uu);
    }
    for (int j = 0; j < U_BS; ++j) {
        const F64 uk = (j + 0.5) * (umax / NBS);
        const F64 off = L * (uk - upk);
        item(fma(off, caz, bs[0]), fma(off, saz, bs[1]), F64(0.0), 800 + j);
    }
    return nfb;
}
}
