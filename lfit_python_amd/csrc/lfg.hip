// lfg.hip -- MI355X (gfx950) kernels and the C ABI of liblfg_hip.so.
//
// Pipeline for one batch of walkers (one emcee half-step), on the caller's
// stream only:
//   k_setup     one lane per (walker, eclipse): parameter gather, L1, findi,
//               strip/beam frame, eclipse Roche priors; one lane per walker:
//               LCModel dphi prior + Prior.ln_prob sum; one lane per
//               (walker, eclipse): the ballistic stream to the disc edge
//   k_elements  one lane per (walker, eclipse, element): eclipse interval of
//               every WD / disc / bright-spot element, donor surface tiles
//   k_lnlike    one workgroup per (walker, eclipse): element tables staged in
//               LDS, lanes stride the phase axis (coalesced), exposure
//               integration, fused chi^2 with a wavefront/LDS reduction
//               and, for the walker's last eclipse, ln_prob = ln_prior + sum_e ln_like_e
// Replaces, per walker, mcmcfit.ln_prob (mcmcfit.py:37-41) -> Node.ln_prob
// (model.py:476-498) -> lfit.CV.calcFlux (CVModel.py:138).
#include <hip/hip_runtime.h>
#include <atomic>
#include <stdint.h>
#include <stdlib.h>

#include <type_traits>

#include "lfg.h"
#include "lfg_device.hpp"
#include "lfg_tables.hpp"

using namespace lfg;

// Diagnostic builds that read device counters back (lfg_debug_*) keep every
// kernel in this translation unit (see lfg_pair_launch_split below)
#if defined(LFG_PROFILE_PAIR) || defined(LFG_COUNT_ITERS) || defined(LFG_COUNT_QUIET)
#define LFG_ONE_TU 1
#endif

namespace {

constexpr int SETUP_BLOCK = 64;
#ifndef LFG_ELEM_BLOCK
#define LFG_ELEM_BLOCK 64  // one wave: the item chunks dispatch at wave granularity (36.0 vs 37.6 us at 256, 36.5 at 128)
#endif
constexpr int ELEM_BLOCK = LFG_ELEM_BLOCK;
#ifndef LFG_ELEM_IPL
#define LFG_ELEM_IPL 1  // items per k_elements lane
#endif
#ifndef ELEM_MINW
#define ELEM_MINW 4  // minimum waves per SIMD of k_elements: <= 128 VGPRs, no spill (at 5 waves / 96 VGPRs the
                     // speculative setup lanes spilled ~100 B/lane; 4 waves measured 3 % faster)
#endif
// per-pair weight block written by k_elements: disc ring weights, the disc
// total 2 pi [P(rdisc) - P(rin)], spot element weights
constexpr int WT_DISC = 0, WT_TD = NDISC_R, WT_BS = 24, WT_N = WT_BS + NBS;
// Eclipse intervals are stored once per mirror pair (MODEL_SPEC 5: the
// mirrored element's interval is [-b, -a]): NU_WDD symmetry-unique WD/disc
// items, then the NBS spot elements, NELU (a, b) pairs per pair in all.  The
// WD/disc slots are in sweep order: slot g holds unique item uitem(g), a
// stride-37 permutation (a wave's lanes sweep items of different rings and
// azimuths, so their LDS atomics spread), and k_lnlike's sweep element g in
// [0, NWD + NDISC) is slot g mod NU_WDD, mirrored for g >= NU_WDD: it reads
// its items as coalesced rows, half the bytes of a table of every element.
constexpr int NU_WDD = (NWD + NDISC) / 2, NELU = NU_WDD + NBS;
__device__ __forceinline__ int uitem(int g) { return (g * 37) % NU_WDD; }
__device__ __forceinline__ int uslot(int u) { return (u * 473) % NU_WDD; }
static_assert(NU_WDD == 700 && (37 * 473) % 700 == 1, "sweep permutation inverse");
__device__ __forceinline__ double2 mirror_ab(double2 ab)
{
    return (ab.x < ab.y) ? make_double2(-ab.y, -ab.x) : make_double2(1.0, -1.0);
}
// sweep element g of a pair's table (g < NWD + NDISC)
__device__ __forceinline__ double2 sweep_ab(const double2* __restrict__ AB, int g)
{
    return (g < NU_WDD) ? AB[g] : mirror_ab(AB[g - NU_WDD]);
}
// per unique donor tile: vx, vy, vz, arc centre, arc half-width (phase units)
constexpr int DON_STRIDE = 5;


struct Ws {
    double* geo;
    int* status;
    int* bstatus;   // [pairs] stream status (k_setup stream lanes), folded into status by k_elements
    double2* ab;    // [pairs][NELU] eclipse intervals (a, b) of the symmetry-unique elements
    double* donor;  // [pairs][NDONOR/4][DON_STRIDE] symmetry-unique donor tiles
    double* wts;    // [pairs][WT_N] ring / spot weights
    double* prior;
    double* lle;
    double* res;    // [pairs][gp_n] GP trees: residuals y - flux (k_lnlike<2> -> k_gp_like)
    double* gpx;    // [pairs][gp_n] GP trees: e^{-lam dx} of each point (k_lnlike<2> -> k_gp_like)
    int* gpb;       // [pairs][gp_n] GP trees: each point's changepoint block
    // speculative setup (lfg_stretch_step_half_spec): per half parity h and
    // candidate c (the partner's move rejected / accepted) the k_setup
    // outputs of the next half, formed inside the previous half's k_elements
    double* geoC;   // [2][2][pairs][NGEO]
    int* statusC;   // [2][2][pairs]
    int* bstatusC;  // [2][2][pairs]
    double* priorC; // [2][2][W]
    double* qC;     // [2][2][W][ndim]
    double* zfC;    // [2][2][W]
    int* jk;        // [2][W] the partner (in the other half) of walker w's proposal
    int* accflag;   // [2][accstride] by the parity of the half that wrote it: 1 where walker
                    // j accepted its move (a rank's shard of W walkers needs every partner's:
                    // nacc = the half); two copies, so a launch that accepts moves of half h
                    // while it selects candidates by half 1 - h's flags reads one, writes the other
    size_t accstride;
    double* snap;   // [2][accstride][ndim] k_pair: the rows of each half of pos as they were
                    // when the launch that reads them began (SetupArgs.ppos)
    size_t total;
};

inline size_t align256(size_t v) { return (v + 255) & ~size_t(255); }

Ws carve(void* base, int W, int E, int gp_n = 0, int ndim_spec = 0, int nacc = 0)
{
    const size_t pairs = size_t(W) * size_t(E);
    Ws ws{};
    char* p = static_cast<char*>(base);
    size_t off = 0;
    auto take = [&](size_t bytes) { char* r = p ? p + off : nullptr; off += align256(bytes); return r; };
    ws.geo = reinterpret_cast<double*>(take(pairs * LFG_NGEO * sizeof(double)));
    ws.status = reinterpret_cast<int*>(take(pairs * sizeof(int)));
    ws.bstatus = reinterpret_cast<int*>(take(pairs * sizeof(int)));
    ws.ab = reinterpret_cast<double2*>(take(pairs * NELU * sizeof(double2)));
    ws.donor = reinterpret_cast<double*>(take(pairs * (NDONOR / 4) * DON_STRIDE * sizeof(double)));
    ws.wts = reinterpret_cast<double*>(take(pairs * WT_N * sizeof(double)));
    ws.prior = reinterpret_cast<double*>(take(size_t(W) * sizeof(double)));
    ws.lle = reinterpret_cast<double*>(take(pairs * sizeof(double)));
    ws.res = gp_n > 0 ? reinterpret_cast<double*>(take(pairs * size_t(gp_n) * sizeof(double))) : nullptr;
    ws.gpx = gp_n > 0 ? reinterpret_cast<double*>(take(pairs * size_t(gp_n) * sizeof(double))) : nullptr;
    ws.gpb = gp_n > 0 ? reinterpret_cast<int*>(take(pairs * size_t(gp_n) * sizeof(int))) : nullptr;
    if (ndim_spec > 0) {
        ws.geoC = reinterpret_cast<double*>(take(4 * pairs * LFG_NGEO * sizeof(double)));
        ws.statusC = reinterpret_cast<int*>(take(4 * pairs * sizeof(int)));
        ws.bstatusC = reinterpret_cast<int*>(take(4 * pairs * sizeof(int)));
        ws.priorC = reinterpret_cast<double*>(take(4 * size_t(W) * sizeof(double)));
        ws.qC = reinterpret_cast<double*>(take(4 * size_t(W) * ndim_spec * sizeof(double)));
        ws.zfC = reinterpret_cast<double*>(take(4 * size_t(W) * sizeof(double)));
        ws.jk = reinterpret_cast<int*>(take(2 * size_t(W) * sizeof(int)));
        ws.accstride = size_t(W > nacc ? W : nacc);
        ws.accflag = reinterpret_cast<int*>(take(2 * ws.accstride * sizeof(int)));
        ws.snap = reinterpret_cast<double*>(take(2 * ws.accstride * ndim_spec * sizeof(double)));
    }
    ws.total = off;
    return ws;
}

// Philox draws of the stretch move (defined with k_propose below)
__device__ inline uint4 draw(unsigned long long seed, unsigned long long step, int half, int purpose, int i);
__device__ inline double u53(unsigned a, unsigned b);

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
    int* bstatus;  // stream lanes' status
    int gp;        // GP likelihood: per-pair hyper-parameters and changepoints
    const int* gp_gather;
    const double* gp_base;
    // inline stretch-move proposal (lfg_stretch_step_half; pos nullptr: off):
    // walker w of the batch is the proposal for ensemble walker half * W + w,
    // formed from pos as k_propose does; the walker lanes store it in qout
    const double* pos;
    double a;
    unsigned long long seed, step;
    int half;
    double* qout;
    double* zfout;
    // the batch is walkers lo .. lo + W - 1 of the ns-walker half (ns = W,
    // lo = 0 on one process; a rank's shard with lfg_stretch_step_shard)
    int lo, ns;
    int fixed_invalid;  // lfg_tree.fixed_invalid: every prior lane gives -inf
    const double* prior_c;  // lfg_tree.prior_c (nullable): [ndim][2] Prior.ln_prob constants
    // speculative setup of the next half (lfg_stretch_step_half_spec): cand 1
    // forms the proposal from the partner's own proposal of the half before
    // (step_prev, the other half), i.e. as if the partner's move is accepted;
    // cand 0 from the partner's current position.  jkout: the partner index.
    int cand;
    unsigned long long step_prev;
    int* jkout;
    // nullable: the partner half's positions as they were when this launch
    // began ([ns][ndim]; k_pair's speculative lanes, whose launch accepts
    // moves of that half while they read it)
    const double* ppos;
    // deferred acceptance (k_pair<_, true>, lfg_stretch_step_shard_fold):
    // this half's previous moves are accepted by the launch these lanes run
    // in, so a row of this half is its snapshot fsnap [ns][ndim] (taken by
    // the launch before) re-formed as the proposal of step fstep where the
    // gathered verdict fv [ns] says accepted (not NaN).  fv nullptr: nothing
    // pending, the rows are read from pos
    const double* fv;
    const double* fsnap;
    unsigned long long fstep;
};

// where a lane reads walker w's parameters: the walker row, or the
// stretch-move proposal s + z (c_j - s) ... written as k_propose writes it;
// with ci the partner's position is itself the proposal cj + zj (ci - cj)...
// of the half before (speculative setup, candidate 1)
struct Prop {
    const double* s;
    const double* cj;
    double z;
    const double* ci;
    double zj;
    // deferred acceptance (FOLD): s and ci are snapshot rows; where their
    // pending move was accepted, the row is the proposal spp + sz (s - spp)
    // (cpp, cz for ci), as k_apply_verdicts will write it
    const double* spp;
    double sz;
    const double* cpp;
    double cz;
};

// the stretch-move draw of walker i of half h at step t: z and the partner
__device__ __forceinline__ int stretch_draw(const SetupArgs& A, unsigned long long t, int h, int i, double& z)
{
    const uint4 r = draw(A.seed, t, h, 0, i);
    const double zr = (A.a - 1.0) * u53(r.x, r.y) + 1.0;
    z = zr * zr / A.a;
    return int(__umulhi(r.z, unsigned(A.ns)));
}

template <bool FOLD = false>
__device__ inline Prop make_prop(const SetupArgs& A, int w)
{
    if (!A.pos) return Prop{A.walkers + size_t(w) * A.ndim, nullptr, 0.0, nullptr, 0.0, nullptr, 0.0, nullptr, 0.0};
    const int ns = A.ns, i = A.lo + w;  // walker i of the half, as k_propose's lane i
    const uint4 r = draw(A.seed, A.step, A.half, 0, i);
    const double u = u53(r.x, r.y);
    const double zr = (A.a - 1.0) * u + 1.0;
    const int j = int(__umulhi(r.z, unsigned(ns)));
    if (A.jkout && A.cand == 0) A.jkout[w] = j;
    Prop P{A.pos + size_t(A.half * ns + i) * A.ndim,
           A.ppos ? A.ppos + size_t(j) * A.ndim : A.pos + size_t((1 - A.half) * ns + j) * A.ndim, zr * zr / A.a,
           nullptr, 0.0, nullptr, 0.0, nullptr, 0.0};
    const double* other = A.pos + size_t(1 - A.half) * ns * A.ndim;  // the partner half's rows (FOLD: final)
    if (FOLD && A.fv) {  // this half's rows as the pending verdicts leave them
        P.s = A.fsnap + size_t(i) * A.ndim;
        if (!isnan(A.fv[i])) P.spp = other + size_t(stretch_draw(A, A.fstep, A.half, i, P.sz)) * A.ndim;
    }
    if (A.cand) {  // partner j's proposal in the other half (step_prev), as its own make_prop forms it
        const int hp = 1 - A.half;
        const uint4 rj = draw(A.seed, A.step_prev, hp, 0, j);
        const double zrj = (A.a - 1.0) * u53(rj.x, rj.y) + 1.0;
        const int ij = int(__umulhi(rj.z, unsigned(ns)));
        P.ci = A.pos + size_t(A.half * ns + ij) * A.ndim;
        P.zj = zrj * zrj / A.a;
        if (FOLD && A.fv) {
            P.ci = A.fsnap + size_t(ij) * A.ndim;
            if (!isnan(A.fv[ij])) P.cpp = other + size_t(stretch_draw(A, A.fstep, A.half, ij, P.cz)) * A.ndim;
        }
    }
    return P;
}

// CV parameter count of eclipse e.  P is pinned to a register first: written
// as `npars ? npars[e] : P` the compiler selected between the two ADDRESSES
// and, to give the kernel argument P one, copied it into scratch
// column of eclipse parameter k of (walker-eclipse) gather row r: the tree's
// gather map, or the identity (lfg_flux / lfg_lnprob without a tree).  A
// branch, not a pointer select: a select between the kernel argument and the
// constant identity table made every read a flat load
__device__ __forceinline__ int gat_at(const SetupArgs& A, int i)
{
    return A.gather ? A.gather[i] : i % 18;
}

__device__ __forceinline__ int npars_of(const SetupArgs& A, int e)
{
    int P = A.P;
    asm volatile("" : "+s"(P));
    return A.npars ? A.npars[e] : P;
}

template <bool FOLD = false>
__device__ __forceinline__ double gather_par(const SetupArgs& A, const Prop& P, int g)
{
    if (g < 0) return A.consts[-1 - g];
    if (!P.cj) return P.s[g];
    if (!FOLD) {
        const double cj = P.ci ? fma(P.cj[g] - P.ci[g], P.zj, P.ci[g]) : P.cj[g];
        return fma(P.s[g] - cj, P.z, cj);
    }
    // FOLD: an accepted pending move re-formed exactly as k_apply_verdicts
    // (k_accept_regen) writes it: fma(old - partner, z, partner)
    double s = P.s[g], cj = P.cj[g];
    if (P.spp) s = fma(s - P.spp[g], P.sz, P.spp[g]);
    if (P.ci) {
        double ci = P.ci[g];
        if (P.cpp) ci = fma(ci - P.cpp[g], P.cz, P.cpp[g]);
        cj = fma(cj - ci, P.zj, ci);
    }
    return fma(s - cj, P.z, cj);
}

// Diagnostic build only (-DLFG_PROFILE_SETUP): s_memtime cycle counts of the
// phases of each lane into g_setup_cyc[slot][lane] (lfg_debug_setup_cycles):
//  0-3 setup lane: gather, roche_init, findi, total; 4-7 stream lane: gather,
//  roche_init, bspot, total; 8 prior lane total, 9 the same in 100 MHz
//  s_memrealtime ticks (calibrates the shader clock), 10 its roche_init + findphi
#ifdef LFG_PROFILE_SETUP
__device__ unsigned long long g_setup_cyc[11][4096];
#define LFG_T0(v) unsigned long long v = __builtin_amdgcn_s_memtime()
#define LFG_CY(slot, i, v) \
    do { const unsigned long long now_ = __builtin_amdgcn_s_memtime(); \
         if ((i) < 4096) g_setup_cyc[slot][i] = now_ - (v); (v) = now_; } while (0)
#else
#define LFG_T0(v)
#define LFG_CY(slot, i, v)
#endif

// ------------------------------------------------------- stream lanes of k_setup
// One lane per (walker, eclipse): the ballistic stream to the disc edge
// (MODEL_SPEC 4.5, the stream table), the spot-dependent Roche prior
// (CVModel.py:215-316) and the strip shape (MODEL_SPEC 5.3: peak, tail end).
// Needs only q, rdisc, az, exp1 and exp2, so these lanes run beside the setup
// lanes of the same launch; the stream status goes to bstatus and is folded
// into the pair status by k_elements.
template <bool FOLD = false>
__device__ inline void bspot_lane(const SetupArgs& A, int t)
{
    LFG_T0(tl);
    const int w = t / A.E, e = t - w * A.E;
    const Prop P = make_prop<FOLD>(A, w);
    const int np = npars_of(A, e);
    const double q = gather_par<FOLD>(A, P, gat_at(A, e * 18 + 4));
    const double rdisc = gather_par<FOLD>(A, P, gat_at(A, e * 18 + 6));
    const double az = gather_par<FOLD>(A, P, gat_at(A, e * 18 + 10));
    const double a1 = (np == 18) ? gather_par<FOLD>(A, P, gat_at(A, e * 18 + 14)) : 2.0;  // MODEL_SPEC 5.3 simple: 2, 1
    const double a2 = (np == 18) ? gather_par<FOLD>(A, P, gat_at(A, e * 18 + 15)) : 1.0;
    double* G = A.geo + size_t(t) * LFG_NGEO;
#ifdef LFG_PROFILE_SETUP
    unsigned long long tb = tl;
    LFG_CY(4, t, tb);
#endif
    Roche R;
    QPatch qp;
    int st = (isfinite(q) && isfinite(rdisc) && isfinite(az)) ? roche_init(R, q, &qp) : ST_BAD_ARGS;
    LFG_CY(5, t, tb);
    double bs[4] = {0.0, 0.0, 0.0, 0.0};
    if (st == ST_OK) st = bspot<false>(R, rdisc * R.xl1, bs, &qp);
    LFG_CY(6, t, tb);
    double rprior = 0.0;
    if (st != ST_OK) {
        rprior = -INFINITY;
    } else {
        double alpha = atan2(bs[1], bs[0]) / DEG;
        if (alpha < 0.0) alpha = 90.0 - alpha;
        const double tangent = alpha + 90.0;
        const double minaz = fmax(0.0, tangent - AZ_SLOPE), maxaz = fmin(178.0, tangent + AZ_SLOPE);
        if (az < minaz || az > maxaz) rprior = -INFINITY;
    }
    G[G_BSX] = bs[0]; G[G_BSY] = bs[1];
    G[G_RPRIOR_BS] = A.roche_priors ? rprior : 0.0;
    if (a1 > 0.0 && a2 > 0.0 && isfinite(a1) && isfinite(a2)) {  // else the setup lane fails the pair
        const double upk = pow(a1 / a2, 1.0 / a2);
        const double lnpk = a1 * log(upk) - pow(upk, a2);
        const double umax = bs_umax(a1, a2, lnpk);
        G[G_UPK] = upk; G[G_UMAX] = umax; G[G_LNPK] = lnpk;
        G[G_EXP1] = a1; G[G_EXP2] = a2;
        // a profile that over- or underflows (exp2 -> 0) is bad geometry,
        // checked after the stream as the oracle does (MODEL_SPEC 6)
        if (st == ST_OK && !(isfinite(upk) && isfinite(lnpk) && isfinite(umax))) st = ST_BAD_GEOMETRY;
    }
    A.bstatus[t] = st;
    LFG_CY(7, t, tl);
}

// per-walker lane: LCModel.ln_prior dphi check (CVModel.py:452-473) and
// Node.ln_prior over the variable parameters (model.py:439-449); with the
// fused stretch move it also stores the proposal
template <bool FOLD = false>
__device__ inline void prior_lane(const SetupArgs& A, int w)
{
    LFG_T0(tl);
#ifdef LFG_PROFILE_SETUP
    unsigned long long trl = __builtin_amdgcn_s_memrealtime(), tr = tl;  // 100 MHz: calibrates s_memtime
#endif
    const Prop P = make_prop<FOLD>(A, w);
    double lp = 0.0;
    if (A.roche_priors) {
        // LCModel.ln_prior: dphi <= findphi(q, 90) - 1e-6, findphi from the
        // q series of the stream table (~1e-16; the solver outside its range)
        const double q = gather_par<FOLD>(A, P, gat_at(A, 4));
        const double dphi = gather_par<FOLD>(A, P, gat_at(A, 5));
        const QPatch qp = q_patch(q);
        double maxphi;
        if (qp.iq >= 0) {
            maxphi = q_series(kStPhi90, qp);
        } else {
            Roche R;
            if (roche_init(R, q) != ST_OK || findphi_fast(R, 90.0, maxphi) != ST_OK) maxphi = -INFINITY;
        }
        if (!(dphi <= maxphi - DPHI_TOL)) lp = -INFINITY;
        LFG_CY(10, w, tr);
    }
    // the walker's parameters in chunks of PCH: each chunk's loads are issued
    // back to back (one memory latency per chunk, not per parameter), then
    // the proposal is stored and the chunk's prior terms summed in order
    constexpr int PCH = 16;
    double* qo = A.pos ? A.qout + size_t(w) * A.ndim : nullptr;
    for (int d0 = 0; d0 < A.ndim; d0 += PCH) {
        double v[PCH];
#pragma unroll
        for (int k = 0; k < PCH; ++k) v[k] = (d0 + k < A.ndim) ? gather_par<FOLD>(A, P, d0 + k) : 0.0;
        if (qo) {  // store the proposal: k_lnlike copies an accepted one into pos
#pragma unroll
            for (int k = 0; k < PCH; ++k)
                if (d0 + k < A.ndim) qo[d0 + k] = v[k];
        }
        if (A.prior_type && A.prior_c) {
            // Prior.ln_prob from the tree's constants (include/lfg.h): the
            // terms c0 - z^2/2 (gauss) or c0, summed in order, and one log of
            // the chunk's product of log_uniform / mod_jeff arguments.  The
            // product is kept as mantissa x 2^pex (frexp per factor: the
            // mantissas lie in [1/2, 1), so 16 of them never leave the normal
            // range and no partial product loses digits)
            double prod = 1.0;
            int pex = 0;
            bool ok = true;
#pragma unroll
            for (int k = 0; k < PCH; ++k) {
                const int d = d0 + k;
                if (d < A.ndim) {
                    const int ty = A.prior_type[d];
                    const double p1 = A.prior_p1[d], p2 = A.prior_p2[d], c0 = A.prior_c[2 * d];
                    const double z = (v[k] - p1) * A.prior_c[2 * d + 1];
                    const double term = (ty <= 1) ? fma(-0.5 * z, z, c0) : c0;
                    lp += term;
                    int fe;
                    const double fm = frexp((ty == 3) ? v[k] : (ty == 4 ? v[k] + p1 : 1.0), &fe);
                    prod *= fm;
                    pex += fe;
                    // scipy's pdf underflows to 0 (log -> -inf) below e^-745.13
                    ok = ok && ((ty <= 1) ? (term > PDF_LN_MIN && (ty == 0 || v[k] > 0.0))
                                          : (ty == 4 ? (v[k] > 0.0 && v[k] < p2)
                                                     : (ty <= 3 && v[k] > p1 && v[k] < p2)));
                }
            }
            lp = ok ? lp - fma(double(pex), LN2, log(prod)) : -INFINITY;
        } else if (A.prior_type) {
#pragma unroll
            for (int k = 0; k < PCH; ++k) {
                const int d = d0 + k;
                if (d < A.ndim)
                    lp += prior_lnprob(A.prior_type[d], A.prior_p1[d], A.prior_p2[d], A.prior_norm[d], v[k]);
            }
        }
    }
    if (qo) A.zfout[w] = (A.ndim - 1.0) * log(P.z);
    A.prior[w] = A.fixed_invalid ? -INFINITY : lp;
    LFG_CY(8, w, tl);
#ifdef LFG_PROFILE_SETUP
    if (w < 4096) g_setup_cyc[9][w] = __builtin_amdgcn_s_memrealtime() - trl;
#endif
}

// one lane of k_setup: t < npairs setup lanes, then W prior lanes, then
// npairs stream lanes
template <bool FOLD = false>
__device__ __forceinline__ void setup_any(const SetupArgs& A, int t)
{
    const int npairs = A.W * A.E;
    if (t >= 2 * npairs + A.W) return;
    if (t >= npairs + A.W) {  // stream lanes (own waves: npairs + W is a multiple of 64 in the bench)
        bspot_lane<FOLD>(A, t - npairs - A.W);
        return;
    }
    if (t >= npairs) {
        prior_lane<FOLD>(A, t - npairs);
        return;
    }

    // setup lane: one per (walker, eclipse)
    LFG_T0(tl);
    const int w = t / A.E, e = t - (t / A.E) * A.E;
    const Prop P = make_prop<FOLD>(A, w);
    const int np = npars_of(A, e);
    double p[18];
    bool finite = (np == 14 || np == 18);
#pragma unroll  // p[] stays in registers (a rolled loop kept it in scratch)
    for (int k = 0; k < 18; ++k) {
        p[k] = (k < np) ? gather_par<FOLD>(A, P, gat_at(A, e * 18 + k)) : 0.0;
        finite = finite && isfinite(p[k]);
    }
    if (np == 14) { p[14] = 2.0; p[15] = 1.0; p[16] = 90.0; p[17] = 0.0; }  // MODEL_SPEC 5.3
    double* G = A.geo + size_t(t) * LFG_NGEO;
#ifdef LFG_PROFILE_SETUP
    unsigned long long tf = tl;
    LFG_CY(0, t, tf);
#endif
    // what does not depend on the inclination is formed and stored before
    // findi, so that only q's Roche record and dphi stay live through the
    // solve (this lane also runs, twice, inside k_elements' register budget:
    // lfg_stretch_step_half_spec); the few values needed after it are read
    // back from the record
    {
        const double tilt = p[16] * DEG, psi = (p[10] - 90.0 + p[17]) * DEG;
        double st_, ct_, sp_, cp_, saz, caz;
        sincos(tilt, &st_, &ct_);
        sincos(psi, &sp_, &cp_);
        sincos(p[10] * DEG, &saz, &caz);
        G[G_CAZ] = caz; G[G_SAZ] = saz;
        G[G_NB0] = st_ * cp_; G[G_NB1] = st_ * sp_; G[G_NB2] = ct_;
        G[G_BDEN] = fabs(st_);  // |sin tilt| until the inclination is known
        G[G_ULIMB] = p[7]; G[G_DEXP] = p[12];
        G[G_FIS] = p[11]; G[G_PHI0] = p[13];
        G[G_WDF] = p[0]; G[G_DF] = p[1]; G[G_SF] = p[2]; G[G_RSF] = p[3];
    }
    int st = ST_OK;
    double rprior = 0.0;
    Roche R;
    if (!finite) st = ST_BAD_ARGS;
    else st = roche_init(R, p[4]);
    LFG_CY(1, t, tf);
    bool bad_geo = false;
    if (st == ST_OK) {
        // SimpleEclipse.ln_prior Roche checks not involving the stream (CVModel.py:215-316)
        if (p[6] * R.xl1 > DISC_MAX_A) rprior = -INFINITY;
        const double rwd = p[8], scale = p[9];
        if (scale > rwd * 3.0 || scale < rwd / 3.0) rprior = -INFINITY;
        // geometry (MODEL_SPEC 6), reported after findi's status
        const double rwd_a = p[8] * R.xl1, rdisc_a = p[6] * R.xl1;
        bad_geo = !(rwd_a > 0.0) || !(rdisc_a > rwd_a) || !(rdisc_a < R.xl1) || !(p[9] > 0.0) || !(p[14] > 0.0) ||
                  !(p[15] > 0.0);
        G[G_Q] = R.q; G[G_CA] = R.cA; G[G_CB] = R.cB; G[G_MU] = R.mu;
        G[G_XL1] = R.xl1; G[G_PL1] = R.pl1; G[G_RS] = R.Rs; G[G_RS2] = R.Rs2;
        G[G_RWD] = rwd_a; G[G_RDISC] = rdisc_a; G[G_REFF] = eggleton(R.q);
        G[G_L] = p[9] * R.xl1;
    } else {
        rprior = -INFINITY;
    }
    const double dphi = p[5];
    double inc = 0.0;
    if (st == ST_OK) st = findi_fast(R, dphi, inc);
    LFG_CY(2, t, tf);
    if (st == ST_OK && bad_geo) st = ST_BAD_GEOMETRY;

    A.status[t] = st;
    G[G_RPRIOR] = A.roche_priors ? rprior : 0.0;
    if (st != ST_OK) return;

    double s, c;
    sincos(inc * DEG, &s, &c);
    const double fis = G[G_FIS];
    const double nmax = G[G_BDEN] * s + G[G_NB2] * c;
    G[G_S] = s; G[G_C] = c; G[G_INC] = inc;
    G[G_BDEN] = fis + (1.0 - fis) * fmax(nmax, 0.0);
    const double sce = s * cos(PI * dphi);
    G[G_RCAL] = sqrt(1.0 - sce * sce);
    if (A.gp) {
        // SimpleGPEclipse.create_GP / calcChangepoints (CVModel.py:529-648):
        // amplitudes exp(ln_amp), metric exp(ln_tau); the changepoint
        // distance from the cache unless q, dphi or rwd moved > 120 %.  A
        // walker that trips the rule needs wdphases (ten nested eclipse
        // solves): it is marked pending (G_GP_OK = 2) and k_gp_dcp solves the
        // ten limb points in parallel lanes before k_lnlike<2> (kept out of
        // this lane, whose registers the speculative copies inside
        // k_elements share)
        const int* gg = A.gp_gather + e * 3;
        const double ain = exp(gather_par<FOLD>(A, P, gg[0])), aout = exp(gather_par<FOLD>(A, P, gg[1]));
        const double tau = exp(gather_par<FOLD>(A, P, gg[2]));
        const double* B = A.gp_base + e * 4;
        const double q = R.q, rwd = p[8];
        const bool pend = fabs(B[1] - dphi) / dphi > 1.2 || fabs(B[0] - q) / q > 1.2 || fabs(B[2] - rwd) / rwd > 1.2;
        const bool ok = tau > 0.0 && isfinite(ain) && isfinite(aout);
        G[G_GP_AIN] = ain;
        G[G_GP_AOUT] = aout;
        G[G_GP_LAM] = sqrt(3.0 / tau);
        G[G_GP_DCP] = B[3];
        G[G_GP_DPHI] = dphi;
        G[G_GP_RWD] = rwd;
        G[G_GP_OK] = !ok ? 0.0 : (pend ? 2.0 : (isfinite(B[3]) ? 1.0 : 0.0));
    }
    LFG_CY(3, t, tl);
}

#ifndef LFG_NOLICM_TU  // (lfg_pair_split.hip compiles k_pair only)
__global__ __launch_bounds__(SETUP_BLOCK) void k_setup(SetupArgs A)
{
    setup_any(A, blockIdx.x * SETUP_BLOCK + threadIdx.x);
}
#endif

// ------------------------------------------------------------- k_elements
// One lane per symmetry-unique element.  The WD/disc grids are mirror
// symmetric under y -> -y and the donor grid under y -> -y and z -> -z; the
// Roche potential shares those symmetries, so a mirrored element's eclipse
// interval is [-b, -a] and a mirrored tile's vector has y (and/or z) negated.
// Unique items per (walker, eclipse): WD 200, disc 500, spot 100, donor 100.
// Output: eclipse intervals as (a, b) pairs and the 100 unique donor tile
// vectors; weights depend on ring only and are formed in k_lnlike.
#ifdef LFG_COUNT_ITERS
__device__ unsigned long long g_iter_dbg[64];

#endif
constexpr int U_WD = NWD / 2, U_DISC = NDISC / 2, U_BS = NBS, U_DON = NDONOR / 4;
constexpr int NUNIQ = U_WD + U_DISC + U_BS + U_DON;
// unique-item order: WD, disc, donor, then the spot
constexpr int U_MAIN = U_WD + U_DISC + U_DON;

__device__ __forceinline__ int wd_ring_of(int u)  // ring of unique WD tile u (ring ir starts at 2 ir^2)
{
    int ir = int(sqrt(u * 0.5));
    if (2 * (ir + 1) * (ir + 1) <= u) ++ir;
    if (2 * ir * ir > u) --ir;
    return ir;
}

// element weights (MODEL_SPEC 5.1-5.3): per WD ring, per disc ring, per spot element
__device__ inline double wd_ring_weight(int ir, double ul) { return fma(kWdA[ir], 1.0 - ul, kWdB[ir] * ul); }

// radial integral of r^(1 - dexp) dr over the disc annuli (MODEL_SPEC 5.2):
// the boundary term P(r) = r^ex / ex, or ln r when ex = 2 - dexp vanishes
template <typename GPtr>
__device__ inline double disc_boundary(int i, GPtr G)
{
    const double rin = G[G_RWD];
    const double r = rin + i * ((G[G_RDISC] - rin) / NDISC_R);
    const double ex = 2.0 - G[G_DEXP];
    return (fabs(ex) < 1e-10) ? log(r) : pow(r, ex) / ex;
}

template <typename GPtr>
__device__ inline double disc_ring_weight(int ir, GPtr G)
{
    return (TWO_PI / NDISC_AZ) * (disc_boundary(ir + 1, G) - disc_boundary(ir, G));
}

template <typename GPtr>
__device__ inline double bs_weight(int j, GPtr G)
{
    const double uk = (j + 0.5) * (G[G_UMAX] / NBS);
    return exp(G[G_EXP1] * log(uk) - pow(uk, G[G_EXP2]) - G[G_LNPK]);
}

// A walker whose ln_prior is -inf (a Prior.ln_prob term, the LCModel dphi
// check, or a Roche prior of this eclipse) has ln_prob = -inf whatever its
// likelihood: Node.ln_prob never calls ln_like for it (model.py:476-498).
// Tree calls skip such pairs in k_elements, k_lnlike and k_gp_like alike, so
// that no kernel reads tables the others did not write.  (Stretch proposals
// outside the prior box are common: in a long config-2 chain most of the
// proposals that sent element solves to the nested fallback were of this
// kind, tools/fallback_hunt.py.)
__device__ __forceinline__ bool prior_rejects(double lprior, const double* G)
{
    return !(lprior + G[G_RPRIOR] + G[G_RPRIOR_BS] > -INFINITY);
}

// k_elements' side jobs in lfg_stretch_step_half_spec:
//  - sel: this half's k_setup outputs were formed speculatively inside the
//    previous half's k_elements for both fates of each walker's partner;
//    the pair takes candidate c = accflag[jk[w]] and its first block copies
//    it into the standard workspace slots k_lnlike reads
//  - spec: the leading nspecblk blocks run the k_setup lanes of the next half
//    for both candidates (setup_any on S[0], S[1])
struct ElemSpec {
    const int* jk;  // nullptr: no selection
    const int* accflag;
    const double* geoC;
    const int* statusC;
    const int* bstatusC;
    const double* priorC;
    const double* qC;
    const double* zfC;
    double* prior;
    double* q;
    double* zf;
    int* bstatus;
    int E, ndim;
    const double* lprior;  // tree calls: the batch's Prior sums (k_setup), prior_rejects skips; nullptr: none
    SetupArgs S[2];
    int nspec;     // lanes per candidate (0: no speculative setup)
    int nspecblk;  // leading blocks that run them
};

// where one pair's element results go: the global workspace tables
// (k_elements) or the block's LDS (k_pair)
struct ElemOut {
    double2* abw;  // [NU_WDD] WD/disc intervals, slot uslot(u)
    double2* abs;  // [NBS] spot intervals
    double* don;   // [U_DON][DON_STRIDE] donor tiles
    double* wtd;   // [NDISC_R + 1] disc ring weights, then the disc total
    double* wbs;   // [NBS] spot element weights
};

// the disc ring weights (MODEL_SPEC 5.2) by the lanes of items v = NUNIQ +
// i, i = 0..NDISC_R, consecutive lanes of one wave: lane i holds the boundary
// term P(r_i) and ring i's weight is the difference of neighbours (one pow
// per lane of one wave, instead of two in a ring-start lane of every disc wave)
template <typename GPtr>
__device__ __forceinline__ void ring_weight_lane(int rb, GPtr G, double* __restrict__ wtd)
{
    const double P = disc_boundary(rb, G);
    const int lane = int(threadIdx.x) & 63, l0 = lane - rb;  // lane of P(r_0)
    const double Pn = __shfl(P, min(lane + 1, l0 + NDISC_R), 64);
    const double Pt = __shfl(P, l0 + NDISC_R, 64);
    if (rb < NDISC_R) wtd[rb] = (TWO_PI / NDISC_AZ) * (Pn - P);
    if (rb == 0) wtd[NDISC_R] = TWO_PI * (Pt - P);
}

// results of an item go to a sink: wd_disc(u, a, b), spot(j, a, b, w),
// donor(uu, vx, vy, vz, centre, half-width)
template <typename GPtr, typename Sink>
__device__ __forceinline__ void element_item_to(int v, GPtr G, Sink& K);

// the sink of k_elements (and k_pair's point-major fallback): the tables
struct MemSink {
    const ElemOut& O;
    __device__ __forceinline__ void mark() {}
    __device__ __forceinline__ void wd_disc(int u, double a, double b) { O.abw[uslot(u)] = make_double2(a, b); }
    __device__ __forceinline__ void spot(int j, double a, double b, double w)
    {
        O.abs[j] = make_double2(a, b);
        O.wbs[j] = w;
    }
    __device__ __forceinline__ void donor(int uu, double vx, double vy, double vz, double cen, double hw)
    {
        double* D = O.don + uu * DON_STRIDE;
        D[0] = vx;
        D[1] = vy;
        D[2] = vz;
        D[3] = cen;
        D[4] = hw;
    }
};

template <typename GPtr>
__device__ __forceinline__ void element_item(int v, GPtr G, const ElemOut& O)
{
    MemSink K{O};
    element_item_to(v, G, K);
}

// one k_elements lane's item v of pair `pair` (v >= NUNIQ: the disc ring
// weights of the last chunk's spare lanes)
__device__ __forceinline__ void element_lane(int v, int pair, int npairs, const double* __restrict__ G, int st0, int bst,
                                             int* status, double2* __restrict__ AB, double* __restrict__ DON,
                                             double* __restrict__ WT, const ElemSpec& X)
{
    double* Wp = WT + size_t(pair) * WT_N;
    if (v >= NUNIQ) {  // the last chunk's spare lanes
        const int rb = v - NUNIQ;
        if (rb > NDISC_R || st0 != ST_OK) return;
        ring_weight_lane(rb, G, Wp + WT_DISC);
        return;
    }
    static_assert((NUNIQ % ELEM_BLOCK) + NDISC_R + 1 <= ELEM_BLOCK, "ring-weight lanes fit in the last chunk");
    static_assert(WT_TD == WT_DISC + NDISC_R, "disc total follows the ring weights");
    if (st0 != ST_OK) return;
    if (bst != ST_OK) {
        if (v == 0 && !X.jk) status[pair] = bst;
        return;
    }
    if (X.lprior) {  // the walker's ln_prior is -inf: nothing to evaluate (k_lnlike skips it too)
        const int w = pair / X.E;
        const double lp = X.jk ? X.priorC[size_t(X.accflag[X.jk[w]]) * (npairs / X.E) + w] : X.lprior[w];
        if (prior_rejects(lp, G)) return;
    }
    double2* ABp = AB + size_t(pair) * NELU;
    element_item(v, G, ElemOut{ABp, ABp + NU_WDD, DON + size_t(pair) * U_DON * DON_STRIDE, Wp + WT_DISC, Wp + WT_BS});
}

// item v (v < NUNIQ) of a pair: item order WD, disc, spot, donor; k_elements
// deals the chunks of 64 items out in its own dispatch order (kOrder)
template <typename GPtr, typename Sink>
__device__ __forceinline__ void element_item_to(int v, GPtr G, Sink& K)
{
    constexpr int V_BS = U_WD + U_DISC;
    const int u = (v < V_BS) ? v : (v < V_BS + U_BS ? U_MAIN + (v - V_BS) : v - U_BS);
    const Roche R{G[G_Q], G[G_CA], G[G_CB], G[G_MU], G[G_XL1], G[G_PL1], G[G_RS], G[G_RS2]};
    const double s = G[G_S], c = G[G_C];

    if (u >= U_WD + U_DISC && u < U_MAIN) {  // donor tile (MODEL_SPEC 5.4), phi' in (0, pi/2)
        const int uu = u - (U_WD + U_DISC);
        const int it = uu / (NDONOR_P / 4), ip = uu - it * (NDONOR_P / 4);
        const double stc = kDonSt[it], ctc = kDonCt[it];
        const double dx = -ctc, dy = stc * kDonCp[ip], dz = stc * kDonSp[ip];
        double lo = 0.0, hi = R.Rs, r = G[G_REFF];
        if (!(r > lo && r < hi)) r = 0.5 * hi;
        double gx, gy, gz;
        for (int itr = 0; itr < ROOT_MAXIT; ++itr) {
            const double X0 = fma(r, dx, 1.0), X1 = r * dy, X2 = r * dz;
            const double f = rpot_grad(R, X0, X1, X2, gx, gy, gz) - R.pl1;
            const double df = gx * dx + gy * dy + gz * dz;
            if (f > 0.0) hi = r; else lo = r;
            const double stp = f * rcp_fast(df);  // (an IEEE quotient: ~10 dependent issue slots more a step)
            if (df > 0.0 && fabs(stp) <= ROOT_LAST) { r -= stp; break; }  // last Newton step
            double rn = (df > 0.0) ? r - stp : 0.5 * (lo + hi);
            if (!(rn > lo && rn < hi)) rn = 0.5 * (lo + hi);
            r = rn;
        }
        rgrad(R, fma(r, dx, 1.0), r * dy, r * dz, gx, gy, gz);
        const double ig = rsqrt(gx * gx + gy * gy + gz * gz);
        const double nx = gx * ig, ny = gy * ig, nz = gz * ig;
        const double dA = r * r * kDonOmega[it] / (nx * dx + ny * dy + nz * dz);
        const double vx = dA * nx, vy = dA * ny, vz = dA * nz;
        // visibility arc: v.e = s rho cos(theta + alpha) + c vz > 0 with
        // rho cos(alpha) = vx, rho sin(alpha) = vy  ->  |theta + alpha| < acos(kappa)
        const double srho = s * sqrt(vx * vx + vy * vy);
        const double kap = (srho > 0.0) ? -c * vz / srho : (c * vz > 0.0 ? -2.0 : 2.0);
        const double cen = -atan2(vy, vx) * (1.0 / TWO_PI), hw = acos(fmin(fmax(kap, -1.0), 1.0)) * (1.0 / TWO_PI);
        K.mark();
        K.donor(uu, vx, vy, vz, cen, hw);
        return;
    }

    // the element of unique item u (its mirror's interval is implied)
    double Px, Py, Pz;
    if (u < U_WD) {  // white dwarf tile (MODEL_SPEC 5.1), cos(psi) > 0 half
        const int ir = wd_ring_of(u);
        const double rc = kWdRc[ir], mu0 = kWdMu0[ir];
        const double cp = kWdCos[u], sp = kWdSin[u];
        const double rw = G[G_RWD];
        Px = rw * (-rc * sp * c + mu0 * s);
        Py = rw * (rc * cp);
        Pz = rw * (rc * sp * s + mu0 * c);
    } else if (u < U_WD + U_DISC) {  // disc (MODEL_SPEC 5.2), alpha in (0, pi)
        const int uu = u - U_WD;
        const int ir = uu / (NDISC_AZ / 2), j = uu - ir * (NDISC_AZ / 2);
        const double rin = G[G_RWD];
        const double rc = rin + (ir + 0.5) * ((G[G_RDISC] - rin) / NDISC_R);
        Px = rc * kDiscCos[j];
        Py = rc * kDiscSin[j];
        Pz = 0.0;
    } else {  // bright-spot strip (MODEL_SPEC 5.3): no mirror partner
        const int j = u - U_MAIN;
        const double uk = (j + 0.5) * (G[G_UMAX] / NBS);
        const double off = G[G_L] * (uk - G[G_UPK]);
        Px = fma(off, G[G_CAZ], G[G_BSX]);
        Py = fma(off, G[G_SAZ], G[G_BSY]);
        Pz = 0.0;
    }
    double a, b;
#ifdef LFG_COUNT_ITERS
    // diagnostic build: per region (WD, disc, spot) sums of iterations
    // [cone, ingress, egress], their per-wave maxima, fallbacks, items, eclipsed
    bool fb = false;
    int nit[3] = {0, 0, 0};
    double gs[2] = {0.0, 0.0};
    element_interval_fast(R, Px, Py, Pz, s, c, G[G_RCAL], G[G_REFF], a, b, &fb, nit, gs);
    {
        const int reg = (u < U_WD) ? 0 : (u < U_WD + U_DISC ? 1 : 2);
        unsigned long long* C = g_iter_dbg + reg * 16;
        for (int i = 0; i < 3; ++i) {
            atomicAdd(C + i, (unsigned long long)nit[i]);
            int m = nit[i];
            for (int off = 32; off > 0; off >>= 1) m = max(m, __shfl_xor(m, off, 64));
            if ((threadIdx.x & 63) == 0) atomicAdd(C + 3 + i, (unsigned long long)m);
        }
        if ((threadIdx.x & 63) == 0) atomicAdd(C + 9, 1ull);
        atomicAdd(C + 6, fb ? 1ull : 0ull);
        if (fb) {  // slots 48..63: count, then up to 15 (pair << 16 | item) records
            const unsigned long long k = atomicAdd(g_iter_dbg + 48, 1ull);
            if (k < 15) g_iter_dbg[49 + k] = (static_cast<unsigned long long>(blockIdx.x) << 16) | unsigned(u);
        }
        atomicAdd(C + 7, 1ull);
        atomicAdd(C + 8, (a < b) ? 1ull : 0ull);
        if (a < b && !fb) {  // initial-guess error of the tangency solves: bins < 1e-4, 1e-3, 1e-2, 3e-2, 1e-1, more
            const double er = fmax(fabs(gs[0] - a * TWO_PI), fabs(gs[1] - b * TWO_PI));
            const int bin = er < 1e-4 ? 0 : er < 1e-3 ? 1 : er < 1e-2 ? 2 : er < 3e-2 ? 3 : er < 1e-1 ? 4 : 5;
            atomicAdd(C + 10 + bin, 1ull);
        }
    }
#else
    element_interval_fast(R, Px, Py, Pz, s, c, G[G_RCAL], G[G_REFF], a, b);
#endif
    K.mark();
    if (u >= U_MAIN) K.spot(u - U_MAIN, a, b, bs_weight(u - U_MAIN, G));
    else K.wd_disc(u, a, b);
}

#ifdef LFG_PROFILE_ELEM  // diagnostic build only: per-wave start / end (s_memrealtime, 100 MHz), HW_ID, kind
__device__ unsigned long long g_elem_wav[4][32768];
__device__ __forceinline__ void elem_stamp(unsigned long long t0, int kind)
{
    if ((threadIdx.x & 63) == 0 && blockIdx.x < 32768) {
        unsigned hw;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        g_elem_wav[0][blockIdx.x] = t0;
        g_elem_wav[1][blockIdx.x] = __builtin_amdgcn_s_memrealtime();
        g_elem_wav[2][blockIdx.x] = hw;
        g_elem_wav[3][blockIdx.x] = kind;
    }
}
#endif

#ifndef LFG_NOLICM_TU  // (lfg_pair_split.hip compiles k_pair only)
__global__ __launch_bounds__(ELEM_BLOCK) __attribute__((amdgpu_waves_per_eu(ELEM_MINW))) void k_elements(const double* __restrict__ geo, int* status, int npairs,
                                                         double2* __restrict__ AB, double* __restrict__ DON,
                                                         double* __restrict__ WT, const int* __restrict__ bstatus,
                                                         ElemSpec X)
{
#ifdef LFG_PROFILE_ELEM
    const unsigned long long pt0 = __builtin_amdgcn_s_memrealtime();
#endif
    if (int(blockIdx.x) < X.nspecblk) {  // speculative setup lanes of the next half
        // candidate c's lanes fill blocks [c * nb, (c + 1) * nb): c is uniform
        // in a block, so X.S[c] is selected in scalar registers (a lane-varying
        // c made the compiler keep both SetupArgs in a private array)
        const int nb = (X.nspec + int(blockDim.x) - 1) / int(blockDim.x);
        const int c = int(blockIdx.x) < nb ? 0 : 1;
        const int t = (int(blockIdx.x) - c * nb) * int(blockDim.x) + int(threadIdx.x);
        if (t < X.nspec) setup_any(X.S[__builtin_amdgcn_readfirstlane(c)], t);
#ifdef LFG_PROFILE_ELEM
        elem_stamp(pt0, 0);
#endif
        return;
    }
    const unsigned bid = blockIdx.x - unsigned(X.nspecblk);
    // blocks cover the NUNIQ unique items of every pair in chunks of
    // blockDim.x (the spot items fill the last chunk); block b takes pair
    // b % npairs, so that (with npairs a multiple of 8 and blocks dealt
    // round-robin over the XCDs) a pair's tables are written on the XCD whose
    // L2 k_lnlike block `pair` reads them from -- speed only.  Item 0 folds
    // the stream lanes' status into the pair status (MODEL_SPEC 6 order:
    // setup failures first); every item skips a pair that failed either.
    const int pair = int(bid % unsigned(npairs));
    // LFG_ELEM_IPL items per lane, one after the other (chunks of
    // ELEM_BLOCK * LFG_ELEM_IPL items)
    // chunks in dispatch order: the donor's (latency-bound 1-D roots, few
    // VALU instructions) and the spot's and outer disc's (four Newton steps)
    // first, the WD's and inner disc's (three) last, so that the second
    // round of waves ends on short ones (profiles/r03/elem_timeline_*.txt:
    // the kernel span 27.4 -> 25.2 us at config 2)
    static_assert(ELEM_BLOCK * LFG_ELEM_IPL == 64 && (NUNIQ + NDISC_R + 1 + 63) / 64 == 15, "chunk order table");
    constexpr int kOrder[15] = {13, 14, 12, 11, 10, 9, 8, 7, 6, 5, 4, 3, 2, 1, 0};
    const int ck = kOrder[bid / unsigned(npairs)];
    const int v0 = ck * (int(blockDim.x) * LFG_ELEM_IPL) + int(threadIdx.x);
    const double* G = geo + size_t(pair) * LFG_NGEO;
    int st0, bst;
    if (X.jk) {
        const int w = pair / X.E, e = pair - w * X.E;
        const size_t cp = size_t(X.accflag[X.jk[w]]) * npairs + pair;  // candidate slot of the pair
        G = X.geoC + cp * LFG_NGEO;
        st0 = X.statusC[cp];
        bst = X.bstatusC[cp];
        if (bid < unsigned(npairs)) {  // the pair's first block: the selected candidate into the standard slots
            const int l = int(threadIdx.x);
            double* Gd = const_cast<double*>(geo) + size_t(pair) * LFG_NGEO;
            if (l < LFG_NGEO) Gd[l] = G[l];
            if (l == LFG_NGEO) status[pair] = (st0 != ST_OK) ? st0 : bst;
            if (l == LFG_NGEO + 1) X.bstatus[pair] = bst;
            if (e == 0) {
                const size_t cw = size_t(X.accflag[X.jk[w]]) * (npairs / X.E) + w;
                for (int d = l; d < X.ndim; d += int(blockDim.x)) X.q[size_t(w) * X.ndim + d] = X.qC[cw * X.ndim + d];
                if (l == LFG_NGEO + 2) X.prior[w] = X.priorC[cw];
                if (l == LFG_NGEO + 3) X.zf[w] = X.zfC[cw];
            }
        }
    } else {
        st0 = status[pair];
        bst = bstatus[pair];
    }
#pragma unroll 1
    for (int k = 0; k < LFG_ELEM_IPL; ++k)
        element_lane(v0 + k * int(blockDim.x), pair, npairs, G, st0, bst, status, AB, DON, WT, X);
#ifdef LFG_PROFILE_ELEM
    elem_stamp(pt0, 1 + ck);  // 1 + chunk of the pair's items
#endif
}
#endif

// interval of element k (MODEL_SPEC 5 numbering) from a pair's table: the
// unique item of k's mirror pair, mirrored when k is the partner
__device__ inline double2 elem_ab(const double2* __restrict__ AB, int k)
{
    if (k >= NWD + NDISC) return AB[NU_WDD + (k - NWD - NDISC)];
    int u;
    bool mir;
    if (k < NWD) {  // ring ir holds 4 (2 ir + 1) tiles; j in [0, q4) u [3 q4, nk) are the unique ones
        int ir = int(sqrt(k * 0.25));
        if (4 * (ir + 1) * (ir + 1) <= k) ++ir;
        if (4 * ir * ir > k) --ir;
        const int nk = 4 * (2 * ir + 1), q4 = nk / 4;
        int j = k - 4 * ir * ir;
        mir = j >= q4 && j < 3 * q4;
        if (mir) j = (j < nk / 2) ? nk / 2 - 1 - j : 3 * nk / 2 - 1 - j;
        u = 2 * ir * ir + ((j < q4) ? j : j - 2 * q4);
    } else {
        const int ir = (k - NWD) / NDISC_AZ;
        int j = k - NWD - ir * NDISC_AZ;
        mir = j >= NDISC_AZ / 2;
        if (mir) j = NDISC_AZ - 1 - j;
        u = U_WD + ir * (NDISC_AZ / 2) + j;
    }
    const double2 ab = AB[uslot(u)];
    return mir ? mirror_ab(ab) : ab;
}

// test/inspection only: per-element weights and the full 400-tile donor
#ifndef LFG_NOLICM_TU  // (lfg_pair_split.hip compiles k_pair only)
__global__ void k_expand(const double* __restrict__ geo, const int* __restrict__ status, int npairs,
                         const double2* __restrict__ AB, const double* __restrict__ DON, double* __restrict__ A,
                         double* __restrict__ B, double* __restrict__ WG, double* __restrict__ DFULL)
{
    const long t = long(blockIdx.x) * blockDim.x + threadIdx.x;
    const int pair = int(t / NEL), k = int(t - long(pair) * NEL);
    if (pair >= npairs || status[pair] != ST_OK) return;
    const double* G = geo + size_t(pair) * LFG_NGEO;
    const double2 ab = elem_ab(AB + size_t(pair) * NELU, k);
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
        const double* v = DON + (size_t(pair) * U_DON + k) * DON_STRIDE;
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
#endif

// --------------------------------------------------------------- k_lnlike
// Cross-lane sums and scans by DPP (no LDS round trips; __shfl_xor /
// __shfl_up would also hoist one address VGPR per offset out of every loop
// and keep it live through k_lnlike).
// v of the lane CTRL's DPP pattern names (0 where the source lane is outside
// the row or the row is not in RM): two 32-bit DPP moves, no LDS round trip
template <int CTRL, int RM>
__device__ __forceinline__ long long dpp64(long long v)
{
    if constexpr (RM == 0xf) {
        // every row enabled: bound_ctrl writes the 0 itself where the source
        // lane is outside the row (no v_mov of an "old" 0 per move)
        const int lo = __builtin_amdgcn_mov_dpp(static_cast<int>(v), CTRL, 0xf, 0xf, true);
        const int hi = __builtin_amdgcn_mov_dpp(static_cast<int>(v >> 32), CTRL, 0xf, 0xf, true);
        return (static_cast<long long>(hi) << 32) | static_cast<unsigned>(lo);
    } else {  // disabled rows keep the old value: 0
        const int lo = __builtin_amdgcn_update_dpp(0, static_cast<int>(v), CTRL, RM, 0xf, false);
        const int hi = __builtin_amdgcn_update_dpp(0, static_cast<int>(v >> 32), CTRL, RM, 0xf, false);
        return (static_cast<long long>(hi) << 32) | static_cast<unsigned>(lo);
    }
}

template <int CTRL, int RM>
__device__ __forceinline__ double dppd(double v)
{
    return __longlong_as_double(dpp64<CTRL, RM>(__double_as_longlong(v)));
}

// sum over the wave, the same value in every lane: the DPP inclusive scan
// (row_shr 1, 2, 4, 8, row_bcast:15, row_bcast:31; no LDS round trips, the
// bpermute butterfly waited one per step) and lane 63's total read back
__device__ __forceinline__ double wave_sum(double v)
{
    v += dppd<0x111, 0xf>(v);
    v += dppd<0x112, 0xf>(v);
    v += dppd<0x114, 0xf>(v);
    v += dppd<0x118, 0xf>(v);
    v += dppd<0x142, 0xa>(v);
    v += dppd<0x143, 0xc>(v);
    const long long t = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane(static_cast<int>(t), 63);
    const int hi = __builtin_amdgcn_readlane(static_cast<int>(t >> 32), 63);
    return __longlong_as_double((static_cast<long long>(hi) << 32) | static_cast<unsigned>(lo));
}

struct LikeArgs {
    const double* geo;
    const int* status;
    const double2* AB;
    const double* DON;
    const double* WT;
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
    const int* gp_ecl;  // GP mode: [E][2] first and last changepoint eclipse numbers
    // fused k_combine (MODE 1, 2): ln_prob = ln_prior + sum_e ln_like_e
    const double* prior;  // [W] Prior.ln_prob sums + LCModel prior (k_setup)
    double* lnp;          // nullable, [W]
    bool combine;         // form ln_prob at all
    // fused stretch-move acceptance (lfg_stretch_lnprob_accept; pos nullptr:
    // off): walker w of this batch is the proposal for ensemble walker
    // half * W + w, with W = the batch size = half the ensemble
    double* pos;
    double* lnp_ens;
    const double* qprop;
    const double* zfac;
    int ndim, half;
    unsigned long long seed, step;
    int* naccept;
    double* res;  // MODE 2: [pairs][N] residuals for k_gp_like
    double* gpx;  // MODE 2: [pairs][N] e^{-lam dx} per point (the filter's transitions)
    int* gpb;     // MODE 2: [pairs][N] changepoint block per point
    const int* bstatus;  // fused element phase: the stream lanes' status (folded into status here)
    int* accflag;        // nullable, [W]: 1 where the walker's move was accepted (speculative setup)
};



// ln_prob of walker w once all its eclipses' ln_like are in lle
// (Node.ln_prob, model.py:476-498; what k_combine does), then the
// Metropolis step of the stretch move for it when fused (k_accept's rule)
__device__ inline void combine_walker(const LikeArgs& L, int w)
{
    double lp = L.prior[w];
    for (int e = 0; e < L.E; ++e) {
        const double* G = L.geo + (size_t(w) * L.E + e) * LFG_NGEO;
        lp += G[G_RPRIOR] + G[G_RPRIOR_BS];
    }
    double v;
    if (!isfinite(lp)) {
        for (int e = 0; e < L.E; ++e) L.lle[size_t(w) * L.E + e] = -INFINITY;
        v = -INFINITY;
    } else {
        double ll = 0.0;
        for (int e = 0; e < L.E; ++e) ll += L.lle[size_t(w) * L.E + e];
        v = lp + ll;
    }
    if (L.lnp) L.lnp[w] = v;
    if (L.pos) {
        const int wg = L.half * L.npairs / L.E + w;  // ensemble index (npairs / E = batch walkers)
        const uint4 r = draw(L.seed, L.step, L.half, 1, w);
        const double lu = log(u53(r.x, r.y));
        if (lu < L.zfac[w] + v - L.lnp_ens[wg]) {
            double* p = L.pos + size_t(wg) * L.ndim;
            const double* qi = L.qprop + size_t(w) * L.ndim;
            for (int d = 0; d < L.ndim; ++d) p[d] = qi[d];
            L.lnp_ens[wg] = v;
            if (L.naccept) L.naccept[wg] += 1;
            if (L.accflag) L.accflag[w] = 1;
        } else if (L.accflag) {
            L.accflag[w] = 0;
        }
    }
}

// end of k_lnlike (all threads; lle[pair] written by thread 0): with one
// eclipse per walker and fused acceptance, thread 0 decides with the
// prefetched draw and the copy of the accepted proposal is spread over the
// first ndim lanes; otherwise thread 0 runs combine_after
__device__ inline void finish_walker(const LikeArgs& L, int pair, int tid, bool acc1, const double* sq,
                                     const double* sacc1, int* sflag);

__device__ inline void combine_after(const LikeArgs& L, int pair)
{
    // one eclipse per walker: at once; E > 1: k_combine_walkers does it
    // after the launch (L.combine is false then)
    if (L.combine) combine_walker(L, pair / L.E);
}

// ---- sweeps over phase-sorted tiles of points (MODEL_SPEC 6 restated) ----
// Every eclipse / visibility term is a sum over elements of w_k g_k(p), where
// g_k is non-zero on a contiguous run of points once the points are sorted:
//  * window mode (exposure windows [lo_p, hi_p], lo and hi non-decreasing):
//    element [a, b] overlaps points [P1, P4) and covers [P2, P3) whole, with
//    P1 = #{hi <= a}, P2 = #{lo < a}, P3 = #{hi <= b}, P4 = #{lo < b};
//  * point mode (zero widths, or the donor's visibility arcs): a < ph < b on
//    points [#{ph <= a}, #{ph < b}).
// Whole-covered runs go into a difference array, partly covered points get
// w |[a,b] n [lo,hi]| / (hi - lo) directly.  Sums are 2^-61 fixed point in
// int64 so LDS atomics add them exactly, independent of order.
constexpr int LIKE_THREADS = 512;
constexpr int ACC_LDS = 24;  // proposal coordinates of the fused acceptance kept in LDS (the rest re-read)
#ifndef LIKE_MINW
#define LIKE_MINW 4  // minimum waves per SIMD: two 512-lane blocks per CU (<= 128 VGPRs; LDS < 80 KB)
#endif
constexpr int LIKE_TILE = LIKE_THREADS;  // one point per thread per tile
constexpr int LIKE_NC = 2 * LIKE_TILE;   // cells of the phase index
#ifndef LFG_WALK
#define LFG_WALK 2  // unrolled forward steps of the cell walk before the loop
#endif
constexpr double FX_SCALE = 2305843009213693952.0;  // 2^61
constexpr double FX_INV = 1.0 / FX_SCALE;

struct PhaseIndex {  // sorted phases v[0..m) with a uniform-cell start table
    const double* v;
    const int* cell;
    int m;
    double t0, ginv;
};

__device__ __forceinline__ int cell_of(const PhaseIndex& X, double v)
{
    const double u = (v - X.t0) * X.ginv;
    return u <= 0.0 ? 0 : (u >= double(LIKE_NC) ? LIKE_NC : int(u));
}

// #{v_p < x} (or #{v_p <= x} when LE).  cell[ci(x)] counts the points whose
// cell index is below x's, all of which lie below x (ci is monotone), so the
// walk only goes forward: usually zero or one point, two unrolled steps
template <bool LE>
__device__ __forceinline__ int count_below(const PhaseIndex& X, double x)
{
    int j = X.cell[cell_of(X, x)];
    const int last = X.m - 1;
    bool adv = false;
#pragma unroll
    for (int k = 0; k < LFG_WALK; ++k) {
        const double vj = X.v[min(j, last)];
        adv = (j <= last) & (LE ? (vj <= x) : (vj < x));
        j += adv ? 1 : 0;
    }
    if (adv)  // clustered points: keep walking
        while (j <= last && (LE ? (X.v[j] <= x) : (X.v[j] < x))) ++j;
    return j;
}

// count_below<false> for Q queries in lockstep, so that their LDS chains overlap
template <int Q>
__device__ __forceinline__ void count_lt_multi(const PhaseIndex& X, const double (&x)[Q], int (&j)[Q])
{
    const int last = X.m - 1;
#pragma unroll
    for (int q = 0; q < Q; ++q) j[q] = X.cell[cell_of(X, x[q])];
    bool adv[Q];
#pragma unroll
    for (int k = 0; k < LFG_WALK; ++k) {
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            const double vj = X.v[min(j[q], last)];
            adv[q] = (j[q] <= last) & (vj < x[q]);
            j[q] += adv[q] ? 1 : 0;
        }
    }
#pragma unroll
    for (int q = 0; q < Q; ++q)
        if (adv[q])
            while (j[q] <= last && X.v[j[q]] < x[q]) ++j[q];
}

// count_le_back for Q queries in lockstep
template <int Q>
__device__ __forceinline__ void count_le_back_multi(const double* __restrict__ hi, const double (&x)[Q],
                                                    const int (&J)[Q], int (&out)[Q])
{
    bool back[Q];
#pragma unroll
    for (int q = 0; q < Q; ++q) {
        back[q] = (J[q] > 0) & (hi[max(J[q] - 1, 0)] > x[q]);
        out[q] = J[q] - (back[q] ? 1 : 0);
    }
#pragma unroll
    for (int q = 0; q < Q; ++q)
        if (back[q])
            while (out[q] > 0 && hi[out[q] - 1] > x[q]) --out[q];
}

// #{hi <= x} given J = #{lo < x}: hi > lo, so the answer is <= J; the points
// straddling x (usually one) are stepped over backwards
__device__ __forceinline__ int count_le_back(const double* __restrict__ hi, int J, double x)
{
    const bool back = (J > 0) & (hi[max(J - 1, 0)] > x);
    J -= back ? 1 : 0;
    if (back)
        while (J > 0 && hi[J - 1] > x) --J;
    return J;
}

// cell[g] = #{p : ci(v_p) < g} with ci(v) = floor((v - t0) ginv) clamped to
// [-1, NC] exactly as cell_of computes it: point p fills the cells
// (ci(v_{p-1}), ci(v_p)], the last point also the cells above its own
__device__ __forceinline__ PhaseIndex phase_index(const double* v, const int* cell, int m)
{
    const double span = v[m - 1] - v[0];
    return PhaseIndex{v, cell, m, v[0], span > 0.0 ? LIKE_NC / span : 0.0};
}

__device__ __forceinline__ void build_cells(const double* __restrict__ v, int m, int* __restrict__ cell, int tid)
{
    const PhaseIndex X = phase_index(v, cell, m);
    const double t0 = X.t0, ginv = X.ginv;
    auto ci = [&](double x) {
        const double u = (x - t0) * ginv;
        return u < 0.0 ? -1 : (u >= double(LIKE_NC) ? LIKE_NC : int(u));
    };
    if (tid < m) {
        const int g0 = tid ? ci(v[tid - 1]) : -1, g1 = ci(v[tid]);
        for (int g = g0 + 1; g <= g1; ++g) cell[g] = tid;
        if (tid == m - 1)
            for (int g = g1 + 1; g <= LIKE_NC; ++g) cell[g] = m;
    }
}

__device__ __forceinline__ long long to_fx(double x) { return static_cast<long long>(rint(x * FX_SCALE)); }

__device__ __forceinline__ void fx_add(unsigned long long* acc, int p, long long q)
{
    atomicAdd(acc + p, static_cast<unsigned long long>(q));
}

// the runs of element [a, b] over the tile's windows [lo_p, hi_p] (lo, hi
// sorted, hi >= lo): it overlaps [P1, P4) and covers [P2, P3) whole.  A
// zero-width window is a point: covered when a <= ph <= b, never partial.
struct Runs {
    int P1, P2, P3, P4;
};

__device__ __forceinline__ Runs element_runs(double a, double b, const PhaseIndex& X, const double* __restrict__ hi)
{
    Runs R;
    R.P2 = count_below<false>(X, a);
    R.P4 = count_below<false>(X, b);
    R.P1 = count_le_back(hi, R.P2, a);
    R.P3 = count_le_back(hi, R.P4, b);
    return R;
}

// adds wn * (covered fraction) of element [a, b] given its runs
__device__ __forceinline__ void apply_runs(const Runs& R, double a, double b, double wn, const PhaseIndex& X,
                                           const double* __restrict__ hi, const double* __restrict__ iw,
                                           unsigned long long* acc)
{
    const int P1 = R.P1, P2 = R.P2, P3 = R.P3, P4 = R.P4;
    int e0 = P4, s1 = P4;  // partial runs [P1, e0) and [s1, P4)
    if (P2 < P3) {         // whole-covered run (slot m is never read)
        const long long q = to_fx(wn);
        fx_add(acc, P2, q);
        if (P3 < X.m) fx_add(acc, P3, -q);
        e0 = P2;
        s1 = P3;
    }
    for (int r = 0; r < 2; ++r) {
        const int pe = r ? P4 : e0;
        for (int p = r ? s1 : P1; p < pe; ++p) {
            const double ov = fmin(b, hi[p]) - fmax(a, X.v[p]);
            if (ov > 0.0) {
                const long long q = to_fx(wn * ov * iw[p]);
                fx_add(acc, p, q);
                if (p + 1 < X.m) fx_add(acc, p + 1, -q);
            }
        }
    }
}

// apply_runs for NI intervals of one lane with every LDS read issued before
// the first atomic: a read waits for all the lane's earlier LDS operations
// (one in-order counter), so reads between atomics waited for each atomic's
// round trip.  The first K windows of each partial run are read up front
// (windows that tile the phase axis give one at each end); longer partial
// runs finish one window at a time after the atomics.  The same entries as
// apply_runs: identical integer sums.
template <int NI>
__device__ __forceinline__ void apply_runs_batched(const Runs (&R)[NI], const double (&a)[NI], const double (&b)[NI],
                                                   double wn, const PhaseIndex& X, const double* __restrict__ hi,
                                                   const double* __restrict__ iw, unsigned long long* acc)
{
    constexpr int K = 2;
    const int last = X.m - 1;
    int ps[NI][2], pn[NI][2];
    long long q[NI][2][K];
#pragma unroll
    for (int k = 0; k < NI; ++k) {
        const bool whole = R[k].P2 < R[k].P3;
        const int e0 = whole ? R[k].P2 : R[k].P4, s1 = whole ? R[k].P3 : R[k].P4;
        ps[k][0] = R[k].P1;
        pn[k][0] = e0 - R[k].P1;
        ps[k][1] = s1;
        pn[k][1] = R[k].P4 - s1;
#pragma unroll
        for (int e = 0; e < 2; ++e)
#pragma unroll
            for (int i = 0; i < K; ++i) {
                const int p = min(ps[k][e] + i, last);
                const double ov = fmin(b[k], hi[p]) - fmax(a[k], X.v[p]);
                q[k][e][i] = (i < pn[k][e] && ov > 0.0) ? to_fx(wn * ov * iw[p]) : 0;
            }
    }
    const long long qw = to_fx(wn);
#pragma unroll
    for (int k = 0; k < NI; ++k) {
        if (R[k].P2 < R[k].P3) {
            fx_add(acc, R[k].P2, qw);
            if (R[k].P3 < X.m) fx_add(acc, R[k].P3, -qw);
        }
#pragma unroll
        for (int e = 0; e < 2; ++e)
#pragma unroll
            for (int i = 0; i < K; ++i) {
                const int p = ps[k][e] + i;
                if (q[k][e][i] != 0) {
                    fx_add(acc, p, q[k][e][i]);
                    if (p + 1 < X.m) fx_add(acc, p + 1, -q[k][e][i]);
                }
            }
    }
#pragma unroll
    for (int k = 0; k < NI; ++k)
#pragma unroll
        for (int e = 0; e < 2; ++e)
            for (int p = ps[k][e] + K; p < ps[k][e] + pn[k][e]; ++p) {
                const double ov = fmin(b[k], hi[p]) - fmax(a[k], X.v[p]);
                if (ov > 0.0) {
                    const long long qq = to_fx(wn * ov * iw[p]);
                    fx_add(acc, p, qq);
                    if (p + 1 < X.m) fx_add(acc, p + 1, -qq);
                }
            }
}

// ring of unique WD/disc item u: WD ring r holds 2 r^2 <= u < 2 (r + 1)^2,
// disc rings follow (NDISC_AZ / 2 items each)
__device__ __forceinline__ int uring(int u)
{
    if (u >= U_WD) return NWD_RINGS + (u - U_WD) / (NDISC_AZ / 2);
    int r = int(sqrtf(float(u) * 0.5f));
    r += (2 * (r + 1) * (r + 1) <= u) ? 1 : 0;
    r -= (2 * r * r > u) ? 1 : 0;
    return r;
}

// inclusive wave prefix sum: Hillis-Steele within each row of 16 lanes
// (row_shr 1, 2, 4, 8), then row_bcast:15 into rows 1 and 3 and
// row_bcast:31 into rows 2 and 3 (gfx9 DPP).  Six dependent VALU steps; the
// ds_bpermute form waited an LDS round trip per step.
__device__ __forceinline__ long long wave_scan_incl(long long v, int lane)
{
    (void)lane;
    v += dpp64<0x111, 0xf>(v);
    v += dpp64<0x112, 0xf>(v);
    v += dpp64<0x114, 0xf>(v);
    v += dpp64<0x118, 0xf>(v);
    v += dpp64<0x142, 0xa>(v);
    v += dpp64<0x143, 0xc>(v);
    return v;
}

// the wave's total of v (all 64 lanes active), in every lane
__device__ __forceinline__ long long wave_total(long long v)
{
    v = wave_scan_incl(v, 0);
    const int lo = __builtin_amdgcn_readlane(static_cast<int>(v), 63);
    const int hi = __builtin_amdgcn_readlane(static_cast<int>(v >> 32), 63);
    return (static_cast<long long>(hi) << 32) | static_cast<unsigned>(lo);
}

// inclusive prefix of NA difference arrays at index tid (one entry per thread)
// (ext, nullable: second copies of arrays 0 and 1, summed in; the integer
// sums are exact, so the split changes no bit of the result)
template <int NA>
__device__ __forceinline__ void block_scan(unsigned long long (*acc)[LIKE_TILE + 1], long long (*part)[LIKE_THREADS / 64],
                                           int tid, long long* out,
                                           const unsigned long long (*ext)[LIKE_TILE + 1] = nullptr)
{
    const int lane = tid & 63, wv = tid >> 6;
    constexpr int NW = LIKE_THREADS / 64;
    for (int i = 0; i < NA; ++i) {
        const unsigned long long a = acc[i][tid] + ((ext && i < 2) ? ext[i][tid] : 0ull);
        out[i] = wave_scan_incl(static_cast<long long>(a), lane);
        if (lane == 63) part[i][wv] = out[i];
    }
    __syncthreads();
    // exclusive prefix over the waves, formed by every wave for itself (one
    // barrier, not three): lanes 0..NW-1 read the NW wave totals of an array
    // in one LDS read, a 3-step DPP row scan sums them, and lane wv - 1's
    // inclusive prefix is this wave's offset
    static_assert(NW == 8, "wave totals fit one DPP row");
    for (int i = 0; i < NA; ++i) {
        long long t = (lane < NW) ? part[i][lane] : 0;
        t += dpp64<0x111, 0xf>(t);
        t += dpp64<0x112, 0xf>(t);
        t += dpp64<0x114, 0xf>(t);
        if (wv > 0) {
            const int lo = __builtin_amdgcn_readlane(static_cast<int>(t), wv - 1);
            const int hi = __builtin_amdgcn_readlane(static_cast<int>(t >> 32), wv - 1);
            out[i] += (static_cast<long long>(hi) << 32) | static_cast<unsigned>(lo);
        }
    }
}

__device__ __forceinline__ double wrap_phase(double ph) { return ph - floor(ph + 0.5); }

// sincospi out of line: inlined into the tile loop, its polynomial constants
// are hoisted into ~20 loop-invariant VGPRs
// sin, cos of pi x and of pi y in one call (the sub-bin queries: the line of
// sight at the first sub-bin and its turn per sub-bin)
__device__ __noinline__ double4 sincospi2_ool(double x, double y)
{
    double sx, cx, sy, cy;
    sincospi(x, &sx, &cx);
    sincospi(y, &sy, &cy);
    return make_double4(sx, cx, sy, cy);
}

__device__ __noinline__ double2 sincospi_ool(double x)
{
    double sn, cs;
    sincospi(x, &sn, &cs);
    return make_double2(sn, cs);
}

// tile buffers of one sweep pass: windows [lo, hi] with inverse widths, and
// the sub-bin centre phases (donor), each with its cell index
struct TileBufs {
    double lo[LIKE_TILE], hi[LIKE_TILE], iw[LIKE_TILE];
    int cell[LIKE_NC + 1];
};

// writes this thread's window; returns 4 for an invalid width (check_sorted
// returns 4 for an out-of-order window): either sends the tile to the direct path
__device__ __forceinline__ int put_window(TileBufs& T, int tid, bool own, double ph, double hw)
{
    if (!own) return 0;
    T.lo[tid] = ph - hw;
    T.hi[tid] = ph + hw;
    T.iw[tid] = 1.0 / (2.0 * hw);
    return (hw >= 0.0) ? 0 : 4;  // negative or NaN widths take the direct path
}

__device__ __forceinline__ int check_sorted(const TileBufs& T, int tid, bool own)
{
    return (own && tid && (T.lo[tid] < T.lo[tid - 1] || T.hi[tid] < T.hi[tid - 1])) ? 4 : 0;
}

// spot element (lane < NBS) and donor tile (last NDONOR lanes) contributions
// of one sub-bin pass into acc[0] (spot eclipse) and acc[1..3] (donor sum v)
__device__ __forceinline__ void sweep_spot_donor(int tid, const PhaseIndex& XW, const TileBufs& TW,
                                                 const PhaseIndex& XP, const double2* sab, const double* sbw,
                                                 double itb, const double* sdq, double ivs,
                                                 unsigned long long (*acc)[LIKE_TILE + 1])
{
    if (tid < NBS) {
        const double2 abB = sab[tid];
        const double wB = sbw[tid] * itb;
        if (abB.x < abB.y) apply_runs(element_runs(abB.x, abB.y, XW, TW.hi), abB.x, abB.y, wB, XW, TW.hi, TW.iw, acc[0]);
    } else if (tid >= LIKE_THREADS - NDONOR) {
        const int mr = (tid - (LIKE_THREADS - NDONOR)) & 3;
        const double* dq = sdq + ((tid - (LIKE_THREADS - NDONOR)) >> 2) * DON_STRIDE;
        const double vx = dq[0], vy = (mr & 1) ? -dq[1] : dq[1], vz = (mr & 2) ? -dq[2] : dq[2];
        const double cen = (mr & 1) ? -dq[3] : dq[3];
        const double hw = (mr & 2) ? 0.5 - dq[4] : dq[4];
        if (hw > 0.0) {
            const long long qx = to_fx(vx * ivs), qy = to_fx(vy * ivs), qz = to_fx(vz * ivs);
            // visible for phases in (cen - hw, cen + hw) mod 1
            double x1 = -INFINITY, x2 = INFINITY, y1 = 0.0, y2 = 0.0;
            bool two = false;
            if (hw < 0.5) {
                const double lo = cen - hw, hi = cen + hw;
                if (lo < -0.5) { x2 = hi; y1 = lo + 1.0; y2 = INFINITY; two = true; }
                else if (hi > 0.5) { x1 = lo; y1 = -INFINITY; y2 = hi - 1.0; two = true; }
                else { x1 = lo; x2 = hi; }
            }
            for (int i = 0; i < (two ? 2 : 1); ++i) {
                const int P = count_below<true>(XP, i ? y1 : x1), Q = count_below<false>(XP, i ? y2 : x2);
                if (P < Q) {
                    fx_add(acc[1], P, qx);
                    fx_add(acc[2], P, qy);
                    fx_add(acc[3], P, qz);
                    if (Q < XP.m) {
                        fx_add(acc[1], Q, -qx);
                        fx_add(acc[2], Q, -qy);
                        fx_add(acc[3], Q, -qz);
                    }
                }
            }
        }
    }
}

// direct (point-major) WD and disc eclipse fractions of one window: the
// fallback for unsorted or mixed windows.  Inlined: k_lnlike takes it as a
// whole pass of its own, where little is live (an out-of-line call anywhere
// in the kernel spilled ~14 live values to scratch in every block)
__device__ __forceinline__ double2 direct_wd_disc(const double2* __restrict__ AB, const double* __restrict__ swr,
                                               double phc, double wk, double twd, double td)
{
    double ewd = 0.0, ed = 0.0;
    const double lo = phc - wk, hi = phc + wk;
    auto cover = [&](double2 ab) {
        return (wk > 0.0) ? fmax(fmin(ab.y, hi) - fmax(ab.x, lo), 0.0) : ((phc > ab.x && phc < ab.y) ? 1.0 : 0.0);
    };
    for (int ring = 0; ring < NWD_RINGS + NDISC_R; ++ring) {  // each unique item and its mirror
        const int u0 = ring < NWD_RINGS ? 2 * ring * ring : U_WD + (ring - NWD_RINGS) * (NDISC_AZ / 2);
        const int u1 = ring < NWD_RINGS ? 2 * (ring + 1) * (ring + 1) : u0 + NDISC_AZ / 2;
        double acc = 0.0;
        for (int u = u0; u < u1; ++u) {
            const double2 ab = AB[uslot(u)];
            acc += cover(ab) + cover(mirror_ab(ab));
        }
        if (ring < NWD_RINGS) ewd = fma(swr[ring], acc, ewd); else ed = fma(swr[ring], acc, ed);
    }
    const double nrm = (wk > 0.0) ? 1.0 / (2.0 * wk) : 1.0;
    return make_double2(ewd * nrm * (1.0 / twd), ed * nrm * (1.0 / td));
}

// direct (point-major) spot eclipse fraction of one window
__device__ __forceinline__ double direct_spot(const double2* ABs, const double* sbw, double ph, double h, double itb)
{
    double eb = 0.0;
    const double l2 = ph - h, h2 = ph + h;
    for (int k = 0; k < NBS; ++k) {
        const double2 ab = ABs[k];
        eb = fma(sbw[k], (h > 0.0) ? fmax(fmin(ab.y, h2) - fmax(ab.x, l2), 0.0)
                                   : ((ph > ab.x && ph < ab.y) ? 1.0 : 0.0), eb);
    }
    return eb * ((h > 0.0) ? 1.0 / (2.0 * h) : 1.0) * itb;
}

// direct donor sum for one line of sight e = (e0, e1, c)
__device__ __forceinline__ double direct_donor(const double* DONp, double e0, double e1, double c)
{
    double D = 0.0;
    for (int q = 0; q < U_DON; ++q) {
        // max(A + Y, 0) + max(A - Y, 0) = max(A + max(Y, A), 0), A = vx e0 +- vz c
        const double* d5 = DONp + q * DON_STRIDE;
        const double y = fabs(d5[1] * e1), z = d5[2] * c;
        const double A1 = fma(d5[0], e0, z), A2 = fma(d5[0], e0, -z);
        D += fmax(A1 + fmax(y, A1), 0.0) + fmax(A2 + fmax(y, A2), 0.0);
    }
    return D;
}



// ---- S > 1: the spot and donor from per-pair breakpoint tables ----
// With sub-bins the spot's eclipse and the donor's visibility are needed at
// N S sub-phases.  Instead of one sweep (every spot element and donor tile
// located in the pass's windows, a block scan) per tile and sub-bin, the
// pair's breakpoints are bucketed once into TCELLS uniform cells (counting
// sort in LDS) with int64 fixed-point prefix sums per cell, and every
// sub-bin is a lookup: the prefix of its cell plus the few entries of the
// cell (MODEL_SPEC 3, 5.3-5.4 restated; the sums are exact integers, so
// entry order inside a cell does not matter).
//  * donor (point mode at the sub-bin centre th): V(th) = sum of the tile
//    vectors visible at th; tile arc (cen - hw, cen + hw) mod 1: +q at its
//    start (counted for th > start), -q at its end (counted for th >= end);
//    arcs wrapping past +-1/2 and always-visible tiles go into V0, and
//    breakpoints outside the cells' range [t0, t1] are folded into V0 or dropped;
//  * spot (window [lo, hi]): E = C(lo) + [sum over elements with a
//    breakpoint inside (lo, hi) of the partial overlaps] / (hi - lo), with
//    C(x) = the weight of the elements covering x (a_k <= x < b_k): +W_k at
//    a_k, -W_k at b_k, both counted for x >= pos.  Zero-width windows: the
//    elements with a_k < ph < b_k.
constexpr int TCELLS = 256;
constexpr int TD_MAX = 2 * NDONOR, TS_MAX = 2 * NBS;
struct SubTables {
    long long dpre[TCELLS][3];   // donor: V at each cell's start (V0 + cells below), fixed point
    long long spre[TCELLS];      // spot: covering weight at each cell's start
    int dend[TCELLS], send[TCELLS];  // entry counts -> exclusive offsets -> (after the scatter) cell ends
    double spos[TS_MAX];
    int scode[TS_MAX];           // element k: 2 k + (1: end b_k)
    long long dv0[3];
    double dt0, dginv, st0, sginv;
};
struct SubEntries {              // donor entries (in sacc rows 2..5: free when S > 1)
    double dpos[TD_MAX];
    int dcode[TD_MAX];           // tile t (0..399 as the donor lanes number them): 2 t + (1: end)
};
static_assert(sizeof(SubEntries) <= 4 * (LIKE_TILE + 1) * sizeof(unsigned long long), "donor entries fit sacc[2..5]");

__device__ __forceinline__ int tcell(double x, double t0, double ginv)
{
    const double u = (x - t0) * ginv;
    return u <= 0.0 ? 0 : (u >= double(TCELLS - 1) ? TCELLS - 1 : int(u));
}

// donor tile t's fixed-point vector (mirror image t & 3 of unique tile t >> 2),
// exactly as its lane forms it
__device__ __forceinline__ void donor_q(const double* sdq, int t, double ivs, long long& qx, long long& qy, long long& qz)
{
    const int mr = t & 3;
    const double* dq = sdq + (t >> 2) * DON_STRIDE;
    qx = to_fx(dq[0] * ivs);
    qy = to_fx(((mr & 1) ? -dq[1] : dq[1]) * ivs);
    qz = to_fx(((mr & 2) ? -dq[2] : dq[2]) * ivs);
}

// wave-wide min / max, every lane: DPP row shifts as wave_sum does, with each
// lane's own value standing in where the source lane is absent (the
// min / max identity), then lane 63's result
template <bool MAX>
__device__ __forceinline__ double wave_ext(double v)
{
    auto step = [&](auto ctrl_tag, auto rm_tag) {
        constexpr int CTRL = decltype(ctrl_tag)::value, RM = decltype(rm_tag)::value;
        const long long b = __double_as_longlong(v);
        const int lo = __builtin_amdgcn_update_dpp(static_cast<int>(b), static_cast<int>(b), CTRL, RM, 0xf, false);
        const int hi = __builtin_amdgcn_update_dpp(static_cast<int>(b >> 32), static_cast<int>(b >> 32), CTRL, RM, 0xf,
                                                   false);
        const double o = __longlong_as_double((static_cast<long long>(hi) << 32) | static_cast<unsigned>(lo));
        v = MAX ? fmax(v, o) : fmin(v, o);
    };
    using I = std::integral_constant<int, 0>;
    (void)sizeof(I);
    step(std::integral_constant<int, 0x111>{}, std::integral_constant<int, 0xf>{});
    step(std::integral_constant<int, 0x112>{}, std::integral_constant<int, 0xf>{});
    step(std::integral_constant<int, 0x114>{}, std::integral_constant<int, 0xf>{});
    step(std::integral_constant<int, 0x118>{}, std::integral_constant<int, 0xf>{});
    step(std::integral_constant<int, 0x142>{}, std::integral_constant<int, 0xa>{});
    step(std::integral_constant<int, 0x143>{}, std::integral_constant<int, 0xc>{});
    const long long t = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane(static_cast<int>(t), 63);
    const int hi = __builtin_amdgcn_readlane(static_cast<int>(t >> 32), 63);
    return __longlong_as_double((static_cast<long long>(hi) << 32) | static_cast<unsigned>(lo));
}
// OR of the low four bits of v over the wave (four ballots)
__device__ __forceinline__ int wave_or4(int v)
{
    return (__ballot(v & 1) ? 1 : 0) | (__ballot(v & 2) ? 2 : 0) | (__ballot(v & 4) ? 4 : 0) | (__ballot(v & 8) ? 8 : 0);
}
__device__ __forceinline__ double wave_min(double v) { return wave_ext<false>(v); }
__device__ __forceinline__ double wave_max(double v) { return wave_ext<true>(v); }

// exclusive prefix over TCELLS cells of NA int64 arrays held one cell per
// thread (threads >= TCELLS pass zeros); totals of each wave through part[]
template <int NA>
__device__ __forceinline__ void cell_scan(long long (&v)[NA], long long (*part)[LIKE_THREADS / 64], int tid)
{
    const int lane = tid & 63, wv = tid >> 6;
    long long incl[NA];
#pragma unroll
    for (int i = 0; i < NA; ++i) {
        incl[i] = wave_scan_incl(v[i], lane);
        if (lane == 63) part[i][wv] = incl[i];
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < NA; ++i) {
        long long off = 0;
        for (int k = 0; k < wv; ++k) off += part[i][k];
        v[i] = incl[i] - v[i] + off;
    }
}

// spot eclipse fraction of window [lo, hi] (h = (hi - lo) / 2; h = 0: point ph = lo)
__device__ __forceinline__ double sub_spot(const SubTables& T, const double2* sab, const double* sbw, double itb,
                                           double lo, double hi, double amin, double bmax)
{
    const bool pt = !(hi > lo);
    if (pt ? !(lo > amin && lo < bmax) : !(hi > amin && lo < bmax)) return 0.0;
    const int g0 = tcell(lo, T.st0, T.sginv), g1 = pt ? g0 : tcell(hi, T.st0, T.sginv);
    long long C = T.spre[g0];
    double corr = 0.0;
    for (int g = g0; g <= g1; ++g) {
        for (int i = g ? T.send[g - 1] : 0; i < T.send[g]; ++i) {
            const double pos = T.spos[i];
            const int code = T.scode[i], k = code >> 1;
            const bool end = code & 1;
            if (g == g0 && pos <= lo) {
                const long long W = to_fx(sbw[k] * itb);
                // point mode: eclipsed when a_k < ph < b_k (MODEL_SPEC 5; the oracle's rule)
                C += end ? -W : ((pt && pos == lo) ? 0 : W);
            } else if (!pt && pos < hi) {
                const double2 ab = sab[k];
                const double wn = sbw[k] * itb;
                if (!end) corr = fma(wn, fmin(ab.y, hi) - ab.x, corr);
                else if (ab.x <= lo) corr = fma(-wn, hi - ab.y, corr);
            }
        }
    }
    const double e = double(C) * FX_INV;
    return pt ? e : fma(corr, 1.0 / (hi - lo), e);
}

// covering weight C(lo) of the spot (fixed point) from the cell table, and
// the cursor: the first entry (cells sorted by position) past lo
__device__ __forceinline__ long long spot_C(const SubTables& T, const double* sbw, double itb, double lo, int& cur)
{
    const int g = tcell(lo, T.st0, T.sginv);
    long long C = T.spre[g];
    int i = g ? T.send[g - 1] : 0;
    for (const int ie = T.send[g]; i < ie && T.spos[i] <= lo; ++i) {
        const int code = T.scode[i];
        const long long W = to_fx(sbw[code >> 1] * itb);
        C += (code & 1) ? -W : W;
    }
    cur = i;
    return C;
}

// donor entries sorted (after step (e) of the table build) by position,
// an end before a start at equal positions: the entries counted at phase th
// (starts with pos < th, ends with pos <= th) are then a prefix of the list,
// and a lane walking up in phase keeps a cursor into it
__device__ __forceinline__ bool donor_counted(double pos, int code, double th)
{
    return (code & 1) ? pos <= th : pos < th;
}

__device__ __forceinline__ void donor_apply(const double* sdq, int code, double ivs, long long& vx, long long& vy,
                                            long long& vz)
{
    long long qx, qy, qz;
    donor_q(sdq, code >> 1, ivs, qx, qy, qz);
    if (code & 1) { vx -= qx; vy -= qy; vz -= qz; }
    else { vx += qx; vy += qy; vz += qz; }
}

// donor sum vector V (fixed point) at phase th, and the cursor: the first
// entry not counted at th
__device__ __forceinline__ int sub_donor(const SubTables& T, const SubEntries& D, const double* sdq, double ivs,
                                         double th, long long& vx, long long& vy, long long& vz)
{
    const int g = tcell(th, T.dt0, T.dginv);
    vx = T.dpre[g][0];
    vy = T.dpre[g][1];
    vz = T.dpre[g][2];
    int i = g ? T.dend[g - 1] : 0;
    for (const int ie = T.dend[g]; i < ie; ++i) {
        const int code = D.dcode[i];
        if (!donor_counted(D.dpos[i], code, th)) break;
        donor_apply(sdq, code, ivs, vx, vy, vz);
    }
    return i;
}


// this lane's breakpoints of the S > 1 tables (<= 2): donor tile t (lanes
// nt - NDONOR ..) or spot element (lanes < NBS); formed twice (count, then
// scatter) instead of held across the barriers between.  v0: how many times
// the tile's vector goes into V0 (+-1, 0)
__device__ __forceinline__ void lane_breakpoints(int tid, const double* sdq, const double2* sab, double t0d, double t1d,
                                                 double& p0, double& p1, bool& in0, bool& in1, int& v0)
{
    // slot 0: the start (code 2 x), slot 1: the end (code 2 x + 1); fixed
    // slots (a compacted pair indexed by a count went to scratch)
    in0 = in1 = false;
    p0 = p1 = 0.0;
    v0 = 0;
    if (tid >= LIKE_THREADS - NDONOR) {
        const int t = tid - (LIKE_THREADS - NDONOR), mr = t & 3;
        const double* dq5 = sdq + (t >> 2) * DON_STRIDE;
        const double cen = (mr & 1) ? -dq5[3] : dq5[3];
        const double hw = (mr & 2) ? 0.5 - dq5[4] : dq5[4];
        if (!(hw > 0.0)) return;
        double sp = NAN, ep = NAN;  // start (counted for th > sp), end (counted for th >= ep)
        if (hw >= 0.5) {
            v0 = 1;
        } else {
            const double lo = cen - hw, hi = cen + hw;
            if (lo < -0.5) { v0 = 1; ep = hi; sp = lo + 1.0; }
            else if (hi > 0.5) { v0 = 1; ep = hi - 1.0; sp = lo; }
            else { sp = lo; ep = hi; }
        }
        if (sp == sp) {  // a start below the range counts for every phase; at or above t1 for none
            if (sp < t0d) v0 += 1;
            else if (sp < t1d) { p0 = sp; in0 = true; }
        }
        if (ep == ep) {
            if (ep <= t0d) v0 -= 1;
            else if (ep <= t1d) { p1 = ep; in1 = true; }
        }
    } else if (tid < NBS) {
        const double2 ab = sab[tid];
        if (ab.x < ab.y) {
            p0 = ab.x;
            p1 = ab.y;
            in0 = in1 = true;
        }
    }
}


// S > 1: the spot and donor terms of one point, summed over its S sub-bins
// (spot eclipse over each sub-bin window, donor at each sub-bin centre, from
// the tables).  The donor vector is looked up at the first sub-bin and
// carried forward by the sorted-entry cursor (the next entry's position in
// registers: usually one compare per sub-bin), and the line of sight is
// rotated from sub-bin to sub-bin (one sincospi per point); a sub-bin past
// +-1/2 starts over.  The beaming denominator and the donor normalisation
// divide the point's sums once.
__device__ __forceinline__ double2 sub_point(const SubTables& T, const SubEntries& D, const double2* sab, const double* sbw,
                                             const double* sdq, const double* snorm, const double* shull, const double* SG,
                                             double ph0, double wk, int S)
{
    // the pair's constants are read from LDS at each use (volatile: held in
    // registers over the loop they pushed k_lnlike past its budget)
    // (LDS address space spelled out: through volatile generic pointers the
    // reads were flat loads, which wait on the vector-memory counter too)
    using lds_cvd = const volatile __attribute__((address_space(3))) double*;
    const lds_cvd VG = (lds_cvd)SG;
    const lds_cvd VN = (lds_cvd)snorm;
    const int nd = T.dend[TCELLS - 1], nsp = T.send[TCELLS - 1];
    const double h = wk / S, ih = 0.5 / h;
    double sbs = 0.0, srs = 0.0, ph = 0.0, sn = 0.0, cs = 1.0, rs = 0.0, rc = 1.0;
    double fx = 0.0, fy = 0.0, fz = 0.0, npos = INFINITY;
    long long vx = 0, vy = 0, vz = 0, Cs = 0;
    int cur = 0, ncode = 0, scur = 0;
    bool sv = false;  // Cs / scur hold C at this sub-bin's lo
    for (int j = 0; j < S; ++j) {
        const double phn = wrap_phase(ph0 - wk + (2 * j + 1) * h);
        bool chg = false;
        if (j == 0 || !(phn >= ph)) {  // a fresh lookup
            sv = false;
#ifdef LFG_ABL_FRESH  // diagnostic ablation: no donor table lookup
            cur = nd;
#else
            cur = sub_donor(T, D, sdq, VN[1], phn, vx, vy, vz);
#endif
            chg = true;
            const double4 e4 = sincospi2_ool(2.0 * phn, 4.0 * h);  // the turn per sub-bin: 2 pi (2 h)
            sn = e4.x;
            cs = e4.y;
            rs = e4.z;
            rc = e4.w;
        } else {
            while (donor_counted(npos, ncode, phn)) {  // npos = inf past the last entry
                donor_apply(sdq, ncode, VN[1], vx, vy, vz);
                chg = true;
                ++cur;
                npos = cur < nd ? D.dpos[cur] : INFINITY;
                ncode = cur < nd ? D.dcode[cur] : 0;
            }
            const double c2 = fma(cs, rc, -sn * rs);
            sn = fma(sn, rc, cs * rs);
            cs = c2;
        }
        if (chg) {
            if (j == 0 || !(phn >= ph)) {
                npos = cur < nd ? D.dpos[cur] : INFINITY;
                ncode = cur < nd ? D.dcode[cur] : 0;
            }
            fx = double(vx);
            fy = double(vy);
            fz = double(vz);
        }
        ph = phn;
        // spot: windows of a point abut, so C(lo) is carried from window to
        // window by a cursor over the position-sorted entries (the entries
        // inside a window give its partial overlaps); zero widths: points
        double ebj = 0.0;
        const double lo = ph - h, hi = ph + h;
#ifdef LFG_ABL_SPOT  // diagnostic ablation: no spot eclipse
        if (false) {
#else
        if (!(h > 0.0)) {
#endif
            ebj = sub_spot(T, sab, sbw, VN[0], lo, hi, shull[2], shull[3]);
        } else if (hi > shull[2] && lo < shull[3]) {
            const double itb = VN[0];
            if (!sv) Cs = spot_C(T, sbw, itb, lo, scur);
            sv = true;
            long long Cn = Cs;
            double corr = 0.0;
            for (; scur < nsp && T.spos[scur] <= hi; ++scur) {
                const int code = T.scode[scur], k = code >> 1;
                const double wn = sbw[k] * itb;
                const double2 ab = sab[k];
                const long long W = to_fx(wn);
                if (!(code & 1)) {
                    Cn += W;
                    corr = fma(wn, fmin(ab.y, hi) - ab.x, corr);
                } else {
                    Cn -= W;
                    if (ab.x <= lo) corr = fma(-wn, hi - ab.y, corr);
                }
            }
            ebj = fma(corr, ih, double(Cs) * FX_INV);
            Cs = Cn;
        } else {
            sv = false;
        }
        const double sg = VG[G_S], cg = VG[G_C];
        const double e0 = sg * cs, e1 = -sg * sn;
        srs = fma(e0, fx, fma(e1, fy, fma(cg, fz, srs)));
        const double fis = VG[G_FIS];
        sbs = fma(fis + (1.0 - fis) * fmax(VG[G_NB0] * e0 + VG[G_NB1] * e1 + VG[G_NB2] * cg, 0.0), 1.0 - ebj, sbs);
    }
    const double bden = VG[G_BDEN];
    return make_double2(bden > 0.0 ? sbs / bden : 0.0, srs * (FX_INV * VN[3]) / VN[2]);
}

#ifdef LFG_PROFILE_LIKE  // diagnostic build only: phase stamps (first tile) into spare geo slots 41..46
// (thread 0), and the earliest / latest wave of each block per phase (g_like_wav)
__device__ unsigned long long g_like_wav[2][6][4096];
#ifdef LFG_PROFILE_LIKE_WAVES  // per-wave stamps (global atomics: they perturb the timing)
constexpr bool LIKE_WAVES = true;
#else
constexpr bool LIKE_WAVES = false;
#endif
#define LIKE_STAMP(i)                                                                                       \
    if (t0 == 0) {                                                                                          \
        const unsigned long long now_ = __builtin_amdgcn_s_memtime() - tstart;                             \
        if (tid == 0) const_cast<double*>(G)[41 + (i)] = double(now_);                                       \
        if (LIKE_WAVES && lane == 0 && blockIdx.x < 4096) {                                                  \
            atomicMin(&g_like_wav[0][i][blockIdx.x], now_);                                                  \
            atomicMax(&g_like_wav[1][i][blockIdx.x], now_);                                                  \
        }                                                                                                   \
    }
// prologue stamps of thread 0 (and of the block's last lane) per block: lfg_debug_like_cycles
__device__ unsigned long long g_like_cyc[8][4096];
#define LIKE_PRO(k)                                                                                 \
    if ((tid == 0 || tid == LIKE_THREADS - 1) && blockIdx.x < 4096)                                  \
        g_like_cyc[(k) + (tid ? 4 : 0)][blockIdx.x] = __builtin_amdgcn_s_memtime() - tstart
#else
#define LIKE_STAMP(i)
#define LIKE_PRO(k)
#endif

__device__ inline void finish_walker(const LikeArgs& L, int pair, int tid, bool acc1, const double* sq,
                                     const double* sacc1, int* sflag)
{
    if (!acc1) {
        if (tid == 0) combine_after(L, pair);
        return;
    }
    __syncthreads();  // sflag is free; lle[pair] is this block's own write
    const int wg = L.half * L.npairs + pair;
    if (tid == 0) {
        const double* G = L.geo + size_t(pair) * LFG_NGEO;
        const double lp = L.prior[pair] + G[G_RPRIOR] + G[G_RPRIOR_BS];
        double v;
        if (!isfinite(lp)) {
            L.lle[pair] = -INFINITY;
            v = -INFINITY;
        } else {
            v = lp + L.lle[pair];
        }
        if (L.lnp) L.lnp[pair] = v;
        const bool a = sacc1[0] < sacc1[1] + v - sacc1[2];
        if (a) {
            L.lnp_ens[wg] = v;
            if (L.naccept) L.naccept[wg] += 1;
        }
        sflag[0] = a ? 1 : 0;
        if (L.accflag) L.accflag[pair] = a ? 1 : 0;
    }
    __syncthreads();
    if (sflag[0] && tid < L.ndim)
        L.pos[size_t(wg) * L.ndim + tid] = (tid < ACC_LDS) ? sq[tid] : L.qprop[size_t(pair) * L.ndim + tid];
}

// MODE 0: flux (and components) only; 1: fused chi^2 -> ln_like; 2: GP
// ln_like of the residuals (a Kalman filter over each tile's sorted points,
// run by wave 0 while the other waves wait at the tile barrier)
// SUB: nsub > 1 (the table path for the spot and donor, MODE as above); the
// host launches SUB = (nsub > 1), so each instantiation holds only its path
template <int MODE, bool SUB>
__global__ __launch_bounds__(LIKE_THREADS, LIKE_MINW) void k_lnlike(LikeArgs L)
{
    constexpr bool CHI = MODE != 0, GP = MODE == 2;
#ifdef LFG_PROFILE_LIKE
    const unsigned long long tstart = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) {  // block start (100 MHz wall clock) and the CU it runs on
        const_cast<double*>(L.geo)[size_t(blockIdx.x) * LFG_NGEO + 47] = double(__builtin_amdgcn_s_memrealtime());
        unsigned hw;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        const_cast<double*>(L.geo)[size_t(blockIdx.x) * LFG_NGEO + 40] = double(hw);
    }
#endif
    __shared__ double swr[NWD_RINGS + NDISC_R];
    __shared__ double swn[NWD_RINGS + NDISC_R];  // ring weights / component totals (the sweep's wn)
    __shared__ double sbw[NBS];
    __shared__ double2 sab[NBS];                  // spot intervals
    __shared__ double sdq[U_DON * DON_STRIDE];    // unique donor tiles
    __shared__ double sacc1[3];                   // fused acceptance: ln u, zfac, old ln_prob
    __shared__ double snorm[4];                   // 1 / spot total, 1 / donor |v| sum, donor norm, |v| sum
    __shared__ double sgeo[LFG_NGEO];             // the pair's geometry record, read at use in the tile loop
    // TA: WD/disc windows.  S = 1: the spot sweep reuses TA's windows, and
    // SU.s1.X holds second copies of the WD and disc difference arrays, taken
    // by the odd lanes of the sweep (half the same-address LDS atomics where
    // contacts cluster; four WD copies measured no faster), sph / scp the
    // donor's phases and their cells.  S > 1: SU.tb, the pair's breakpoint
    // tables (spot and donor), with the donor entries in sacc rows 2..5.
    __shared__ TileBufs TA;
    __shared__ union SubU_ {
        struct {
            unsigned long long X[2][LIKE_TILE + 1];
            double sph[LIKE_TILE];  // point phases (donor)
            int scp[LIKE_NC + 1];
        } s1;
        SubTables tb;
    } SU;
    double* const sph = SU.s1.sph;
    int* const scp = SU.s1.scp;
    __shared__ double shull[4];  // WD/disc and spot element hulls: min a, max b (eclipsed elements)
    __shared__ double shw[4][LIKE_THREADS / 64];  // their wave partials
    __shared__ double sqr[2][LIKE_THREADS / 64];  // S > 1: wave partials of the sub-bin phase range
    __shared__ unsigned long long sacc[6][LIKE_TILE + 1];
    __shared__ long long spart[6][LIKE_THREADS / 64];
    __shared__ double red[3][LIKE_THREADS / 64];
    __shared__ int sflag[2];

    constexpr int nt = LIKE_THREADS, nw = LIKE_THREADS / 64;
    const int pair = blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int e = (L.E == 1) ? 0 : pair % L.E;  // (one eclipse: no division constants held)
    // one eclipse: off = {0, max_n} (lfg.h), so the point loads need not
    // wait on a load of the offsets (one memory round trip of the prologue)
    const bool offs = L.off && L.E > 1;
    const int o0 = offs ? L.off[e] : 0;
    const int n = offs ? L.off[e + 1] - o0 : L.N;
    const double* G = L.geo + size_t(pair) * LFG_NGEO;
    const double* Wt = L.WT + size_t(pair) * WT_N;
    const double2* AB = L.AB + size_t(pair) * NELU;
    const double* DONp = L.DON + size_t(pair) * U_DON * DON_STRIDE;
    // tree calls: a walker whose ln_prior is -inf was not solved by k_elements
    // (prior_rejects); the pair goes straight to the -inf finish (a local
    // status value only: the status array keeps the model's own code)
    constexpr int ST_PRIOR_SKIP = -1;
    const bool prej = CHI && L.prior && prior_rejects(L.prior[L.E == 1 ? pair : pair / L.E], G);
    if constexpr (GP) {
        // the Kalman filter's state-independent factors of the pair's points
        // (e^{-lam dx}, changepoint block), for k_gp_like: one point per
        // thread here instead of ~60 instructions per point in the filter's
        // serial lane (formed before the prologue: no registers held)
        const double lam = G[G_GP_LAM], dcp = G[G_GP_DCP], ph0 = G[G_PHI0];
        const int ge0 = L.gp_ecl[2 * e], ge1 = L.gp_ecl[2 * e + 1];
        for (int p = tid; p < n; p += LIKE_THREADS) {
            const double xp = L.x[o0 + p];
            const double dx = xp - (p > 0 ? L.x[o0 + p - 1] : xp);
            const size_t q = size_t(pair) * L.N + p;
            L.gpx[q] = exp(-(lam * dx));
            L.gpb[q] = gp_block(xp, ge0, ge1, dcp, ph0);
        }
    }

    // fused acceptance with one eclipse per walker: the proposal's coordinates
    // (one per lane), the uniform draw and the old ln_prob are fetched here,
    // off the tail of the block (combine_walker does it for E > 1)
    const bool acc1 = CHI && !GP && L.pos && L.E == 1;
    // the proposal's coordinates wait in LDS (a register held through the
    // whole block would be spilled: the kernel is at its 128-VGPR budget)
    __shared__ double sq[ACC_LDS];
    if (acc1 && tid < L.ndim && tid < ACC_LDS) sq[tid] = L.qprop[size_t(pair) * L.ndim + tid];
    // each thread's own data point y, ye: fetched with the prologue's loads
    // into this thread's LDS slot (no registers held through the passes, and
    // no memory round trip where chi^2 is formed)
    __shared__ double sy[CHI ? LIKE_TILE : 1], sye[CHI ? LIKE_TILE : 1];
    if (CHI && tid < n) {
        sy[tid] = L.y[o0 + tid];
        if (!GP) sye[tid] = L.ye[o0 + tid];
    }
    int st;
    double s, c, ul, td;
    double px = 0.0, pw = 0.0;  // tile-0 point of this thread (y, ye: read where chi^2 is formed)
    // this thread's sweep items, held in registers for every tile: WD/disc
    // elements tid + i nt (sweep_ab) with their ring weights, spot element
    // tid (< NBS), donor tile (last NDONOR lanes)
    constexpr int NI = (NWD + NDISC + nt - 1) / nt;
    double2 abk[NI];
    double2 abB = make_double2(1.0, -1.0);
    double wB = 0.0;
    double dq[DON_STRIDE] = {0.0, 0.0, 0.0, 0.0, 0.0};
    double gv = 0.0;     // one geometry word per lane for sgeo
    double wring = 0.0;  // ring weights for the direct path
    // every global load of the prologue is issued before anything waits on
    // one (the status included): a single memory round trip
    st = L.status[pair];
    if (st == ST_OK && prej) st = ST_PRIOR_SKIP;
    s = G[G_S];
    c = G[G_C];
    ul = G[G_ULIMB];
    td = Wt[WT_TD];
    if (!SUB && tid < n) {  // (S > 1: at the first tile, after the table build it would be held through)
        px = L.x[o0 + tid];
        pw = L.w ? L.w[o0 + tid] : 0.0;
    }
    for (int i = 0; i < NI; ++i) {
        const int g = tid + i * nt;
        abk[i] = (g < NWD + NDISC) ? sweep_ab(AB, g) : make_double2(1.0, -1.0);
    }
    if (tid < NBS) {
        abB = AB[NU_WDD + tid];
        wB = Wt[WT_BS + tid];
    } else if (tid >= nt - NDONOR) {
        const int t = tid - (nt - NDONOR);
        for (int i = 0; i < DON_STRIDE; ++i) dq[i] = DONp[(t >> 2) * DON_STRIDE + i];
    }
    if (tid >= NBS + NWD_RINGS + NDISC_R && tid < NBS + NWD_RINGS + NDISC_R + G_COUNT)
        gv = G[tid - (NBS + NWD_RINGS + NDISC_R)];
    if (tid >= NBS && tid < NBS + NWD_RINGS) wring = wd_ring_weight(tid - NBS, ul);
    else if (tid >= NBS + NWD_RINGS && tid < NBS + NWD_RINGS + NDISC_R)
        wring = Wt[WT_DISC + tid - NBS - NWD_RINGS];
    // the acceptance draw by the block's last lane, after its prologue loads
    // are in flight (in wave 0 the Philox rounds and the log delayed every
    // load of that wave's prologue)
    if (acc1 && tid == nt - 1) {
        const uint4 r = draw(L.seed, L.step, L.half, 1, pair);
        sacc1[0] = log(u53(r.x, r.y));
        sacc1[1] = L.zfac[pair];
        sacc1[2] = L.lnp_ens[L.half * L.npairs + pair];
    }

    LIKE_PRO(0);
    if (st != ST_OK) {
        for (int p = tid; p < n && !CHI; p += nt) {  // flux outputs: MODE 0 only (the tree paths pass none)
            if (L.flux) L.flux[size_t(pair) * n + p] = NAN;
            if (L.comps)
                for (int m = 0; m < 4; ++m) L.comps[(size_t(m) * L.npairs + pair) * n + p] = NAN;
        }
        if (CHI && !GP) {  // GP trees: k_gp_like sees the status and finishes the pair
            if (tid == 0) L.lle[pair] = -INFINITY;
            finish_walker(L, pair, tid, acc1, sq, sacc1, sflag);
        }
        return;
    }
    double tb = 0.0, dn = 0.0, vs = 0.0;
    if (tid < NBS) {
        sbw[tid] = wB;
        tb = wB;
    } else if (tid >= nt - NDONOR) {
        // donor normalisation at quadrature (theta = pi/2): e = (0, -s, c)
        const int mr = (tid - (nt - NDONOR)) & 3;
        const double vy = (mr & 1) ? -dq[1] : dq[1], vz = (mr & 2) ? -dq[2] : dq[2];
        dn = fmax(-s * vy + c * vz, 0.0);
        vs = fabs(dq[0]) + fabs(dq[1]) + fabs(dq[2]);
    }
    if (tid >= NBS && tid < NBS + NWD_RINGS + NDISC_R) swr[tid - NBS] = wring;
    {
        if (tid >= NBS + NWD_RINGS + NDISC_R && tid < NBS + NWD_RINGS + NDISC_R + G_COUNT)
            sgeo[tid - (NBS + NWD_RINGS + NDISC_R)] = gv;
        if (tid < NBS) sab[tid] = abB;
        else if (tid >= nt - NDONOR && ((tid - (nt - NDONOR)) & 3) == 0)
            for (int i = 0; i < DON_STRIDE; ++i) sdq[((tid - (nt - NDONOR)) >> 2) * DON_STRIDE + i] = dq[i];
    }
    // hulls of the eclipsed WD/disc and spot intervals (tiles outside skip
    // them): only when there is more than one tile or sub-bin tables
    const bool hull = SUB || n > LIKE_TILE;
    if (hull) {
        double wa = INFINITY, wb = -INFINITY, sa = INFINITY, sb = -INFINITY;
#pragma unroll
        for (int i = 0; i < NI; ++i)
            if (abk[i].x < abk[i].y) { wa = fmin(wa, abk[i].x); wb = fmax(wb, abk[i].y); }
        if (tid < NBS && abB.x < abB.y) { sa = abB.x; sb = abB.y; }
        wa = wave_min(wa); wb = wave_max(wb); sa = wave_min(sa); sb = wave_max(sb);
        if (lane == 0) { shw[0][wv] = wa; shw[1][wv] = wb; shw[2][wv] = sa; shw[3][wv] = sb; }
    }
    tb = wave_sum(tb);
    dn = wave_sum(dn);
    vs = wave_sum(vs);
    if (lane == 0) { red[0][wv] = tb; red[1][wv] = dn; red[2][wv] = vs; }
    LIKE_PRO(1);
    __syncthreads();
    LIKE_PRO(2);
    if (wv == 0) {  // block-uniform normalisers live in LDS (read at use: no registers held)
        // the nw wave partials: lanes 0..nw-1 read them at once and three
        // independent DPP wave sums add them (a serial loop in one lane
        // waited on every LDS read in turn)
        double p0 = 0.0, p1 = 0.0, p2 = 0.0;
        if (lane < nw) { p0 = red[0][lane]; p1 = red[1][lane]; p2 = red[2][lane]; }
        p0 = wave_sum(p0);
        p1 = wave_sum(p1);
        p2 = wave_sum(p2);
        if (lane == 0) {
            snorm[0] = 1.0 / p0;
            snorm[1] = 1.0 / p2;
            snorm[2] = p1;
            snorm[3] = p2;
        }
        if (hull && lane < 4) {
            double h = (lane & 1) ? -INFINITY : INFINITY;
            for (int k = 0; k < nw; ++k) h = (lane & 1) ? fmax(h, shw[lane][k]) : fmin(h, shw[lane][k]);
            shull[lane] = h;
        }
    }
    const double twd = TWO_PI * ((1.0 - ul) * 0.5 + ul / 3.0);  // 2 pi [F(1) - F(0)]
    if (tid >= NBS && tid < NBS + NWD_RINGS + NDISC_R)  // visible to the sweep after the pass barrier
        swn[tid - NBS] = wring * ((tid - NBS < NWD_RINGS) ? 1.0 / twd : 1.0 / td);

    // geometry constants of the tile loop come from sgeo at each use (vector
    // loads of G would hold ~13 doubles in VGPRs through every pass)
    const double* SG = sgeo;
    const int S = L.nsub;
    constexpr bool TAB = SUB;  // sub-bins: the spot and donor from breakpoint tables
    SubEntries& DE = *reinterpret_cast<SubEntries*>(&sacc[2][0]);
    if (TAB) {
        SubTables& T = SU.tb;
        // (a) the range of every sub-bin centre of the pair (the donor cells
        // span it), and the tables zeroed
        double qlo = INFINITY, qhi = -INFINITY;
        for (int p = tid; p < n; p += nt) {
            const double xp = L.x[o0 + p], wp = L.w ? L.w[o0 + p] : 0.0;
            const double a0 = xp - SG[G_PHI0], hp = wp / S;
            for (int j = 0; j < S; ++j) {
                const double ph = wrap_phase(a0 - wp + (2 * j + 1) * hp);
                qlo = fmin(qlo, ph);
                qhi = fmax(qhi, ph);
            }
        }
        for (int g = tid; g < TCELLS; g += nt) {
            T.dpre[g][0] = T.dpre[g][1] = T.dpre[g][2] = 0;
            T.spre[g] = 0;
            T.dend[g] = T.send[g] = 0;
        }
        if (tid < 3) T.dv0[tid] = 0;
        qlo = wave_min(qlo);
        qhi = wave_max(qhi);
        if (lane == 0) { sqr[0][wv] = qlo; sqr[1][wv] = qhi; }
        __syncthreads();
        double t0d = INFINITY, t1d = -INFINITY;
        for (int k = 0; k < nw; ++k) { t0d = fmin(t0d, sqr[0][k]); t1d = fmax(t1d, sqr[1][k]); }
        const double dginv = (t1d > t0d) ? TCELLS / (t1d - t0d) : 0.0;
        const double st0 = shull[2], sginv = (shull[3] > shull[2]) ? TCELLS / (shull[3] - shull[2]) : 0.0;
        if (tid == 0) { T.dt0 = t0d; T.dginv = dginv; T.st0 = st0; T.sginv = sginv; }
        // (b) this lane's breakpoints (<= 2): counts and fixed-point sums per cell
        {
            const double itb = snorm[0], ivs = snorm[1];
            double p0, p1;
            bool in0, in1;
            int v0;
            lane_breakpoints(tid, sdq, sab, t0d, t1d, p0, p1, in0, in1, v0);
            if (tid >= nt - NDONOR) {
                long long q[3];
                donor_q(sdq, tid - (nt - NDONOR), ivs, q[0], q[1], q[2]);
                if (v0)
                    for (int k = 0; k < 3; ++k)
                        atomicAdd(reinterpret_cast<unsigned long long*>(&T.dv0[k]),
                                  static_cast<unsigned long long>(v0 * q[k]));
#pragma unroll
                for (int b = 0; b < 2; ++b) {
                    if (!(b ? in1 : in0)) continue;
                    const int g = tcell(b ? p1 : p0, t0d, dginv);
                    atomicAdd(&T.dend[g], 1);
                    for (int k = 0; k < 3; ++k)
                        atomicAdd(reinterpret_cast<unsigned long long*>(&T.dpre[g][k]),
                                  static_cast<unsigned long long>(b ? -q[k] : q[k]));
                }
            } else if (in0) {
                const long long W = to_fx(sbw[tid] * itb);
#pragma unroll
                for (int b = 0; b < 2; ++b) {
                    const int g = tcell(b ? p1 : p0, st0, sginv);
                    atomicAdd(&T.send[g], 1);
                    atomicAdd(reinterpret_cast<unsigned long long*>(&T.spre[g]),
                              static_cast<unsigned long long>(b ? -W : W));
                }
            }
        }
        __syncthreads();
        // (c) exclusive prefixes over the cells: entry offsets, V0 + sums below, covering weights
        long long v[6] = {0, 0, 0, 0, 0, 0};
        if (tid < TCELLS) {
            v[0] = T.dend[tid];
            v[1] = T.send[tid];
            v[2] = T.dpre[tid][0];
            v[3] = T.dpre[tid][1];
            v[4] = T.dpre[tid][2];
            v[5] = T.spre[tid];
        }
        cell_scan<6>(v, spart, tid);
        if (tid < TCELLS) {
            T.dend[tid] = int(v[0]);
            T.send[tid] = int(v[1]);
            T.dpre[tid][0] = v[2] + T.dv0[0];
            T.dpre[tid][1] = v[3] + T.dv0[1];
            T.dpre[tid][2] = v[4] + T.dv0[2];
            T.spre[tid] = v[5];
        }
        __syncthreads();
        // (d) the entries into cell order; afterwards dend / send hold each cell's end
        {
            double p0, p1;
            bool in0, in1;
            int v0;
            lane_breakpoints(tid, sdq, sab, t0d, t1d, p0, p1, in0, in1, v0);
            const int base = (tid >= nt - NDONOR) ? 2 * (tid - (nt - NDONOR)) : 2 * tid;
#pragma unroll
            for (int b = 0; b < 2; ++b) {
                if (!(b ? in1 : in0)) continue;
                const double pos = b ? p1 : p0;
                if (tid >= nt - NDONOR) {
                    const int slot = atomicAdd(&T.dend[tcell(pos, t0d, dginv)], 1);
                    DE.dpos[slot] = pos;
                    DE.dcode[slot] = base + b;
                } else {
                    const int slot = atomicAdd(&T.send[tcell(pos, st0, sginv)], 1);
                    T.spos[slot] = pos;
                    T.scode[slot] = base + b;
                }
            }
        }
        __syncthreads();
        // (e) each cell's donor entries in order (sub_point's cursor): position,
        // an end before a start at equal positions; a few entries per cell.
        // The spot's entries by position too
        if (tid < TCELLS) {
            const int i0 = tid ? T.dend[tid - 1] : 0, i1 = T.dend[tid];
            for (int i = i0 + 1; i < i1; ++i) {
                const double p = DE.dpos[i];
                const int c = DE.dcode[i];
                int k = i;
                for (; k > i0; --k) {
                    const double pk = DE.dpos[k - 1];
                    const int ck = DE.dcode[k - 1];
                    if (!(pk > p || (pk == p && (c & 1) && !(ck & 1)))) break;
                    DE.dpos[k] = pk;
                    DE.dcode[k] = ck;
                }
                DE.dpos[k] = p;
                DE.dcode[k] = c;
            }
            // the spot's entries of the cell by position (sub_point's spot cursor)
            const int j0 = tid ? T.send[tid - 1] : 0, j1 = T.send[tid];
            for (int i = j0 + 1; i < j1; ++i) {
                const double p = T.spos[i];
                const int c = T.scode[i];
                int k = i;
                for (; k > j0 && T.spos[k - 1] > p; --k) {
                    T.spos[k] = T.spos[k - 1];
                    T.scode[k] = T.scode[k - 1];
                }
                T.spos[k] = p;
                T.scode[k] = c;
            }
        }
        __syncthreads();
    }
    for (int t0 = 0; t0 < n; t0 += LIKE_TILE) {
        double chi = 0.0;  // this tile's chi^2 (summed per wave into red[1] at the tile's end)
        const int m = min(LIKE_TILE, n - t0);
        LIKE_STAMP(0);
        const bool own = tid < m;
        if ((t0 > 0 || SUB) && own) {
            // the point index re-formed from a fresh (volatile) read of the
            // offset: o0 + tid would otherwise be held, spilled, over the tiles
            const int p = (offs ? *reinterpret_cast<const volatile int*>(L.off + e) : 0) + t0 + tid;
            px = L.x[p];
            pw = L.w ? L.w[p] : 0.0;
            if (CHI && t0 > 0) {
                sy[tid] = L.y[p];
                if (!GP) sye[tid] = L.ye[p];
            }
        }
        // MODEL_SPEC 3: a negative width is a zero one (point evaluation at the
        // centre for every S); NaN stays NaN
        const double wk = own ? (pw < 0.0 ? 0.0 : pw) : 0.0;
        const double ph0 = own ? px - SG[G_PHI0] : 0.0;
        const double phc = wrap_phase(ph0);
        double fw = 0.0, fd = 0.0, sbs = 0.0, srs = 0.0;
        // the pass over the points' own windows: the WD and disc (and, S = 1,
        // the spot on the same windows and the donor at the point phases)
        if (tid == 0) { sflag[0] = 0; sflag[1] = 0; }
        int flA = put_window(TA, tid, own, phc, wk);
        if (!TAB && own) sph[tid] = phc;
        for (int i = 0; i < (TAB ? 2 : 6); ++i) sacc[i][tid] = 0ull;
        if (!TAB) {
            SU.s1.X[0][tid] = 0ull;
            SU.s1.X[1][tid] = 0ull;
        }
        if (tid == 0)
            for (int i = 0; i < (TAB ? 2 : 6); ++i) sacc[i][nt] = 0ull;
        // does this point's window reach the WD/disc hull?  (any does: the tile
        // sweeps; one tile and no sub-bins: always)
        if (hull && own && wk >= 0.0 && !(phc + wk < shull[0] || phc - wk > shull[1])) flA |= 8;
        __syncthreads();
        flA |= check_sorted(TA, tid, own);
        // the flags OR-ed over the wave first: one LDS atomic per wave
        // (a same-address atomic per point serialised the hull bit)
        const int wfA = wave_or4(flA);
        if (lane == 0 && wfA) atomicOr(&sflag[0], wfA);
        build_cells(TA.lo, m, TA.cell, tid);
        if (!TAB) {
            const int flB = (flA & 7) | ((own && tid && sph[tid] < sph[tid - 1]) ? 4 : 0);
            const int wfB = wave_or4(flB);
            if (lane == 0 && wfB) atomicOr(&sflag[1], wfB);
            build_cells(sph, m, scp, tid);
        }
        __syncthreads();
        // any unsorted / mixed window (or invalid width) of the tile: the
        // pass goes point-major (every element against each point)
        const bool dir = (sflag[0] & 7) != 0 || (!TAB && sflag[1] != 0);
#ifdef LFG_ABL_WDD  // diagnostic ablation: no WD/disc sweep
        const bool wdd = false;
#else
        const bool wdd = !hull || (sflag[0] & 8) != 0;  // the WD/disc elements touch the tile
#endif
        LIKE_STAMP(1);
        double eb = 0.0, R3 = 0.0, R4 = 0.0, R5 = 0.0;
        if (dir) {
            if (own) {
                const double ulg = SG[G_ULIMB];
                const double2 f2 = direct_wd_disc(AB, swr, phc, wk, TWO_PI * ((1.0 - ulg) * 0.5 + ulg / 3.0), Wt[WT_TD]);
                fw = f2.x;
                fd = f2.y;
                if (!TAB) eb = direct_spot(sab, sbw, phc, wk, snorm[0]);
            }
            __syncthreads();  // every wave has read sflag before the next tile resets it
        } else {
            if (wdd) {
                if constexpr (TAB) {
                    // re-read per tile (L2): held over the tiles they would not
                    // leave the sub-bin queries their registers.  The pointer is
                    // laundered through an empty asm so that the compiler cannot
                    // reuse the prologue's loads of the same (restrict) table:
                    // it kept those values live through the table build, 48 B
                    // of scratch per lane
                    const double2* ABt = AB;
                    asm volatile("" : "+s"(ABt));
#pragma unroll
                    for (int i = 0; i < NI; ++i) {
                        const int g = tid + i * nt;
                        abk[i] = (g < NWD + NDISC) ? sweep_ab(ABt, g) : make_double2(1.0, -1.0);
                    }
                }
                const PhaseIndex X = phase_index(TA.lo, TA.cell, m);
                double qx[2 * NI];
                int J[2 * NI], Jb[2 * NI];
#pragma unroll
                for (int i = 0; i < NI; ++i) {
                    qx[2 * i] = abk[i].x;
                    qx[2 * i + 1] = abk[i].y;
                }
                count_lt_multi<2 * NI>(X, qx, J);
                count_le_back_multi<2 * NI>(TA.hi, qx, J, Jb);
#pragma unroll
                for (int i = 0; i < NI; ++i)
                    if (abk[i].x < abk[i].y) {
                        const int g = tid + i * nt;
                        const int u = uitem(g < NU_WDD ? g : g - NU_WDD);
                        apply_runs(Runs{Jb[2 * i], J[2 * i], Jb[2 * i + 1], J[2 * i + 1]}, abk[i].x, abk[i].y,
                                   swn[uring(u)], X, TA.hi, TA.iw,
                                   ((!TAB && (lane & 1)) ? SU.s1.X : sacc)[(u < U_WD) ? 0 : 1]);
                    }
            }
            LIKE_STAMP(2);
            if (!TAB)
                sweep_spot_donor(tid, phase_index(TA.lo, TA.cell, m), TA, phase_index(sph, scp, m), sab, sbw,
                                 snorm[0], sdq, snorm[1], sacc + 2);
            __syncthreads();
            LIKE_STAMP(3);
            long long r[6] = {0, 0, 0, 0, 0, 0};
            if (!TAB) block_scan<6>(sacc, spart, tid, r, SU.s1.X);
            else if (wdd) block_scan<2>(sacc, spart, tid, r);
            LIKE_STAMP(4);
            fw = double(r[0]) * FX_INV;
            fd = double(r[1]) * FX_INV;
            eb = double(r[2]) * FX_INV;
            R3 = double(r[3]);
            R4 = double(r[4]);
            R5 = double(r[5]);
        }
        const double sg = SG[G_S], cg = SG[G_C];
        const double bden = SG[G_BDEN], fis = SG[G_FIS];
        if (!TAB) {
            const double2 scp2 = sincospi_ool(2.0 * phc);  // |2 ph| <= 1: cheap exact reduction
            const double e0 = sg * scp2.y, e1 = -sg * scp2.x;
            double D = 0.0;
            if (!dir) D = (e0 * R3 + e1 * R4 + cg * R5) * (FX_INV * snorm[3]);
            else if (own) D = direct_donor(sdq, e0, e1, cg);
            double beam = 0.0;
            if (bden > 0.0)
                beam = (fis + (1.0 - fis) * fmax(SG[G_NB0] * e0 + SG[G_NB1] * e1 + SG[G_NB2] * cg, 0.0)) / bden;
            sbs = beam * (1.0 - eb);
            srs = D / snorm[2];
        } else if (own) {
#ifdef LFG_ABL_SUBPOINT  // diagnostic ablation: no sub-bin spot / donor terms
            const double2 r2 = make_double2(ph0 * 1e-30, wk * 1e-30);
#else
            const double2 r2 = sub_point(SU.tb, DE, sab, sbw, sdq, snorm, shull, SG, ph0, wk, S);
#endif
            sbs = r2.x;
            srs = r2.y;
        }
        // no barrier before the next tile rewrites the tile buffers: every
        // read of TA / sph / scp / sacc / sflag of this tile precedes the
        // block scan's barriers or the direct path's barrier (after them only
        // registers, part[], the tables and the pass-invariant LDS are read,
        // none of which the next tile's prologue writes); a table tile that
        // skipped the scan waits here instead
        if (TAB && !dir && !wdd) __syncthreads();
        if (own) {
            const double nw0 = isnan(wk) ? NAN : 1.0;  // MODEL_SPEC 3: a NaN width gives a NaN flux
            const double fwv = nw0 * SG[G_WDF] * (1.0 - fw), fdv = nw0 * SG[G_DF] * (1.0 - fd);
            const double fb = nw0 * SG[G_SF] * sbs / S, fr = nw0 * SG[G_RSF] * srs / S;
            const double f = fwv + fdv + fb + fr;
            const int pi = t0 + tid;
            if (!CHI && L.flux) L.flux[size_t(pair) * n + pi] = f;
            if (!CHI && L.comps) {
                L.comps[(size_t(0) * L.npairs + pair) * n + pi] = fwv;
                L.comps[(size_t(1) * L.npairs + pair) * n + pi] = fdv;
                L.comps[(size_t(2) * L.npairs + pair) * n + pi] = fb;
                L.comps[(size_t(3) * L.npairs + pair) * n + pi] = fr;
            }
            if (CHI && !GP) {
                const double r = (sy[tid] - f) / sye[tid];
                chi += isnan(f) ? INFINITY : r * r;
            }
            if (GP) L.res[size_t(pair) * L.N + pi] = sy[tid] - f;  // the filter runs in k_gp_like
        }
        if (CHI && !GP) {  // red[1] is free after the prologue; each wave owns its slot
            chi = wave_sum(chi);
            if (lane == 0) red[1][wv] = (t0 == 0) ? chi : red[1][wv] + chi;
        }
        LIKE_STAMP(5);
    }
    if (CHI && !GP) {
        __syncthreads();
        if (tid == 0) {
            double tot = 0.0;
            for (int i = 0; i < nw; ++i) tot += red[1][i];
            L.lle[pair] = -0.5 * tot;
        }
        finish_walker(L, pair, tid, acc1, sq, sacc1, sflag);
    }
}

// ------------------------------------------------------------------ k_pair
// k_elements and k_lnlike<1, false> of one (walker, eclipse) pair in ONE
// workgroup, for trees whose eclipses fit one tile (max_n <= LIKE_TILE, S =
// 1, no GP): the element intervals never leave the workgroup, the half-step
// is one launch instead of two (no kernel boundary behind a 10 MB table
// write-back, no re-fetch of the tables), and the interval sweep runs inside
// the element phase: a lane that has solved an element adds its runs to the
// LDS difference arrays at once, while other waves are still solving.
//  * prologue: every thread forms its point's window and phase (and its
//    predecessor's, for the sortedness flags and the phase-index cells, so
//    no barrier is needed for them), the disc ring weights (21 lanes);
//  * element phase: 16 jobs, wave w takes job w and grabs the next free one
//    from an LDS counter twice more.  Job 0: this block's share of the
//    speculative setup lanes of the next half (setup_any, as k_elements'
//    leading blocks run them); jobs 1..15: the 15 chunks of 64 items, longest
//    first.  Each solved item is swept (element and mirror for WD/disc, the
//    four mirrored donor tiles) with k_lnlike's run / point-mode rules.  The
//    spot and donor sums are accumulated unnormalised (int64 fixed point at
//    2^-54 / 2^-58, exact) with their totals, and normalised per point;
//  * after the phase barrier: the block scan, each point's flux, chi^2, the
//    fused acceptance.  Unsorted or invalid windows: the tables go to LDS and
//    the point-major pass runs instead (as k_lnlike's).
// With the fused acceptance the block writes its walker's row of pos while
// the speculative lanes of other blocks read partner rows of the same half:
// those lanes read the snapshot (SetupArgs.ppos) that the launch before took
// of that half, and this launch snapshots the other half for the next one.
typedef const __attribute__((address_space(4))) double* CGeo;
constexpr int DCP_LANES = 16, DCP_NTHETA = 10;  // k_gp_dcp / k_pair<true>: limb points of wdphases

// The arguments of k_pair's prologue chains, contiguous, read at the entry in
// one batch of scalar loads (kernarg_copy): the compiler otherwise issued them
// in ~10 rounds, each behind an s_waitcnt for every outstanding load, ahead of
// the candidate chain.  Copies of the LikeArgs / ElemSpec / PairArgs fields
// of the same names (fill_hot, on the host, before each launch), typed by
// address space: the uniform read-only words constant (scalar loads), the
// points global (a copied generic pointer would make flat loads)
typedef const __attribute__((address_space(4))) int* KInt;
typedef const __attribute__((address_space(4))) double* KDbl;
typedef const __attribute__((address_space(1))) double* GDbl;
struct PairHot {
    KInt accflag;   // X.accflag (the partner half's flags: this launch writes the other half's)
    KDbl fv;        // fv (FOLD)
    KInt jk;        // X.jk
    KInt statusC;   // X.statusC, X.bstatusC, X.priorC, X.geoC (this half's candidates; the
    KInt bstatusC;  //   speculative lanes write the next half's)
    KDbl priorC;
    KDbl geoC;
    KDbl geo;       // L.geo, L.status, L.bstatus, L.prior (read before B0; wave 7 writes
    KInt status;    //   the standard slots after it)
    KInt bstatus;
    KDbl prior;
    KInt off;       // L.off, L.x, L.w
    GDbl x;
    GDbl w;
    unsigned long long jseed, jstep;
    int jhalf, jlo, jns, E, N, npairs;
};

struct PairArgs {
    LikeArgs L;
    ElemSpec X;                // candidate selection (X.jk) and speculative lanes (X.nspec, X.S)
    const double* snap_src;    // nullable: rows [ns][ndim] of the other half of pos, copied to snap_dst
    double* snap_dst;
    int spl;                   // speculative lanes per block that has them (64: wave 0's job 0)
    int nbc;                   // blocks [0, nbc) carry candidate 0's lanes, [nbc, 2 nbc) candidate 1's
    // with X.jk: walker w's partner j in the other half, drawn here as the
    // speculative lanes drew it (make_prop: draw(seed, step, half, 0, lo + w),
    // j = umulhi(r.z, ns)) instead of read back from X.jk, one dependent
    // global load less before the candidate is known
    unsigned long long jseed, jstep;
    int jhalf, jlo, jns;
    int prio;  // blocks [0, prio) take the wave priorities (PAIR_PRIO; pair_prio)
    // FOLD (lfg_stretch_step_shard_fold): the partner half's moves of the
    // half-step before are accepted here, from the verdicts every rank
    // gathered (fv [jns]: ln_prob where accepted, NaN where not; nullptr:
    // nothing pending), each workgroup taking rows w, w + nwk, ...; the pair's
    // candidate is chosen by the same verdicts, and the launch leaves its own
    // verdicts in vout [npairs] (the next exchange's payload)
    const double* fv = nullptr;
    double* vout = nullptr;
    double* fpos = nullptr;   // the ensemble [W][ndim], ln_prob [W], counters [W]
    double* flnp = nullptr;
    int* fnacc = nullptr;
    double* fsnap = nullptr;  // [jns][ndim]: this half's rows, for the next launch's speculative lanes
    unsigned long long fstep = 0;  // the step of the pending moves' proposals
    double fa = 2.0;               // the stretch scale a
    PairHot hot{};                 // fill_hot
};

// PairArgs.hot from the fields it copies (every k_pair launch, last)
static void fill_hot(PairArgs& A)
{
    PairHot& H = A.hot;
    H.accflag = (KInt)A.X.accflag;
    H.fv = (KDbl)A.fv;
    H.jk = (KInt)A.X.jk;
    H.statusC = (KInt)A.X.statusC;
    H.bstatusC = (KInt)A.X.bstatusC;
    H.priorC = (KDbl)A.X.priorC;
    H.geoC = (KDbl)A.X.geoC;
    H.geo = (KDbl)A.L.geo;
    H.status = (KInt)A.L.status;
    H.bstatus = (KInt)A.L.bstatus;
    H.prior = (KDbl)A.L.prior;
    H.off = (KInt)A.L.off;
    H.x = (GDbl)A.L.x;
    H.w = (GDbl)A.L.w;
    H.jseed = A.jseed;
    H.jstep = A.jstep;
    H.jhalf = A.jhalf;
    H.jlo = A.jlo;
    H.jns = A.jns;
    H.E = A.L.E;
    H.N = A.L.N;
    H.npairs = A.L.npairs;
}

// The kernel-argument segment as a typed constant pointer whose value the
// compiler cannot see through.  k_pair's arguments are ~1 KB; the compiler
// loaded the speculative lanes' two SetupArgs (560 B, used by wave 0 of a few
// blocks) at every wave's entry and spilled them into VGPR lanes, a chain of
// ~15 dependent scalar-load waits (~3 us) ahead of the candidate chain.
// Fields read through this pointer are loaded where they are used.
template <typename T>
__device__ __forceinline__ const __attribute__((address_space(4))) T* opaque_kernargs()
{
    auto p = (const __attribute__((address_space(4))) T*)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(p));
    return p;
}

// a by-value copy of a kernel-argument struct read through such a pointer
// (word by word: the struct's copy constructor takes a generic reference)
template <typename T>
__device__ __forceinline__ T kernarg_copy(const __attribute__((address_space(4))) T* p)
{
    static_assert(sizeof(T) % 8 == 0, "whole words");
    const auto* src = reinterpret_cast<const __attribute__((address_space(4))) unsigned long long*>(p);
    unsigned long long w[sizeof(T) / 8];
#pragma unroll
    for (int i = 0; i < int(sizeof(T) / 8); ++i) w[i] = src[i];
    T out;
    __builtin_memcpy(&out, w, sizeof(T));
    return out;
}

// the chunks of k_pair's element jobs 1..15, longest first (spot, outer
// disc, donor, inner disc, WD: the Newton steps per region)
__constant__ int kJobChunk[15] = {11, 12, 10, 9, 8, 13, 14, 7, 6, 5, 4, 3, 2, 1, 0};

// fixed-point scales of k_pair's unnormalised spot and donor sums, as
// factors into to_fx's 2^61: spot weights <= 1 (100 of them: 2^54), donor
// vectors (their |v| sums stay far below 2^5: 2^58)
constexpr double PAIR_SPOT_S = 1.0 / 128.0, PAIR_DON_S = 1.0 / 8.0;

#ifdef LFG_PROFILE_PAIR  // diagnostic build only: s_memrealtime (100 MHz) stamps of each block's phases
__device__ unsigned long long g_pair_t[24][4096];
#define PAIR_STAMP(slot, cond)                                                     \
    do {                                                                           \
        if ((cond) && blockIdx.x < 4096) g_pair_t[slot][blockIdx.x] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
__device__ unsigned long long g_pair_w[4][8][4096];
__device__ unsigned long long g_long_t[8][4096];  // the LONG table build's steps (thread 0 after each barrier)
#define LONG_TSTAMP(k)                                                                      \
    do {                                                                                    \
        if (tid == 0 && blockIdx.x < 4096) g_long_t[k][blockIdx.x] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
__device__ unsigned long long g_pair_j[3][16][4096];  // per chunk: job start, sink entry, end
#define PAIR_WSTAMP(k)                                                                                  \
    do {                                                                                                \
        if (lane == 0 && blockIdx.x < 4096) g_pair_w[k][wv][blockIdx.x] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
#else
#define PAIR_STAMP(slot, cond)
#define LONG_TSTAMP(k)
#define PAIR_WSTAMP(k)
#endif

// wave priority in a launch of at most two rounds (blocks [0, A.prio)): the
// issue arbiter favours the older of a CU's two workgroups, so one finished
// ~10 us before the other and the CU ran its last phases on half its waves.
// Element waves drop their priority with each job they start (3, 2, 1, then
// 0), so both workgroups advance together; the speculative setup waves
// (latency-bound, and the longest job) keep 3.  In a launch of many rounds
// the older workgroup's early finish lets the next round's start, so the
// default order stays (pair_prio)
#define PAIR_PRIO(p)                                                    \
    do {                                                                \
        if (int(blockIdx.x) < A.prio) __builtin_amdgcn_s_setprio(p);    \
    } while (0)

// k_pair's sweep of one solved item (the element phase's sink): element runs
// over the tile's windows (WD, disc, spot) and the donor tiles' visibility
// arcs over the point phases, into the LDS difference arrays; or, for a tile
// that goes point-major, the tables
struct PairSink {
    bool dir;
    int lane;
    PhaseIndex XW, XP;      // windows (lo, cells) and point phases (sph, scp)
    const double* hi;
    const double* iw;
    unsigned long long (*acc)[LIKE_TILE + 1];   // sacc
    unsigned long long (*acc2)[LIKE_TILE + 1];  // second WD/disc copies (odd lanes)
    unsigned long long* tot;                    // [2] spot weight and donor quadrature sums
    const double* swt;      // disc ring weights, disc total
    double ul, itwd, s, c;  // ulimb, 1 / (2 pi (F(1) - F(0))), sin / cos i
    double2* ab;            // point-major: the WD/disc intervals, spot intervals and weights, donor tiles
    double2* sab;
    double* sbw;
    double* sdq;
    unsigned long long* mk;  // diagnostic builds: where mark() stamps the sink's entry
    // lane-local sums flushed once per wave (flush): the spot weight and donor
    // quadrature totals, and the donor arcs that open at the tile's first point
    // (all 64 lanes of a wave added these to the same LDS word: 64-way conflicts)
    long long tspot, tdon, bx, by, bz;

    __device__ __forceinline__ void mark()
    {
#ifdef LFG_PROFILE_PAIR
        if (mk) *mk = __builtin_amdgcn_s_memrealtime();
#endif
    }
    __device__ __forceinline__ void wd_disc(int u, double a, double b)
    {
#ifdef LFG_ABL_SINK_WD  // (diagnostic builds) the sink skipped: LDS counter attribution only
        return;
#endif
        if (dir) {
            ab[uslot(u)] = make_double2(a, b);
            return;
        }
        if (!(a < b)) return;
        const int ir = uring(u);
        const double wn = (u < U_WD) ? wd_ring_weight(ir, ul) * itwd : swt[ir - NWD_RINGS] * (1.0 / swt[NDISC_R]);
        double q[4] = {a, b, -b, -a};  // the element and its mirror [-b, -a]
        int J[4], Jb[4];
        count_lt_multi<4>(XW, q, J);
        count_le_back_multi<4>(hi, q, J, Jb);
        unsigned long long* A = ((lane & 1) ? acc2 : acc)[(u < U_WD) ? 0 : 1];
        const Runs RR[2] = {Runs{Jb[0], J[0], Jb[1], J[1]}, Runs{Jb[2], J[2], Jb[3], J[3]}};
        const double aa[2] = {a, -b}, bb[2] = {b, -a};
        apply_runs_batched<2>(RR, aa, bb, wn, XW, hi, iw, A);
    }
    __device__ __forceinline__ void spot(int j, double a, double b, double w)
    {
        sab[j] = make_double2(a, b);
        sbw[j] = w;
        tspot += to_fx(w * PAIR_SPOT_S);
#ifdef LFG_ABL_SINK_SPOT  // (diagnostic builds) the runs skipped: LDS counter attribution only
        if (false) {
#else
        if (!dir && a < b) {
#endif
            const Runs RR[1] = {element_runs(a, b, XW, hi)};
            const double aa[1] = {a}, bb[1] = {b};
            apply_runs_batched<1>(RR, aa, bb, w * PAIR_SPOT_S, XW, hi, iw, acc[2]);
        }
    }
    __device__ __forceinline__ void donor(int uu, double vx0, double vy0, double vz0, double cen0, double hw0)
    {
        double* D = sdq + uu * DON_STRIDE;
        D[0] = vx0;
        D[1] = vy0;
        D[2] = vz0;
        D[3] = cen0;
        D[4] = hw0;
        long long tn = 0;
        // the arcs' point ranges first (LDS reads), then their entries
        int PA[4][2], QA[4][2];
#pragma unroll
        for (int mr = 0; mr < 4; ++mr) {  // the tile's mirror images, as k_lnlike's donor lanes form them
            const double vy = (mr & 1) ? -vy0 : vy0, vz = (mr & 2) ? -vz0 : vz0;
            const double cen = (mr & 1) ? -cen0 : cen0;
            const double hw = (mr & 2) ? 0.5 - hw0 : hw0;
            tn += to_fx(fmax(-s * vy + c * vz, 0.0) * PAIR_DON_S);
            PA[mr][0] = QA[mr][0] = PA[mr][1] = QA[mr][1] = 0;
#ifdef LFG_ABL_SINK_DON  // (diagnostic builds) the arcs skipped: LDS counter attribution only
            continue;
#endif
            if (dir || !(hw > 0.0)) continue;
            // visible for phases in (cen - hw, cen + hw) mod 1
            double x1 = -INFINITY, x2 = INFINITY, y1 = 0.0, y2 = 0.0;
            bool two = false;
            if (hw < 0.5) {
                const double lo = cen - hw, hi2 = cen + hw;
                if (lo < -0.5) { x2 = hi2; y1 = lo + 1.0; y2 = INFINITY; two = true; }
                else if (hi2 > 0.5) { x1 = lo; y1 = -INFINITY; y2 = hi2 - 1.0; two = true; }
                else { x1 = lo; x2 = hi2; }
            }
            PA[mr][0] = count_below<true>(XP, x1);
            QA[mr][0] = count_below<false>(XP, x2);
            if (two) {
                PA[mr][1] = count_below<true>(XP, y1);
                QA[mr][1] = count_below<false>(XP, y2);
            }
        }
        const long long qx = to_fx(vx0 * PAIR_DON_S), qy0 = to_fx(vy0 * PAIR_DON_S), qz0 = to_fx(vz0 * PAIR_DON_S);
#pragma unroll
        for (int mr = 0; mr < 4; ++mr) {
            const long long qy = (mr & 1) ? -qy0 : qy0, qz = (mr & 2) ? -qz0 : qz0;
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const int P = PA[mr][i], Q = QA[mr][i];
                if (P < Q) {
                    if (P == 0) {
                        bx += qx;
                        by += qy;
                        bz += qz;
                    } else {
                        fx_add(acc[3], P, qx);
                        fx_add(acc[4], P, qy);
                        fx_add(acc[5], P, qz);
                    }
                    if (Q < XP.m) {
                        fx_add(acc[3], Q, -qx);
                        fx_add(acc[4], Q, -qy);
                        fx_add(acc[5], Q, -qz);
                    }
                }
            }
        }
        tdon += tn;
    }
    // the lane-local sums into LDS: every lane of the wave calls it, after its
    // last item (the integer sums are exact in any order)
    __device__ __forceinline__ void flush()
    {
        const long long t0 = wave_total(tspot), t1 = wave_total(tdon);
        const long long x = wave_total(bx), y = wave_total(by), z = wave_total(bz);
        if (lane == 0) {
            if (t0) atomicAdd(tot, static_cast<unsigned long long>(t0));
            if (t1) atomicAdd(tot + 1, static_cast<unsigned long long>(t1));
            if (x) fx_add(acc[3], 0, x);
            if (y) fx_add(acc[4], 0, y);
            if (z) fx_add(acc[5], 0, z);
        }
    }
};

// point-major WD and disc eclipse fractions of one window (k_pair's
// unsorted-tile pass: direct_wd_disc with the ring weights formed here)
__device__ __forceinline__ double2 pair_direct_wd_disc(const double2* __restrict__ AB, double ul,
                                                       const double* __restrict__ swt, double phc, double wk,
                                                       double twd, double td)
{
    double ewd = 0.0, ed = 0.0;
    const double lo = phc - wk, hi = phc + wk;
    auto cover = [&](double2 ab) {
        return (wk > 0.0) ? fmax(fmin(ab.y, hi) - fmax(ab.x, lo), 0.0) : ((phc > ab.x && phc < ab.y) ? 1.0 : 0.0);
    };
    for (int ring = 0; ring < NWD_RINGS + NDISC_R; ++ring) {  // each unique item and its mirror
        const int u0 = ring < NWD_RINGS ? 2 * ring * ring : U_WD + (ring - NWD_RINGS) * (NDISC_AZ / 2);
        const int u1 = ring < NWD_RINGS ? 2 * (ring + 1) * (ring + 1) : u0 + NDISC_AZ / 2;
        double acc = 0.0;
        for (int u = u0; u < u1; ++u) {
            const double2 ab = AB[uslot(u)];
            acc += cover(ab) + cover(mirror_ab(ab));
        }
        const double wr = ring < NWD_RINGS ? wd_ring_weight(ring, ul) : swt[ring - NWD_RINGS];
        if (ring < NWD_RINGS) ewd = fma(wr, acc, ewd); else ed = fma(wr, acc, ed);
    }
    const double nrm = (wk > 0.0) ? 1.0 / (2.0 * wk) : 1.0;
    return make_double2(ewd * nrm * (1.0 / twd), ed * nrm * (1.0 / td));
}

// a point's window: phase, lo, hi (k_lnlike's put_window arithmetic)
__device__ __forceinline__ void pair_window(double x, double w, double phi0, double& ph, double& lo, double& hi,
                                            double& hw)
{
    ph = wrap_phase(x - phi0);
    hw = w;
    lo = ph - hw;
    hi = ph + hw;
}

// the cells of phase index (v sorted, v[0] = v0, v[m-1] = v1) that point p
// fills, as build_cells does, from p's own value and its predecessor's
__device__ __forceinline__ void pair_cells(int* cell, int p, int m, double vprev, double vown, double v0, double v1)
{
    const double span = v1 - v0, ginv = span > 0.0 ? LIKE_NC / span : 0.0;
    auto ci = [&](double x) {
        const double u = (x - v0) * ginv;
        return u < 0.0 ? -1 : (u >= double(LIKE_NC) ? LIKE_NC : int(u));
    };
    const int g0 = p ? ci(vprev) : -1, g1 = ci(vown);
    for (int g = g0 + 1; g <= g1; ++g) cell[g] = p;
    if (p == m - 1)
        for (int g = g1 + 1; g <= LIKE_NC; ++g) cell[g] = m;
}

// ---- LONG: eclipses of any length and sub-binned exposures in k_pair ----
// The element phase stores every solved item (k_pair's point-major sinks:
// WD/disc intervals, spot intervals and weights, donor tiles) and the pair's
// breakpoints are then bucketed into per-pair tables in LDS, so that every
// point is evaluated on its own, with no tile loop, block scan or barrier per
// 512 points (config 5: 10 000 points x 5 sub-bins):
//  * WD and disc (one table each, the symmetry-unique elements; a mirror
//    element [-b, -a] is the unique one seen from -phase): the eclipsed
//    fraction of window [lo, hi] is the integral of the covering weight,
//      int_lo^hi C(t) dt = C(lo) (hi - lo) + sum_{lo <= pos < hi} q (hi - pos),
//    with q = +w at a start a_k and -w at an end b_k; each sorted entry holds
//    C just after it (int64 fixed point, exact), so C(lo) is one read once the
//    first entry at or above lo is found -- in its cell (1 024 per table over
//    the table's own hull, a few entries even where the WD contacts crowd);
//    a zero-width window takes the elements with a_k < ph < b_k;
//  * spot and donor at the sub-bins: the S > 1 breakpoint tables of k_lnlike
//    (SubTables, SubEntries, sub_point), built here from LDS.
// Each wave takes a range of blocks of 64 points, its lanes interleaved
// (MODEL_SPEC 3 for every width, order and wrap: no sortedness is assumed).
constexpr int NE_W = 2 * U_WD, NE_D = 2 * U_DISC;  // WD / disc table entries (two per unique element)
constexpr int LONG_FC = 4 * TCELLS;                 // cells per WD/disc table (the sub-bin tables: TCELLS)
struct LongTabs {
    int fend[2][LONG_FC];       // WD / disc cells: counts -> exclusive offsets -> (after the scatter) cell ends
    double epos[NE_W + NE_D];   // entries: WD [0, NE_W), disc after
    long long ecb[NE_W + NE_D];  // build: q; after the sort and scan: C just after the entry
    double t0[2], ginv[2], amin[2], bmax[2];  // per table: LONG_FC cells over its hull
    double snorm[4];            // sub_point's: 1 / spot total, 1 / donor |v| sum, donor norm, |v| sum
    double shull[4];            // [2], [3]: the spot hull (sub_point)
    double sgeo[LFG_NGEO];      // the record, for sub_point's LDS reads
    double part[8][LIKE_THREADS / 64];  // wave partials of the hulls and sums
};

// the WD/disc cell of x in table t (clamped to the table's cells)
__device__ __forceinline__ int long_cell(double x, double t0, double ginv)
{
    const double u = (x - t0) * ginv;
    return u <= 0.0 ? 0 : (u >= double(LONG_FC - 1) ? LONG_FC - 1 : int(u));
}

// a value the whole block holds alike, into scalar registers
__device__ __forceinline__ double uni(double x)
{
    const long long b = __double_as_longlong(x);
    const int lo = __builtin_amdgcn_readfirstlane(static_cast<int>(b));
    const int hi = __builtin_amdgcn_readfirstlane(static_cast<int>(b >> 32));
    return __longlong_as_double((static_cast<long long>(hi) << 32) | static_cast<unsigned>(lo));
}

// the point phase's per-pair constants, read once from LDS into scalar
// registers: every lane's lookups and sub-bin terms use them, and the LDS
// pipe -- which the lookups keep busy -- serves no broadcasts in the loop
struct LongU {
    double t0[2], gf[2], amin[2], bmax[2];  // WD/disc tables: cells and hulls
    int n[2];                               // entries per table
    double itb, ivs, dnorm, vsum, sa, sb;   // spot / donor norms, the spot hull
    double nbs0, nbs1, nbc, fis, omf;       // the record's terms of the sub-bin sums (MODEL_SPEC 6), folded
    double sg, cg, ibden, dsc;              // the sums' scales
    double invS;                            // 1 / sub-bins
    int nd, nsp;                            // donor / spot entries
};

__device__ __forceinline__ LongU long_uniforms(const LongTabs& W, const SubTables& T, int S)
{
    LongU K;
    K.invS = uni(1.0 / S);
    for (int t = 0; t < 2; ++t) {
        K.t0[t] = uni(W.t0[t]);
        K.gf[t] = uni(W.ginv[t]);
        K.amin[t] = uni(W.amin[t]);
        K.bmax[t] = uni(W.bmax[t]);
        K.n[t] = __builtin_amdgcn_readfirstlane(W.fend[t][LONG_FC - 1]);
    }
    K.itb = uni(W.snorm[0]); K.ivs = uni(W.snorm[1]); K.dnorm = uni(W.snorm[2]); K.vsum = uni(W.snorm[3]);
    K.sa = uni(W.shull[2]); K.sb = uni(W.shull[3]);
    const double sg = W.sgeo[G_S], cg = W.sgeo[G_C], fis = W.sgeo[G_FIS], bden = W.sgeo[G_BDEN];
    K.sg = uni(sg); K.cg = uni(cg); K.fis = uni(fis); K.omf = uni(1.0 - fis);
    K.nbs0 = uni(W.sgeo[G_NB0] * sg); K.nbs1 = uni(-W.sgeo[G_NB1] * sg); K.nbc = uni(W.sgeo[G_NB2] * cg);
    K.ibden = uni(bden > 0.0 ? 1.0 / bden : 0.0);
    K.dsc = uni(FX_INV * W.snorm[3] / W.snorm[2]);
    K.nd = __builtin_amdgcn_readfirstlane(T.dend[TCELLS - 1]);
    K.nsp = __builtin_amdgcn_readfirstlane(T.send[TCELLS - 1]);
    return K;
}

// the first entry of table t at or above x: the entries of the cells below
// x's all lie below it, those of the cells above all above (the cell index
// is monotone in position)
#ifdef LFG_PROFILE_PAIR
#define LONG_CNT(c, k) (c)[k]++
#else
#define LONG_CNT(c, k)
#endif
__device__ __forceinline__ int long_find(const LongTabs& W, const LongU& K, int t, double x, int* ctr = nullptr)
{
    const int f = long_cell(x, K.t0[t], K.gf[t]);
    const double* ep = W.epos + (t ? NE_W : 0);
    int i = f ? W.fend[t][f - 1] : 0;
    const int ie = W.fend[t][f];
    while (i < ie && ep[i] < x) {
        ++i;
        LONG_CNT(ctr, 0);
    }
    return i;
}

// eclipsed fraction of table t over window [lo, hi] (hi > lo): the integral
// of the covering weight over the window / its width (iw = FX_INV / (hi - lo))
__device__ __forceinline__ double long_window(const LongTabs& W, const LongU& K, int t, double lo, double hi,
                                              double iw, int* ctr = nullptr)
{
    if (!(hi > K.amin[t] && lo < K.bmax[t])) return 0.0;
    LONG_CNT(ctr, 2);
    const int base = t ? NE_W : 0, n = K.n[t];
    int i = long_find(W, K, t, lo, ctr);
    long long Cp = i ? W.ecb[base + i - 1] : 0;
    const long long C = Cp;
    double corr = 0.0;
    for (; i < n && W.epos[base + i] < hi; ++i) {
        const long long cb = W.ecb[base + i];
        corr = fma(double(cb - Cp), hi - W.epos[base + i], corr);
        Cp = cb;
        LONG_CNT(ctr, 1);
    }
    return fma(corr, iw, double(C) * FX_INV);
}

// table t at a point (zero-width window): the elements with a_k < ph < b_k
// (the starts below ph, the ends at or below it)
__device__ __forceinline__ double long_point(const LongTabs& W, const LongU& K, int t, double ph)
{
    if (!(ph > K.amin[t] && ph < K.bmax[t])) return 0.0;
    const int base = t ? NE_W : 0, n = K.n[t];
    int i = long_find(W, K, t, ph);
    long long Cp = i ? W.ecb[base + i - 1] : 0, C = Cp;
    for (; i < n && W.epos[base + i] == ph; ++i) {
        const long long cb = W.ecb[base + i];
        if (cb - Cp < 0) C += cb - Cp;
        Cp = cb;
    }
    return double(C) * FX_INV;
}

// WD and disc eclipsed fractions of a point's window (phase phc, half-width
// wk >= 0): the unique elements over [lo, hi] and, for their mirrors, over
// [-hi, -lo]
__device__ __forceinline__ double2 long_wd_disc(const LongTabs& W, const LongU& K, double phc, double wk,
                                               int* ctr = nullptr)
{
    if (wk > 0.0) {
        const double lo = phc - wk, hi = phc + wk, iw = FX_INV / (hi - lo);  // -lo - -hi = hi - lo exactly
        return make_double2(long_window(W, K, 0, lo, hi, iw, ctr) + long_window(W, K, 0, -hi, -lo, iw, ctr),
                            long_window(W, K, 1, lo, hi, iw, ctr) + long_window(W, K, 1, -hi, -lo, iw, ctr));
    }
    return make_double2(long_point(W, K, 0, phc) + long_point(W, K, 0, -phc),
                        long_point(W, K, 1, phc) + long_point(W, K, 1, -phc));
}

// sub_point with its donor cursor carried from point to point (SubCur): a
// point whose first sub-bin lies at or above the last one's phase walks on
// from there instead of a fresh lookup (a thread's run of sorted points);
// the line of sight is formed afresh at each point's first sub-bin
// the donor cursor runs two entries ahead: the next entry's position, code
// and tile vector (fixed point as a double: long_tables' step (g)) and the one after's
// position and code are in registers, their loads issued a crossing earlier
// -- a crossing applies the vector and moves the pipe on without waiting on LDS
// the donor sum V of the point phase, in fixed-point units but held as a
// double: the sub-bin sums take it without an int64 -> double conversion per
// sub-bin (12 instructions; 2.72 -> 2.91 M evals/s at config 5).  The sum
// over a thread's crossings rounds, ~1e-15 of V's scale, against exact int64
// (the tables' cell prefixes and the tiles' vectors stay exact)
using LongV = double;
struct SubCur {
    double ph, npos, n2pos;
    LongV nq[3];  // the next entry's tile vector (fixed point, before the mirror's signs)
    LongV vx, vy, vz;
    int cur, ncode, n2code;
    double dkw = -1.0, dk = 0.0;  // sub_point_quiet's Dirichlet kernel of width dkw
};

__device__ __forceinline__ void subcur_fill(const SubEntries& D, const double* sdq, int nd, SubCur& U)
{
    U.npos = U.cur < nd ? D.dpos[U.cur] : INFINITY;
    U.ncode = U.cur < nd ? D.dcode[U.cur] : 0;
    U.n2pos = U.cur + 1 < nd ? D.dpos[U.cur + 1] : INFINITY;
    U.n2code = U.cur + 1 < nd ? D.dcode[U.cur + 1] : 0;
    const LongV* dq = reinterpret_cast<const LongV*>(sdq + ((U.ncode >> 1) >> 2) * DON_STRIDE);
    U.nq[0] = dq[0]; U.nq[1] = dq[1]; U.nq[2] = dq[2];
}

#ifndef LFG_LW_BASE
#define LFG_LW_BASE 3
#endif
#ifndef LFG_LW_WD
#define LFG_LW_WD 2
#endif
#ifndef LFG_LW_SPOT
#define LFG_LW_SPOT 3
#endif
// a point's estimated cost in the LONG point phase (the partition of the
// points over the threads): windows in the WD/disc hulls walk the tables,
// those in the spot hull the spot entries at every sub-bin
__device__ __forceinline__ int long_weight(const LongU& K, double ph0, double w)
{
    const double phc = wrap_phase(ph0), wk = w < 0.0 ? 0.0 : w, lo = phc - wk, hi = phc + wk;
    bool wd = false;
    for (int t = 0; t < 2; ++t)
        wd = wd || (hi >= K.amin[t] && lo <= K.bmax[t]) || (-lo >= K.amin[t] && -hi <= K.bmax[t]);
    const bool sp = hi >= K.sa && lo <= K.sb;
    // weights from A/B runs at config 5 (wave ranges with interleaved lanes):
    // 5/3/1 2.39 M evals/s, 5/8/2 2.34, 5/1/1 2.31, uniform 2.36 (round 5);
    // round 6, with the quiet points in closed form: the spot hull's points
    // all take the sub-bin loop (LFG_LW_* to retune)
    return LFG_LW_BASE + (wd ? LFG_LW_WD : 0) + (sp ? LFG_LW_SPOT : 0);
}

// a crossing of entry cur: its vector into V (the mirror image's signs on the
// unique tile's fixed-point vector), then the pipe one entry on
__device__ __forceinline__ void subcur_cross(const SubEntries& D, const double* sdq, int nd, SubCur& U)
{
    const int code = U.ncode, mr = (code >> 1) & 3;
    const LongV qx = U.nq[0], qy = (mr & 1) ? -U.nq[1] : U.nq[1], qz = (mr & 2) ? -U.nq[2] : U.nq[2];
    if (code & 1) { U.vx -= qx; U.vy -= qy; U.vz -= qz; }
    else { U.vx += qx; U.vy += qy; U.vz += qz; }
    ++U.cur;
    U.npos = U.n2pos;
    U.ncode = U.n2code;
    const LongV* dq = reinterpret_cast<const LongV*>(sdq + ((U.ncode >> 1) >> 2) * DON_STRIDE);
    U.nq[0] = dq[0]; U.nq[1] = dq[1]; U.nq[2] = dq[2];
    U.n2pos = U.cur + 1 < nd ? D.dpos[U.cur + 1] : INFINITY;
    U.n2code = U.cur + 1 < nd ? D.dcode[U.cur + 1] : 0;
}

__device__ __forceinline__ double2 sub_point_c(const SubTables& T, const SubEntries& D, const double2* sab,
                                               const double* sbw, const double* sdq, const LongU& K, double ph0,
                                               double wk, int S, SubCur& U)
{
    const int nd = K.nd, nsp = K.nsp;
    const double h = wk * K.invS, ih = 0.5 / h;
    // the first sub-bin's line of sight and the turn per sub-bin
    const double phA = wrap_phase(ph0 - wk + h);
    const double4 eA = sincospi2_ool(2.0 * phA, 4.0 * h);
    double sbs = 0.0, srs1 = 0.0, srs2 = 0.0, sn = 0.0, cs = 1.0, rs = 0.0, rc = 1.0;
    long long Cs = 0;
    int scur = 0;
    bool sv = false;  // Cs / scur hold C at this sub-bin's lo
    for (int j = 0; j < S; ++j) {
        const double phn = wrap_phase(ph0 - wk + (2 * j + 1) * h);
        if (!(phn >= U.ph)) {  // a fresh lookup (the first point, a step back in phase)
            {  // sub_donor with the tiles' fixed-point vectors
                const int g = tcell(phn, T.dt0, T.dginv);
                U.vx = LongV(T.dpre[g][0]);
                U.vy = LongV(T.dpre[g][1]);
                U.vz = LongV(T.dpre[g][2]);
                int i = g ? T.dend[g - 1] : 0;
                for (const int ie = T.dend[g]; i < ie; ++i) {
                    const int code = D.dcode[i];
                    if (!donor_counted(D.dpos[i], code, phn)) break;
                    const int mr = (code >> 1) & 3;
                    const LongV* dq = reinterpret_cast<const LongV*>(sdq + ((code >> 1) >> 2) * DON_STRIDE);
                    const LongV qx = dq[0], qy = (mr & 1) ? -dq[1] : dq[1], qz = (mr & 2) ? -dq[2] : dq[2];
                    if (code & 1) { U.vx -= qx; U.vy -= qy; U.vz -= qz; }
                    else { U.vx += qx; U.vy += qy; U.vz += qz; }
                }
                U.cur = i;
            }
            subcur_fill(D, sdq, nd, U);
        } else {
            while (donor_counted(U.npos, U.ncode, phn))  // npos = inf past the last entry
                subcur_cross(D, sdq, nd, U);
        }
        if (j == 0 || !(phn >= U.ph)) {
            const double4 e4 = j == 0 ? eA : sincospi2_ool(2.0 * phn, 4.0 * h);  // the turn per sub-bin: 2 pi (2 h)
            sn = e4.x;
            cs = e4.y;
            rs = e4.z;
            rc = e4.w;
        } else {
            const double c2 = fma(cs, rc, -sn * rs);
            sn = fma(sn, rc, cs * rs);
            cs = c2;
        }
        U.ph = phn;
        // spot: as sub_point (the windows of a point abut; each point starts afresh)
        double ebj = 0.0;
        const double lo = phn - h, hi = phn + h;
        if (!(h > 0.0)) {
            ebj = sub_spot(T, sab, sbw, K.itb, lo, hi, K.sa, K.sb);
        } else if (hi > K.sa && lo < K.sb) {
            const double itb = K.itb;
            if (!sv) Cs = spot_C(T, sbw, itb, lo, scur);
            sv = true;
            long long Cn = Cs;
            double corr = 0.0;
            for (; scur < nsp && T.spos[scur] <= hi; ++scur) {
                const int code = T.scode[scur], k = code >> 1;
                const double wn = sbw[k] * itb;
                const double2 ab = sab[k];
                const long long Wq = to_fx(wn);
                if (!(code & 1)) {
                    Cn += Wq;
                    corr = fma(wn, fmin(ab.y, hi) - ab.x, corr);
                } else {
                    Cn -= Wq;
                    if (ab.x <= lo) corr = fma(-wn, hi - ab.y, corr);
                }
            }
            ebj = fma(corr, ih, double(Cs) * FX_INV);
            Cs = Cn;
        } else {
            sv = false;
        }
        // e = (s cos, -s sin, c) at the sub-phase: the donor term V . e and
        // the spot's beaming term fis + (1 - fis) max(nb . e, 0) (sg, cg folded in)
        srs1 = fma(cs, double(U.vx), fma(-sn, double(U.vy), srs1));
        srs2 += double(U.vz);
        sbs = fma(fma(K.omf, fmax(fma(K.nbs0, cs, fma(K.nbs1, sn, K.nbc)), 0.0), K.fis), 1.0 - ebj, sbs);
    }
    return make_double2(sbs * K.ibden, fma(K.sg, srs1, K.cg * srs2) * K.dsc);
}

// ---- LONG quiet points: sub_point_c's sums in closed form ----
// A point is quiet when, over its window [ph - w, ph + w] (S sub-bins):
//  * no donor entry is counted between its first and its last sub-bin (the
//    donor vector V is the same at every sub-bin),
//  * the window is off the spot's hull (no sub-bin sees the spot eclipsed),
//  * the beaming term b(phi) = nbs0 cos 2 pi phi + nbs1 sin 2 pi phi + nbc
//    keeps one sign (neither of its two zero crossings lies in the window),
//  * the window neither wraps at +-0.5 nor has a zero or NaN width.
// The sub-bins' lines of sight then sum to D (cos, sin)(2 pi ph) with the
// Dirichlet kernel D = sin(2 pi w) / sin(2 pi w / S) (the sub-bin centres lie
// symmetrically about ph, 2 h apart), every sum of sub_point_c is linear in
// them, and the point costs one sincospi instead of S sub-bin steps.
// (Config 5: ~80 % of the points; the sub-bin sums were 57 % of the point
// phase's VALU instructions.)  The others run sub_point_c.
struct LongB {          // the beaming term's zero crossings, per pair (uniform)
    double z0, z1;      // phases in [-0.5, 0.5)
    int any;            // 0: b keeps one sign over the orbit
};

__device__ __forceinline__ LongB long_beam_zeros(const LongU& K)
{
    LongB B{0.0, 0.0, 0};
    const double R = sqrt(K.nbs0 * K.nbs0 + K.nbs1 * K.nbs1);
    if (R > fabs(K.nbc)) {  // b = R cos(2 pi phi - t) + nbc crosses zero twice
        const double t = atan2(K.nbs1, K.nbs0), a = acos(-K.nbc / R);
        B.z0 = uni(wrap_phase((t - a) * (1.0 / TWO_PI)));
        B.z1 = uni(wrap_phase((t + a) * (1.0 / TWO_PI)));
        B.any = 1;
    }
    return B;
}

// sin(x) / x, |x| < 0.1: the series to x^10 (error < 2e-22)
__device__ __forceinline__ double sinc_small(double x)
{
    const double x2 = x * x;
    return fma(x2, fma(x2, fma(x2, fma(x2, fma(x2, -1.0 / 39916800.0, 1.0 / 362880.0), -1.0 / 5040.0),
                               1.0 / 120.0), -1.0 / 6.0), 1.0);
}

// true and the sums (as sub_point_c returns them) for a quiet point; false
// for the others.  Either way U is left at the point's first sub-bin, as
// sub_point_c's first step leaves it (the cursor walks on from there)
__device__ __forceinline__ bool sub_point_quiet(const SubTables& T, const SubEntries& D, const double* sbw,
                                                const double* sdq, const LongU& K, const LongB& B, double ph0,
                                                double wk, int S, SubCur& U, double2& out)
{
    const double h = wk * K.invS;
#ifdef LFG_COUNT_QUIET  // (diagnostic builds, with LFG_COUNT_ITERS: lfg_diag_iters) why points are not quiet
#define QCNT(k) atomicAdd(g_iter_dbg + 56 + (k), 1ull)
    QCNT(0);
#else
#define QCNT(k)
#endif
#ifdef LFG_ABL_QNONE  // (diagnostic builds) every point through the queue and sub_point_c
    return false;
#endif
    if (!(h > 0.0)) { QCNT(1); return false; }  // zero or NaN widths
    const double phc = wrap_phase(ph0), lo = phc - wk, hi = phc + wk;
    constexpr double EPS = 1e-9;   // margins on the phase tests (the sub-bin loop's own phases round)
#ifndef LFG_ABL_QALL  // (diagnostic builds: every point in closed form, a timing floor; wrong sums)
    if (!(lo > -0.5 + EPS && hi < 0.5 - EPS)) { QCNT(2); return false; }
    // the spot: the window off its hull, or inside it (then no spot entry may lie in the window)
    const bool inspot = hi + EPS > K.sa && lo - EPS < K.sb;
    if (inspot && !(lo - EPS > K.sa && hi + EPS < K.sb)) { QCNT(3); return false; }
    if (B.any && ((B.z0 > lo - EPS && B.z0 < hi + EPS) || (B.z1 > lo - EPS && B.z1 < hi + EPS))) { QCNT(4); return false; }
#endif
    // the donor vector at the first sub-bin, as sub_point_c finds it
    const int nd = K.nd;
    const double ph1 = wrap_phase(ph0 - wk + h);
    if (!(ph1 >= U.ph)) {
        const int g = tcell(ph1, T.dt0, T.dginv);
        U.vx = LongV(T.dpre[g][0]);
        U.vy = LongV(T.dpre[g][1]);
        U.vz = LongV(T.dpre[g][2]);
        int i = g ? T.dend[g - 1] : 0;
        for (const int ie = T.dend[g]; i < ie; ++i) {
            const int code = D.dcode[i];
            if (!donor_counted(D.dpos[i], code, ph1)) break;
            const int mr = (code >> 1) & 3;
            const LongV* dq = reinterpret_cast<const LongV*>(sdq + ((code >> 1) >> 2) * DON_STRIDE);
            const LongV qx = dq[0], qy = (mr & 1) ? -dq[1] : dq[1], qz = (mr & 2) ? -dq[2] : dq[2];
            if (code & 1) { U.vx -= qx; U.vy -= qy; U.vz -= qz; }
            else { U.vx += qx; U.vy += qy; U.vz += qz; }
        }
        U.cur = i;
        subcur_fill(D, sdq, nd, U);
    } else {
        while (donor_counted(U.npos, U.ncode, ph1)) subcur_cross(D, sdq, nd, U);
    }
    U.ph = ph1;
    const double phS = wrap_phase(ph0 - wk + (2 * S - 1) * h);  // the last sub-bin
#ifndef LFG_ABL_QALL
    // an entry counted by a later sub-bin moves V inside the window: the
    // sub-bin loop (a closed form per crossing, Dirichlet kernels of the
    // sub-bins after it, held more registers than the loop has: 25-42
    // spilled VGPRs, slower than the loop on 4 % of the points)
    if (donor_counted(U.npos, U.ncode, phS)) { QCNT(5); return false; }
#endif
    // the spot's covering weight at the first sub-bin's lo, as sub_point_c
    // takes it (spot_C); with no entry up to the last sub-bin's hi it is the
    // eclipsed fraction of every sub-bin
    double E = 0.0;
    if (inspot) {
        int cur;
        const long long C = spot_C(T, sbw, K.itb, ph1 - h, cur);
        if (cur < K.nsp && T.spos[cur] <= phS + h + EPS) { QCNT(3); return false; }
        E = double(C) * FX_INV;
    }
    // the Dirichlet kernel of the sub-bins' turn (2 pi 2 h per sub-bin)
    const double x = TWO_PI * wk, xs = TWO_PI * h;
    double Dk;
    if (wk == U.dkw) {  // the lane's last width (the cursor keeps its kernel): config 5 +1.5 %
        Dk = U.dk;
    } else {
        if (x < 0.1) {
            Dk = S * (sinc_small(x) / sinc_small(xs));
        } else {
            const double2 a = sincospi_ool(2.0 * wk), b = sincospi_ool(2.0 * h);
            Dk = a.x / b.x;
        }
        U.dkw = wk;
        U.dk = Dk;
    }
    // (sin, cos) at the window's centre, inlined: out of line while the
    // unit was compiled with machine LICM (inlined, its hoisted constants
    // spilled: config 5 -13 %); without the pass inlined is +0.7 %
    // (profiles/r06/long/ab_sincospi_inline_nolicm.txt)
    double esn, ecs;
    sincospi(2.0 * phc, &esn, &ecs);
    const double2 e = make_double2(esn, ecs);
    const double Scs = Dk * e.y, Ssn = Dk * e.x;
    const double srs1 = fma(Scs, double(U.vx), -Ssn * double(U.vy)), srs2 = S * double(U.vz);
    const double bc = fma(K.nbs0, e.y, fma(K.nbs1, e.x, K.nbc));  // b at the centre: its sign in the window
    const double sbs = (1.0 - E) * (bc > 0.0 ? fma(K.omf, fma(K.nbs0, Scs, fma(K.nbs1, Ssn, S * K.nbc)), S * K.fis)
                                             : S * K.fis);
    out = make_double2(sbs * K.ibden, fma(K.sg, srs1, K.cg * srs2) * K.dsc);
    QCNT(6);
    return true;
#undef QCNT
}

// the LONG tables from the element phase's results in LDS (all threads of
// the block, after the phase barrier; seven barriers).  abw: the WD/disc
// intervals by sweep slot; the spot (sab, sbw), the donor tiles (sdq), the
// disc ring weights (swt) and the spot / donor fixed-point totals (stot) as
// k_pair's point-major sinks leave them.  The tables must be zero (k_pair's
// prologue clears them).  Step (g) rewrites each unique donor tile's first
// three sdq words as its fixed-point vector in doubles (the point phase's form)
__device__ __forceinline__ void long_tables(LongTabs& W, SubTables& T, SubEntries& D, const double2* abw,
                                            const double2* sab, const double* sbw, double* sdq,
                                            const double* swt, const unsigned long long* stot, double ul, double itwd,
                                            long long (*spart)[LIKE_THREADS / 64], int tid)
{
    constexpr int nt = LIKE_THREADS, nw = LIKE_THREADS / 64;
    const int lane = tid & 63, wv = tid >> 6;
    // (a) hulls of the WD/disc and spot intervals, the donor |v| sum
    double amin[2] = {INFINITY, INFINITY}, bmax[2] = {-INFINITY, -INFINITY}, sa = INFINITY, sb = -INFINITY, vs = 0.0;
    for (int g = tid; g < NU_WDD; g += nt) {
        const double2 ab = abw[g];
        const int t = uitem(g) < U_WD ? 0 : 1;
        if (ab.x < ab.y) {
            amin[t] = fmin(amin[t], ab.x);
            bmax[t] = fmax(bmax[t], ab.y);
        }
    }
    if (tid < NBS && sab[tid].x < sab[tid].y) { sa = sab[tid].x; sb = sab[tid].y; }
    if (tid < U_DON)  // the four mirror images of a tile have the same |vx| + |vy| + |vz|
        vs = 4.0 * (fabs(sdq[tid * DON_STRIDE]) + fabs(sdq[tid * DON_STRIDE + 1]) + fabs(sdq[tid * DON_STRIDE + 2]));
    for (int t = 0; t < 2; ++t) {
        amin[t] = wave_min(amin[t]);
        bmax[t] = wave_max(bmax[t]);
    }
    sa = wave_min(sa); sb = wave_max(sb); vs = wave_sum(vs);
    if (lane == 0) {
        W.part[0][wv] = amin[0]; W.part[1][wv] = bmax[0]; W.part[2][wv] = sa; W.part[3][wv] = sb; W.part[4][wv] = vs;
        W.part[5][wv] = amin[1]; W.part[6][wv] = bmax[1];
    }
    __syncthreads();
    LONG_TSTAMP(0);
    amin[0] = amin[1] = INFINITY; bmax[0] = bmax[1] = -INFINITY; sa = INFINITY; sb = -INFINITY; vs = 0.0;
    for (int k = 0; k < nw; ++k) {  // every thread forms the block's values (no barrier for a broadcast)
        amin[0] = fmin(amin[0], W.part[0][k]); bmax[0] = fmax(bmax[0], W.part[1][k]);
        amin[1] = fmin(amin[1], W.part[5][k]); bmax[1] = fmax(bmax[1], W.part[6][k]);
        sa = fmin(sa, W.part[2][k]); sb = fmax(sb, W.part[3][k]); vs += W.part[4][k];
    }
    // the cells of table t over its own hull (the WD contacts crowd a narrower one)
    double t0[2], ginv[2];
    for (int t = 0; t < 2; ++t) {
        t0[t] = amin[t];
        ginv[t] = (bmax[t] > amin[t]) ? LONG_FC / (bmax[t] - amin[t]) : 0.0;
    }
    const double st0 = sa, sginv = (sb > sa) ? TCELLS / (sb - sa) : 0.0;
    constexpr double t0d = -0.5, t1d = 0.5, dginv = TCELLS;  // donor cells: the whole phase circle
    const double itb = 1.0 / (double(static_cast<long long>(stot[0])) * (FX_INV / PAIR_SPOT_S)), ivs = 1.0 / vs;
    if (tid == 0) {
        for (int t = 0; t < 2; ++t) { W.t0[t] = t0[t]; W.ginv[t] = ginv[t]; W.amin[t] = amin[t]; W.bmax[t] = bmax[t]; }
        W.snorm[0] = itb;
        W.snorm[1] = ivs;
        W.snorm[2] = double(static_cast<long long>(stot[1])) * (FX_INV / PAIR_DON_S);
        W.snorm[3] = vs;
        W.shull[0] = fmin(amin[0], amin[1]); W.shull[1] = fmax(bmax[0], bmax[1]); W.shull[2] = sa; W.shull[3] = sb;
        T.dt0 = t0d; T.dginv = dginv; T.st0 = st0; T.sginv = sginv;
    }
    // (b) counts and fixed-point sums per cell
    auto wd_entry = [&](int g, double2& ab, int& t, long long& q) {
        ab = abw[g];
        if (!(ab.x < ab.y)) return false;
        const int u = uitem(g), ir = uring(u);
        t = u < U_WD ? 0 : 1;
        q = to_fx(u < U_WD ? wd_ring_weight(ir, ul) * itwd : swt[ir - NWD_RINGS] * (1.0 / swt[NDISC_R]));
        return true;
    };
    for (int g = tid; g < NU_WDD; g += nt) {
        double2 ab;
        int t;
        long long q;
        if (!wd_entry(g, ab, t, q)) continue;
        (void)q;
        atomicAdd(&W.fend[t][long_cell(ab.x, t0[t], ginv[t])], 1);
        atomicAdd(&W.fend[t][long_cell(ab.y, t0[t], ginv[t])], 1);
    }
    {
        double p0, p1;
        bool in0, in1;
        int v0;
        lane_breakpoints(tid, sdq, sab, t0d, t1d, p0, p1, in0, in1, v0);
        long long c0[3] = {0, 0, 0};  // this lane's share of V0, summed per wave below
        if (tid >= nt - NDONOR) {
            long long q[3];
            donor_q(sdq, tid - (nt - NDONOR), ivs, q[0], q[1], q[2]);
            for (int k = 0; k < 3; ++k) c0[k] = v0 * q[k];
#pragma unroll
            for (int b = 0; b < 2; ++b) {
                if (!(b ? in1 : in0)) continue;
                const int g = tcell(b ? p1 : p0, t0d, dginv);
                atomicAdd(&T.dend[g], 1);
                for (int k = 0; k < 3; ++k)
                    atomicAdd(reinterpret_cast<unsigned long long*>(&T.dpre[g][k]),
                              static_cast<unsigned long long>(b ? -q[k] : q[k]));
            }
        } else if (in0) {
            const long long Wq = to_fx(sbw[tid] * itb);
#pragma unroll
            for (int b = 0; b < 2; ++b) {
                const int g = tcell(b ? p1 : p0, st0, sginv);
                atomicAdd(&T.send[g], 1);
                atomicAdd(reinterpret_cast<unsigned long long*>(&T.spre[g]), static_cast<unsigned long long>(b ? -Wq : Wq));
            }
        }
        // V0: the wave's sum, one atomic per component (half the donor lanes
        // add to these three words; per-lane atomics serialised on them)
        for (int k = 0; k < 3; ++k) {
            const long long w = wave_scan_incl(c0[k], lane);
            if (lane == 63 && w != 0)
                atomicAdd(reinterpret_cast<unsigned long long*>(&T.dv0[k]), static_cast<unsigned long long>(w));
        }
    }
    __syncthreads();
    LONG_TSTAMP(1);
    // (c) exclusive prefixes over the cells: each wave scans one whole array
    // (a lane its run of consecutive cells, then the wave's 64 sums), so no
    // part sums cross waves and one barrier ends the step
    static_assert(TCELLS == 4 * 64 && LONG_FC == 16 * 64 && nw == 8, "eight arrays, one per wave");
    (void)spart;
    {
        const int a = wv;  // 0, 1: the WD/disc cells; 2..7: the sub-bin tables' cells
        auto get = [&](int g) -> long long {
            switch (a) {
            case 0: return W.fend[0][g];
            case 1: return W.fend[1][g];
            case 2: return T.dend[g];
            case 3: return T.send[g];
            case 4: return T.dpre[g][0];
            case 5: return T.dpre[g][1];
            case 6: return T.dpre[g][2];
            default: return T.spre[g];
            }
        };
        auto set = [&](int g, long long x) {
            switch (a) {
            case 0: W.fend[0][g] = int(x); break;
            case 1: W.fend[1][g] = int(x); break;
            case 2: T.dend[g] = int(x); break;
            case 3: T.send[g] = int(x); break;
            case 4: T.dpre[g][0] = x + T.dv0[0]; break;
            case 5: T.dpre[g][1] = x + T.dv0[1]; break;
            case 6: T.dpre[g][2] = x + T.dv0[2]; break;
            default: T.spre[g] = x; break;
            }
        };
        if (a < 2) {  // 16 cells per lane, int counts: loaded once, in one round trip
            constexpr int PER = LONG_FC / 64;
            int* f = W.fend[a] + PER * lane;
            int c[PER];
            int own = 0;
#pragma unroll
            for (int j = 0; j < PER; ++j) {
                c[j] = f[j];
                own += c[j];
            }
            int run = int(wave_scan_incl(own, lane)) - own;
#pragma unroll
            for (int j = 0; j < PER; ++j) {
                f[j] = run;
                run += c[j];
            }
        } else {
            constexpr int PER = TCELLS / 64;
            const int g0 = PER * lane;
            long long c[PER];
            long long own = 0;
#pragma unroll
            for (int j = 0; j < PER; ++j) {
                c[j] = get(g0 + j);
                own += c[j];
            }
            long long run = wave_scan_incl(own, lane) - own;
#pragma unroll
            for (int j = 0; j < PER; ++j) {
                set(g0 + j, run);
                run += c[j];
            }
        }
    }
    __syncthreads();
    LONG_TSTAMP(2);
    // (d) the entries into cell order; afterwards cend / dend / send hold the cell ends
    for (int g = tid; g < NU_WDD; g += nt) {
        double2 ab;
        int t;
        long long q;
        if (!wd_entry(g, ab, t, q)) continue;
        const int base = t ? NE_W : 0;
        const int ia = atomicAdd(&W.fend[t][long_cell(ab.x, t0[t], ginv[t])], 1);
        W.epos[base + ia] = ab.x;
        W.ecb[base + ia] = q;
        const int ib = atomicAdd(&W.fend[t][long_cell(ab.y, t0[t], ginv[t])], 1);
        W.epos[base + ib] = ab.y;
        W.ecb[base + ib] = -q;
    }
    {
        double p0, p1;
        bool in0, in1;
        int v0;
        lane_breakpoints(tid, sdq, sab, t0d, t1d, p0, p1, in0, in1, v0);
        const int base = (tid >= nt - NDONOR) ? 2 * (tid - (nt - NDONOR)) : 2 * tid;
#pragma unroll
        for (int b = 0; b < 2; ++b) {
            if (!(b ? in1 : in0)) continue;
            const double pos = b ? p1 : p0;
            if (tid >= nt - NDONOR) {
                const int slot = atomicAdd(&T.dend[tcell(pos, t0d, dginv)], 1);
                D.dpos[slot] = pos;
                D.dcode[slot] = base + b;
            } else {
                const int slot = atomicAdd(&T.send[tcell(pos, st0, sginv)], 1);
                T.spos[slot] = pos;
                T.scode[slot] = base + b;
            }
        }
    }
    __syncthreads();
    LONG_TSTAMP(3);
    // (e) every cell's entries in order: each entry counts the entries of its
    // cell that sort before it and moves to that rank (all entries at once;
    // an insertion sort per cell took O(n^2) steps in the cells where the WD
    // contacts crowd).  WD/disc by (position, weight), donor by position with
    // an end before a start (sub_point's cursor), spot by (position, code):
    // total orders, so the tables (and long_window's double sums) do not
    // depend on the atomics' slot order
    {
        constexpr int RW = (NE_W + NE_D + nt - 1) / nt, RD = (TD_MAX + nt - 1) / nt;
        double wp[RW], dp[RD], sp = 0.0;
        long long wq[RW];
        int wslot[RW], dc[RD], dslot[RD], sc = 0, sslot = -1;
#pragma unroll
        for (int r = 0; r < RW; ++r) {
            wslot[r] = -1;
            wp[r] = 0.0;
            wq[r] = 0;
            const int i = tid + r * nt, t = i < NE_W ? 0 : 1, base = t ? NE_W : 0, li = i - base;
            if (i >= NE_W + NE_D || li >= W.fend[t][LONG_FC - 1]) continue;
            const double p = W.epos[i];
            const long long q = W.ecb[i];
            const int g = long_cell(p, t0[t], ginv[t]), c0 = g ? W.fend[t][g - 1] : 0, c1 = W.fend[t][g];
            int rank = 0;
#pragma unroll 4
            for (int k = c0; k < c1; ++k) {
                const double pk = W.epos[base + k];
                const long long qk = W.ecb[base + k];
                rank += (pk < p || (pk == p && (qk < q || (qk == q && k < li)))) ? 1 : 0;
            }
            wp[r] = p;
            wq[r] = q;
            wslot[r] = base + c0 + rank;
        }
        const int ndn = T.dend[TCELLS - 1], nsn = T.send[TCELLS - 1];
#pragma unroll
        for (int r = 0; r < RD; ++r) {
            dslot[r] = -1;
            dp[r] = 0.0;
            dc[r] = 0;
            const int i = tid + r * nt;
            if (i >= ndn) continue;
            const double p = D.dpos[i];
            const int c = D.dcode[i], g = tcell(p, t0d, dginv), c0 = g ? T.dend[g - 1] : 0, c1 = T.dend[g];
            int rank = 0;
#pragma unroll 4
            for (int k = c0; k < c1; ++k) {
                const double pk = D.dpos[k];
                const int ck = D.dcode[k];
                rank += (pk < p || (pk == p && ((ck & 1) > (c & 1) || ((ck & 1) == (c & 1) && (ck < c || (ck == c && k < i))))))
                            ? 1 : 0;
            }
            dp[r] = p;
            dc[r] = c;
            dslot[r] = c0 + rank;
        }
        if (tid < nsn) {
            const double p = T.spos[tid];
            const int c = T.scode[tid], g = tcell(p, st0, sginv), c0 = g ? T.send[g - 1] : 0, c1 = T.send[g];
            int rank = 0;
#pragma unroll 4
            for (int k = c0; k < c1; ++k) {
                const double pk = T.spos[k];
                const int ck = T.scode[k];
                rank += (pk < p || (pk == p && (ck < c || (ck == c && k < tid)))) ? 1 : 0;
            }
            sp = p;
            sc = c;
            sslot = c0 + rank;
        }
        __syncthreads();
    LONG_TSTAMP(4);
#pragma unroll
        for (int r = 0; r < RW; ++r)
            if (wslot[r] >= 0) {
                W.epos[wslot[r]] = wp[r];
                W.ecb[wslot[r]] = wq[r];
            }
#pragma unroll
        for (int r = 0; r < RD; ++r)
            if (dslot[r] >= 0) {
                D.dpos[dslot[r]] = dp[r];
                D.dcode[dslot[r]] = dc[r];
            }
        if (sslot >= 0) {
            T.spos[sslot] = sp;
            T.scode[sslot] = sc;
        }
    }
    __syncthreads();
    LONG_TSTAMP(5);
    // (f) C just after each sorted WD/disc entry: the running sum of the
    // weights in table order (exact int64), a wave per table, a lane a run
    if (wv < 2) {
        const int t = wv, n = W.fend[t][LONG_FC - 1], B = (n + 63) >> 6, k0 = min(lane * B, n), k1 = min(k0 + B, n);
        long long* q = W.ecb + (t ? NE_W : 0);
        long long own = 0;
        for (int k = k0; k < k1; ++k) own += q[k];
        long long run = wave_scan_incl(own, lane) - own;
        for (int k = k0; k < k1; ++k) {
            run += q[k];
            q[k] = run;
        }
    }
    // (g) each unique donor tile's vector in fixed point (held as doubles),
    // in place of its raw components (the point phase adds them at its donor
    // crossings; a mirror image's components differ in sign only, and to_fx
    // is odd)
    if (tid >= 128 && tid < 128 + U_DON) {  // waves 2.. (0 and 1 run (f))
        double* dq = sdq + (tid - 128) * DON_STRIDE;
        const long long q0 = to_fx(dq[0] * ivs), q1 = to_fx(dq[1] * ivs), q2 = to_fx(dq[2] * ivs);
        LongV* dl = reinterpret_cast<LongV*>(dq);
        dl[0] = q0;
        dl[1] = q1;
        dl[2] = q2;
    }
    __syncthreads();
    LONG_TSTAMP(6);
}

// GP (GP trees, MODE 2 of k_lnlike): instead of chi^2 the residuals, each
// point's e^{-lam dx} and changepoint block go to the workspace for
// k_gp_like, and a walker that tripped the changepoint cache rule has its
// distance solved here (k_gp_dcp's ten limb points, on wave 0's lanes 32..)
// LONG: eclipses longer than a tile and sub-binned exposures (the LONG
// tables above, long_tables / long_wd_disc / sub_point): the element phase
// keeps the point-major sinks, and after the phase barrier the tables are
// built and every wave evaluates a cost-balanced range of the points
template <bool GP, bool FOLD = false, bool LONG = false>
__global__ __launch_bounds__(LIKE_THREADS, LIKE_MINW) void k_pair(PairArgs A)
{
    static_assert(!(GP && LONG), "GP trees keep the one-tile layout or the two kernels");
    const LikeArgs& L = A.L;
    const ElemSpec& X = A.X;
    __shared__ double swt[NDISC_R + 1];           // disc ring weights and the disc total (prologue)
    __shared__ double sbw[NBS];
    __shared__ double2 sab[NBS];
    __shared__ double sdq[U_DON * DON_STRIDE];
    __shared__ double sacc1[3];
    __shared__ TileBufs TA;
    __shared__ double sph[LIKE_TILE];
    // the second WD/disc difference arrays and the point-phase cells; or,
    // for a tile that goes point-major, the WD/disc intervals
    __shared__ union PairU_ {
        struct {
            unsigned long long X[2][LIKE_TILE + 1];
            int scp[LIKE_NC + 1];
        } s;
        double2 ab[NU_WDD];
    } SU;
    __shared__ unsigned long long sacc[6][LIKE_TILE + 1];
    __shared__ unsigned long long stot[2];
    __shared__ long long spart[6][LIKE_THREADS / 64];
    __shared__ double red[LIKE_THREADS / 64];
    __shared__ int sflagw[LIKE_THREADS / 64];
    __shared__ int sflag[1];
    __shared__ int sjob;
    __shared__ double sq[ACC_LDS];
    __shared__ double sy[LIKE_TILE], sye[LIKE_TILE];
    // LONG only (the one-tile instantiations reference none of these)
    __shared__ LongTabs LT;
    __shared__ SubTables LST;
    __shared__ SubEntries LSE;
    __shared__ double2 Lab[NU_WDD];
    __shared__ long long lspart[10][LIKE_THREADS / 64];

    constexpr int nt = LIKE_THREADS, nw = LIKE_THREADS / 64;
    // the prologue's arguments in one batch of scalar loads (PairHot)
    const PairHot H = kernarg_copy(&opaque_kernargs<PairArgs>()->hot);
    const int pair = blockIdx.x, npairs = H.npairs;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
#ifdef LFG_ABL_EMPTY  // (diagnostic builds) the launch alone: traffic and instructions of an empty k_pair
    if (pair >= 0) return;
#endif
    PAIR_STAMP(0, tid == 0);
#ifdef LFG_PROFILE_PAIR
    if (tid == 0 && blockIdx.x < 4096) {
        unsigned hw, xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        g_pair_t[14][blockIdx.x] = hw;
        g_pair_t[18][blockIdx.x] = xcc;
    }
#endif
    const int E = H.E;
    const int w = (E == 1) ? pair : pair / E, e = (E == 1) ? 0 : pair - w * E;
    const int nwk = npairs / E;  // walkers of the batch
    const bool offs = H.off && E > 1;
    const int o0 = offs ? H.off[e] : 0;
    const int n = offs ? H.off[e + 1] - o0 : H.N;

    // the point loads the windows need, issued first: they overlap the
    // candidate chain below (own point, predecessor, first and last)
    const bool own = !LONG && tid < n;
    const int m = n;
    const int pl = own ? tid : 0;
    const GDbl xe = H.x + o0;
    double xw_own = 0.0, xw_prv = 0.0, xw_0 = 0.0, xw_1 = 0.0;
    double ww_own = 0.0, ww_prv = 0.0, ww_0 = 0.0, ww_1 = 0.0;
    if (!LONG && n > 0) {
        xw_own = xe[pl];
        xw_prv = xe[pl > 0 ? pl - 1 : 0];
        xw_0 = xe[0];
        xw_1 = xe[n - 1];
    }
    PAIR_STAMP(20, tid == 0 && n != -7);
    if (!LONG && H.w && n > 0) {
        const GDbl we = H.w + o0;
        ww_own = we[pl];
        ww_prv = we[pl > 0 ? pl - 1 : 0];
        ww_0 = we[0];
        ww_1 = we[n - 1];
    }
    // ---- prologue: the pair's candidate (speculative setup) or standard
    // slots.  Only what the phase barrier B0 waits for is done here (the
    // barrier waits for every wave's outstanding memory operations): both
    // candidates' per-pair words are loaded alongside the selection chain
    // (jk -> accflag), and the copies into the standard slots, the snapshot
    // and the acceptance's prefetch follow B0 (wave 7's first task)
    const double* G;
    int st0, bst, cand = 0;
    double lpr = 0.0, zf = 0.0, rpr, phi0;
    if (H.jk) {
        const size_t c0 = size_t(pair), c1 = size_t(npairs) + pair;
        const int sa0 = H.statusC[c0], sa1 = H.statusC[c1], sb0 = H.bstatusC[c0], sb1 = H.bstatusC[c1];
        const double lp0 = H.priorC[w], lp1 = H.priorC[size_t(nwk) + w];
        const KDbl G0 = H.geoC + c0 * LFG_NGEO;
        const KDbl G1 = H.geoC + c1 * LFG_NGEO;
        const double rp0 = G0[G_RPRIOR] + G0[G_RPRIOR_BS], rp1 = G1[G_RPRIOR] + G1[G_RPRIOR_BS];
        const double ph0 = G0[G_PHI0], ph1 = G1[G_PHI0];
        const int jw = int(__umulhi(draw(H.jseed, H.jstep, H.jhalf, 0, H.jlo + w).z, unsigned(H.jns)));
        PAIR_STAMP(21, tid == 0 && jw != -7);
        if (FOLD)  // the partner's pending verdict: accepted unless NaN
            cand = __builtin_amdgcn_readfirstlane(int(!isnan(H.fv[__builtin_amdgcn_readfirstlane(jw)])));
        else
            cand = __builtin_amdgcn_readfirstlane(H.accflag[__builtin_amdgcn_readfirstlane(jw)]);
        PAIR_STAMP(10, tid == 0 && cand >= 0);
        G = (const double*)(cand ? G1 : G0);
        st0 = cand ? sa1 : sa0;
        bst = cand ? sb1 : sb0;
        lpr = cand ? lp1 : lp0;
        rpr = cand ? rp1 : rp0;
        phi0 = cand ? ph1 : ph0;
    } else {
        G = (const double*)(H.geo + size_t(pair) * LFG_NGEO);
        st0 = H.status[pair];
        bst = H.bstatus[pair];
        if (H.prior) lpr = H.prior[w];
        rpr = G[G_RPRIOR] + G[G_RPRIOR_BS];
        phi0 = G[G_PHI0];
    }
    // the record through the constant address space: its reads are scalar
    // loads into SGPRs, as in k_elements (the launch writes no record it
    // reads: the standard slot it copies into is not G when X.jk is set)
    const CGeo Gc = (CGeo)(G);
    const int stp = (st0 != ST_OK) ? st0 : bst;  // MODEL_SPEC 6 order: setup failures first
    const bool prej = H.prior && !(lpr + rpr > -INFINITY);  // prior_rejects
    const int st = (stp == ST_OK && prej) ? -1 : stp;  // -1: prior-rejected, straight to the -inf finish
    const bool acc1 = L.pos && E == 1;
    // this thread's point (one tile: m = n points): window and phase into LDS,
    // its sortedness against the predecessor, and the cells it fills of the
    // two phase indices (windows' lo, point phases), formed from its own and
    // its predecessor's windows, so that no barrier separates them
    int fl = 0;
    if (own) {
        double ph, lo, hi, hw;
        pair_window(xw_own, ww_own, phi0, ph, lo, hi, hw);
        PAIR_STAMP(11, tid == 0 && ph != 12345.0);
        TA.lo[tid] = lo;
        TA.hi[tid] = hi;
        TA.iw[tid] = 1.0 / (2.0 * hw);
        sph[tid] = ph;
        double php = 0.0, lop = 0.0, hip = 0.0, hwp, ph0, lo0, hi0, hw0, ph1, lo1, hi1, hw1;
        if (tid) pair_window(xw_prv, ww_prv, phi0, php, lop, hip, hwp);
        pair_window(xw_0, ww_0, phi0, ph0, lo0, hi0, hw0);
        pair_window(xw_1, ww_1, phi0, ph1, lo1, hi1, hw1);
        fl = (hw >= 0.0) ? 0 : 4;  // negative or NaN widths: point-major
        if (tid && (lo < lop || hi < hip || ph < php)) fl = 4;
        pair_cells(TA.cell, tid, m, lop, lo, lo0, lo1);
        pair_cells(SU.s.scp, tid, m, php, ph, ph0, ph1);
    }
    {
        const int wf = wave_or4(fl);
        if (lane == 0) sflagw[wv] = wf;
    }
    if constexpr (LONG) {  // the tables' counters and sums; the record for sub_point's LDS reads
        for (int i = tid; i < 2 * LONG_FC; i += nt) (&LT.fend[0][0])[i] = 0;
        if (tid < TCELLS) {
            LST.dpre[tid][0] = LST.dpre[tid][1] = LST.dpre[tid][2] = 0;
            LST.spre[tid] = 0;
            LST.dend[tid] = LST.send[tid] = 0;
        } else if (tid < TCELLS + 3) {
            LST.dv0[tid - TCELLS] = 0;
        } else if (tid >= nt - LFG_NGEO) {
            LT.sgeo[tid - (nt - LFG_NGEO)] = G[tid - (nt - LFG_NGEO)];
        }
    } else {
        for (int i = 0; i < 6; ++i) sacc[i][tid] = 0ull;
        SU.s.X[0][tid] = 0ull;
        SU.s.X[1][tid] = 0ull;
    }
    if (tid == 0) {
        if constexpr (!LONG) {
            for (int i = 0; i < 6; ++i) sacc[i][nt] = 0ull;
            SU.s.X[0][nt] = 0ull;
            SU.s.X[1][nt] = 0ull;
        }
        stot[0] = stot[1] = 0ull;
        sjob = (X.nspec > 0 && pair < 2 * A.nbc) ? 8 : 9;
    }
    PAIR_STAMP(19, tid == 0);
    // the disc ring weights (MODEL_SPEC 5.2): wave 7's lanes 0..NDISC_R
    if (st == ST_OK && wv == 7 && lane <= NDISC_R) ring_weight_lane(lane, Gc, swt);
    __syncthreads();  // B0: windows, cells, flags, zeroed sums, ring weights, sjob
    PAIR_STAMP(16, tid == 0);

    bool dir = LONG;  // LONG: the point-major sinks always
    if (!LONG)
        for (int k = 0; k < nw; ++k) dir = dir || sflagw[k] != 0;
    // this thread's data point (read after the phase barrier), the GP
    // filter's transition factor of the point (k_gp_like)
    if (own) {
        sy[tid] = L.y[o0 + tid];
        if (!GP) sye[tid] = L.ye[o0 + tid];
        if (GP) {
            const double xp = L.x[o0 + tid], dx = xp - (tid ? L.x[o0 + tid - 1] : xp);
            L.gpx[size_t(pair) * L.N + tid] = exp(-(Gc[G_GP_LAM] * dx));
        }
    }
    // GP: the changepoint distance is solved in this launch (the cache rule
    // tripped, G_GP_OK = 2); wave 0 then owns the slot's G_GP_DCP / G_GP_OK
    const bool pend = GP && st == ST_OK && Gc[G_GP_OK] == 2.0;
    // FOLD: rows w, w + nwk, ... of each half (wave 7's lanes): the snapshot
    // of this half's (final in this launch) for the next launch's speculative
    // lanes, and the pending verdicts of the partner half's, an accepted row
    // becoming its proposal (k_accept_regen's arithmetic)
    auto fold_rows = [&](int l) {
        const int ns = A.jns, h = L.half, hp = 1 - h, nd = L.ndim, r = (ns + nwk - 1) / nwk;
        for (int f = l; f < r * nd; f += 64) {
            const int k = f / nd, d = f - k * nd, j = w + k * nwk;
            if (j < ns) A.fsnap[size_t(j) * nd + d] = A.fpos[(size_t(h) * ns + j) * nd + d];
        }
        if (A.fv) {
            for (int f = l; f < r * nd; f += 64) {
                const int k = f / nd, d = f - k * nd, j = w + k * nwk;
                if (j >= ns) continue;
                const double v = A.fv[j];
                const uint4 rr = draw(L.seed, A.fstep, hp, 0, j);
                if (isnan(v)) continue;
                const double zr = (A.fa - 1.0) * u53(rr.x, rr.y) + 1.0, z = zr * zr / A.fa;
                const double* cj = A.fpos + (size_t(h) * ns + int(__umulhi(rr.z, unsigned(ns)))) * nd;
                double* row = A.fpos + (size_t(hp) * ns + j) * nd;
                row[d] = fma(row[d] - cj[d], z, cj[d]);
                if (d == 0) {
                    A.flnp[size_t(hp) * ns + j] = v;
                    if (A.fnacc) A.fnacc[size_t(hp) * ns + j] += 1;
                }
            }
        }
    };
    if (wv == 7) {
        // housekeeping off the prologue's critical path: the selected candidate
        // into the standard slots (API readers, k_combine_walkers, k_gp_like),
        // the pair status, the snapshot of the other half's rows for the next
        // launch's speculative lanes, the fused acceptance's prefetch
        const int l = lane;
        if (X.jk) {
            const size_t cw = size_t(cand) * nwk + w;
            double* Gd = const_cast<double*>(L.geo) + size_t(pair) * LFG_NGEO;
            // (a pending changepoint's two words are wave 0's: one writer each)
            if (l < LFG_NGEO && !(pend && (l == G_GP_DCP || l == G_GP_OK))) Gd[l] = G[l];
            if (l == 48) X.bstatus[pair] = bst;
            if (e == 0) {
                const double* qc = X.qC + cw * X.ndim;
                for (int d = l; d < X.ndim; d += 64) X.q[size_t(w) * X.ndim + d] = qc[d];
                if (l == 49) X.prior[w] = lpr;
                if (l == 50) X.zf[w] = X.zfC[cw];
            }
        }
        if (l == 51) const_cast<int*>(L.status)[pair] = stp;
        if (A.snap_dst && e == 0)
            for (int d = l; d < L.ndim; d += 64) A.snap_dst[size_t(w) * L.ndim + d] = A.snap_src[size_t(w) * L.ndim + d];
        if (FOLD) {
            fold_rows(l);
            if (l == 63) {  // the verdict's draw, zf and old ln_prob
                const int ns = A.jns, h = L.half;
                const uint4 r1 = draw(L.seed, L.step, h, 1, A.jlo + w);
                sacc1[0] = log(u53(r1.x, r1.y));
                sacc1[1] = X.jk ? X.zfC[size_t(cand) * nwk + w] : L.zfac[w];
                sacc1[2] = A.flnp[size_t(h) * ns + A.jlo + w];
            }
        }
        if (acc1) {
            const double* qsrc = X.jk ? X.qC + (size_t(cand) * nwk + w) * X.ndim : L.qprop + size_t(w) * L.ndim;
            for (int d = l; d < L.ndim && d < ACC_LDS; d += 64) sq[d] = qsrc[d];
            if (l == 63) {
                const uint4 r = draw(L.seed, L.step, L.half, 1, pair);
                sacc1[0] = log(u53(r.x, r.y));
                sacc1[1] = X.jk ? X.zfC[size_t(cand) * nwk + w] : L.zfac[w];
                sacc1[2] = L.lnp_ens[L.half * npairs + pair];
            }
        }
    }
    // ---- element phase: 16 jobs.  Job 0: this block's speculative setup
    // lanes of the next half; jobs 1..15: the 15 item chunks, longest first
    // (kJobChunk).  Wave w takes job w, then grabs the next free job from
    // sjob, at most twice (8 waves x 3 >= 16): the waves finish together
    // whatever the pair's Newton counts (a static two-chunk split waited
    // ~8 us at the phase barrier on its slowest wave)
    // the speculative lanes fill whole waves: wave 0 of the first 2 nbc blocks
    // (a few lanes in every block's wave 0 cost each of them the lanes' whole
    // instruction stream: SIMD issue slots of ~10x the work)
    const bool specblk = X.nspec > 0 && pair < 2 * A.nbc;
    if (wv == 0 && specblk) {
        PAIR_PRIO(3);
        if (lane < A.spl) {
            // candidate uniform per block: X.S[c] stays in scalar registers
            const int c = pair < A.nbc ? 0 : 1;
            const int t = (pair - c * A.nbc) * A.spl + lane;
            if (t < X.nspec) {  // the SetupArgs loaded here, not at the kernel's entry (opaque_kernargs)
                const SetupArgs Sc = kernarg_copy(&opaque_kernargs<PairArgs>()->X.S[__builtin_amdgcn_readfirstlane(c)]);
                setup_any<FOLD>(Sc, t);
            }
#ifdef LFG_PROFILE_PAIR
            if (lane == 0 && blockIdx.x < 4096) {
                const int np = X.S[0].W * X.S[0].E;
                g_pair_t[17][blockIdx.x] = t >= X.nspec ? 9 : (t < np ? 0 : (t < np + X.S[0].W ? 1 : 2));
            }
#endif
        }
    }
    __shared__ double sdcp;
    if (GP) {
        // the changepoint distance: the cache's, or (cache rule tripped,
        // G_GP_OK = 2) dist_cp = (dphi + phi4 - phi3) / 2 from ten limb
        // points' egress phases (CVModel.py:561-570; k_gp_dcp's solve)
        if (pend && wv == 0 && lane >= 32 && lane < 32 + DCP_LANES) {
            const int k = lane - 32;
            bool ok = Gc[G_GP_RWD] > 0.0;
            double b = NAN;
            if (ok && k < DCP_NTHETA) {
                const Roche R{Gc[G_Q], Gc[G_CA], Gc[G_CB], Gc[G_MU], Gc[G_XL1], Gc[G_PL1], Gc[G_RS], Gc[G_RS2]};
                const double s = Gc[G_S], c = Gc[G_C], r1 = Gc[G_GP_RWD];
                double dphi_c;
                if (findphi_fast(R, Gc[G_INC], dphi_c) == ST_OK) {
                    double sth, cth, sp, cp, a;
                    sincos(PI * dphi_c, &sth, &cth);
                    sincos(TWO_PI * k / DCP_NTHETA, &sp, &cp);
                    if (!element_interval(R, r1 * (cp * sth - sp * c * cth), r1 * (cp * cth + sp * c * sth),
                                          r1 * (sp * s), s, c, eggleton(R.q), a, b))
                        b = NAN;
                }
            }
            double lo = isnan(b) ? INFINITY : b, hi = isnan(b) ? -INFINITY : b;
            for (int off = DCP_LANES / 2; off > 0; off >>= 1) {
                lo = fmin(lo, __shfl_xor(lo, off, DCP_LANES));
                hi = fmax(hi, __shfl_xor(hi, off, DCP_LANES));
            }
            if (k == 0) {
                ok = ok && lo <= hi;  // no eclipsed limb point: wdphases fails
                const double d = ok ? (Gc[G_GP_DPHI] + (hi - lo)) / 2.0 : NAN;
                double* Gd = const_cast<double*>(L.geo) + size_t(pair) * LFG_NGEO;  // the standard slot
                Gd[G_GP_DCP] = d;
                Gd[G_GP_OK] = ok ? 1.0 : 0.0;
                sdcp = d;
            }
        } else if (!pend && tid == 0) {
            sdcp = Gc[G_GP_DCP];
        }
    }
    if (st == ST_OK && m > 0) {
        const double ul = Gc[G_ULIMB];
        const double itwd = 1.0 / (TWO_PI * ((1.0 - ul) * 0.5 + ul / 3.0));
        auto make_sink = [&]() {
            if constexpr (LONG)  // the point-major sinks only (no tile arrays in this instantiation)
                return PairSink{true, lane, PhaseIndex{}, PhaseIndex{}, nullptr, nullptr, nullptr, nullptr, stot, swt,
                                ul, itwd, Gc[G_S], Gc[G_C], Lab, sab, sbw, sdq};
            else
                return PairSink{dir, lane, phase_index(TA.lo, TA.cell, m), phase_index(sph, SU.s.scp, m), TA.hi,
                                TA.iw, sacc, SU.s.X, stot, swt, ul, itwd, Gc[G_S], Gc[G_C], SU.ab, sab, sbw, sdq};
        };
        PairSink K = make_sink();
        // chunk c: items v = 64 c + lane of one region each (c < 11: WD and
        // disc; 11, 12: spot; 13, 14: donor), so that no wave runs two
        // regions' code one after the other
        auto chunk = [&](int j) {
            const int c = kJobChunk[j - 1];
            constexpr int V_BS = U_WD + U_DISC, V_DON = V_BS + U_BS;
            const int r0 = c < 11 ? 0 : (c < 13 ? V_BS : V_DON), c0 = c < 11 ? 0 : (c < 13 ? 11 : 13);
            const int r1 = c < 11 ? V_BS : (c < 13 ? V_DON : NUNIQ);
            const int v = r0 + (c - c0) * 64 + lane < r1 ? r0 + (c - c0) * 64 + lane : -1;
#ifdef LFG_PROFILE_PAIR
            const bool rec = lane == 0 && blockIdx.x < 4096;
            if (rec) g_pair_j[0][c][blockIdx.x] = __builtin_amdgcn_s_memrealtime();
            K.mk = rec ? &g_pair_j[1][c][blockIdx.x] : nullptr;
#endif
            if (v >= 0) element_item_to(v, Gc, K);
#ifdef LFG_PROFILE_PAIR
            if (rec) g_pair_j[2][c][blockIdx.x] = __builtin_amdgcn_s_memrealtime();
#endif
        };
        auto grab = [&]() {
            int j = 0;
            if (lane == 0) j = atomicAdd(&sjob, 1);
            return __builtin_amdgcn_readfirstlane(j);  // every lane is active: the first is lane 0
        };
        // straight-line calls, not a loop: a loop's invariant constants (the
        // transcendental polynomials) were hoisted and spilled to scratch
        // (a block without speculative lanes starts wave w on job w + 1)
        // wave priority falls with each job a wave starts, so that the two
        // workgroups of a CU advance together (the issue arbiter otherwise
        // favours the older workgroup's waves)
#ifndef LFG_ABL_ELEM  // (diagnostic builds) no element jobs: the prologue, setup lanes and likelihood alone
        PAIR_PRIO(3);
        if (!specblk) chunk(wv + 1);
        else if (wv > 0) chunk(wv);
        int j = grab();
        PAIR_PRIO(2);
        if (j < 16) chunk(j);
        j = grab();
        PAIR_PRIO(1);
        if (j < 16) chunk(j);
        PAIR_PRIO(0);
#else
        (void)chunk;
        (void)grab;
#endif
        K.flush();
    }
    static_assert(11 * 64 >= U_WD + U_DISC && 10 * 64 < U_WD + U_DISC, "11 chunks of WD/disc");
    static_assert(U_BS > 64 && U_BS <= 128 && U_DON > 64 && U_DON <= 128, "two spot and two donor chunks");
    PAIR_STAMP(1 + wv, lane == 0);
    __syncthreads();  // B1: the sums (or the tables)
    PAIR_STAMP(9, tid == 0);

    if (st != ST_OK) {
        if (GP) return;  // k_gp_like sees the status (or the prior) and finishes the pair
        if (FOLD) {  // ln_prob -inf (combine_walker's value): rejected unless the old one is -inf too
            if (tid == 0) {
                L.lle[pair] = -INFINITY;
                if (L.lnp) L.lnp[pair] = -INFINITY;
                const double v = -INFINITY;
                A.vout[pair] = (sacc1[0] < sacc1[1] + v - sacc1[2]) ? v : NAN;
            }
            return;
        }
        if (tid == 0) L.lle[pair] = -INFINITY;
        finish_walker(L, pair, tid, acc1, sq, sacc1, sflag);
        return;
    }
    // ---- each point's flux and chi^2 (GP: residual, changepoint block)
    double chi = 0.0;
#ifdef LFG_ABL_LIKE  // (diagnostic builds) no likelihood phase: chi^2 = 0
    if (false) {
    } else
#endif
    if constexpr (LONG) {
        // the pair's tables, then this wave's range of the points (lanes interleaved)
        const double ul = Gc[G_ULIMB];
        long_tables(LT, LST, LSE, Lab, sab, sbw, sdq, swt, stot, ul, 1.0 / (TWO_PI * ((1.0 - ul) * 0.5 + ul / 3.0)),
                    lspart, tid);
        PAIR_STAMP(12, tid == 0);
        const int S = L.nsub;
        const double* xe = L.x + o0;
        const double* we = L.w ? L.w + o0 : nullptr;
        const double* ye = L.y + o0;
        const double* ee = L.ye + o0;
        const double fwd = Gc[G_WDF], fds = Gc[G_DF], fsp = Gc[G_SF], frs = Gc[G_RSF];
#ifdef LFG_PROFILE_PAIR
        unsigned long long tl_wd = 0, tl_sub = 0;
        int lctr[3] = {0, 0, 0};
#endif
        SubCur SC{INFINITY, INFINITY, INFINITY, {0, 0, 0}, LongV(0), LongV(0), LongV(0), 0, 0, 0
        };
        const LongU KU = long_uniforms(LT, LST, S);
        const double fspS = uni(fsp / S), frsS = uni(frs / S);
        // each wave a contiguous range of the points, its lanes interleaved
        // (a thread's points follow one another 64 apart, and its donor
        // cursor walks on from point to point).  A dynamic queue of 4-point
        // chunks balanced the eclipse's points over the waves but doubled the
        // total (every chunk starts with fresh lookups; and its chi^2 order
        // was not fixed)
        // The runs are cut where the running estimated cost (long_weight, in
        // index order) passes equal shares: a thread in the eclipse takes
        // fewer points, and the waves end together (the eclipse's waves took
        // 2-3 times the others' time with equal counts)
        // The points in blocks of 64 (one step of a wave's loop): each block's
        // estimated cost (long_weight, one coalesced pass, a wave per block),
        // their prefix, and each wave takes the blocks where the running cost
        // passes its eighth of the total; its lanes interleaved, so every step
        // reads 64 consecutive points and the lanes of a wave stand at
        // neighbouring phases (the same branches of the lookups)
        constexpr int LAB_INTS = int(NU_WDD * sizeof(double2) / sizeof(int));  // the spent interval table, as ints
        int p0, p1;
        {
            constexpr int nw = LIKE_THREADS / 64;
            const int nch = (n + 63) >> 6;
            int* cw = reinterpret_cast<int*>(Lab);  // the WD/disc intervals are spent
            int b0, b1;
            if (nch + 1 <= LAB_INTS - 8 * 128) {  // (the point phase's queues take the last 8 x 128 ints)
                for (int c = wv; c < nch; c += nw) {
                    const int p = c * 64 + lane;
                    int wt = p < n ? long_weight(KU, xe[p] - phi0, we ? we[p] : 0.0) : 0;
                    for (int off = 32; off > 0; off >>= 1) wt += __shfl_xor(wt, off);
                    if (lane == 0) cw[c] = wt;
                }
                __syncthreads();
                if (wv == 0) {  // exclusive prefix over the blocks, in place; the total at nch
                    const int B = (nch + 63) >> 6, q0 = min(lane * B, nch), q1 = min(q0 + B, nch);
                    long long own = 0;
                    for (int c = q0; c < q1; ++c) own += cw[c];
                    long long run = wave_scan_incl(own, lane) - own;
                    for (int c = q0; c < q1; ++c) {
                        const int v = cw[c];
                        cw[c] = int(run);
                        run += v;
                    }
                    if (lane == 63) cw[nch] = int(run);
                }
                __syncthreads();
                const long long T = cw[nch];
                auto first = [&](int w) {  // the first block whose cost before it reaches w / nw of the total
                    const long long tgt = (T * w) / nw;
                    int a = 0, b = nch;
                    while (a < b) {
                        const int mid = (a + b) >> 1;
                        if (cw[mid] >= tgt) b = mid;
                        else a = mid + 1;
                    }
                    return a;
                };
                b0 = wv ? first(wv) : 0;
                b1 = wv + 1 < nw ? first(wv + 1) : nch;
            } else {  // more blocks than the spent LDS holds: equal shares
                b0 = nch * wv / nw;
                b1 = nch * (wv + 1) / nw;
            }
            p0 = __builtin_amdgcn_readfirstlane(b0) * 64 + lane;
            p1 = min(__builtin_amdgcn_readfirstlane(b1) * 64, n);
        }
        // Pass 1 over the wave's points (steps of 64, lanes interleaved): the
        // WD/disc windows, and the sub-bin sums in closed form where the point
        // is quiet (sub_point_quiet).  The other points go to the wave's queue
        // (a ring of LQ_CAP indices in the spent interval table, in index
        // order); each time it holds 64 they run sub_point_c with every lane
        // busy (pass 2), and the rest after the last step.  Every point's
        // chi^2 term is added once, by the lane that finishes it.
        constexpr int LQ_CAP = 128;
        int* const lq = reinterpret_cast<int*>(Lab) + (LAB_INTS - 8 * LQ_CAP) + wv * LQ_CAP;
        const LongB KB = long_beam_zeros(KU);
        int qhead = 0, qtail = 0;  // uniform over the wave
        auto full_point = [&](int p) {  // sub_point_c's path for point p
            const double xp = xe[p], wp = we ? we[p] : 0.0, yp = ye[p], ep = ee[p];
            const double wk = wp < 0.0 ? 0.0 : wp;  // MODEL_SPEC 3 (NaN stays NaN)
            const double ph0 = xp - phi0, phc = wrap_phase(ph0);
            const double2 f2 = long_wd_disc(LT, KU, phc, wk);
            const double2 r2 = sub_point_c(LST, LSE, sab, sbw, sdq, KU, ph0, wk, S, SC);
            const double f = isnan(wk) ? NAN : fwd * (1.0 - f2.x) + fds * (1.0 - f2.y) + fspS * r2.x + frsS * r2.y;
            const double rr = (yp - f) / ep;
            chi += isnan(f) ? INFINITY : rr * rr;
        };
        auto run_queue = [&](int cnt) {  // pass 2: cnt <= 64 queued points, one per lane
            if (lane < cnt) full_point(lq[(qhead + lane) & (LQ_CAP - 1)]);
            qhead += cnt;
            // the queued points lie behind pass 1 (the cursor's fresh lookup
            // took them), and walking the cursor back up from there re-crossed
            // every entry in between: pass 1's next point looks afresh (one cell)
            SC.ph = INFINITY;
        };
        const int pw0 = p0 - lane;  // the wave's first point (uniform)
        // the next step's phase and width, in flight during this one
        double xn = p0 < p1 ? xe[p0] : 0.0, wn = (p0 < p1 && we) ? we[p0] : 0.0;
        for (int base = pw0; base < p1; base += 64) {
            const int p = base + lane;
            bool defer = false;
            if (p < p1) {
#ifdef LFG_ABL_GLOAD  // (diagnostic builds) no global loads in the point loop: a synthetic grid
                const double xp = -0.3 + p * 6.0006e-5, wp = 3.0003e-5, yp = 1.0, ep = 0.004;
                (void)xn; (void)wn;
#else
                const double xp = xn, wp = wn, yp = ye[p], ep = ee[p];
                if (p + 64 < p1) {
                    xn = xe[p + 64];
                    wn = we ? we[p + 64] : 0.0;
                }
#endif
                const double wk = wp < 0.0 ? 0.0 : wp;  // MODEL_SPEC 3 (NaN stays NaN)
                const double ph0 = xp - phi0, phc = wrap_phase(ph0);
                double2 r2;
#ifdef LFG_ABL_LSUB
                r2 = make_double2(phc * 1e-30, wk * 1e-30);
                const bool quiet = true;
#else
                const bool quiet = sub_point_quiet(LST, LSE, sbw, sdq, KU, KB, ph0, wk, S, SC, r2);
#endif
                if (quiet) {
#ifdef LFG_ABL_LWD
                    const double2 f2 = make_double2(phc * 1e-30, wk * 1e-30);
#else
                    const double2 f2 = long_wd_disc(LT, KU, phc, wk);
#endif
                    // k_lnlike's sum, term for term (MODEL_SPEC 3: a NaN width, a NaN flux)
                    const double f = fwd * (1.0 - f2.x) + fds * (1.0 - f2.y) + fspS * r2.x + frsS * r2.y;
                    const double rr = (yp - f) / ep;
                    chi += isnan(f) ? INFINITY : rr * rr;
                } else {
                    defer = true;
                }
            }
            const unsigned long long m = __ballot(defer);
            if (defer)
                lq[(qtail + __builtin_amdgcn_mbcnt_hi(unsigned(m >> 32), __builtin_amdgcn_mbcnt_lo(unsigned(m), 0u))) &
                   (LQ_CAP - 1)] = p;
            qtail += __popcll(m);
#ifdef LFG_PROFILE_PAIR  // (diagnostic builds) the block's quiet and queued points
            const unsigned long long mact = __ballot(p < p1);
            if (lane == 0 && blockIdx.x < 4096) {
                atomicAdd(&g_pair_t[22][blockIdx.x], (unsigned long long)__popcll(mact & ~m));
                atomicAdd(&g_pair_t[23][blockIdx.x], (unsigned long long)__popcll(m));
            }
#endif
            if (qtail - qhead >= 64) run_queue(64);
        }
        if (qtail > qhead) run_queue(qtail - qhead);
        PAIR_WSTAMP(0);  // (diagnostic builds) this wave's points done
#ifdef LFG_PROFILE_PAIR
        {
            unsigned long long a = tl_wd, b = tl_sub;
            for (int off = 32; off > 0; off >>= 1) {
                a = max(a, (unsigned long long)__shfl_xor((long long)a, off));
                b = max(b, (unsigned long long)__shfl_xor((long long)b, off));
            }
            if (lane == 0 && blockIdx.x < 4096) { g_pair_w[1][wv][blockIdx.x] = a; g_pair_w[2][wv][blockIdx.x] = b; }
            // walk steps / window entries / windows in a hull: the wave's max lane (16 bits each)
            int c0 = lctr[0], c1 = lctr[1], c2 = lctr[2];
            for (int off = 32; off > 0; off >>= 1) {
                c0 = max(c0, __shfl_xor(c0, off));
                c1 = max(c1, __shfl_xor(c1, off));
                c2 = max(c2, __shfl_xor(c2, off));
            }
            if (lane == 0 && blockIdx.x < 4096)
                g_pair_w[3][wv][blockIdx.x] = (unsigned long long)(c0 & 0xffff) | ((unsigned long long)(c1 & 0xffff) << 16) |
                                              ((unsigned long long)(c2 & 0xffff) << 32);
        }
#endif
    } else if (m > 0) {
        const double s = Gc[G_S], c = Gc[G_C], ul = Gc[G_ULIMB];
        const double twd = TWO_PI * ((1.0 - ul) * 0.5 + ul / 3.0);  // 2 pi [F(1) - F(0)]
        const double wspot = double(static_cast<long long>(stot[0])) * (FX_INV / PAIR_SPOT_S);
        const double dn = double(static_cast<long long>(stot[1])) * (FX_INV / PAIR_DON_S);
        const double phc = own ? sph[tid] : 0.0;
        double fw = 0.0, fd = 0.0, eb = 0.0, R3 = 0.0, R4 = 0.0, R5 = 0.0;
        if (dir) {
            if (own) {
                const double wk = L.w ? L.w[o0 + tid] : 0.0;
                const double2 f2 = pair_direct_wd_disc(SU.ab, ul, swt, phc, wk, twd, swt[NDISC_R]);
                // MODEL_SPEC 3: a NaN width gives a NaN flux (such a tile is
                // always point-major: its window fails the sortedness test)
                fw = isnan(wk) ? NAN : f2.x;
                fd = f2.y;
                eb = direct_spot(sab, sbw, phc, wk, 1.0 / wspot);
            }
        } else {
            long long r[6] = {0, 0, 0, 0, 0, 0};
            block_scan<6>(sacc, spart, tid, r, SU.s.X);
            PAIR_STAMP(12, tid == 0);
            fw = double(r[0]) * FX_INV;
            fd = double(r[1]) * FX_INV;
            eb = double(r[2]) * (FX_INV / PAIR_SPOT_S) / wspot;
            R3 = double(r[3]);
            R4 = double(r[4]);
            R5 = double(r[5]);
        }
        const double2 scp2 = sincospi_ool(2.0 * phc);
        const double e0 = s * scp2.y, e1 = -s * scp2.x;
        double D = 0.0;
        if (!dir) D = (e0 * R3 + e1 * R4 + c * R5) * (FX_INV / PAIR_DON_S);
        else if (own) D = direct_donor(sdq, e0, e1, c);
        double beam = 0.0;
        const double bden = Gc[G_BDEN], fis = Gc[G_FIS];
        if (bden > 0.0) beam = (fis + (1.0 - fis) * fmax(Gc[G_NB0] * e0 + Gc[G_NB1] * e1 + Gc[G_NB2] * c, 0.0)) / bden;
        const double sbs = beam * (1.0 - eb), srs = D / dn;
        if (own) {
            const double f = Gc[G_WDF] * (1.0 - fw) + Gc[G_DF] * (1.0 - fd) + Gc[G_SF] * sbs + Gc[G_RSF] * srs;
            if (GP) {
                const size_t q = size_t(pair) * L.N + tid;
                L.res[q] = sy[tid] - f;
                L.gpb[q] = gp_block(L.x[o0 + tid], L.gp_ecl[2 * e], L.gp_ecl[2 * e + 1], sdcp, Gc[G_PHI0]);
            } else {
                const double rr = (sy[tid] - f) / sye[tid];
                chi = isnan(f) ? INFINITY : rr * rr;
            }
        }
    }
    if (GP) return;  // k_gp_like forms ln_like from the residuals
    chi = wave_sum(chi);
    if (lane == 0) red[wv] = chi;
    __syncthreads();
    // the finish (finish_walker's arithmetic) from the values thread 0
    // holds: its ln_like, and the prior terms of the candidate it selected
    // (what the standard slots hold now), without a barrier and a global
    // round trip for each
    if (tid == 0) {
        double tot = 0.0;
        for (int i = 0; i < nw; ++i) tot += red[i];
        const double lp = lpr + Gc[G_RPRIOR] + Gc[G_RPRIOR_BS];  // finish_walker's sum, term for term
        const double lle = isfinite(lp) ? -0.5 * tot : -INFINITY;
        L.lle[pair] = lle;
        PAIR_STAMP(13, true);
        if (FOLD) {  // this pair's verdict for the exchange (k_accept_regen's test)
            const double v = isfinite(lp) ? lp + lle : -INFINITY;
            if (L.lnp) L.lnp[pair] = v;
            A.vout[pair] = (sacc1[0] < sacc1[1] + v - sacc1[2]) ? v : NAN;
        } else if (!acc1) {
            combine_after(L, pair);
        } else {
            const int wg = L.half * L.npairs + pair;
            const double v = isfinite(lp) ? lp + lle : -INFINITY;
            if (L.lnp) L.lnp[pair] = v;
            const bool a = sacc1[0] < sacc1[1] + v - sacc1[2];
            if (a) {
                L.lnp_ens[wg] = v;
                if (L.naccept) L.naccept[wg] += 1;
            }
            sflag[0] = a ? 1 : 0;
            if (L.accflag) L.accflag[pair] = a ? 1 : 0;
        }
    }
    if (acc1) {
        __syncthreads();
        const int wg = L.half * L.npairs + pair;
        if (sflag[0] && tid < L.ndim)
            L.pos[size_t(wg) * L.ndim + tid] = (tid < ACC_LDS) ? sq[tid] : L.qprop[size_t(pair) * L.ndim + tid];
    }
    PAIR_STAMP(15, tid == 0);
}

// -------------------------------------------------------------- k_gp_dcp
// GP trees: the changepoint distance of pairs whose walker tripped the
// cache rule (k_setup marked them G_GP_OK = 2): dist_cp = (dphi + phi4 -
// phi3) / 2 with phi3 / phi4 = wdphases(q, i, rwd, 10) (CVModel.py:561-570,
// MODEL_SPEC 10.2-10.3).  16 lanes per pair, lane k < 10 solves limb point k
// (the nested eclipse solver), min / max by shuffles; other pairs return at
// once.  Runs after k_elements (the pair's record is in the standard slot)
// and before k_lnlike<2>, which reads G_GP_DCP.
#ifndef LFG_NOLICM_TU  // (lfg_pair_split.hip compiles k_pair only)
__global__ __launch_bounds__(64) void k_gp_dcp(double* __restrict__ geo, const int* __restrict__ status, int npairs)
{
    const int pair = int(blockIdx.x) * (64 / DCP_LANES) + int(threadIdx.x) / DCP_LANES;
    const int k = int(threadIdx.x) % DCP_LANES;
    if (pair >= npairs) return;
    double* G = geo + size_t(pair) * LFG_NGEO;
    if (G[G_GP_OK] != 2.0) return;  // uniform over the pair's 16 lanes
    bool ok = status[pair] == ST_OK && G[G_GP_RWD] > 0.0;
    double b = NAN;
    if (ok && k < DCP_NTHETA) {
        const Roche R{G[G_Q], G[G_CA], G[G_CB], G[G_MU], G[G_XL1], G[G_PL1], G[G_RS], G[G_RS2]};
        const double s = G[G_S], c = G[G_C], r1 = G[G_GP_RWD];
        double dphi_c;
        if (findphi_fast(R, G[G_INC], dphi_c) == ST_OK) {  // as wdphases: the egress phase of the WD centre
            double sth, cth, sp, cp, a;
            sincos(PI * dphi_c, &sth, &cth);
            sincos(TWO_PI * k / DCP_NTHETA, &sp, &cp);
            if (!element_interval(R, r1 * (cp * sth - sp * c * cth), r1 * (cp * cth + sp * c * sth), r1 * (sp * s), s,
                                  c, eggleton(R.q), a, b))
                b = NAN;
        }
    }
    double lo = isnan(b) ? INFINITY : b, hi = isnan(b) ? -INFINITY : b;
    for (int off = DCP_LANES / 2; off > 0; off >>= 1) {
        lo = fmin(lo, __shfl_xor(lo, off, DCP_LANES));
        hi = fmax(hi, __shfl_xor(hi, off, DCP_LANES));
    }
    if (k == 0) {
        ok = ok && lo <= hi;  // no eclipsed limb point: wdphases fails
        G[G_GP_DCP] = ok ? (G[G_GP_DPHI] + (hi - lo)) / 2.0 : NAN;
        G[G_GP_OK] = ok ? 1.0 : 0.0;
    }
}
#endif

// -------------------------------------------------------------- k_gp_like
// GP trees (MODEL_SPEC 10.4): the Kalman filter over each pair's residuals
// (k_lnlike<2> wrote them), parallel in time.  The recursion is serial in
// the points and its dependent chain (D -> S -> 1/S -> D, ~14 FP64 ops of
// 32-48 cycles each for a lone wave, tools/lat_probe.hip) set the time when
// one lane or one quad ran a pair's 300 points.  So a pair's points are cut
// into GP_SEG segments, each filtered by a quad of lanes at once:
//  * element pass (per segment s, its quad): the filter conditioned on the
//    unknown prior state x_s at the segment's first point -- the mean is
//    A x_s + c, the covariance starts at 0, and the segment's data give
//    exp(-1/2 x_s^T J x_s + eta^T x_s - kappa / 2).  Lane r owns row r of
//    D (= P - P_inf), column r of A, c_r, row r of J and eta_r; rows and
//    gains travel by DPP quad permutes.
//  * combine (one lane per pair, serial over the segments, 4x4 algebra):
//    integrate x_s against its prior N(mu, Sigma), add the segment's ln_like,
//    carry the filtered end state (A mu_post + c, A Sigma_post A^T + P_end)
//    through the gap's transition (and a block start) to the next segment.
// tests/gp_kalman.py:gp_lnlike_segments restates it; equal to the dense
// likelihood to ~1e-15.
//
// Coordinates: Jordan form of each 2-state block.  With K = [[lam, 1],
// [-lam^2, -lam]] (K^2 = 0), Phi(d) = e^{-u} (I + d K); z = (x0, lam x0 + x1)
// turns it into e^{-u} T, T = [[1, d], [0, 1]].  The observation is still z0
// and P_inf = a [[1, lam], [lam, 2 lam^2]] per block.
//
// Then ln_like = sum of the segments' and, as k_lnlike does, ln_prob and the
// acceptance of the walker once its last eclipse is in.  Pairs of a wave
// take one eclipse of consecutive walkers (equal point counts, shared x / ye).
constexpr int GP_BLOCK = 64;
#ifndef LFG_GP_CHUNK
#define LFG_GP_CHUNK 8
#endif
constexpr int GP_CHUNK = LFG_GP_CHUNK;
constexpr int GP_SEG = 8;                     // segments per pair
constexpr int GP_LPP = 4 * GP_SEG;            // lanes per pair: a quad per segment
constexpr int GP_PAIRS = GP_BLOCK / GP_LPP;   // pairs per wave
constexpr int GP_EL = 16;                     // doubles of a lane's element row in LDS

// v of lane (quad base + PERM's selector for this lane): DPP quad_perm on both halves
template <int PERM>
__device__ __forceinline__ double quad_perm(double v)
{
    // every lane of a quad is a valid source: no "old" value (update_dpp's
    // copy of it cost a v_mov per permute)
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_mov_dpp(static_cast<int>(b), PERM, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_mov_dpp(static_cast<int>(b >> 32), PERM, 0xf, 0xf, false);
    return __longlong_as_double((static_cast<long long>(hi) << 32) | static_cast<unsigned>(lo));
}
constexpr int QP_NEXT = 0xF5;  // [1, 1, 3, 3]: the odd row of each block
constexpr int QP_B0 = 0x00, QP_B1 = 0x55, QP_B2 = 0xAA, QP_B3 = 0xFF;  // broadcast lane 0 / 1 / 2 / 3

// P_inf (z coordinates) entry (i, j) of a pair: blocks ain, aout
__device__ __forceinline__ double gp_pinf(int i, int j, double ain, double aout, double lam)
{
    if ((i >> 1) != (j >> 1)) return 0.0;
    const double a = (i >> 1) ? aout : ain;
    const int k = (i & 1) + (j & 1);
    return k == 0 ? a : (k == 1 ? a * lam : 2.0 * a * lam * lam);
}

#ifndef LFG_NOLICM_TU  // (lfg_pair_split.hip compiles k_pair only)
__global__ __launch_bounds__(GP_BLOCK) __attribute__((amdgpu_waves_per_eu(2))) void k_gp_like(LikeArgs L)
{
    __shared__ double sel[GP_PAIRS][GP_SEG][4][GP_EL];
    __shared__ double sgap[GP_PAIRS][GP_SEG][4];  // the gap into each segment (the combine's transition)
    const int nw = L.npairs / L.E, nwb = (nw + GP_PAIRS - 1) / GP_PAIRS;
    const int e = int(blockIdx.x) / nwb;
    const int lane = int(threadIdx.x), pp = lane / GP_LPP, sg = (lane / 4) % GP_SEG, r = lane & 3;
    const int w = (int(blockIdx.x) - e * nwb) * GP_PAIRS + pp;
    const bool live = w < nw;
    const int pair = live ? w * L.E + e : 0;
    const int o0 = L.off ? L.off[e] : 0;
    const int n = L.off ? L.off[e + 1] - o0 : L.N;
    const double* G = L.geo + size_t(pair) * LFG_NGEO;
    const bool run = live && L.status[pair] == ST_OK && G[G_GP_OK] != 0.0 &&
                     !(L.prior && prior_rejects(L.prior[pair / L.E], G));
    const double ain = G[G_GP_AIN], aout = G[G_GP_AOUT], lam = G[G_GP_LAM];
    const double* res = L.res + size_t(pair) * L.N;
    const double* gx = L.gpx + size_t(pair) * L.N;
    const int* gb = L.gpb + size_t(pair) * L.N;
    const double* xs = L.x + o0;
    const double* yes = L.ye + o0;
    if (run) {
        // ---- element pass: segment sg of the pair, lane r of its quad
        const int i0 = (n * sg) / GP_SEG, i1 = (n * (sg + 1)) / GP_SEG;
        const double pc0 = gp_pinf(r, 0, ain, aout, lam), pc2 = gp_pinf(r, 2, ain, aout, lam);
        const bool even = (r & 1) == 0, hrow = r >= 2;
        // P starts at 0: D = -P_inf; A = I; c = 0
        double D0 = -gp_pinf(r, 0, ain, aout, lam), D1 = -gp_pinf(r, 1, ain, aout, lam);
        double D2 = -gp_pinf(r, 2, ain, aout, lam), D3 = -gp_pinf(r, 3, ain, aout, lam);
        double A0 = r == 0 ? 1.0 : 0.0, A1 = r == 1 ? 1.0 : 0.0, A2 = r == 2 ? 1.0 : 0.0, A3 = r == 3 ? 1.0 : 0.0;
        double c = 0.0, J0 = 0.0, J1 = 0.0, J2 = 0.0, J3 = 0.0, eta = 0.0;
        double q2 = 0.0, lnS = 0.0, xprev = (i0 > 0 && i0 < n) ? xs[i0 - 1] : 0.0;
        int bp = (i0 > 0 && i0 < n) ? gb[i0 - 1] : -1;
        bool bad = false;
        double cx[GP_CHUNK], cy[GP_CHUNK], cr[GP_CHUNK], ce[GP_CHUNK];
        int cb[GP_CHUNK];
        auto fetch = [&](int p0) {
#pragma unroll
            for (int k = 0; k < GP_CHUNK; ++k) {
                const int q = min(p0 + k, i1 - 1);
                cx[k] = xs[q];
                cy[k] = yes[q];
                cr[k] = res[q];
                ce[k] = gx[q];
                cb[k] = gb[q];
            }
        };
        if (i1 > i0) fetch(i0);
        if (i1 > i0) {  // the gap into this segment (the combine's transition): lane r of the quad
            // writes entry r (d, e^{-lam d}, block start), read back in the combine
            // instead of a dependent global load per segment (k_gp_like 42.0 -> 40.4 us,
            // profiles/r06/ab_gp_combine.txt)
            const bool fr = cb[0] >= 0 && cb[0] != bp;
            sgap[pp][sg][r] = r == 0 ? cx[0] - xprev : (r == 1 ? ce[0] : (fr ? 1.0 : 0.0));
        }
        for (int p0 = i0; p0 < i1; p0 += GP_CHUNK) {
            double dk[GP_CHUNK], ek[GP_CHUNK], Ek[GP_CHUNK], ye2[GP_CHUNK], rv[GP_CHUNK];
            int blk[GP_CHUNK];
#pragma unroll
            for (int k = 0; k < GP_CHUNK; ++k) {
                const double dd = cx[k] - (k ? cx[k - 1] : xprev);
                dk[k] = dd;
                ek[k] = ce[k];  // e^{-lam dd}, formed in k_lnlike<2>
                Ek[k] = ce[k] * ce[k];
                ye2[k] = cy[k] * cy[k];
                rv[k] = cr[k];
                blk[k] = cb[k];
                bad = bad || (p0 + k < i1 && p0 + k > 0 && !(dd >= 0.0)) || (p0 + k < i1 && !isfinite(cr[k]));
            }
            xprev = cx[GP_CHUNK - 1];
            if (p0 + GP_CHUNK < i1) fetch(p0 + GP_CHUNK);  // in flight during the recursion
            double prodS = 1.0;  // one log per chunk (S ~ ye^2: eight factors stay far from underflow)
#pragma unroll
            for (int k = 0; k < GP_CHUNK; ++k) {
                if (p0 + k >= i1) break;
                // a new block: its process starts stationary and independent
                // of x_s: rows / columns 2, 3 of D and rows 2, 3 of A and c
                // restart at 0 (zero scales in the prediction; the block
                // start at the segment's first point is the combine's)
                const bool fresh = blk[k] >= 0 && blk[k] != bp;
                bp = blk[k];
                if (p0 + k > i0) {  // predict: D <- e^{-2u} T D T^T, A <- e^{-u} T A, c <- e^{-u} T c
                    const double d = dk[k], dr = even ? d : 0.0, ex = ek[k];
                    const double kr = (fresh && hrow) ? 0.0 : 1.0, kc = fresh ? 0.0 : 1.0;
                    const double n0 = quad_perm<QP_NEXT>(D0), n1 = quad_perm<QP_NEXT>(D1);
                    const double n2 = quad_perm<QP_NEXT>(D2), n3 = quad_perm<QP_NEXT>(D3);
                    const double nc = quad_perm<QP_NEXT>(c);
                    const double t0 = fma(dr, n0, D0), t1 = fma(dr, n1, D1);
                    const double t2 = fma(dr, n2, D2), t3 = fma(dr, n3, D3);
                    const double Eg = Ek[k] * kr, Eh = Eg * kc;
                    D0 = Eg * fma(d, t1, t0);
                    D1 = Eg * t1;
                    D2 = Eh * fma(d, t3, t2);
                    D3 = Eh * t3;
                    const double exh = ex * kc;
                    A0 = ex * fma(d, A1, A0);
                    A1 = ex * A1;
                    A2 = exh * fma(d, A3, A2);
                    A3 = exh * A3;
                    c = (ex * kr) * fma(dr, nc, c);
                }
                const double a = (blk[k] >= 0) ? 1.0 : 0.0;
                // k = P h, h = (1, 0, a, 0), P = D + P_inf: this row's gain
                const double kk = (D0 + pc0) + a * (D2 + pc2);
                const double k0 = quad_perm<QP_B0>(kk), k1 = quad_perm<QP_B1>(kk);
                const double k2 = quad_perm<QP_B2>(kk), k3 = quad_perm<QP_B3>(kk);
                const double c0 = quad_perm<QP_B0>(c), c2 = quad_perm<QP_B2>(c);
                const double hA = fma(a, A2, A0);  // (h^T A)_r
                const double h0 = quad_perm<QP_B0>(hA), h1 = quad_perm<QP_B1>(hA);
                const double h2 = quad_perm<QP_B2>(hA), h3 = quad_perm<QP_B3>(hA);
                const double S = fma(a, k2, k0) + ye2[k];
                const double vt = rv[k] - fma(a, c2, c0);
                const double iS = rcp_fast(S);  // v_rcp_f64 (2.5e-8) + one Newton step: ~1 ulp
                bad = bad || !(S > 0.0) || !isfinite(vt);
                q2 = fma(vt * vt, iS, q2);
                prodS *= S;
                const double g = hA * iS;
                J0 = fma(g, h0, J0);
                J1 = fma(g, h1, J1);
                J2 = fma(g, h2, J2);
                J3 = fma(g, h3, J3);
                eta = fma(g, vt, eta);
                c = fma(kk, vt * iS, c);
                A0 = fma(-k0, g, A0);
                A1 = fma(-k1, g, A1);
                A2 = fma(-k2, g, A2);
                A3 = fma(-k3, g, A3);
                const double j = kk * iS;
                D0 = fma(-j, k0, D0);
                D1 = fma(-j, k1, D1);
                D2 = fma(-j, k2, D2);
                D3 = fma(-j, k3, D3);
            }
            lnS += log(prodS);
        }
        double* o = sel[pp][sg][r];
        o[0] = D0; o[1] = D1; o[2] = D2; o[3] = D3;
        o[4] = A0; o[5] = A1; o[6] = A2; o[7] = A3;
        o[8] = c;
        o[9] = J0; o[10] = J1; o[11] = J2; o[12] = J3;
        o[13] = eta;
        o[14] = q2 + lnS;
        o[15] = bad ? 1.0 : 0.0;
    }
    __syncthreads();
    // ---- combine: serial over the segments, the 4x4 algebra spread over 16
    // lanes of the pair (lane (ci, cj) holds entry (ci, cj) of Sigma and of
    // each product; rows / columns are exchanged through LDS; vectors are
    // formed in every lane).  Every lane of the wave runs it (barriers):
    // lanes 16..31 of a pair repeat 0..15 without writing, and pairs that
    // are not evaluated compute on unset data and are discarded.
    __shared__ double smat[GP_PAIRS][5][16];
    double* const SGb = smat[pp][0];  // Sigma
    double* const CBb = smat[pp][1];  // C = I + J Sigma
    double* const CIb = smat[pp][2];  // C^-1
    double* const SPb = smat[pp][3];  // Sigma_post
    double* const ASb = smat[pp][4];  // A Sigma_post
    const int q16 = lane % GP_LPP, e16 = q16 & 15, ci = e16 >> 2, cj = e16 & 3;
    const bool wr = q16 < 16;
    const double pij = gp_pinf(ci, cj, ain, aout, lam);
    double sgm = pij;  // Sigma_{ci cj}: the stationary prior of the first point
    double mu[4] = {0.0, 0.0, 0.0, 0.0};
    double ll = 0.0;
    bool bad = false;
    for (int s = 0; s < GP_SEG; ++s) {
        const int i0 = (n * s) / GP_SEG, i1 = (n * (s + 1)) / GP_SEG;
        if (i1 <= i0) continue;  // an empty segment: nothing observed, no transition (n is the wave's)
        const double* El = &sel[pp][s][0][0];
        bad = bad || El[15] != 0.0 || El[GP_EL + 15] != 0.0;
        if (s > 0 && i0 > 0) {  // the gap from the previous segment's last point
            const double d = sgap[pp][s][0], ex = sgap[pp][s][1], E = ex * ex;
            const bool fresh = sgap[pp][s][2] != 0.0;
            mu[0] = ex * fma(d, mu[1], mu[0]);
            mu[1] = ex * mu[1];
            mu[2] = fresh ? 0.0 : ex * fma(d, mu[3], mu[2]);
            mu[3] = fresh ? 0.0 : ex * mu[3];
            // Sigma <- E T (Sigma - P_inf) T^T + P_inf, T = [[1, d], [0, 1]] per block
            if (wr) SGb[e16] = sgm - pij;
            __syncthreads();
            const bool ei = (ci & 1) == 0, ej = (cj & 1) == 0;
            const double t0 = SGb[e16] + (ei ? d * SGb[e16 + 4] : 0.0);
            const double t1 = ej ? SGb[e16 + 1] + (ei ? d * SGb[e16 + 5] : 0.0) : 0.0;
            const double sgx = fma(E, ej ? fma(d, t1, t0) : t0, pij);
            sgm = (fresh && (ci >= 2 || cj >= 2)) ? pij : sgx;
            __syncthreads();
        }
        // C = I + J Sigma
        if (wr) SGb[e16] = sgm;
        __syncthreads();
        {
            double v = (ci == cj) ? 1.0 : 0.0;
#pragma unroll
            for (int k = 0; k < 4; ++k) v = fma(El[ci * GP_EL + 9 + k], SGb[k * 4 + cj], v);
            if (wr) CBb[e16] = v;
        }
        __syncthreads();
        // det C by 2x2 minors (every lane), C^-1_{ci cj} = cof_{cj ci} / det
        // with the cofactor a 3x3 determinant of C less row cj, column ci
        double det;
        {
            const double* m = CBb;
            const double s0 = fma(m[0], m[5], -m[4] * m[1]), s1 = fma(m[0], m[6], -m[4] * m[2]);
            const double s2 = fma(m[0], m[7], -m[4] * m[3]), s3 = fma(m[1], m[6], -m[5] * m[2]);
            const double s4 = fma(m[1], m[7], -m[5] * m[3]), s5 = fma(m[2], m[7], -m[6] * m[3]);
            const double c5 = fma(m[10], m[15], -m[14] * m[11]), c4 = fma(m[9], m[15], -m[13] * m[11]);
            const double c3 = fma(m[9], m[14], -m[13] * m[10]), c2 = fma(m[8], m[15], -m[12] * m[11]);
            const double c1 = fma(m[8], m[14], -m[12] * m[10]), c0 = fma(m[8], m[13], -m[12] * m[9]);
            det = (fma(s0, c5, -s1 * c4) + fma(s2, c3, s3 * c2)) + fma(s5, c0, -s4 * c1);
            const int r0 = cj == 0 ? 1 : 0, r1 = cj <= 1 ? 2 : 1, r2 = cj <= 2 ? 3 : 2;
            const int k0 = ci == 0 ? 1 : 0, k1 = ci <= 1 ? 2 : 1, k2 = ci <= 2 ? 3 : 2;
            const double a00 = m[r0 * 4 + k0], a01 = m[r0 * 4 + k1], a02 = m[r0 * 4 + k2];
            const double a10 = m[r1 * 4 + k0], a11 = m[r1 * 4 + k1], a12 = m[r1 * 4 + k2];
            const double a20 = m[r2 * 4 + k0], a21 = m[r2 * 4 + k1], a22 = m[r2 * 4 + k2];
            const double d3 = a00 * fma(a11, a22, -a12 * a21) - a01 * fma(a10, a22, -a12 * a20) +
                              a02 * fma(a10, a21, -a11 * a20);
            const double cof = ((ci + cj) & 1) ? -d3 : d3;
            if (wr) CIb[e16] = cof / det;
        }
        bad = bad || !(det > 0.0);
        __syncthreads();
        // Sigma_post = Sigma C^-1
        {
            double v = 0.0;
#pragma unroll
            for (int k = 0; k < 4; ++k) v = fma(SGb[ci * 4 + k], CIb[k * 4 + cj], v);
            if (wr) SPb[e16] = v;
        }
        __syncthreads();
        // vectors (every lane): u = eta - J mu, Sigma_post u, the segment's ln_like
        double u[4], emu = 0.0, mJm = 0.0;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            double jm = 0.0;
#pragma unroll
            for (int k = 0; k < 4; ++k) jm = fma(El[i * GP_EL + 9 + k], mu[k], jm);
            const double et = El[i * GP_EL + 13];
            u[i] = et - jm;
            emu = fma(et, mu[i], emu);
            mJm = fma(mu[i], jm, mJm);
        }
        double uSu = 0.0, mp[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            double su = 0.0;
#pragma unroll
            for (int k = 0; k < 4; ++k) su = fma(SPb[i * 4 + k], u[k], su);
            uSu = fma(u[i], su, uSu);
            mp[i] = mu[i] + su;
        }
        ll += (emu - 0.5 * log(det)) + 0.5 * (uSu - mJm - El[14]);
        // the filtered end state: A mp + c (every lane), A Sigma_post A^T + P_end
        // (lane j of the element's quad wrote column j of A: A_ik = El[k][4 + i])
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            double v = El[i * GP_EL + 8];
#pragma unroll
            for (int k = 0; k < 4; ++k) v = fma(El[k * GP_EL + 4 + i], mp[k], v);
            mu[i] = v;
        }
        {
            double v = 0.0;
#pragma unroll
            for (int k = 0; k < 4; ++k) v = fma(El[k * GP_EL + 4 + ci], SPb[k * 4 + cj], v);
            if (wr) ASb[e16] = v;
        }
        __syncthreads();
        {
            double v = El[ci * GP_EL + cj] + pij;  // P_end = D_end + P_inf
#pragma unroll
            for (int k = 0; k < 4; ++k) v = fma(ASb[ci * 4 + k], El[k * GP_EL + 4 + cj], v);
            sgm = v;
        }
        __syncthreads();
    }
    if (!live || q16 != 0) return;
    double lle = -INFINITY;
    if (run) {
        const double v = ll - 0.5 * n * 1.8378770664093454836;  // log(2 pi)
        lle = (bad || !isfinite(v)) ? -INFINITY : v;
    }
    L.lle[pair] = lle;
    combine_after(L, pair);
}
#endif

// -------------------------------------------------------------- k_combine
// E > 1: ln_prob (and the fused acceptance) of every walker once all its
// eclipses' ln_like are written, one lane per walker, in a launch of its own.
// (The last-finishing block of each walker used to do it after a device-scope
// fence: on MI355X that fence writes back the block's whole L2, and the 12 288
// fences of a config-3 launch cost a third of k_lnlike: 898 -> 587 us.)
// One wave per walker: the lanes fetch the E Roche priors and ln_like at
// once (the walker's chain of 2E dependent-latency loads in one lane was 43 us
// per config-3 launch), lane 0 adds them in combine_walker's order (the
// same sums, bit for bit), and the lanes copy an accepted proposal.
#ifndef LFG_NOLICM_TU  // (lfg_pair_split.hip compiles k_pair only)
__global__ __launch_bounds__(256) void k_combine_walkers(LikeArgs L)
{
    const int w = int(blockIdx.x) * 4 + int(threadIdx.x >> 6), lane = int(threadIdx.x & 63);
    if (w >= L.npairs / L.E) return;
    const size_t p0 = size_t(w) * L.E;
    double lp = L.prior[w];
    double ll = 0.0;
    for (int e0 = 0; e0 < L.E; e0 += 64) {
        const int e = e0 + lane;
        double g = 0.0, l = 0.0;
        if (e < L.E) {
            const double* G = L.geo + (p0 + e) * LFG_NGEO;
            g = G[G_RPRIOR] + G[G_RPRIOR_BS];
            l = L.lle[p0 + e];
        }
        const int m = min(64, L.E - e0);
        for (int k = 0; k < m; ++k) {  // in eclipse order, as combine_walker
            lp += __shfl(g, k, 64);
            ll += __shfl(l, k, 64);
        }
    }
    double v;
    if (!isfinite(lp)) {
        for (int e = lane; e < L.E; e += 64) L.lle[p0 + e] = -INFINITY;
        v = -INFINITY;
    } else {
        v = lp + ll;
    }
    if (L.lnp && lane == 0) L.lnp[w] = v;
    if (!L.pos) return;
    const int wg = L.half * L.npairs / L.E + w;  // ensemble index (npairs / E = batch walkers)
    bool acc = false;
    if (lane == 0) {
        const uint4 r = draw(L.seed, L.step, L.half, 1, w);
        acc = log(u53(r.x, r.y)) < L.zfac[w] + v - L.lnp_ens[wg];
        if (acc) {
            L.lnp_ens[wg] = v;
            if (L.naccept) L.naccept[wg] += 1;
        }
        if (L.accflag) L.accflag[w] = acc ? 1 : 0;
    }
    if (__shfl(acc ? 1 : 0, 0, 64))
        for (int d = lane; d < L.ndim; d += 64) L.pos[size_t(wg) * L.ndim + d] = L.qprop[size_t(w) * L.ndim + d];
}
#endif

#ifndef LFG_NOLICM_TU  // (lfg_pair_split.hip compiles k_pair only)
__global__ void k_combine(int W, int E, const double* __restrict__ prior, const double* __restrict__ geo,
                          double* __restrict__ lle, double* __restrict__ lnp)
{
    const int w = blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= W) return;
    double lp = prior[w];
    for (int e = 0; e < E; ++e) {
        const double* G = geo + (size_t(w) * E + e) * LFG_NGEO;
        lp += G[G_RPRIOR] + G[G_RPRIOR_BS];
    }
    if (!lle) {  // ln_prior only (lfg_lnprior)
        lnp[w] = isfinite(lp) ? lp : -INFINITY;
        return;
    }
    if (!isfinite(lp)) {
        for (int e = 0; e < E; ++e) lle[size_t(w) * E + e] = -INFINITY;
        lnp[w] = -INFINITY;
        return;
    }
    double ll = 0.0;
    for (int e = 0; e < E; ++e) ll += lle[size_t(w) * E + e];
    lnp[w] = lp + ll;
}
#endif

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
// step counter: by value, or (stepp != nullptr) from device memory so that
// a captured HIP graph replays with the current step
#ifndef LFG_NOLICM_TU  // (lfg_pair_split.hip compiles k_pair only)
__global__ void k_propose(const double* __restrict__ pos, int W, int ndim, int half, double a,
                          unsigned long long seed, unsigned long long step,
                          const unsigned long long* __restrict__ stepp, double* __restrict__ q,
                          double* __restrict__ zfac)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const int ns = W / 2;
    if (i >= ns) return;
    if (stepp) step = *stepp;
    const uint4 r = draw(seed, step, half, 0, i);
    const double u = u53(r.x, r.y);
    const double zr = (a - 1.0) * u + 1.0;
    const double z = zr * zr / a;
    const int j = int(__umulhi(r.z, unsigned(ns)));  // partner in the other half
    const double* s = pos + size_t(half * ns + i) * ndim;
    const double* cj = pos + size_t((1 - half) * ns + j) * ndim;
    double* out = q + size_t(i) * ndim;
    for (int d = 0; d < ndim; ++d) out[d] = fma(s[d] - cj[d], z, cj[d]);  // c_j + z (s - c_j), as make_prop
    zfac[i] = (ndim - 1.0) * log(z);
}
#endif

// Metropolis acceptance: accept if ln u < factor + lnp_new - lnp_old
#ifndef LFG_NOLICM_TU  // (lfg_pair_split.hip compiles k_pair only)
__global__ void k_accept(double* __restrict__ pos, double* __restrict__ lnp, int W, int ndim, int half,
                         const double* __restrict__ q, const double* __restrict__ zfac,
                         const double* __restrict__ lnp_new, unsigned long long seed, unsigned long long step,
                         const unsigned long long* __restrict__ stepp, int* __restrict__ naccept)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const int ns = W / 2;
    if (i >= ns) return;
    if (stepp) step = *stepp;
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
#endif

// k_accept with the proposal re-formed from the same draws (k_propose's
// arithmetic): the sharded half-step keeps only its own shard of q, and the
// partner half is unchanged until this half is accepted
// one wave per walker of the half (four per 256-lane block): the draws and
// the decision are wave-uniform (scalar ALU and scalar loads), and an
// accepted walker's row moves with one load round over the lanes (lane d:
// dimension d) instead of one lane's serial chunks of 8
constexpr int REGEN_WAVES = 4;
#ifndef LFG_NOLICM_TU  // (lfg_pair_split.hip compiles k_pair only)
__global__ __launch_bounds__(64 * REGEN_WAVES) void k_accept_regen(double* __restrict__ pos, double* __restrict__ lnp, int W, int ndim, int half,
                               double a, const double* __restrict__ lnp_new, unsigned long long seed,
                               unsigned long long step, int* __restrict__ naccept, int* __restrict__ accflag)
{
    const int i = __builtin_amdgcn_readfirstlane(int(blockIdx.x) * REGEN_WAVES + int(threadIdx.x >> 6));
    const int lane = threadIdx.x & 63;
    const int ns = W / 2;
    if (i >= ns) return;
    const int w = half * ns + i;
    const uint4 r0 = draw(seed, step, half, 0, i);
    const double zr = (a - 1.0) * u53(r0.x, r0.y) + 1.0;
    const double z = zr * zr / a;
    const uint4 r = draw(seed, step, half, 1, i);
    const double lu = log(u53(r.x, r.y));
    const double diff = (ndim - 1.0) * log(z) + lnp_new[i] - lnp[w];
    const bool acc = lu < diff;
    if (acc) {
        const int j = int(__umulhi(r0.z, unsigned(ns)));
        double* p = pos + size_t(w) * ndim;
        const double* cj = pos + size_t((1 - half) * ns + j) * ndim;
        for (int d = lane; d < ndim; d += 64) p[d] = fma(p[d] - cj[d], z, cj[d]);
        if (lane == 0) {
            lnp[w] = lnp_new[i];
            if (naccept) naccept[w] += 1;
        }
    }
    if (accflag && lane == 0) accflag[i] = acc ? 1 : 0;  // the speculative setup's candidate choice
}
#endif

// the deferred acceptance's two halves outside k_pair<_, true>:
//  k_apply_verdicts: half `half`'s gathered verdicts (ln_prob where the move
//  was accepted, NaN where not) applied to the ensemble, the proposal
//  re-formed from its draws as k_accept_regen does (the flush at a chain's
//  end, and the fold's fallback); one wave per walker
//  k_verdict: a shard's verdicts from its ln_prob (k_accept_regen's test)
#ifndef LFG_NOLICM_TU  // (lfg_pair_split.hip compiles k_pair only)
__global__ __launch_bounds__(64 * REGEN_WAVES) void k_apply_verdicts(double* __restrict__ pos, double* __restrict__ lnp,
                                                                      int W, int ndim, int half, double a,
                                                                      const double* __restrict__ verdict,
                                                                      unsigned long long seed, unsigned long long step,
                                                                      int* __restrict__ naccept, int* __restrict__ accflag)
{
    const int i = __builtin_amdgcn_readfirstlane(int(blockIdx.x) * REGEN_WAVES + int(threadIdx.x >> 6));
    const int lane = threadIdx.x & 63;
    const int ns = W / 2;
    if (i >= ns) return;
    const double v = verdict[i];
    const bool acc = !isnan(v);
    if (acc) {
        const int w = half * ns + i;
        const uint4 r0 = draw(seed, step, half, 0, i);
        const double zr = (a - 1.0) * u53(r0.x, r0.y) + 1.0;
        const double z = zr * zr / a;
        const int j = int(__umulhi(r0.z, unsigned(ns)));
        double* p = pos + size_t(w) * ndim;
        const double* cj = pos + size_t((1 - half) * ns + j) * ndim;
        for (int d = lane; d < ndim; d += 64) p[d] = fma(p[d] - cj[d], z, cj[d]);
        if (lane == 0) {
            lnp[w] = v;
            if (naccept) naccept[w] += 1;
        }
    }
    if (accflag && lane == 0) accflag[i] = acc ? 1 : 0;
}
#endif

#ifndef LFG_NOLICM_TU  // (lfg_pair_split.hip compiles k_pair only)
__global__ void k_verdict(const double* __restrict__ lnp_new, const double* __restrict__ lnp,
                          const double* __restrict__ zfac, int n, int lo, int ns, int half, unsigned long long seed,
                          unsigned long long step, double* __restrict__ vout)
{
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const uint4 r = draw(seed, step, half, 1, lo + k);
    const double v = lnp_new[k];
    vout[k] = (log(u53(r.x, r.y)) < zfac[k] + v - lnp[size_t(half) * ns + lo + k]) ? v : NAN;
}
#endif

// ------------------------------------------------------ k_gp, k_wdphases
__device__ __forceinline__ double readlane_f64(double v, int j)
{
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane(int(b), j), hi = __builtin_amdgcn_readlane(int(b >> 32), j);
    return __longlong_as_double((static_cast<long long>(hi) << 32) | static_cast<unsigned>(lo));
}

// one wave per residual vector: lanes load 64 points at a time, every lane
// runs the (wave-uniform) filter over them through readlane broadcasts
#ifndef LFG_NOLICM_TU  // (lfg_pair_split.hip compiles k_pair only)
__global__ __launch_bounds__(64) void k_gp(const double* __restrict__ x, const double* __restrict__ ye,
                                           const double* __restrict__ res, int N, const double* __restrict__ hyp,
                                           const double* __restrict__ blocks, int nb, double* __restrict__ lnlike)
{
    const int w = blockIdx.x, lane = threadIdx.x;
    const double* r = res + size_t(w) * N;
    const double* bk = blocks + size_t(w) * nb * 2;
    GPFilter F;
    F.init(hyp[3 * w], hyp[3 * w + 1], hyp[3 * w + 2]);
    for (int c0 = 0; c0 < N; c0 += 64) {
        const int p = c0 + lane;
        double xv = 0.0, yv = 1.0, rv = 0.0;
        int bv = -1;
        if (p < N) {
            xv = x[p];
            yv = ye[p];
            rv = r[p];
            for (int k = 0; k < nb; ++k)
                if (xv >= bk[2 * k] && xv <= bk[2 * k + 1]) bv = k;
        }
        const int m = min(64, N - c0);
        for (int j = 0; j < m; ++j)
            F.step(readlane_f64(xv, j), readlane_f64(yv, j), readlane_f64(rv, j), __builtin_amdgcn_readlane(bv, j));
    }
    if (lane == 0) lnlike[w] = F.lnlike();
}
#endif

#ifndef LFG_NOLICM_TU  // (lfg_pair_split.hip compiles k_pair only)
__global__ void k_wdphases(const double* __restrict__ q, const double* __restrict__ inc,
                           const double* __restrict__ r1, int n, int ntheta, double* __restrict__ ph3,
                           double* __restrict__ ph4, int* __restrict__ status)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    Roche R;
    double a = NAN, b = NAN;
    int st = roche_init(R, q[i]);
    if (st == ST_OK) st = wdphases(R, inc[i], r1[i], ntheta, a, b);
    ph3[i] = (st == ST_OK) ? a : NAN;
    ph4[i] = (st == ST_OK) ? b : NAN;
    status[i] = st;
}
#endif

// ---------------------------------------------------------------- k_roche
#ifndef LFG_NOLICM_TU  // (lfg_pair_split.hip compiles k_pair only)
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
#endif

inline int launch_ok() { return hipGetLastError() == hipSuccess ? LFG_OK : LFG_E_LAUNCH; }

#ifndef LFG_NOLICM_TU
// k_setup (setup, prior and stream lanes) then k_elements, on the caller's
// stream.  ev (nullable, LFG_NEV events): 0 before k_setup, 1 after k_setup,
// 2 after k_elements
// k_setup (unless the speculative candidates stand in for it) then k_elements
int run_front(const SetupArgs& S, const Ws& ws, hipStream_t st, void* const* ev, bool elements = true,
              const ElemSpec* X = nullptr, bool setup = true)
{
    auto mark = [&](int i) {
        if (ev && ev[i]) (void)hipEventRecord(static_cast<hipEvent_t>(ev[i]), st);
    };
    const int npairs = S.W * S.E;
    const int nlanes = 2 * npairs + S.W;
    mark(0);
    if (setup) {
        hipLaunchKernelGGL(k_setup, dim3((nlanes + SETUP_BLOCK - 1) / SETUP_BLOCK), dim3(SETUP_BLOCK), 0, st, S);
        if (launch_ok() != LFG_OK) return LFG_E_LAUNCH;
    }
    mark(1);
    if (elements) {
        constexpr int chunks = (NUNIQ + ELEM_BLOCK * LFG_ELEM_IPL - 1) / (ELEM_BLOCK * LFG_ELEM_IPL);
        ElemSpec none{};
        const ElemSpec& XS = X ? *X : none;
        hipLaunchKernelGGL(k_elements, dim3(unsigned(npairs) * chunks + unsigned(XS.nspecblk)), dim3(ELEM_BLOCK), 0,
                           st, ws.geo, ws.status, npairs, ws.ab, ws.donor, ws.wts, ws.bstatus, XS);
        if (launch_ok() != LFG_OK) return LFG_E_LAUNCH;
    }
    mark(2);
    return LFG_OK;
}
#endif  // LFG_NOLICM_TU

}  // namespace

// k_pair's fold and LONG instantiations are compiled in lfg_pair_split.hip:
// this source again, without machine LICM (-mllvm -disable-machine-licm).
// At the 128-VGPR ceiling the pass hoisted literal constants and cheap loop
// invariants into VGPRs and the register allocator then spilled: LONG's
// point loop reloaded five doubles from scratch per point (48 B per lane,
// 41.6 MB of PMC traffic per config-5 launch), the fold variant 32 B.
// Without it LONG spills 16 B and the fold variant none: config 5
// 3.39 -> 3.52 M evals/s; config 4's one-of-eight fold shard 12.71 -> 12.76
// and 12.36 -> 12.77 M on two boxes (profiles/r06/ab_split_nolicm.txt).  The
// speculative one-tile k_pair (config 2) measured no different and GP trees
// 5 % slower, so they stay here, compiled with the pass.
enum { PAIR_SPLIT_LONG = 0, PAIR_SPLIT_FOLD = 1, PAIR_SPLIT_FOLD_LONG = 2 };
__attribute__((visibility("hidden"))) void lfg_pair_launch_split(int variant, unsigned grid, hipStream_t st,
                                                                   const void* args);

#ifndef LFG_NOLICM_TU
namespace {
// launch k_pair<false, FOLD, LONG> (not both false) with the arguments A
void launch_pair_split(int variant, unsigned grid, hipStream_t st, const PairArgs& A)
{
#ifdef LFG_ONE_TU
    if (variant == PAIR_SPLIT_LONG) hipLaunchKernelGGL((k_pair<false, false, true>), dim3(grid), dim3(LIKE_THREADS), 0, st, A);
    else if (variant == PAIR_SPLIT_FOLD) hipLaunchKernelGGL((k_pair<false, true>), dim3(grid), dim3(LIKE_THREADS), 0, st, A);
    else hipLaunchKernelGGL((k_pair<false, true, true>), dim3(grid), dim3(LIKE_THREADS), 0, st, A);
#else
    lfg_pair_launch_split(variant, grid, st, &A);
#endif
}
}  // namespace

extern "C" {

size_t lfg_workspace_size(int W, int E)
{
    if (W <= 0 || E <= 0) return 0;
    return carve(nullptr, W, E).total;
}

size_t lfg_workspace_size_tree(int W, const lfg_tree* T)
{
    if (W <= 0 || !T || T->E <= 0) return 0;
    return carve(nullptr, W, T->E, T->gp ? T->max_n : 0, T->ndim).total;  // + lfg_stretch_step_half_spec's
}

int lfg_flux(const double* pars, int W, int P, const double* x, const double* w, int N, int nsub,
             double* flux, double* comps, int* status, void* wsp, size_t ws_bytes, void* stream)
{
    if (W <= 0 || N < 0 || nsub < 1 || (P != 14 && P != 18) || !pars || (!x && N > 0)) return LFG_E_ARGS;
    Ws ws = carve(wsp, W, 1);
    if (!wsp || ws_bytes < ws.total) return LFG_E_WORKSPACE;
    hipStream_t st = static_cast<hipStream_t>(stream);
    SetupArgs S{pars, W, P, 1, P, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, 0,
                ws.geo, ws.status, ws.prior, ws.bstatus, 0, nullptr, nullptr};
    int rc = run_front(S, ws, st, nullptr);
    if (rc) return rc;
    if (N > 0) {
        LikeArgs L{ws.geo, ws.status, ws.ab, ws.donor, ws.wts, 1, nullptr, N, x, nullptr, nullptr, w,
                   nsub, flux, comps, nullptr, W, nullptr, nullptr, nullptr, false, nullptr,
                   nullptr, nullptr, nullptr, 0, 0, 0ull, 0ull, nullptr};
        L.bstatus = ws.bstatus;
        if (nsub > 1) hipLaunchKernelGGL((k_lnlike<0, true>), dim3(W), dim3(LIKE_THREADS), 0, st, L);
        else hipLaunchKernelGGL((k_lnlike<0, false>), dim3(W), dim3(LIKE_THREADS), 0, st, L);
        if ((rc = launch_ok())) return rc;
    }
    if (status && hipMemcpyAsync(status, ws.status, sizeof(int) * W, hipMemcpyDeviceToDevice, st) != hipSuccess)
        return LFG_E_LAUNCH;
    return LFG_OK;
}

// k_pair serves trees whose eclipses fit one tile with S = 1 (GP trees
// included); k_elements + k_lnlike serve the rest, and every tree when
// LFG_PAIR=0 is in the environment (the A/B switch of the two layouts)
// k_pair's workgroups all resident at once: two per CU (72.9 KB of LDS each)
// PairArgs.prio: the workgroups that take the wave-priority scheme
// (PAIR_PRIO).  Launches of at most two rounds (two workgroups per CU
// resident): all of them -- the one-round launches of config 2 and of the
// weak-scaling shards, and the two-round 1 024-pair shard of config 4 over 8
// ranks, whose projected 1 -> 8 speed-up rose 5.7x -> 6.1x with it (A/B,
// rounds 1 and 2 both prioritised vs none: 173 vs 183 us per step).  Longer
// launches none: there an early finish lets the next round's workgroup in
// (the GP example's 6 rounds: 1.92 vs 1.95 M evals/s with the scheme on)
static int pair_prio(int npairs)
{
    int dev = 0, cus = 0;  // the current device's (the runtime caches the attribute)
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        cus = 0;
    return npairs <= 4 * cus ? npairs : 0;
}

// the trees k_pair can serve: one-tile eclipses, S = 1 (kind 1); and, with
// the LONG tables, chi^2 trees of any eclipse length and sub-binning (kind 2)
static bool pair_fits(int nsub, int max_n, int ndim) { return nsub == 1 && max_n <= LIKE_TILE && ndim <= LIKE_THREADS; }
static int pair_eligible(int gp, int nsub, int max_n, int ndim)
{
    if (pair_fits(nsub, max_n, ndim)) return 1;
    return (!gp && nsub >= 1 && ndim <= LIKE_THREADS) ? 2 : 0;
}

static bool pair_env()
{
    const char* e = getenv("LFG_PAIR");
    return !(e && e[0] == '0');
}
static std::atomic<int> g_pair_layout{-2};  // -2: not read yet; 0 / 1: lfg_set_layout or the environment

// the kernels a tree runs on: 0 k_elements + k_lnlike, 1 k_pair, 2 k_pair LONG
static int pair_kind(int gp, int nsub, int max_n, int ndim)
{
    int m = g_pair_layout.load(std::memory_order_relaxed);
    if (m == -2) {
        m = pair_env() ? 1 : 0;
        g_pair_layout.store(m, std::memory_order_relaxed);
    }
    return m == 1 ? pair_eligible(gp, nsub, max_n, ndim) : 0;
}

int lfg_set_layout(int mode)
{
    if (mode < -1 || mode > 1) return LFG_E_ARGS;
    int prev = g_pair_layout.load();
    if (prev == -2) prev = pair_env() ? 1 : 0;
    g_pair_layout.store(mode == -1 ? (pair_env() ? 1 : 0) : mode);
    return prev;
}

int lfg_layout(const lfg_tree* T)
{
    if (!T || T->E <= 0) return LFG_E_ARGS;
    return pair_kind(T->gp, T->nsub, T->max_n, T->ndim);
}

int lfg_lnlike(const double* pars, int W, int P, const double* x, const double* w, int N, int nsub, const double* y,
               const double* ye, double* lnlike, int* status, void* wsp, size_t ws_bytes, void* stream)
{
    if (W <= 0 || N < 0 || nsub < 1 || (P != 14 && P != 18) || !pars || !lnlike || (N > 0 && (!x || !y || !ye)))
        return LFG_E_ARGS;
    Ws ws = carve(wsp, W, 1);
    if (!wsp || ws_bytes < ws.total) return LFG_E_WORKSPACE;
    hipStream_t st = static_cast<hipStream_t>(stream);
    SetupArgs S{pars, W, P, 1, P, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, 0,
                ws.geo, ws.status, ws.prior, ws.bstatus, 0, nullptr, nullptr};
    const int kind = pair_kind(0, nsub, N, 0);
    const bool pair = kind > 0;
    int rc = run_front(S, ws, st, nullptr, !pair);
    if (rc) return rc;
    LikeArgs L{ws.geo, ws.status, ws.ab, ws.donor, ws.wts, 1, nullptr, N, x, y, ye, w,
               nsub, nullptr, nullptr, lnlike, W, nullptr, nullptr, nullptr, false, nullptr,
               nullptr, nullptr, nullptr, 0, 0, 0ull, 0ull, nullptr};
    L.bstatus = ws.bstatus;
    PairArgs A{L, ElemSpec{}, nullptr, nullptr, 64, 0, 0ull, 0ull, 0, 0, 0, pair_prio(W)};
    fill_hot(A);
    if (kind == 2) launch_pair_split(PAIR_SPLIT_LONG, unsigned(W), st, A);
    else if (pair) hipLaunchKernelGGL(k_pair<false>, dim3(W), dim3(LIKE_THREADS), 0, st, A);
    else if (nsub > 1) hipLaunchKernelGGL((k_lnlike<1, true>), dim3(W), dim3(LIKE_THREADS), 0, st, L);
    else hipLaunchKernelGGL((k_lnlike<1, false>), dim3(W), dim3(LIKE_THREADS), 0, st, L);
    if ((rc = launch_ok())) return rc;
    if (status && hipMemcpyAsync(status, ws.status, sizeof(int) * W, hipMemcpyDeviceToDevice, st) != hipSuccess)
        return LFG_E_LAUNCH;
    return LFG_OK;
}

struct Accept {  // fused stretch-move acceptance of lfg_stretch_lnprob_accept
    double* pos;
    double* lnp;
    const double* zfac;
    int half;
    unsigned long long seed, step;
    int* naccept;
};

struct Propose {  // inline proposal of lfg_stretch_step_half / _shard
    const double* pos;
    double a;
    double* q;
    double* zfac;
    int half;
    unsigned long long seed, step;
    int lo, ns;  // the batch: walkers lo .. lo + W - 1 of the ns-walker half
};

struct SpecCtl {  // lfg_stretch_step_half_spec
    bool in;   // this half's setup candidates are in the workspace (skip k_setup)
    bool out;  // form the next half's candidates inside this k_elements
};

struct FoldCtl {  // lfg_stretch_step_shard_fold: deferred acceptance
    const double* fv;  // [ns] the partner half's pending verdicts (nullptr: none)
    double* vout;      // [n] this shard's verdicts
    double* pos;       // the ensemble the verdicts apply to
    double* lnp;
    int* naccept;
};

static int apply_verdicts(double* pos, double* lnp, int W, int ndim, int half, double a, const double* verdict,
                          unsigned long long seed, unsigned long long step, int* naccept, int* accflag,
                          hipStream_t st)
{
    const int ns = W / 2;
    hipLaunchKernelGGL(k_apply_verdicts, dim3((ns + REGEN_WAVES - 1) / REGEN_WAVES), dim3(64 * REGEN_WAVES), 0, st,
                       pos, lnp, W, ndim, half, a, verdict, seed, step, naccept, accflag);
    return launch_ok();
}

static int lnprob_impl(const double* walkers, int W, const lfg_tree* T, double* lnp, double* lnlike_e, void* wsp,
                       size_t ws_bytes, void* stream, void* const* ev, const Accept* acc = nullptr,
                       const Propose* prop = nullptr, const SpecCtl* sp = nullptr, const FoldCtl* fold = nullptr)
{
    if (W <= 0 || !T || T->E <= 0 || T->ndim <= 0 || T->nsub < 1 || !walkers || (!lnp && !acc)) return LFG_E_ARGS;
    if (sp && (!prop || (acc && (prop->lo != 0 || prop->ns != W)))) return LFG_E_ARGS;
    if (fold && (!sp || !prop || acc || !lnp || !fold->vout || !fold->pos || !fold->lnp || (sp->in && !fold->fv)))
        return LFG_E_ARGS;
    Ws ws = carve(wsp, W, T->E, T->gp ? T->max_n : 0, sp ? T->ndim : 0, prop ? prop->ns : 0);
    if (!wsp || ws_bytes < ws.total) return LFG_E_WORKSPACE;
    hipStream_t st = static_cast<hipStream_t>(stream);
    // the deferred acceptance runs inside k_pair for one-eclipse chi^2 trees
    // on the k_pair layout; otherwise (and when no candidates are in the
    // workspace: k_setup reads the rows directly) the pending verdicts are
    // applied first, recording the acceptances for the candidate choice, and
    // the shard's verdicts are formed after its ln_prob (k_verdict)
    const double* fv = fold ? fold->fv : nullptr;
    const int kind = pair_kind(T->gp, T->nsub, T->max_n, T->ndim);
    const bool fold_pair = fold && T->E == 1 && !T->gp && kind > 0 &&
                           (!sp->out || 2 * ((2 * W + W + 63) / 64) <= W);
    const unsigned long long fstep = prop && prop->half == 0 ? prop->step - 1 : (prop ? prop->step : 0);
    if (fv && (!fold_pair || !sp->in)) {
        const int rc = apply_verdicts(fold->pos, fold->lnp, 2 * prop->ns, T->ndim, 1 - prop->half, prop->a, fv,
                                      prop->seed, fstep, fold->naccept,
                                      ws.accflag + size_t(1 - prop->half) * ws.accstride, st);
        if (rc) return rc;
        fv = nullptr;
    }
    auto mark = [&](int i) {
        if (ev && ev[i]) (void)hipEventRecord(static_cast<hipEvent_t>(ev[i]), st);
    };
    SetupArgs S{walkers, W, T->ndim, T->E, 18, T->gather, T->npars, T->consts, T->prior_type, T->prior_p1,
                T->prior_p2, T->prior_norm, T->roche_priors, ws.geo, ws.status, ws.prior, ws.bstatus, T->gp,
                T->gp_gather, T->gp_base};
    S.fixed_invalid = T->fixed_invalid;
    S.prior_c = T->prior_c;
    if (prop) {
        S.pos = prop->pos;
        S.a = prop->a;
        S.seed = prop->seed;
        S.step = prop->step;
        S.half = prop->half;
        S.qout = prop->q;
        S.zfout = prop->zfac;
        S.lo = prop->lo;
        S.ns = prop->ns;
    }
    const int npairs = W * T->E;
    ElemSpec X{};
    X.E = T->E;
    X.ndim = T->ndim;
    X.lprior = ws.prior;
    if (sp) {
        const int h = prop->half, hn = 1 - prop->half;
        const size_t P48 = size_t(npairs) * LFG_NGEO;
        if (sp->in) {
            X.jk = ws.jk + size_t(h) * W;
            X.accflag = ws.accflag + size_t(hn) * ws.accstride;  // the partner half's acceptances
            X.geoC = ws.geoC + 2 * h * P48;
            X.statusC = ws.statusC + 2 * h * size_t(npairs);
            X.bstatusC = ws.bstatusC + 2 * h * size_t(npairs);
            X.priorC = ws.priorC + 2 * h * size_t(W);
            X.qC = ws.qC + 2 * h * size_t(W) * T->ndim;
            X.zfC = ws.zfC + 2 * h * size_t(W);
            X.prior = ws.prior;
            X.q = prop->q;
            X.zf = prop->zfac;
            X.bstatus = ws.bstatus;
        }
        if (sp->out) {
            for (int c = 0; c < 2; ++c) {
                SetupArgs& N = X.S[c];
                N = S;
                const size_t k = size_t(2 * hn + c);
                N.half = hn;
                N.step = hn == 0 ? prop->step + 1 : prop->step;
                N.step_prev = prop->step;
                N.cand = c;
                N.geo = ws.geoC + k * P48;
                N.status = ws.statusC + k * npairs;
                N.bstatus = ws.bstatusC + k * npairs;
                N.prior = ws.priorC + k * W;
                N.qout = ws.qC + k * size_t(W) * T->ndim;
                N.zfout = ws.zfC + k * W;
                N.jkout = ws.jk + size_t(hn) * W;
                if (fold_pair && fv) {  // the next half's rows as the pending verdicts leave them
                    N.fv = fv;
                    N.fsnap = ws.snap + size_t(hn) * ws.accstride * T->ndim;
                    N.fstep = N.step - 1;
                }
            }
            X.nspec = 2 * npairs + W;
            X.nspecblk = (2 * ((X.nspec + ELEM_BLOCK - 1) / ELEM_BLOCK) + 7) / 8 * 8;  // keeps the pair -> XCD map
        }
    }
    // k_pair: the element solve and the likelihood of a pair in one
    // workgroup (one-tile eclipses, S = 1; GP trees through k_pair<true> and
    // k_gp_like).  The speculative lanes fill whole waves: wave 0 of blocks
    // [0, 2 nbc), nbc blocks per candidate, so there must be 2 nbc pairs
    const int spl = 64, nbc = (X.nspec + 63) / 64;
    const bool pair_path = kind > 0 && (X.nspec == 0 || 2 * nbc <= npairs);
    if (fold_pair && !pair_path) return LFG_E_ARGS;  // (fold_pair's test is pair_path's)
    // the end of every path but the fold's own: the shard's verdicts from its
    // ln_prob (fold fallback), then the last event
    auto finish = [&]() {
        if (fold) {
            hipLaunchKernelGGL(k_verdict, dim3((W + 63) / 64), dim3(64), 0, st, lnp, fold->lnp, prop->zfac, W,
                               prop->lo, prop->ns, prop->half, prop->seed, prop->step, fold->vout);
            if (launch_ok()) return LFG_E_LAUNCH;
        }
        mark(3);
        return LFG_OK;
    };
    int rc = run_front(S, ws, st, ev, !pair_path, &X, !(sp && sp->in));
    if (rc) return rc;
    double* lle = lnlike_e ? lnlike_e : ws.lle;
    LikeArgs L{ws.geo, ws.status, ws.ab, ws.donor, ws.wts, T->E, T->off, T->max_n, T->x, T->y, T->ye,
               T->w, T->nsub, nullptr, nullptr, lle, npairs, T->gp ? T->gp_ecl : nullptr, ws.prior, lnp,
               true, acc ? acc->pos : nullptr, acc ? acc->lnp : nullptr, walkers, acc ? acc->zfac : nullptr,
               T->ndim, acc ? acc->half : 0, acc ? acc->seed : 0ull, acc ? acc->step : 0ull,
               acc ? acc->naccept : nullptr};
    L.bstatus = ws.bstatus;
    // sharded: k_accept_regen records them
    L.accflag = (sp && acc) ? ws.accflag + size_t(prop->half) * ws.accstride : nullptr;
    L.combine = T->E == 1;  // E > 1: k_combine_walkers after the likelihood kernels
    if (pair_path) {
        PairArgs A{L, X, nullptr, nullptr, spl, nbc, 0ull, 0ull, 0, 0, 0, pair_prio(npairs)};
        if (prop) {
            A.jseed = prop->seed;
            A.jstep = prop->step;
            A.jhalf = prop->half;
            A.jlo = prop->lo;
            A.jns = prop->ns;
        }
        if (fold_pair) {
            const int h = prop->half;
            A.fv = fv;
            A.vout = fold->vout;
            A.fpos = fold->pos;
            A.flnp = fold->lnp;
            A.fnacc = fold->naccept;
            A.fsnap = ws.snap + size_t(h) * ws.accstride * T->ndim;
            A.fstep = fstep;
            A.fa = prop->a;
            A.L.seed = prop->seed;
            A.L.step = prop->step;
            A.L.half = h;
            A.L.zfac = prop->zfac;
            fill_hot(A);
            launch_pair_split(kind == 2 ? PAIR_SPLIT_FOLD_LONG : PAIR_SPLIT_FOLD, unsigned(npairs), st, A);
            if ((rc = launch_ok())) return rc;
            mark(3);
            return LFG_OK;
        }
        if (sp && sp->out && acc && T->E == 1) {
            // this launch accepts moves of half h while its speculative lanes
            // read half h's rows: they read the snapshot of them instead (taken
            // by the launch before, or here), and the launch snapshots half 1 - h
            const int h = prop->half, hn = 1 - h, ns = prop->ns;
            const size_t rows = size_t(ns) * T->ndim;
            double* snap_h = ws.snap + size_t(h) * ws.accstride * T->ndim;
            if (!sp->in && hipMemcpyAsync(snap_h, prop->pos + size_t(h) * rows, rows * sizeof(double),
                                          hipMemcpyDeviceToDevice, st) != hipSuccess)
                return LFG_E_LAUNCH;
            A.X.S[0].ppos = A.X.S[1].ppos = snap_h;
            A.snap_src = prop->pos + size_t(hn) * rows;
            A.snap_dst = ws.snap + size_t(hn) * ws.accstride * T->ndim;
        }
        if (T->gp) {
            L.res = ws.res;
            L.gpx = ws.gpx;
            L.gpb = ws.gpb;
            A.L = L;
            fill_hot(A);
            hipLaunchKernelGGL(k_pair<true>, dim3(npairs), dim3(LIKE_THREADS), 0, st, A);
            if ((rc = launch_ok())) return rc;
            hipLaunchKernelGGL(k_gp_like, dim3(T->E * ((W + GP_PAIRS - 1) / GP_PAIRS)), dim3(GP_BLOCK), 0, st, L);
        } else if (kind == 2) {
            fill_hot(A);
            launch_pair_split(PAIR_SPLIT_LONG, unsigned(npairs), st, A);
        } else {
            fill_hot(A);
            hipLaunchKernelGGL(k_pair<false>, dim3(npairs), dim3(LIKE_THREADS), 0, st, A);
        }
        if ((rc = launch_ok())) return rc;
        if (T->E > 1) {
            hipLaunchKernelGGL(k_combine_walkers, dim3((W + 3) / 4), dim3(256), 0, st, L);
            if ((rc = launch_ok())) return rc;
        }
        return finish();
    }
    if (sp && sp->out && acc && T->E == 1 && pair_eligible(T->gp, T->nsub, T->max_n, T->ndim)) {
        // a k_pair-eligible tree on the two-kernel layout (lfg_set_layout(0)):
        // leave the partner-half snapshot a k_pair launch would have left, so
        // that a layout switch before the chain's next half reads valid rows
        const int hn = 1 - prop->half;
        const size_t rows = size_t(prop->ns) * T->ndim;
        if (hipMemcpyAsync(ws.snap + size_t(hn) * ws.accstride * T->ndim, prop->pos + size_t(hn) * rows,
                           rows * sizeof(double), hipMemcpyDeviceToDevice, st) != hipSuccess)
            return LFG_E_LAUNCH;
    }
    if (sp && sp->out && fold && T->E == 1 && pair_eligible(T->gp, T->nsub, T->max_n, T->ndim)) {
        // the deferred acceptance on the two-kernel layout: a fold k_pair
        // launch snapshots its own half's rows (final until its verdicts are
        // applied) for the next launch's speculative lanes; leave the same
        // snapshot, so that a layout switch before the next half reads it valid
        const int h = prop->half;
        const size_t rows = size_t(prop->ns) * T->ndim;
        if (hipMemcpyAsync(ws.snap + size_t(h) * ws.accstride * T->ndim, prop->pos + size_t(h) * rows,
                           rows * sizeof(double), hipMemcpyDeviceToDevice, st) != hipSuccess)
            return LFG_E_LAUNCH;
    }
    if (T->gp) {
        L.res = ws.res;
        L.gpx = ws.gpx;
        L.gpb = ws.gpb;
        hipLaunchKernelGGL(k_gp_dcp, dim3((npairs + 64 / DCP_LANES - 1) / (64 / DCP_LANES)), dim3(64), 0, st, ws.geo,
                           ws.status, npairs);
        if ((rc = launch_ok())) return rc;
        if (T->nsub > 1) hipLaunchKernelGGL((k_lnlike<2, true>), dim3(npairs), dim3(LIKE_THREADS), 0, st, L);
        else hipLaunchKernelGGL((k_lnlike<2, false>), dim3(npairs), dim3(LIKE_THREADS), 0, st, L);
        if ((rc = launch_ok())) return rc;
        hipLaunchKernelGGL(k_gp_like, dim3(T->E * ((W + GP_PAIRS - 1) / GP_PAIRS)), dim3(GP_BLOCK), 0, st, L);
    } else {
        if (T->nsub > 1) hipLaunchKernelGGL((k_lnlike<1, true>), dim3(npairs), dim3(LIKE_THREADS), 0, st, L);
        else hipLaunchKernelGGL((k_lnlike<1, false>), dim3(npairs), dim3(LIKE_THREADS), 0, st, L);
    }
    if ((rc = launch_ok())) return rc;
    if (T->E > 1) {
        hipLaunchKernelGGL(k_combine_walkers, dim3((W + 3) / 4), dim3(256), 0, st, L);
        if ((rc = launch_ok())) return rc;
    }
    return finish();
}

int lfg_lnprior(const double* walkers, int W, const lfg_tree* T, double* lnprior, void* wsp, size_t ws_bytes,
                void* stream)
{
    if (W <= 0 || !T || T->E <= 0 || T->ndim <= 0 || !walkers || !lnprior) return LFG_E_ARGS;
    Ws ws = carve(wsp, W, T->E);
    if (!wsp || ws_bytes < ws.total) return LFG_E_WORKSPACE;
    hipStream_t st = static_cast<hipStream_t>(stream);
    SetupArgs S{walkers, W, T->ndim, T->E, 18, T->gather, T->npars, T->consts, T->prior_type, T->prior_p1,
                T->prior_p2, T->prior_norm, T->roche_priors, ws.geo, ws.status, ws.prior, ws.bstatus, 0,
                nullptr, nullptr};
    S.fixed_invalid = T->fixed_invalid;
    S.prior_c = T->prior_c;
    const int nlanes = 2 * W * T->E + W;
    hipLaunchKernelGGL(k_setup, dim3((nlanes + SETUP_BLOCK - 1) / SETUP_BLOCK), dim3(SETUP_BLOCK), 0, st, S);
    int rc = launch_ok();
    if (rc) return rc;
    hipLaunchKernelGGL(k_combine, dim3((W + 255) / 256), dim3(256), 0, st, W, T->E, ws.prior, ws.geo, nullptr,
                       lnprior);
    return launch_ok();
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

int lfg_stretch_step_half(double* pos, double* lnp, int W, int half, double a, unsigned long long seed,
                          unsigned long long step, double* q, double* zfac, const lfg_tree* T, int* naccept,
                          double* lnp_new, void* wsp, size_t ws_bytes, void* stream, void* const* ev)
{
    if (W < 4 || (W & 1) || (half != 0 && half != 1) || !(a > 1.0) || !pos || !lnp || !q || !zfac || !T)
        return LFG_E_ARGS;
    const Accept acc{pos, lnp, zfac, half, seed, step, naccept};
    const Propose prop{pos, a, q, zfac, half, seed, step, 0, W / 2};
    return lnprob_impl(q, W / 2, T, lnp_new, nullptr, wsp, ws_bytes, stream, ev, &acc, &prop);
}

int lfg_stretch_step_half_spec(double* pos, double* lnp, int W, int half, double a, unsigned long long seed,
                               unsigned long long step, double* q, double* zfac, const lfg_tree* T, int* naccept,
                               double* lnp_new, int spec_in, int spec_out, void* wsp, size_t ws_bytes, void* stream,
                               void* const* ev)
{
    if (W < 4 || (W & 1) || (half != 0 && half != 1) || !(a > 1.0) || !pos || !lnp || !q || !zfac || !T)
        return LFG_E_ARGS;
    const Accept acc{pos, lnp, zfac, half, seed, step, naccept};
    const Propose prop{pos, a, q, zfac, half, seed, step, 0, W / 2};
    const SpecCtl sp{spec_in != 0, spec_out != 0};
    // the fused-element build has no k_elements to host the candidates: plain half-step
    return lnprob_impl(q, W / 2, T, lnp_new, nullptr, wsp, ws_bytes, stream, ev, &acc, &prop, &sp);
}

int lfg_stretch_step_shard(const double* pos, int W, int half, double a, unsigned long long seed,
                           unsigned long long step, int lo, int n, double* q, double* zfac, const lfg_tree* T,
                           double* lnp_new, void* wsp, size_t ws_bytes, void* stream, void* const* ev)
{
    if (W < 4 || (W & 1) || (half != 0 && half != 1) || !(a > 1.0) || !pos || !q || !zfac || !T || !lnp_new ||
        n <= 0 || lo < 0 || lo + n > W / 2)
        return LFG_E_ARGS;
    const Propose prop{pos, a, q, zfac, half, seed, step, lo, W / 2};
    return lnprob_impl(q, n, T, lnp_new, nullptr, wsp, ws_bytes, stream, ev, nullptr, &prop);
}

int lfg_stretch_step_shard_spec(const double* pos, int W, int half, double a, unsigned long long seed,
                                unsigned long long step, int lo, int n, double* q, double* zfac, const lfg_tree* T,
                                double* lnp_new, int spec_in, int spec_out, void* wsp, size_t ws_bytes,
                                void* stream, void* const* ev)
{
    if (W < 4 || (W & 1) || (half != 0 && half != 1) || !(a > 1.0) || !pos || !q || !zfac || !T || !lnp_new ||
        n <= 0 || lo < 0 || lo + n > W / 2)
        return LFG_E_ARGS;
    const Propose prop{pos, a, q, zfac, half, seed, step, lo, W / 2};
    const SpecCtl sp{spec_in != 0, spec_out != 0};
    return lnprob_impl(q, n, T, lnp_new, nullptr, wsp, ws_bytes, stream, ev, nullptr, &prop, &sp);
}

int lfg_stretch_step_shard_fold(double* pos, double* lnp, int W, int half, double a, unsigned long long seed,
                                unsigned long long step, int lo, int n, double* q, double* zfac, const lfg_tree* T,
                                const double* verdict_prev, double* verdict, double* lnp_new, int* naccept,
                                int spec_in, int spec_out, void* wsp, size_t ws_bytes, void* stream, void* const* ev)
{
    if (W < 4 || (W & 1) || (half != 0 && half != 1) || !(a > 1.0) || !pos || !lnp || !q || !zfac || !T ||
        !lnp_new || !verdict || n <= 0 || lo < 0 || lo + n > W / 2 || (spec_in && !verdict_prev) ||
        (verdict_prev && half == 0 && step == 0))
        return LFG_E_ARGS;
    const Propose prop{pos, a, q, zfac, half, seed, step, lo, W / 2};
    const SpecCtl sp{spec_in != 0, spec_out != 0};
    const FoldCtl fold{verdict_prev, verdict, pos, lnp, naccept};
    return lnprob_impl(q, n, T, lnp_new, nullptr, wsp, ws_bytes, stream, ev, nullptr, &prop, &sp, &fold);
}

int lfg_stretch_apply_verdicts(double* pos, double* lnp, int W, int ndim, int half, double a, unsigned long long seed,
                               unsigned long long step, const double* verdict, int* naccept, void* stream)
{
    if (W < 4 || (W & 1) || ndim <= 0 || (half != 0 && half != 1) || !(a > 1.0) || !pos || !lnp || !verdict)
        return LFG_E_ARGS;
    return apply_verdicts(pos, lnp, W, ndim, half, a, verdict, seed, step, naccept, nullptr,
                          static_cast<hipStream_t>(stream));
}

int lfg_stretch_lnprob_accept(double* pos, double* lnp, int W, int half, const double* q, const double* zfac,
                              const lfg_tree* T, unsigned long long seed, unsigned long long step, int* naccept,
                              double* lnp_new, void* wsp, size_t ws_bytes, void* stream, void* const* ev)
{
    if (W < 4 || (W & 1) || (half != 0 && half != 1) || !pos || !lnp || !q || !zfac || !T) return LFG_E_ARGS;
    const Accept acc{pos, lnp, zfac, half, seed, step, naccept};
    return lnprob_impl(q, W / 2, T, lnp_new, nullptr, wsp, ws_bytes, stream, ev, &acc);
}

static int propose_impl(const double* pos, int W, int ndim, int half, double a, unsigned long long seed,
                        unsigned long long step, const unsigned long long* stepp, double* q, double* zfac,
                        void* stream)
{
    if (W < 4 || (W & 1) || ndim <= 0 || (half != 0 && half != 1) || !(a > 1.0) || !pos || !q || !zfac)
        return LFG_E_ARGS;
    const int ns = W / 2;
    hipLaunchKernelGGL(k_propose, dim3((ns + 63) / 64), dim3(64), 0, static_cast<hipStream_t>(stream), pos, W,
                       ndim, half, a, seed, step, stepp, q, zfac);
    return launch_ok();
}

static int accept_impl(double* pos, double* lnp, int W, int ndim, int half, const double* q, const double* zfac,
                       const double* lnp_new, unsigned long long seed, unsigned long long step,
                       const unsigned long long* stepp, int* naccept, void* stream)
{
    if (W < 4 || (W & 1) || ndim <= 0 || (half != 0 && half != 1) || !pos || !lnp || !q || !zfac || !lnp_new)
        return LFG_E_ARGS;
    const int ns = W / 2;
    hipLaunchKernelGGL(k_accept, dim3((ns + 63) / 64), dim3(64), 0, static_cast<hipStream_t>(stream), pos, lnp,
                       W, ndim, half, q, zfac, lnp_new, seed, step, stepp, naccept);
    return launch_ok();
}

int lfg_stretch_accept_regen(double* pos, double* lnp, int W, int ndim, int half, double a,
                             unsigned long long seed, unsigned long long step, const double* lnp_new, int* naccept,
                             void* stream)
{
    if (W < 4 || (W & 1) || ndim <= 0 || (half != 0 && half != 1) || !(a > 1.0) || !pos || !lnp || !lnp_new)
        return LFG_E_ARGS;
    const int ns = W / 2;
    hipLaunchKernelGGL(k_accept_regen, dim3((ns + REGEN_WAVES - 1) / REGEN_WAVES), dim3(64 * REGEN_WAVES), 0,
                       static_cast<hipStream_t>(stream), pos, lnp, W, ndim, half, a, lnp_new, seed, step, naccept,
                       nullptr);
    return launch_ok();
}

int lfg_stretch_accept_regen_spec(double* pos, double* lnp, int W, int half, double a, unsigned long long seed,
                                  unsigned long long step, const double* lnp_new, int* naccept, const lfg_tree* T,
                                  int n, void* wsp, size_t ws_bytes, void* stream)
{
    if (W < 4 || (W & 1) || (half != 0 && half != 1) || !(a > 1.0) || !pos || !lnp || !lnp_new || !T ||
        T->ndim <= 0 || n <= 0 || n > W / 2)
        return LFG_E_ARGS;
    const Ws ws = carve(wsp, n, T->E, T->gp ? T->max_n : 0, T->ndim, W / 2);
    if (!wsp || ws_bytes < ws.total) return LFG_E_WORKSPACE;
    const int ns = W / 2;
    hipLaunchKernelGGL(k_accept_regen, dim3((ns + REGEN_WAVES - 1) / REGEN_WAVES), dim3(64 * REGEN_WAVES), 0,
                       static_cast<hipStream_t>(stream), pos, lnp, W, T->ndim, half, a, lnp_new, seed, step, naccept,
                       ws.accflag + size_t(half) * ws.accstride);
    return launch_ok();
}

int lfg_stretch_propose(const double* pos, int W, int ndim, int half, double a, unsigned long long seed,
                        unsigned long long step, double* q, double* zfac, void* stream)
{
    return propose_impl(pos, W, ndim, half, a, seed, step, nullptr, q, zfac, stream);
}

int lfg_stretch_accept(double* pos, double* lnp, int W, int ndim, int half, const double* q, const double* zfac,
                       const double* lnp_new, unsigned long long seed, unsigned long long step, int* naccept,
                       void* stream)
{
    return accept_impl(pos, lnp, W, ndim, half, q, zfac, lnp_new, seed, step, nullptr, naccept, stream);
}

int lfg_stretch_propose_dev(const double* pos, int W, int ndim, int half, double a, unsigned long long seed,
                            const unsigned long long* step_dev, double* q, double* zfac, void* stream)
{
    if (!step_dev) return LFG_E_ARGS;
    return propose_impl(pos, W, ndim, half, a, seed, 0, step_dev, q, zfac, stream);
}

int lfg_stretch_accept_dev(double* pos, double* lnp, int W, int ndim, int half, const double* q,
                           const double* zfac, const double* lnp_new, unsigned long long seed,
                           const unsigned long long* step_dev, int* naccept, void* stream)
{
    if (!step_dev) return LFG_E_ARGS;
    return accept_impl(pos, lnp, W, ndim, half, q, zfac, lnp_new, seed, 0, step_dev, naccept, stream);
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
                ws.geo, ws.status, ws.prior, ws.bstatus, 0, nullptr, nullptr};
    int rc = run_front(S, ws, st, nullptr, true);  // the white-box tables come from k_elements
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

int lfg_wdphases(const double* q, const double* inc, const double* r1, int n, int ntheta, double* phi3,
                 double* phi4, int* status, void* stream)
{
    if (n < 0 || ntheta < 1 || (n > 0 && (!q || !inc || !r1 || !phi3 || !phi4 || !status))) return LFG_E_ARGS;
    if (n == 0) return LFG_OK;
    hipLaunchKernelGGL(k_wdphases, dim3((n + 63) / 64), dim3(64), 0, static_cast<hipStream_t>(stream), q, inc, r1,
                       n, ntheta, phi3, phi4, status);
    return launch_ok();
}

int lfg_gp_lnlike(const double* x, const double* ye, const double* res, int W, int N, const double* hyp,
                  const double* blocks, int nb, double* lnlike, void* stream)
{
    if (W <= 0 || N < 0 || nb < 0 || !hyp || !lnlike || (N > 0 && (!x || !ye || !res)) || (nb > 0 && !blocks))
        return LFG_E_ARGS;
    hipLaunchKernelGGL(k_gp, dim3(W), dim3(64), 0, static_cast<hipStream_t>(stream), x, ye, res, N, hyp, blocks, nb,
                       lnlike);
    return launch_ok();
}

#ifdef LFG_PROFILE_LIKE
// diagnostic build only: k_lnlike prologue stamps
int lfg_debug_like_cycles(unsigned long long* host)
{
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_like_cyc), sizeof(g_like_cyc)) == hipSuccess ? 0 : -1;
}

// per-wave phase stamps: host [2][6][4096] (min, max over the block's waves);
// reset (host == nullptr): min slots to ~0, max slots to 0
int lfg_debug_like_waves(unsigned long long* host)
{
    static unsigned long long buf[2][6][4096];
    if (!host) {
        for (int i = 0; i < 6 * 4096; ++i) { (&buf[0][0][0])[i] = ~0ull; (&buf[1][0][0])[i] = 0ull; }
        return hipMemcpyToSymbol(HIP_SYMBOL(g_like_wav), buf, sizeof(buf)) == hipSuccess ? 0 : -1;
    }
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_like_wav), sizeof(g_like_wav)) == hipSuccess ? 0 : -1;
}
#endif

#ifdef LFG_PROFILE_PAIR
// diagnostic build only: k_pair's phase stamps of the last launch, host [20][4096]
int lfg_debug_pair(unsigned long long* host)
{
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_pair_t), sizeof(g_pair_t)) == hipSuccess ? 0 : -1;
}
// its per-chunk job stamps (start, sink entry, end), host [3][16][4096]
int lfg_debug_pair_jobs(unsigned long long* host)
{
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_pair_j), sizeof(g_pair_j)) == hipSuccess ? 0 : -1;
}
// and its per-wave sweep stamps, host [4][8][4096]
int lfg_debug_pair_waves(unsigned long long* host)
{
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_pair_w), sizeof(g_pair_w)) == hipSuccess ? 0 : -1;
}
int lfg_debug_long_tables(unsigned long long* host)
{
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_long_t), sizeof(g_long_t)) == hipSuccess ? 0 : -1;
}
#endif

#ifdef LFG_PROFILE_ELEM
// diagnostic build only: k_elements' per-wave stamps of the last launch, host [4][32768]
int lfg_debug_elem_waves(unsigned long long* host)
{
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_elem_wav), sizeof(g_elem_wav)) == hipSuccess ? 0 : -1;
}
#endif

#ifdef LFG_PROFILE_SETUP
// diagnostic build only: copy the k_setup lane stamps to the host
int lfg_debug_setup_cycles(unsigned long long* host)
{
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_setup_cyc), sizeof(g_setup_cyc)) == hipSuccess ? 0 : -1;
}
#endif

// the hash of the sources and flags this library was built from
// (lfit_python_amd._native.source_hash, passed by build()); the tag string
// lets build() read it back from the file without loading it
#ifndef LFG_SRC_HASH
#define LFG_SRC_HASH "unhashed"
#endif
__attribute__((used)) const char lfg_src_hash_tag[] = "lfg-src-hash:" LFG_SRC_HASH;

const char* lfg_version(void)
{
    // the layout named is the one lfg_set_layout / LFG_PAIR currently select
    // for eligible trees (pair: k_pair and k_pair LONG; two_kernel: k_elements
    // + k_lnlike); lfg_layout(T) gives a given tree's kernels
    int m = g_pair_layout.load(std::memory_order_relaxed);
    if (m == -2) m = pair_env() ? 1 : 0;
    return m == 1 ? "lfg 0.5.0 gfx950 fp64 layout=pair src=" LFG_SRC_HASH
                  : "lfg 0.5.0 gfx950 fp64 layout=two_kernel src=" LFG_SRC_HASH;
}

#ifdef LFG_COUNT_ITERS
// diagnostic builds only: read and clear the iteration counters of k_elements
int lfg_diag_iters(unsigned long long* out)
{
    if (hipDeviceSynchronize() != hipSuccess || hipMemcpyFromSymbol(out, HIP_SYMBOL(g_iter_dbg), sizeof(g_iter_dbg)) != hipSuccess)
        return LFG_E_LAUNCH;
    unsigned long long z[64] = {};
    return hipMemcpyToSymbol(HIP_SYMBOL(g_iter_dbg), z, sizeof(z)) == hipSuccess ? LFG_OK : LFG_E_LAUNCH;
}
#endif

}  // extern "C"
#endif  // LFG_NOLICM_TU
