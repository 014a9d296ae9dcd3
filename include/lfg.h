/*
 * lfg.h -- C ABI of liblfg_hip.so, the MI355X-native CV eclipse light-curve
 * evaluator.  Drop-in for the lfit.CV.calcFlux() hot path of
 * wildjames/lfit_python (reference at /root/reference).
 *
 * Every entry point takes plain pointers and sizes (no torch types), is
 * re-entrant, never allocates, and enqueues its kernels on the caller's HIP
 * stream (`stream` = hipStream_t, NULL = default stream).  The one piece of
 * process-wide state is the kernel-layout switch (lfg_set_layout, read once
 * from the environment's LFG_PAIR): a measurement and test control that
 * selects between two implementations with identical results; every other
 * input is an argument.  Pointers marked [dev] are device (HBM) pointers; scratch space is
 * passed in as `ws` of at least lfg_workspace_size() bytes.  All arithmetic is
 * FP64.  Return value: LFG_OK or an LFG_E_* code (launch/argument errors).
 * Per-parameter-set model failures are NOT call errors: they are reported in
 * `status` and turn into NaN flux / -inf ln_like, exactly as the reference
 * turns an lfit exception into NaN (CVModel.py:137-144) and -inf
 * (CVModel.py:163-171, model.py:485-493).
 */
#ifndef LFG_H
#define LFG_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LFG_OK               0
#define LFG_E_ARGS          -1
#define LFG_E_WORKSPACE     -2
#define LFG_E_LAUNCH        -3

/* per-parameter-set status (same codes as oracle/lfg_oracle.h) */
#define LFG_ST_OK            0
#define LFG_ST_BAD_Q         1
#define LFG_ST_BAD_DPHI      2
#define LFG_ST_BAD_GEOMETRY  3
#define LFG_ST_BAD_STREAM    4
#define LFG_ST_BAD_ARGS      5

/* element grid of MODEL_SPEC.md section 5 */
#define LFG_NWD      400
#define LFG_NDISC    1000
#define LFG_NBS      100
#define LFG_NDONOR   400
#define LFG_NEL      (LFG_NWD + LFG_NDISC + LFG_NBS)
#define LFG_NGEO     48

/*
 * Compiled model tree: the flat description of a model.py/CVModel.py tree
 * (trunk -> bands -> eclipses) produced by lfit_python_amd.batch.  Replaces
 * the per-walker Python recursion of Node.ln_prob (model.py:476-498).
 *   gather[e*18+k] >= 0 : CV parameter k of eclipse e is walker[gather]
 *   gather[e*18+k] <  0 : it is the constant consts[-1-gather] (isVar = 0)
 * CV parameter order is lfit's (CVModel.py:384-388; README.md:24-43), so the
 * tree's yaw/tilt storage order (CVModel.py:376-380) is swapped in `gather`.
 */
typedef struct lfg_tree lfg_tree;
/* scratch bytes lfg_lnprob & co. need for W walkers of `tree` (GP trees
 * also keep every pair's residuals, W x E x max_n doubles) */
size_t lfg_workspace_size_tree(int W, const lfg_tree* tree);

struct lfg_tree {
    int E;                    /* eclipses (leaves)                          */
    int ndim;                 /* walker vector length                       */
    int nsub;                 /* exposure sub-bins S >= 1 (1 = native)      */
    int max_n;                /* max data points of any eclipse: the max
                                 of off[e+1] - off[e] (off[0] = 0; with one
                                 eclipse the kernels take {0, max_n})       */
    const int* gather;        /* [dev] E*18                                 */
    const int* npars;         /* [dev] E, 14 or 18                          */
    const double* consts;     /* [dev] constant parameter values            */
    const int* off;           /* [dev] E+1 offsets into x/y/ye/w            */
    const double* x;          /* [dev] phases                               */
    const double* y;          /* [dev] fluxes                               */
    const double* ye;         /* [dev] flux errors                          */
    const double* w;          /* [dev] exposure half-widths (lc.w)          */
    const int* prior_type;    /* [dev] ndim; 0 gauss 1 gaussPos 2 uniform
                                 3 log_uniform 4 mod_jeff; NULL = no priors */
    const double* prior_p1;   /* [dev] ndim                                 */
    const double* prior_p2;   /* [dev] ndim                                 */
    const double* prior_norm; /* [dev] ndim: Prior.normalise                */
    int roche_priors;         /* 1: LCModel + eclipse Roche priors
                                 (CVModel.py:193-324, 440-491)             */
    /* Gaussian-process likelihood of GPLCModel trees (CVModel.py:494-711);
     * gp = 0: chi^2 (gp_* unused).  Each eclipse's points must be sorted by
     * phase (lfit_python_amd.batch sorts them). */
    int gp;
    const int* gp_gather;     /* [dev] E*3: ln_ampin_gp, ln_ampout_gp,
                                 ln_tau_gp (walker column or -1-const)      */
    const double* gp_base;    /* [dev] E*4: q, dphi, rwd of the changepoint
                                 cache and its distance dist_cp
                                 (CVModel.py:548-576)                       */
    const int* gp_ecl;        /* [dev] E*2: first and last eclipse number of
                                 the changepoint list (CVModel.py:582-590)  */
    /* 1: a fixed (isVar = 0) parameter lies outside its prior, so
     * Node.ln_prior is -inf for every walker (model.py:439-441 checks every
     * parameter, variable or not); ln_prob = -inf on every path */
    int fixed_invalid;
    /* [dev] ndim x 2, nullable: per-parameter constants of Prior.ln_prob so
     * the prior lanes need no transcendental per parameter:
     *   gauss, gaussPos   c0 = -ln(sqrt(2 pi) p2),  c1 = 1 / p2
     *   uniform           c0 = ln(1 / |p1 - p2|)
     *   log_uniform, mod_jeff  c0 = -ln(normalise)
     * (lfit_python_amd.batch.prior_consts).  NULL: each term from
     * prior_p1/p2/norm directly. */
    const double* prior_c;
};

/* scratch bytes needed for W parameter sets x E eclipses (chi^2 trees and
 * lfg_flux / lfg_elements) */
size_t lfg_workspace_size(int W, int E);

/*
 * Batched lfit.CV.calcFlux (CVModel.py:132-147; lfit API README.md:21-48).
 *   pars   [dev] W x P (P = 14 simple or 18 complex bright spot)
 *   x, w   [dev] N phases and exposure half-widths shared by all W sets
 *          (w = NULL: point evaluation)
 *   flux   [dev] W x N
 *   comps  [dev] nullable, 4 x W x N: white dwarf, disc, bright spot, donor
 *          (lfit's cv.ywd, cv.yd, cv.ys, cv.yrs; CVModel.py:155)
 *   status [dev] W (LFG_ST_*)
 */
int lfg_flux(const double* pars, int W, int P, const double* x,
             const double* w, int N, int nsub, double* flux, double* comps,
             int* status, void* ws, size_t ws_bytes, void* stream);

/*
 * Fused single-eclipse ln_like, no tree: SimpleEclipse.chisq / ln_like
 * (CVModel.py:157-191) of W parameter sets against one light curve,
 * ln_like = -0.5 sum_p ((y_p - flux_p) / ye_p)^2, a NaN flux -> chi^2 = +inf
 * (CVModel.py:163-171); no flux array is materialised and no prior is
 * applied (lfg_lnprob adds the priors through a tree).
 *   pars, x, w, N, nsub, status: as lfg_flux
 *   y, ye   [dev] N data points and errors
 *   lnlike  [dev] W (-inf where status != LFG_ST_OK)
 * Workspace: lfg_workspace_size(W, 1).
 */
int lfg_lnlike(const double* pars, int W, int P, const double* x,
               const double* w, int N, int nsub, const double* y,
               const double* ye, double* lnlike, int* status, void* ws,
               size_t ws_bytes, void* stream);

/*
 * Batched emcee log-probability of a whole walker ensemble through a compiled
 * tree: mcmcfit.ln_prob (mcmcfit.py:37-41) -> Node.ln_prob (model.py:476-498)
 * = ln_prior (model.py:426-474 + Roche priors) + sum_e -0.5 chi^2_e
 * (CVModel.py:157-191), fused: no flux array is materialised.
 *   walkers  [dev] W x ndim
 *   lnp      [dev] W
 *   lnlike_e [dev] nullable, W x E per-eclipse ln_like
 */
int lfg_lnprob(const double* walkers, int W, const lfg_tree* tree,
               double* lnp, double* lnlike_e, void* ws, size_t ws_bytes,
               void* stream);

/*
 * ln_prior alone of a walker ensemble through a compiled tree: Node.ln_prior
 * of the tree root (model.py:426-474) with the LCModel and eclipse Roche
 * priors (CVModel.py:193-324, 440-491), as mcmcfit.ln_prior
 * (mcmcfit.py:30-34) feeds the walker initialisation (mcmc_utils.py:46-72).
 *   walkers [dev] W x ndim;  lnprior [dev] W
 */
int lfg_lnprior(const double* walkers, int W, const lfg_tree* tree,
                double* lnprior, void* ws, size_t ws_bytes, void* stream);

/*
 * White-box access to the element tables of MODEL_SPEC.md section 5 for W
 * parameter sets (tests): a, b, wgt [dev] W x LFG_NEL eclipse intervals
 * (phase) and weights; donor [dev] W x LFG_NDONOR x 3; geo [dev] W x LFG_NGEO;
 * status [dev] W.
 */
int lfg_elements(const double* pars, int W, int P, double* a, double* b,
                 double* wgt, double* donor, double* geo, int* status,
                 void* ws, size_t ws_bytes, void* stream);

/*
 * Batched trm.roche primitives (CVModel.py:222,288,460,561):
 *   op 0 xl1(q = a[i])                     -> out[i]
 *   op 1 findphi(q = a[i], inc = b[i])     -> out[i]
 *   op 2 findi(q = a[i], dphi = b[i])      -> out[i]
 *   op 3 bspot(q = a[i], rad = b[i])       -> out[4i .. 4i+3] = x, y, vx, vy
 * a, b, out, status are [dev]; status[i] = LFG_ST_*.
 */
int lfg_roche(int op, const double* a, const double* b, int n, double* out,
              int* status, void* stream);

/*
 * Same as lfg_lnprob, recording LFG_NEV caller-created hipEvent_t events on
 * `stream` around each phase (bench timing).  NULL entries are skipped.
 *   ev[0] before k_setup (every layout);
 *   ev[1] after k_setup (= ev[0]'s position when the speculative candidates
 *         stand in for it);
 *   ev[2] after k_elements on the two-kernel layout; on the k_pair layout
 *         (lfg_layout = 1) nothing runs between ev[1] and ev[2];
 *   ev[3] after the likelihood kernels: k_lnlike, or k_pair (element solve,
 *         chi^2, ln_prob and the fused acceptance in one launch), followed
 *         for GP trees by k_gp_like and for E > 1 by k_combine_walkers.
 * So ev[2] -> ev[3] times k_pair alone for a one-eclipse chi^2 tree.
 */
#define LFG_NEV 4
int lfg_lnprob_timed(const double* walkers, int W, const lfg_tree* tree,
                     double* lnp, double* lnlike_e, void* ws, size_t ws_bytes,
                     void* stream, void* const* ev);

/*
 * Device-resident affine-invariant stretch move (Goodman & Weare 2010), the
 * move of emcee.EnsembleSampler that the reference drives (mcmcfit.py:283-288,
 * mcmc_utils.py:114-183), with the emcee 2.x fixed red/blue halves:
 * half h in {0, 1} updates walkers [h W/2, (h+1) W/2) against the other half.
 * Random numbers come from Philox4x32-10 keyed by `seed` and counted by
 * (walker, step, half), so every rank of a multi-GPU run draws identical
 * proposals without communicating.
 *   pos [dev] W x ndim (updated in place by accept), lnp [dev] W
 *   q   [dev] W/2 x ndim proposals, zfac [dev] W/2 = (ndim-1) ln z
 *   lnp_new [dev] W/2 ln_prob of q;  naccept [dev] W acceptance counters
 */
int lfg_stretch_propose(const double* pos, int W, int ndim, int half,
                        double a, unsigned long long seed,
                        unsigned long long step, double* q, double* zfac,
                        void* stream);
int lfg_stretch_accept(double* pos, double* lnp, int W, int ndim, int half,
                       const double* q, const double* zfac,
                       const double* lnp_new, unsigned long long seed,
                       unsigned long long step, int* naccept, void* stream);

/*
 * One half-step of the stretch move after the proposal: the batched ln_prob
 * of the proposals q (lfg_lnprob on W/2 walkers) with the Metropolis step of
 * lfg_stretch_accept fused into the kernel that forms each ln_prob (same
 * draws, same result; one launch fewer per half-step).  pos, lnp, naccept
 * as lfg_stretch_accept; lnp_new [dev] nullable W/2; ev: LFG_NEV events or
 * NULL.  Single process only: with walker shards over ranks, use lfg_lnprob,
 * gather, then lfg_stretch_accept.
 */
int lfg_stretch_lnprob_accept(double* pos, double* lnp, int W, int half,
                              const double* q, const double* zfac,
                              const lfg_tree* tree, unsigned long long seed,
                              unsigned long long step, int* naccept,
                              double* lnp_new, void* ws, size_t ws_bytes,
                              void* stream, void* const* ev);

/*
 * A whole half-step of the stretch move in three kernels: the proposals of
 * half `half` are formed inside k_setup (k_propose's arithmetic and draws;
 * written to q / zfac), their ln_prob evaluated, and the Metropolis step
 * fused as in lfg_stretch_lnprob_accept.  Same chain as lfg_stretch_propose
 * + lfg_lnprob + lfg_stretch_accept.  q [dev] W/2 x ndim, zfac [dev] W/2
 * (outputs); the rest as lfg_stretch_lnprob_accept.  Single process only.
 */
int lfg_stretch_step_half(double* pos, double* lnp, int W, int half, double a,
                          unsigned long long seed, unsigned long long step,
                          double* q, double* zfac, const lfg_tree* tree,
                          int* naccept, double* lnp_new, void* ws,
                          size_t ws_bytes, void* stream, void* const* ev);

/*
 * lfg_stretch_step_half with the next half's setup formed speculatively.
 * The proposal of walker k of the next half uses its partner j's position
 * after this half's Metropolis step: j's current position or j's proposal.
 * With spec_out = 1, this call's k_elements also runs the next half's k_setup
 * lanes for both cases (the chip is mostly idle in k_setup, which is bound by
 * dependent FP64 latency), and k_lnlike records which moves it accepted.
 * With spec_in = 1 the call skips k_setup: k_elements takes each pair's
 * candidate for the partner's actual fate.  spec_in = 1 is valid only when
 * the previous call on this workspace was this sampler's other half (the
 * step before for half 0) with spec_out = 1, and pos / lnp were not changed
 * in between; the chain is bit-identical to lfg_stretch_step_half's.  The
 * workspace must come from lfg_workspace_size_tree (it holds the candidates).
 */
int lfg_stretch_step_half_spec(double* pos, double* lnp, int W, int half,
                               double a, unsigned long long seed,
                               unsigned long long step, double* q,
                               double* zfac, const lfg_tree* tree,
                               int* naccept, double* lnp_new, int spec_in,
                               int spec_out, void* ws, size_t ws_bytes,
                               void* stream, void* const* ev);

/*
 * The half-step of one rank when the walkers of each half are sharded over
 * ranks (the replacement of the reference's pool.map over walkers,
 * mcmcfit.py:273-288).  lfg_stretch_step_shard forms the proposals of
 * walkers lo .. lo+n-1 of half `half` inside k_setup (same draws as
 * lfg_stretch_propose's lanes lo .. lo+n-1) and writes their ln_prob to
 * lnp_new [dev] n; q [dev] n x ndim and zfac [dev] n receive the proposals.
 * After the caller has gathered every rank's lnp_new into the W/2 vector,
 * lfg_stretch_accept_regen applies the Metropolis step to the whole half,
 * re-forming each proposal from its draws (bit-identical to k_propose), so
 * no rank needs another rank's q.  Three kernels + collective + one kernel
 * per half-step; the chain equals lfg_stretch_step_half's.
 */
int lfg_stretch_step_shard(const double* pos, int W, int half, double a,
                           unsigned long long seed, unsigned long long step,
                           int lo, int n, double* q, double* zfac,
                           const lfg_tree* tree, double* lnp_new, void* ws,
                           size_t ws_bytes, void* stream, void* const* ev);

/*
 * The sharded half-step with the speculative setup of
 * lfg_stretch_step_half_spec: this call's k_elements also forms the setup
 * of walkers lo .. lo+n-1 of the next half for both fates of each partner
 * (spec_out), and with spec_in the call skips k_setup and takes each pair's
 * candidate by the acceptances lfg_stretch_accept_regen_spec recorded for the
 * whole half.  spec_in = 1 is valid only right after lfg_stretch_step_shard_spec
 * (other half, spec_out = 1, same lo / n / ensemble) and
 * lfg_stretch_accept_regen_spec of that half on the same workspace, which must
 * be sized for W/2 walkers (lfg_workspace_size_tree(W/2, tree)).
 */
int lfg_stretch_step_shard_spec(const double* pos, int W, int half, double a,
                                unsigned long long seed, unsigned long long step,
                                int lo, int n, double* q, double* zfac,
                                const lfg_tree* tree, double* lnp_new,
                                int spec_in, int spec_out, void* ws,
                                size_t ws_bytes, void* stream, void* const* ev);

/*
 * lfg_stretch_accept_regen that also records each walker's acceptance in the
 * workspace of the rank's lfg_stretch_step_shard_spec calls (n: their shard
 * size), for the next half's candidate choice.
 */
int lfg_stretch_accept_regen_spec(double* pos, double* lnp, int W, int half,
                                  double a, unsigned long long seed,
                                  unsigned long long step, const double* lnp_new,
                                  int* naccept, const lfg_tree* tree, int n,
                                  void* ws, size_t ws_bytes, void* stream);
int lfg_stretch_accept_regen(double* pos, double* lnp, int W, int ndim,
                             int half, double a, unsigned long long seed,
                             unsigned long long step, const double* lnp_new,
                             int* naccept, void* stream);

/*
 * The sharded half-step with the acceptance deferred into the next launch
 * (the multi-rank replacement of the reference's pool.map fan-out,
 * mcmcfit.py:273-288, in ONE kernel plus the collective per half-step):
 *
 *   rank r, half h:  lfg_stretch_step_shard_fold(.., verdict_prev = V[1-h],
 *                                                 verdict = v_r, ..)
 *                    all_gather(V[h] <- v_r over ranks)
 *
 * A verdict is the walker's new ln_prob where its move was accepted and NaN
 * where it was not (k_accept_regen's test, made by the rank that evaluated
 * the walker, whose old ln_prob is at hand).  The call applies verdict_prev
 * (the other half's moves of the half-step before: rows re-formed from the
 * draws, lnp, naccept) to pos / lnp / naccept, chooses each pair's
 * speculative candidate by the same verdicts, evaluates walkers lo .. lo+n-1
 * of half `half` (q, zfac, lnp_new [dev] n as lfg_stretch_step_shard) and
 * writes their verdicts to verdict [dev] n.  On the k_pair layout with one
 * eclipse and chi^2 that is one launch; other trees run the apply, the
 * shard's kernels and a verdict kernel in sequence (same results).
 *   verdict_prev [dev] W/2 or NULL (nothing pending: the chain's first call,
 *                or after lfg_stretch_apply_verdicts); it must be the other
 *                half's verdicts of the immediately preceding half-step
 *   spec_in / spec_out as lfg_stretch_step_shard_spec; spec_in = 1 needs
 *                verdict_prev and the same workspace as that call
 * Until the pending verdicts are applied, pos / lnp / naccept of that half
 * hold the state before its last move: lfg_stretch_apply_verdicts(.., half,
 * step of that half's proposal, V[half]) brings them up to date (the flush at
 * the end of a run).  Workspace: lfg_workspace_size_tree(W/2, tree).  The
 * chain equals lfg_stretch_step_shard_spec + lfg_stretch_accept_regen_spec's.
 */
int lfg_stretch_step_shard_fold(double* pos, double* lnp, int W, int half,
                                double a, unsigned long long seed,
                                unsigned long long step, int lo, int n,
                                double* q, double* zfac, const lfg_tree* tree,
                                const double* verdict_prev, double* verdict,
                                double* lnp_new, int* naccept, int spec_in,
                                int spec_out, void* ws, size_t ws_bytes,
                                void* stream, void* const* ev);
int lfg_stretch_apply_verdicts(double* pos, double* lnp, int W, int ndim,
                               int half, double a, unsigned long long seed,
                               unsigned long long step, const double* verdict,
                               int* naccept, void* stream);

/*
 * The same two moves with the step counter read from device memory
 * (step_dev [dev] 1 x uint64), so that one emcee iteration can be captured
 * in a HIP graph and replayed; the caller advances *step_dev after half 1.
 */
int lfg_stretch_propose_dev(const double* pos, int W, int ndim, int half,
                            double a, unsigned long long seed,
                            const unsigned long long* step_dev, double* q,
                            double* zfac, void* stream);
int lfg_stretch_accept_dev(double* pos, double* lnp, int W, int ndim, int half,
                           const double* q, const double* zfac,
                           const double* lnp_new, unsigned long long seed,
                           const unsigned long long* step_dev, int* naccept,
                           void* stream);

/*
 * Batched trm.roche.wdphases(q, iangle, r1, ntheta) (CVModel.py:564): third
 * and fourth contact phases of a sphere of radius r1 at the white dwarf.
 * q, inc (degrees), r1, phi3, phi4, status: [dev] n.
 */
int lfg_wdphases(const double* q, const double* inc, const double* r1, int n,
                 int ntheta, double* phi3, double* phi4, int* status,
                 void* stream);

/*
 * Batched george GP log-likelihood of the kernel SimpleGPEclipse.create_GP
 * builds (CVModel.py:603-648): ampin*Matern32(tau) + ampout*Matern32(tau) on
 * each of nb closed blocks, plus ye^2 on the diagonal (gp.compute(x, ye),
 * CVModel.py:687), for W residual vectors (gp.log_likelihood(r),
 * CVModel.py:691).  Exact, O(N) per set (MODEL_SPEC 10.4).
 *   x, ye   [dev] N, sorted by x (an unsorted x gives -inf)
 *   res     [dev] W x N residuals
 *   hyp     [dev] W x 3: ampin, ampout, tau (george's metric)
 *   blocks  [dev] W x nb x 2: block [lo, hi] in x
 *   lnlike  [dev] W (-inf where not positive definite or not finite)
 */
int lfg_gp_lnlike(const double* x, const double* ye, const double* res, int W,
                  int N, const double* hyp, const double* blocks, int nb,
                  double* lnlike, void* stream);

/*
 * lfit's component objects (MODEL_SPEC 5.6): the unit-normalised flux of one
 * component for W parameter sets, at inclination inc (degrees, not dphi),
 * on a caller-chosen grid.  Replaces
 *   lfit.PyWhiteDwarf(rwd/xl1, ulimb).calcFlux(q, inc, phi, width)   kind 0
 *   lfit.PyDisc(q, rwd/xl1, rdisc, dexp, npts).calcFlux(...)         kind 1
 *   lfit.PySpot(q, rdisc, az, fis, scale, exp1, exp2, tilt, yaw,
 *               complex).calcFlux(...)                                kind 2
 *   lfit.PyDonor(q, npts).calcFlux(...)                              kind 3
 * (testCV.py:27-49, fitEcl.py:21-24).  cpars [dev] W x ncp with ncp = 2
 * (rwd/xl1, ulimb), 3 (rwd/xl1, rdisc/xl1, dexp), 8 (rdisc/xl1, az, fis,
 * scale/xl1, exp1, exp2, tilt, yaw), 0 (donor: cpars unused);
 * q, inc [dev] W; grids: disc n1 rings x n2 azimuths, spot n1 strip
 * elements, donor n1 bands x n2 azimuths (the WD grid is fixed, 400 tiles);
 * x, w [dev] N phases (used as given: no phi0) and exposure half-widths
 * (w = NULL: points); out [dev] W x N; status [dev] W.  Scratch ws of at
 * least lfg_component_workspace_size(kind, W, n1, n2) bytes.
 */
size_t lfg_component_workspace_size(int kind, int W, int n1, int n2);
int lfg_component(int kind, const double* cpars, int ncp, const double* q,
                  const double* inc, int W, int n1, int n2, const double* x,
                  const double* w, int N, double* out, int* status, void* ws,
                  size_t ws_bytes, void* stream);

/* hipEvent helpers for hosts without a HIP binding (ctypes) */
int lfg_event_create(void** ev);
int lfg_event_destroy(void* ev);
int lfg_event_elapsed_ms(void* start, void* stop, float* ms);

const char* lfg_version(void);

/* The kernels a tree's ln_prob runs on: 1 = k_pair (element solve and
 * likelihood of a walker-eclipse pair in one workgroup: eclipses of at most
 * 512 points, nsub = 1), 0 = k_elements + k_lnlike (every other tree);
 * LFG_E_ARGS for a null or empty tree.  For measurement tools. */
int lfg_layout(const lfg_tree* tree);

/* Process-wide layout switch (tests, A/B measurement): 0 = k_elements +
 * k_lnlike for every tree, 1 = k_pair where lfg_layout allows it (the
 * default), -1 = back to the environment's choice (LFG_PAIR=0 selects 0).
 * Returns the previous setting (0 or 1), LFG_E_ARGS for another value.  Not
 * synchronised with launches in flight on other host threads.  A switch
 * between the two halves of a speculative chain (spec_out = 1 then
 * spec_in = 1) is safe: both layouts leave the partner-half snapshot the
 * k_pair launch reads. */
int lfg_set_layout(int mode);

#ifdef __cplusplus
}
#endif
#endif /* LFG_H */
