/*
 * lfg_oracle.h -- CPU FP64 restatement of the CV eclipse light-curve model.
 *
 * TEST INFRASTRUCTURE ONLY.  This library is the parity checker for the HIP
 * product in lfit_python_amd/csrc.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it.  It never sits on the product path.
 *
 * Parity against the real lfit C++ package is UNPINNED: lfit and trm.roche are
 * third-party, unvendored and absent.  What this file
 * restates is MODEL_SPEC.md, our written contract for lfit.CV.calcFlux()
 * (reference call site CVModel.py:138, API README.md:21-48).  The Python layers
 * around the call (priors, routing, chi^2) are pinned by golden fixtures
 * captured from the reference itself (tests/golden/).
 */
#ifndef LFG_ORACLE_H
#define LFG_ORACLE_H

#ifdef __cplusplus
extern "C" {
#endif

/* status codes (shared with include/lfg.h) */
#define LFO_OK            0
#define LFO_BAD_Q         1   /* q <= 0 or not finite                       */
#define LFO_BAD_DPHI      2   /* dphi outside (0, findphi(q,90))            */
#define LFO_BAD_GEOMETRY  3   /* rwd/rdisc/scale/exp out of domain          */
#define LFO_BAD_STREAM    4   /* bspot: the stream misses the disc radius  */
#define LFO_BAD_ARGS      5

/* roche primitives (trm.roche call sites CVModel.py:222,288,460,561) */
double lfo_xl1(double q);
int    lfo_findphi(double q, double inc_deg, double* dphi);
int    lfo_findi(double q, double dphi, double* inc_deg);
int    lfo_bspot(double q, double rad, double out4[4]);
/* eclipse interval (phase) of a point P; returns 1 if eclipsed */
int    lfo_point_interval(double q, double inc_deg, const double P[3],
                          double* a, double* b);

/* trm.roche.wdphases(q, iangle, r1, ntheta) (CVModel.py:564): third and
 * fourth contact phases of a sphere of radius r1 at the WD (MODEL_SPEC 10.2) */
int    lfo_wdphases(double q, double inc_deg, double r1, int ntheta,
                    double* phi3, double* phi4);

/* lfit.CV.calcFlux restatement: pars[14|18] (CV order, README.md:24-43). */
int lfo_flux(const double* pars, int npars, const double* x, const double* w,
             int n, int nsub, double* flux, double* ywd, double* yd,
             double* ys, double* yrs);

/* element tables, for white-box tests: returns counts and fills arrays of
 * length >= LFO_NEL (a, b = eclipse interval in phase, wgt = weight) and
 * donor vectors (LFO_NDONOR x 3). geo[16] receives derived geometry. */
#define LFO_NWD_RINGS   10
#define LFO_NWD         400
#define LFO_NDISC_R     20
#define LFO_NDISC_AZ    50
#define LFO_NDISC       1000
#define LFO_NBS         100
#define LFO_NDONOR_T    20
#define LFO_NDONOR_P    20
#define LFO_NDONOR      400
#define LFO_NEL         (LFO_NWD + LFO_NDISC + LFO_NBS)
int lfo_elements(const double* pars, int npars, double* a, double* b,
                 double* wgt, double* donor, double* geo);

/* Prior.ln_prob (model.py:83-113); type: 0 gauss 1 gaussPos 2 uniform
 * 3 log_uniform 4 mod_jeff; norm = Prior.normalise. */
double lfo_prior_lnprob(int type, double p1, double p2, double norm, double v);

/* Batched tree ln_prob (mcmcfit.py:37-41 -> model.py:476-498), OpenMP over
 * walkers.  gather[E*18]: >=0 index into a walker row, <0 -> consts[-1-g].
 * npars[E] = 14|18.  off[E+1] offsets into x/y/ye/w.  prior_* have length
 * ndim.  Returns number of threads used. */
int lfo_lnprob_batch(const double* walkers, int W, int ndim,
                     int E, const int* gather, const int* npars,
                     const double* consts,
                     const int* off, const double* x, const double* y,
                     const double* ye, const double* w, int nsub,
                     const int* prior_type, const double* prior_p1,
                     const double* prior_p2, const double* prior_norm,
                     double* lnp, double* lnlike_e, int nthreads);

/* GP likelihood (CVModel.py:603-696; MODEL_SPEC 10): exact dense george
 * log-likelihood of residuals r for ampin*M32(tau) + ampout*M32(tau) on each
 * closed block [blk[2k], blk[2k+1]] of x, plus ye^2 on the diagonal */
double lfo_gp_lnlike(const double* x, const double* r, const double* ye, int n,
                     double ampin, double ampout, double tau,
                     const double* blk, int nb);
/* changepoint distance (dphi + phi4 - phi3) / 2 of CVModel.py:560-570 */
int lfo_gp_base_dcp(double q, double dphi, double rwd, double* dcp);
/* lfo_lnprob_batch with the GP likelihood of GPLCModel trees:
 * gp_gather [E*3] ln_ampin_gp, ln_ampout_gp, ln_tau_gp (column or -1-const),
 * gp_base [E*3] q, dphi, rwd of the changepoint cache, gp_ecl [E*2] first and
 * last eclipse number of the changepoint list; NULL gp_gather = chi^2 */
int lfo_lnprob_batch_gp(const double* walkers, int W, int ndim,
                        int E, const int* gather, const int* npars,
                        const double* consts,
                        const int* off, const double* x, const double* y,
                        const double* ye, const double* w, int nsub,
                        const int* prior_type, const double* prior_p1,
                        const double* prior_p2, const double* prior_norm,
                        const int* gp_gather, const double* gp_base,
                        const int* gp_ecl, double* lnp, double* lnlike_e,
                        int nthreads);

/* lfit's component objects (testCV.py:27-49; MODEL_SPEC 5.6): unit-
 * normalised flux of one component at inclination inc_deg, phases x used as
 * given, half-widths w (NULL: points).  kind 0 white dwarf cp = {rwd/xl1,
 * ulimb}; 1 disc cp = {rwd/xl1, rdisc/xl1, dexp}, n1 x n2 rings x azimuths;
 * 2 bright spot cp = {rdisc/xl1, az, fis, scale/xl1, exp1, exp2, tilt, yaw},
 * n1 strip elements; 3 donor, n1 x n2 bands x azimuths. */
int lfo_component(int kind, const double* cp, double q, double inc_deg, int n1, int n2,
                  const double* x, const double* w, int n, double* out);

#ifdef __cplusplus
}
#endif
#endif
