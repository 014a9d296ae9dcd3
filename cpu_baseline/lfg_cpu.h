/*
 * lfg_cpu.h -- the CPU port of the GPU path (cpu_baseline/lfg_cpu.cpp):
 * lfg_device.hpp's setup, stream table and envelope-Newton element solver
 * compiled for the host, mirror symmetry and the interval sweep, OpenMP over
 * parameter sets / walkers.  It is bench.py's CPU baseline and the host twin
 * (lfg_cpu_*) of include/lfg.h's entry points: same argument meaning and
 * status codes, HOST pointers, no workspace or stream; nthreads <= 0: every
 * OpenMP thread.  Not a product path: lfit_python_amd never loads it.
 */
#ifndef LFG_CPU_H
#define LFG_CPU_H

#include "lfg.h"

#ifdef __cplusplus
extern "C" {
#endif

/* lfg_flux's twin (lfit.CV.calcFlux, CVModel.py:132-147): flux [W][N] */
int lfg_cpu_flux(const double* pars, int W, int P, const double* x,
                 const double* w, int N, int nsub, double* flux, int* status,
                 int nthreads);

/* lfg_lnlike's twin (SimpleEclipse.chisq / ln_like, CVModel.py:157-191) */
int lfg_cpu_lnlike(const double* pars, int W, int P, const double* x,
                   const double* w, int N, int nsub, const double* y,
                   const double* ye, double* lnlike, int* status,
                   int nthreads);

/* lfg_lnprob's twin (mcmcfit.ln_prob -> Node.ln_prob) over a tree whose
 * arrays are host pointers; chi^2 or GP trees */
int lfg_cpu_lnprob(const double* walkers, int W, const lfg_tree* tree,
                   double* lnp, int nthreads);

/* the batch form bench.py times (the oracle's lfo_lnprob_batch arguments);
 * returns the OpenMP threads used */
int lfc_lnprob_batch(const double* walkers, int W, int ndim, int E,
                     const int* gather, const int* npars, const double* consts,
                     const int* off, const double* x, const double* y,
                     const double* ye, const double* w, int nsub,
                     const int* prior_type, const double* prior_p1,
                     const double* prior_p2, const double* prior_norm,
                     int roche_priors, double* lnp, int nthreads);
int lfc_lnprob_batch_gp(const double* walkers, int W, int ndim, int E,
                        const int* gather, const int* npars,
                        const double* consts, const int* off, const double* x,
                        const double* y, const double* ye, const double* w,
                        int nsub, const int* prior_type,
                        const double* prior_p1, const double* prior_p2,
                        const double* prior_norm, int roche_priors,
                        const int* gp_gather, const double* gp_base,
                        const int* gp_ecl, double* lnp, int nthreads);

#ifdef __cplusplus
}
#endif
#endif
