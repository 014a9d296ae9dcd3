"""The sampler utilities of the reference's mcmc_utils.py over the
device-resident EnsembleSampler: same names, arguments and file formats.

  initialise_walkers(p, scatter, nwalkers, ln_prior, model)   mcmc_utils.py:46-72
  run_burnin(sampler, startPos, nSteps, storechain=False)      mcmc_utils.py:114-132
  run_mcmc_save(sampler, startPos, nSteps, rState, file, col_names)
                                                                mcmc_utils.py:135-183
  flatchain(chain, npars=None, nskip=0, thin=1)                 mcmc_utils.py:242-249
  readchain(file) / readchain_dask(file)                        mcmc_utils.py:252-300
  readflatchain(file)                                           mcmc_utils.py:303-306

The emcee RNG state the reference threads from the burn-in into production
(`state` -> `rstate0`) is the sampler's Philox counter here
(EnsembleSampler.random_state).  run_mcmc_save keeps the chain on the device
and writes it in bulk chunks instead of re-opening the file for every row
(mcmc_utils.py:157-164); the rows are the reference's format.
"""
import numpy as np

from . import sampler as _sampler


def initialise_walkers(p, scatter, nwalkers, ln_prior, model=None, seed=0):
    """A Gaussian ball around p resampled until every walker has a finite
    ln_prior (mcmc_utils.py:46-72).  ln_prior(p, model) as mcmcfit.ln_prior
    (one vector), or -- marked with `ln_prior.batched = True` -- a function
    of the whole [n, ndim] batch (e.g. batched_ln_prior(evaluator))."""
    if getattr(ln_prior, "batched", False):
        fn = lambda x: np.asarray(ln_prior(x, model))  # noqa: E731
    else:
        fn = lambda x: np.array([ln_prior(v, model) for v in x])  # noqa: E731
    return _sampler.initialise_walkers(p, scatter, nwalkers, fn, seed=seed)


def batched_ln_prior(evaluator):
    """mcmcfit.ln_prior (mcmcfit.py:30-34) for a whole batch on the device
    (lfg_lnprior through a batch.LnProbEvaluator); usable as the ln_prior of
    initialise_walkers."""
    import torch

    def ln_prior(x, model=None):
        return evaluator.ln_prior(torch.as_tensor(np.asarray(x, dtype=np.float64),
                                                  device=evaluator.device)).cpu().numpy()
    ln_prior.batched = True
    return ln_prior


def run_burnin(sampler, startPos, nSteps, storechain=False, progress=False):
    """Burn-in (mcmc_utils.py:114-132): returns (pos, prob, state), with
    state the RNG counter to hand to run_mcmc_save.  The steps run back to
    back on the device (EnsembleSampler.run_mcmc); the reference's
    `for pos, prob, state in sampler.sample(...)` loop also works on the
    sampler, one host copy per step."""
    return sampler.run_mcmc(startPos, nSteps, storechain=storechain)


def run_mcmc_save(sampler, startPos, nSteps, rState, file, col_names='', progress=False, chunk=None,
                  lnprob0=None, **kwargs):
    """Production run written to `file` (mcmc_utils.py:135-183): the header
    line col_names, then '{k:4d} {values} {ln_prob:f}' per walker per step.
    rState (from run_burnin) continues the burn-in's random stream; None
    keeps the sampler's own.  Afterwards sampler.chain holds every step, as
    (nwalkers, nSteps, npars) like emcee's.  With torch.distributed every rank
    runs the steps (the ensemble is replicated) and rank 0 alone writes."""
    if rState is not None:
        sampler.random_state = rState
    W, ndim = sampler.W, sampler.ndim
    writer = bool(file) and getattr(sampler, "rank", 0) == 0
    if writer:
        with open(file, "w") as fh:
            fh.write(col_names)
            if col_names:
                fh.write("\n")
    chunk = chunk or max(1, min(nSteps, (1 << 28) // max(1, W * (ndim + 1) * 8)))
    done, first = 0, True
    while done < nSteps:
        k = min(chunk, nSteps - done)
        sampler.run_mcmc(startPos if first else None, k, storechain=True, lnprob0=lnprob0 if first else None)
        if writer:
            ch, lp = sampler.last_run()
            _sampler.write_chain(file, None, ch.cpu().numpy(), lp.cpu().numpy(), mode="a")
        first = False
        done += k
    return sampler


def flatchain(chain, npars=None, nskip=0, thin=1):
    """All walkers' samples as one [n, npars] array, skipping the first nskip
    steps and keeping every thin-th (mcmc_utils.py:242-249)."""
    if hasattr(chain, "cpu"):  # a device tensor
        chain = chain.cpu().numpy()
    chain = np.asarray(chain)
    if npars is None:
        npars = chain.shape[2]
    return chain[:, nskip::thin, :].reshape((-1, npars))


def readchain(file, **kwargs):
    """chain_prod.txt -> [nwalkers, nprod, npars + 1] (mcmc_utils.py:252-272);
    the last column is ln_prob."""
    return _sampler.read_chain(file)


def readchain_dask(file, **kwargs):
    """The reference's threaded reader (mcmc_utils.py:275-300) falls back to
    readchain when dask is absent; so does this one (same result)."""
    return readchain(file, **kwargs)


def readflatchain(file):
    """A whitespace-separated table read with no header row (e.g. a
    flattened chain) as one array (mcmc_utils.py:303-306: pandas, header=None)."""
    import pandas as pd
    return np.array(pd.read_csv(file, header=None, sep=r"\s+", float_precision="round_trip"))
