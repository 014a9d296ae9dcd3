"""Device-resident MCMC fit driver: the reference's mcmcfit.py with the
walker ensemble on the GPU.

    python -m lfit_python_amd.mcmcfit mcmc_input.dat [--quiet] [--debug] [--seed S]
    torchrun --nproc-per-node N -m lfit_python_amd.mcmcfit mcmc_input.dat   (walker shards over N GPUs)

Same input file keys, checks and outputs as mcmcfit.py:51-343:
  nburn, nprod, nwalkers, first_scatter, second_scatter, fit, double_burnin,
  comp_scat (nthread is read and ignored: the GPU replaces the process pool);
  the initial chi^2 / ln_prior / ln_like / ln_prob report; the exit when the
  start violates the priors or when nwalkers < 2 * npars; the prior-resampled
  walker ball (mcmc_utils.initialise_walkers); burn-in (twice with
  double_burnin, re-centred on the best walker); reset; production written
  to chain_prod.txt in the reference's format (header
  'walker_no <names> ln_prob', one row per walker per step).
Parallel tempering (usePT = 1, ptemcee) and the plots / e-mailed summary are
out of scope; usePT = 1 is refused.
"""
import argparse
import os
import sys

import numpy as np

from . import batch, cvmodel, sampler


def _cfg(cfg, key, conv, default=None):
    if key in cfg:
        return conv(cfg[key])
    if default is None:
        raise KeyError("the input file lacks %r" % key)
    return default


def read_run_config(path):
    """The run keys of mcmcfit.py:118-139."""
    cfg = cvmodel.read_config(path)
    return {
        "nburn": _cfg(cfg, "nburn", int),
        "nprod": _cfg(cfg, "nprod", int),
        "nthread": _cfg(cfg, "nthread", int, 1),
        "nwalkers": _cfg(cfg, "nwalkers", int),
        "ntemps": _cfg(cfg, "ntemps", int, 1),
        "first_scatter": _cfg(cfg, "first_scatter", float),
        "second_scatter": _cfg(cfg, "second_scatter", float),
        "fit": _cfg(cfg, "fit", int, 1),
        "usePT": bool(_cfg(cfg, "usePT", int, 0)),
        "double_burnin": bool(_cfg(cfg, "double_burnin", int, 0)),
        "comp_scat": bool(_cfg(cfg, "comp_scat", int, 0)),
    }


def scatter_vectors(names, run):
    """p0_scatter_1 and p0_scatter_2 of mcmcfit.py:204-246 (the second only
    exists with comp_scat, as in the reference)."""
    s1 = np.full(len(names), run["first_scatter"])
    s2 = None
    if run["comp_scat"]:
        s1 = sampler.comp_scatter(names, run["first_scatter"])
        s2 = s1 * (run["second_scatter"] / run["first_scatter"])
    return s1, s2


def degrees_of_freedom(model):
    """mcmcfit.py:141-148"""
    dof = int(np.sum([ecl.lc.n_data for ecl in model.search_node_type('Eclipse')]))
    return dof - len(model.dynasty_par_names) - 1


def run(input_file, quiet=False, debug=False, seed=0, chain_file="chain_prod.txt", chunk=None, log=print):
    import torch
    dist = torch.distributed
    world = dist.get_world_size() if (dist.is_available() and dist.is_initialized()) else 1
    rank = dist.get_rank() if world > 1 else 0
    say = log if rank == 0 else (lambda *a, **k: None)
    dev = torch.device("cuda", torch.cuda.current_device())

    model = cvmodel.construct_model(input_file, debug)
    rc = read_run_config(input_file)
    say("\nStructure: %s with %d eclipses" % (type(model).__name__, len(model.search_node_type('Eclipse'))))
    dof = degrees_of_freedom(model)
    pars = list(model.dynasty_par_vals)
    say("\n\nInitial guess has a chisq of {:.3f} ({:d} D.o.F.).".format(model.chisq(), dof))
    say("\nFrom the wrapper functions with the above parameters, we get;")
    lp0 = model.ln_prior()
    say("a ln_prior of {:.3f}".format(lp0))
    say("a ln_like of {:.3f}".format(model.ln_like()))
    say("a ln_prob of {:.3f}".format(model.ln_prob()))
    if np.isinf(lp0):
        say("ERROR: Starting position violates priors!")
        say("Offending parameters are:")
        for par, lab in model.descendant_params():
            if not par.isValid:
                say("  -> {}_{}".format(par.name, lab))
        return {"status": "prior_violation"}
    if not rc["fit"]:
        return {"status": "no_fit"}  # mcmcfit.py:181-182: report only
    if rc["usePT"]:
        raise NotImplementedError("parallel tempering (usePT = 1, ptemcee) is out of scope")

    names = model.dynasty_par_names
    npars = len(pars)
    nwalkers = rc["nwalkers"]
    say("\n\nThe MCMC has {:d} variables and {:d} walkers".format(npars, nwalkers))
    say("(It should have at least 2*npars, {:d} walkers)".format(2 * npars))
    if nwalkers < 2 * npars:
        return {"status": "too_few_walkers"}  # mcmcfit.py:195-196
    s1, s2 = scatter_vectors(names, rc)
    if rc["double_burnin"] and s2 is None:
        raise NameError("double_burnin needs comp_scat = 1 (the reference defines p0_scatter_2 only then)")

    tree = batch.compile_tree(model)
    ev = batch.LnProbEvaluator(tree, device=dev, max_walkers=nwalkers)
    prior_fn = lambda p: ev.ln_prior(torch.as_tensor(p, device=dev)).cpu().numpy()
    S = sampler.EnsembleSampler(nwalkers, npars, ev, seed=seed)
    rng_seed = seed
    p0 = sampler.initialise_walkers(np.asarray(pars), s1, nwalkers, prior_fn, seed=rng_seed)

    say("\n\nExecuting the burn-in phase...")
    pos, prob, state = S.run_mcmc(p0, rc["nburn"], storechain=False)
    if rc["double_burnin"]:
        say("Executing the second burn-in phase")
        p0 = sampler.initialise_walkers(pos[np.argmax(prob)], s2, nwalkers, prior_fn, seed=rng_seed + 1)
        pos, prob, state = S.run_mcmc(p0, rc["nburn"], storechain=False)

    S.reset()  # clears the counters; the RNG stream carries on (emcee's rstate0=rState)
    say("Starting the main MCMC chain. Probably going to take a while!")
    nprod = rc["nprod"]
    chunk = chunk or max(1, min(nprod, (1 << 28) // max(1, nwalkers * (npars + 1) * 8)))
    first = True
    done = 0
    while done < nprod:
        k = min(chunk, nprod - done)
        S.run_mcmc(None if not first else pos, k, storechain=True, lnprob0=None if not first else prob)
        if rank == 0:
            ch, lp = S.last_run()
            sampler.write_chain(chain_file, names, ch.cpu().numpy(), lp.cpu().numpy(),
                                mode="w" if first else "a")
        first = False
        done += k
    acc = float(np.mean(S.acceptance_fraction))
    S.close()  # the direct RCCL communicator, before the process group goes
    say("Mean acceptance fraction: {:.3f}".format(acc))
    return {"status": "ok", "chain_file": chain_file, "acceptance": acc, "nwalkers": nwalkers, "npars": npars,
            "nprod": nprod}


def main(argv=None):
    ap = argparse.ArgumentParser(description="Execute an MCMC fit to a dataset (GPU ensemble).")
    ap.add_argument("input", help="The filename for the MCMC parameters' input file.")
    ap.add_argument("--notify", default="", help="accepted for compatibility; e-mail is out of scope")
    ap.add_argument("--debug", action="store_true")
    ap.add_argument("--quiet", action="store_true")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--chain", default="chain_prod.txt")
    args = ap.parse_args(argv)
    import torch
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        local = int(os.environ.get("LOCAL_RANK", "0"))
        torch.cuda.set_device(local)
        torch.distributed.init_process_group("nccl", device_id=torch.device("cuda", local))
    out = run(args.input, quiet=args.quiet, debug=args.debug, seed=args.seed, chain_file=args.chain)
    if torch.distributed.is_initialized():
        torch.distributed.destroy_process_group()
    # the reference leaves through a bare exit() (status 0) for a report-only
    # run (fit = 0) and for too few walkers; a start that violates the priors
    # is an error here (non-zero), so wrapping scripts can tell it apart
    return 1 if out["status"] == "prior_violation" else 0


if __name__ == "__main__":
    sys.exit(main())
