#!/usr/bin/env python3
"""Benchmark: walker ln_prob evaluations per second of the device-resident
emcee loop, on BASELINE.json's metric config (single eclipse, complex bright
spot, 300-point phase grid; config 2 = 1024 walkers per GPU).

A step is one emcee iteration of the whole ensemble: two half-steps of
propose -> batched ln_prob of the proposals (k_setup, k_elements, k_lnlike)
-> accept.  On one GPU a half-step is those three kernels alone
(lfg_stretch_step_half: the proposal formed in k_setup, the acceptance in
k_lnlike); with N ranks each rank evaluates its shard of the half
(lfg_stretch_step_shard), ncclAllGather's the shard's ln_prob on the compute
stream, and every rank accepts (lfg_stretch_accept_regen).  value = walkers
x steps / time, max over ranks, inputs resident in HBM.

Configs (BASELINE.json):
  2   1024 walkers per GPU, weak scaling (the metric's config; default)
  3   3-band x 4-eclipse tree, 2048 walkers per GPU, weak
  4   the 16384-walker ensemble sharded over the N GPUs: strong scaling
      (16384 / N walkers per GPU; at N = 8, 2048 per GPU)
  5   10000 points x 5 sub-samples, 4096 walkers per GPU, weak
  gp  the reference's shipped useGP = 1 example (87 parameters, 6 eclipses,
      its real light curves), 1024 walkers per GPU, weak

Launch: `python bench.py --gpus N` with N > 1 spawns N rank processes itself
(before anything touches the GPU), one per GPU; under torchrun WORLD_SIZE
must equal --gpus.

Kernel timing: the last warmup step records HIP events around every kernel
(include/lfg.h LFG_NEV, on the caller stream all kernels run on) and picks
the dominant kernel; in the timed region every --time-every-th ln_prob call
records a start/stop event pair around that kernel only (default every 20th:
two samples at the driver's 20 steps, ten at 100).  A timing event is a queue
barrier: events around all kernels cost ~20 % of the step, so they stay out
of the timed region; a pair on every 8th call cost 1.2 % of the config-2 line
against none (12.08 vs 12.23 M evals/s, one box, three rounds), every 40th
nothing measurable.

Roofline (MODEL_SPEC.md section 11; the path is FP64-VALU or latency bound,
neither HBM- nor MFMA-bound):
  roofline.achieved / frac   the DOMINANT kernel (k_pair, or k_elements on
      the two-kernel layout, chosen by the warmup's events): its counted FP64
      work per launch (profiles/r04/flops_<config>.json per pair x the pairs
      of a launch) / its average launch time over the timed region (HIP events
      on its stream) / 78.6 TFLOP/s;
  roofline.traffic           HBM bytes per launch of that kernel from the
      committed PMC passes (profiles/*/pmc_traffic_<config>.json), when they
      were taken on the same workload and kernel layout;
  roofline.whole_step        every kernel of the step on the same counts x
      evals/s per GPU;
  roofline.direct_form_equivalent   SURVEY 8(d)'s direct element x point
      count (a rate of equivalent work, not a utilisation);
  roofline.hbm               SURVEY 8(d)'s algorithmic bytes per half-step
      (8 ndim + 8 per walker, 32 N per eclipse per launch) over the step time,
      the element tables kernels hand each other apart (none on k_pair).
Multi-rank lines carry "ranks": the world size, the RCCL communicator's own
count (ncclCommCount), each rank's step time and exchange time.
"""
import argparse
import ctypes
import json
import os
import socket
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# MI355X peaks (/opt/skills/guides/MI355X_MICROARCH.md; FP64 vector = spec)
HBM_PEAK_GBS = 8000.0
FP64_PEAK_TFLOPS = 78.6
PMC_DIR = os.path.join(ROOT, "profiles", "r06")   # pmc_traffic_<config>.json (tools/pmc_traffic.py)

NEV = 4  # LFG_NEV (include/lfg.h)
# (name as rocprofv3 prints it, start event, end event) per kernel layout
# (lfg_layout): k_elements + k_lnlike, or k_pair (both in one workgroup per pair)
KERNELS_TWO = [("k_setup", 0, 1), ("k_elements", 1, 2), ("k_lnlike", 2, 3)]
KERNELS_PAIR = [("k_setup", 0, 1), ("k_pair", 2, 3)]

# Counted FP64 work per (walker, eclipse) pair of the algorithm the kernels
# execute (MODEL_SPEC.md section 11; tools/flop_count.py + tools/like_count.py
# -> profiles/r04/flops_<config>.json): per-kernel figures for the roofline's
# kernel fraction and the whole step, and the direct-form count of SURVEY
# 8(d) (900 roots x geometry + N S (1500 x 3 + 400 x 6 + 40)) kept apart as
# direct_form_equivalent
FLOPS_DIR = os.path.join(ROOT, "profiles", "r04")
FLOPS_TABLE = {"2": "c2", "3": "c3", "4": "c2", "5": "c5", "gp": "gp"}

# builder's intermediate tables per (walker, eclipse) pair:
# what each kernel reads and writes of the tables the kernels hand each other
# (intervals: the 700 symmetry-unique WD/disc elements + 100 spot, 16 B each;
# k_lnlike also reads each point's x, w, y, ye: shared by the eclipse's pairs)
NELU, U_DON, DON_STRIDE = 800, 100, 5
GEO_SETUP, GEO_BSPOT, GEO_READ = 41, 5, 40
WT_N = 124
MATERIALISED_PER_PAIR = {
    "k_setup": 18 * 8 + GEO_SETUP * 8 + 4 + 3 * 8 + GEO_BSPOT * 8 + 4,
    "k_elements": GEO_READ * 8 + 8 + NELU * 16 + U_DON * DON_STRIDE * 8 + WT_N * 8,
    "k_lnlike": GEO_READ * 8 + 4 + NELU * 16 + U_DON * DON_STRIDE * 8 + WT_N * 8 + 8,
    "k_pair": GEO_READ * 8 + 4 + 8,   # the tables stay in the workgroup's LDS
}

CONFIGS = {
    "2": dict(walkers=1024, npts=300, nsub=1, scaling="weak",
              desc="config 2: single eclipse, complex 18-par bright spot, %d phase pts, nsub %d, "
                   "%d walkers/GPU, emcee stretch move"),
    "3": dict(walkers=2048, npts=300, nsub=1, scaling="weak",
              desc="config 3: 3-band x 4-eclipse tree (shared q/dphi/rwd), complex bright spot, %d phase pts "
                   "per eclipse, nsub %d, %d walkers/GPU"),
    "4": dict(walkers_total=16384, npts=300, nsub=1, scaling="strong",
              desc="config 4: 16384-walker ensemble sharded over the GPUs, single eclipse, complex bright spot, "
                   "%d phase pts, nsub %d, %d walkers/GPU"),
    "5": dict(walkers=4096, npts=10000, nsub=5, scaling="weak",
              desc="config 5: single eclipse, complex bright spot, %d phase pts, nsub %d sub-samples, "
                   "%d walkers/GPU"),
    "gp": dict(walkers=1024, npts=None, nsub=1, scaling="weak",
               desc="the reference's useGP = 1 example (test_data/mcmc_input.dat: 87 parameters, 3 bands x 2 "
                    "eclipses, its real light curves, Matern-3/2 GP likelihood), %s pts, nsub %d, %d walkers/GPU"),
}


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs (ranks); N > 1 without torchrun spawns the N ranks here")
    ap.add_argument("--steps", type=int, default=100)  # ~20 ms timed: one host hiccup stays small
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="2", choices=sorted(CONFIGS), help="BASELINE.json config (see above)")
    ap.add_argument("--walkers", type=int, default=None, help="walkers per GPU (default: the config's)")
    ap.add_argument("--npts", type=int, default=None)
    ap.add_argument("--nsub", type=int, default=None)
    ap.add_argument("--shard-path", action="store_true",
                    help="run the multi-rank half-step (lfg_stretch_step_shard + accept_regen) on one rank")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="per CPU baseline (two are timed)")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0: every core this process may run on")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--exchange-path", action="store_true",
                    help="one GPU: a one-rank RCCL group and the multi-rank code path with its real "
                         "exchange (shard kernels, ncclAllGather on the compute stream, k_accept_regen)")
    ap.add_argument("--emulate-rank", default=None, metavar="K/N",
                    help="timing rehearsal of rank K of an N-GPU run on this one GPU (config 4: W = 16384 held, "
                         "W/2/N walkers evaluated per half, a one-rank RCCL exchange of the shard, the acceptance "
                         "over the whole half); also times the fused one-GPU step and reports the implied 1->N ratio")
    ap.add_argument("--seed", type=int, default=20261015)
    ap.add_argument("--time-every", type=int, default=20,
                    help="record the dominant kernel's event pair on every k-th ln_prob call of the timed region")
    args = ap.parse_args(argv)
    cfg = CONFIGS[args.config]
    args.emu = None
    if args.emulate_rank:
        k, n = (int(v) for v in args.emulate_rank.split("/"))
        args.emu = (k, n)
        args.exchange_path = True
    args.npts = args.npts or cfg["npts"]
    args.nsub = args.nsub or cfg["nsub"]
    return args


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _rank_entry(rank, argv, world, port):
    """One spawned rank (fresh interpreter, nothing touched the GPU before)."""
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    run(parse(argv))


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is not None:
        if args.gpus is not None and int(env_world) != args.gpus:
            sys.exit("bench.py: WORLD_SIZE=%s but --gpus %d" % (env_world, args.gpus))
        return run(args)
    n = args.gpus or 1
    if n == 1:
        return run(args)
    # N ranks, one per GPU, spawned before any HIP call in this process
    import torch.multiprocessing as mp
    mp.start_processes(_rank_entry, args=(argv, n, _free_port()), nprocs=n, join=True, start_method="spawn")
    return 0


def walker_count(args, world):
    cfg = CONFIGS[args.config]
    if args.walkers:
        return args.walkers
    if "walkers_total" in cfg:
        tot = cfg["walkers_total"]
        if args.emu:  # one rank of N: the whole ensemble is held, 1/N of each half evaluated
            return tot
        if tot % (2 * world):
            raise SystemExit("config 4: 16384 walkers do not shard over %d ranks" % world)
        return tot // world
    return cfg["walkers"]


def build_model(args, flux_fn):
    from lfit_python_amd import cvmodel, synthetic
    if args.config == "gp":
        return cvmodel.construct_model(os.path.join(ROOT, "tests", "golden", "ref_test_data", "mcmc_input.dat"))
    if args.config == "3":
        return synthetic.config_tree(4, args.npts, flux_fn=flux_fn, nsub=args.nsub)
    return synthetic.config_single(npts=args.npts, flux_fn=flux_fn, nsub=args.nsub)


def flops_per_pair(config, npts, nsub):
    """Counted FP64 FLOPs of one walker-eclipse pair by kernel (MODEL_SPEC.md
    section 11), from the committed table of the configuration's workload.
    Config 4 runs config 2's light curve.  A run whose points x sub-samples
    differ from the table's scales k_lnlike's per-point part (its tiles and
    sub-bin work grow linearly with N S) and says so."""
    path = os.path.join(FLOPS_DIR, "flops_%s.json" % FLOPS_TABLE[config])
    d = json.load(open(path))
    pk = dict(d["per_kernel"])
    direct = float(d["F_direct_form_equivalent_per_pair"])
    note = None
    ns0 = d["npts"] * d["nsub"]
    if config != "gp" and npts * nsub != ns0:
        r = npts * nsub / float(ns0)
        fixed = d["F_like_parts"]["prologue"] + d["F_like_parts"]["wd_disc"]
        pk["k_lnlike"] = fixed + (pk["k_lnlike"] - fixed) * r
        direct = (direct - d["F_acc_total"]) + d["F_acc_total"] * r
        note = "scaled from %s's %d x %d points x sub-samples" % (os.path.basename(path), d["npts"], d["nsub"])
    executed = float(pk["k_elements"] + pk["k_lnlike"])   # the spec path: no k_setup launch per step
    pk["k_pair"] = executed                                # k_elements' and k_lnlike's work in one kernel
    return {"per_kernel": pk, "executed": executed, "direct": direct, "note": note,
            "source": os.path.relpath(path, ROOT)}


# kernels inside each event span of the timed region (the GP pair of kernels
# runs between k_lnlike's events)
SPAN = {"k_setup": ("k_setup",), "k_elements": ("k_elements",),
        "k_lnlike": ("k_lnlike", "k_gp_dcp", "k_gp_like"), "k_pair": ("k_pair", "k_combine_walkers")}


def pmc_row(kernel, config, npts, nsub, pairs):
    """Counter-derived bytes and executed FP64 FLOPs per launch of the event
    span `kernel` (summed over the kernels in it; the one-off initial
    k_lnlike<0> excluded), scaled to `pairs`, from the committed PMC summary
    of this configuration's workload; (None, None) when there is none."""
    path = os.path.join(PMC_DIR, "pmc_traffic_%s.json" % FLOPS_TABLE[config])
    try:
        d = json.load(open(path))
    except (OSError, ValueError):
        return None, None
    meta = d.get("meta", {})
    if config != "gp" and (meta.get("npts"), meta.get("nsub")) != (npts, nsub):
        return None, None
    out = {}
    for name, row in d.get("kernels", {}).items():
        base = name.split("<")[0]
        if base not in SPAN[kernel] or name.startswith("k_lnlike<0"):
            continue
        for k in ("traffic_bytes", "fp64_flops"):
            if k in row:
                out[k] = out.get(k, 0.0) + row[k]
    if not out:
        return None, None
    scale = pairs / float(meta.get("pairs_per_launch", pairs))
    return {k: v * scale for k, v in out.items()}, os.path.relpath(path, ROOT)


def line_value(W, steps, elapsed, emu=None):
    """The line's value: walker ln_prob evaluations per second of the whole
    job.  W is the ensemble over all ranks; each step evaluates every walker
    once (two half-steps of W/2).  Emulating rank K of N (emu = (K, N)), the
    process holds the whole ensemble but evaluates W / N walkers per step:
    only those count."""
    evaluated = W // emu[1] if emu else W
    return evaluated * steps / elapsed


def rank_block(dist, world, backend, own_ms, xch_ms, cnt, dev):
    """The line's "ranks" object (every rank calls it: one all_gather of each
    rank's own ms per step and exchange ms): world size, backend, the RCCL
    communicator's own rank count and user rank (cnt = ncclCommCount,
    ncclCommUserRank of rank 0's communicator, or None), per-rank times"""
    import torch
    mine = torch.tensor([own_ms, xch_ms if xch_ms is not None else float("nan")], dtype=torch.float64, device=dev)
    allr = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(allr, mine)
    per = torch.stack(allr).cpu().numpy()
    return {"world_size": world, "backend": backend,
            "rccl_comm_count": cnt[0] if cnt else None, "rccl_user_rank": cnt[1] if cnt else None,
            "ms_per_step_per_rank": [float(v) for v in per[:, 0]],
            "ms_per_step_min": float(per[:, 0].min()), "ms_per_step_max": float(per[:, 0].max()),
            "exchange_ms_per_half_step": [None if np.isnan(v) else float(v) for v in per[:, 1]],
            "note": "ms_per_step_per_rank: each rank's timed steps before the closing barrier; exchange: events "
                    "around the all_gather on the sampled calls (rccl_comm_count: ncclCommCount of the direct RCCL "
                    "communicator, null when the exchange ran through torch.distributed)"}


def run(args):
    # stdout carries exactly one JSON line: libraries that print to stdout
    # (RCCL's version banner at communicator init) are sent to stderr
    json_out = os.fdopen(os.dup(1), "w")
    sys.stdout.flush()
    os.dup2(2, 1)
    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # LFG_BENCH_BACKEND=gloo rehearses the multi-rank flow with every rank on
    # the GPUs there are (e.g. two ranks on a one-GPU box); the driver's runs
    # use RCCL ("nccl"), one rank per GPU
    backend = os.environ.get("LFG_BENCH_BACKEND", "nccl")
    if backend != "nccl":
        local %= torch.cuda.device_count()
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = None
    if args.exchange_path and world == 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(_free_port()))
        args.shard_path = True
    if world > 1 or args.exchange_path:
        import torch.distributed as dist
        if world == 1:
            dist.init_process_group(backend, rank=0, world_size=1,
                                    **({"device_id": dev} if backend == "nccl" else {}))
        elif backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    from lfit_python_amd import _native, batch, sampler
    from lfit_python_amd.lfit import flux_batch
    _native.require_gpu()
    L = _native.lib()

    def flux_fn(pars, x, w, nsub):
        f, st = flux_batch(np.asarray(pars)[None, :], x, w, nsub=nsub, device=dev)
        assert int(st[0].item()) == 0
        return f[0].cpu().numpy()

    model = build_model(args, flux_fn)
    tree = batch.compile_tree(model, nsub=args.nsub)
    per_gpu = walker_count(args, world)
    W = per_gpu * world
    ev = batch.LnProbEvaluator(tree, device=dev, max_walkers=W)
    p0 = np.array(model.dynasty_par_vals)
    scat = sampler.comp_scatter(model.dynasty_par_names, 0.1)
    init = sampler.initialise_walkers(
        p0, scat, W, lambda p: ev(torch.as_tensor(p, device=dev)).cpu().numpy(), seed=args.seed)
    S = sampler.EnsembleSampler(W, tree.ndim, ev, seed=args.seed)
    S.force_shard = args.shard_path
    S.force_exchange = args.exchange_path
    if args.emu:
        S.emulate_rank(*args.emu)
    S.set_state(init)
    layout = L.lfg_layout(ctypes.byref(ev.ctree))
    KERNELS = KERNELS_PAIR if layout >= 1 else KERNELS_TWO   # 2: k_pair's LONG variant

    # HIP events around kernels of lfg_lnprob calls (include/lfg.h LFG_NEV)
    events = []
    want = [True] * NEV  # which events to record
    every = [1]          # record on every k-th call
    ncall = [0]

    def sampled():
        ncall[0] += 1
        return (ncall[0] - 1) % every[0] == 0

    pool = []  # event sets made before the timed region (hipEventCreate is host work in the loop)

    def make_evs():
        if pool:
            return pool.pop()
        evs = (ctypes.c_void_p * NEV)()
        for i in range(NEV):
            if want[i]:
                h = ctypes.c_void_p()
                _native.check(L.lfg_event_create(ctypes.byref(h)), "lfg_event_create")
                evs[i] = h.value
        return evs

    def timed_half(pos, lnp, half, a, seed, step, q, zfac, naccept, lnp_new=None, spec=False):
        """the single-process path: lfg_stretch_step_half(_spec) with the events"""
        evs = None
        if sampled():
            evs = make_evs()
            events.append((evs, q.shape[0]))
        ev.step_half(pos, lnp, half, a, seed, step, q, zfac, naccept, lnp_new=lnp_new, events=evs, spec=spec)

    def timed_shard(pos, half, a, seed, step, lo, q, zfac, lnp_sh, spec=False, fold=None):
        """the multi-rank path: this rank's lfg_stretch_step_shard(_spec / _fold) with the events"""
        evs = None
        if sampled():
            evs = make_evs()
            events.append((evs, lnp_sh.shape[0]))
        ev.step_shard(pos, half, a, seed, step, lo, q, zfac, lnp_sh, events=evs, spec=spec, fold=fold)

    timed_half.takes_spec = timed_shard.takes_spec = timed_shard.takes_fold = True

    # the per-half-step ln_prob exchange, timed by HIP events on the stream it
    # is enqueued on, on the calls whose shard kernels are sampled too
    xch_events = []
    xch_on = [False]
    plain_gather = S._gather

    def timed_gather(out, mine):
        if not xch_on[0] or (ncall[0] - 1) % every[0]:
            return plain_gather(out, mine)
        # the exchange is enqueued on torch's current stream (comm.py), so
        # torch's events see it
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        plain_gather(out, mine)
        e1.record()
        xch_events.append((e0, e1))
    S._gather = timed_gather

    def set_timing(on):
        if world == 1 and not args.shard_path:
            S.half_timer = timed_half if on else None
        else:
            S.shard_timer = timed_shard if on else None

    def kernel_ms(kernels):
        """mean ms per launch of each (name, a, b) over the recorded calls; frees the events"""
        tot = np.zeros(len(kernels))
        fms = ctypes.c_float()
        for evs, _ in events:
            for k, (_, a, b) in enumerate(kernels):
                _native.check(L.lfg_event_elapsed_ms(evs[a], evs[b], ctypes.byref(fms)), "elapsed")
                tot[k] += fms.value
        n = len(events)
        for evs, _ in events:
            for i in range(NEV):
                if evs[i]:
                    L.lfg_event_destroy(evs[i])
        return tot / max(n, 1), n

    ev._ensure(W)
    for i in range(args.warmup):
        if i == args.warmup - 1:
            set_timing(True)  # calibration: every kernel
        S.step()
    torch.cuda.synchronize()
    set_timing(False)
    dom = len(KERNELS) - 1  # the likelihood kernel unless calibrated
    calib = {}
    if events:
        cal_ms, _ = kernel_ms(KERNELS)
        calib = {n: float(m) for (n, _, _), m in zip(KERNELS, cal_ms)}
        dom = int(np.argmax(cal_ms))
    events.clear()
    kname, ea, eb = KERNELS[dom]
    want[:] = [i in (ea, eb) for i in range(NEV)]
    every[0] = max(1, args.time_every)
    ncall[0] = 0
    calls = 2 * args.steps  # ln_prob calls of the timed region (one per half-step)
    pool.extend(make_evs() for _ in range((calls + every[0] - 1) // every[0]))
    set_timing(True)

    xch_on[0] = True
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        S.step()
    torch.cuda.synchronize()
    own_elapsed = time.perf_counter() - t0   # this rank's own steps, before it waits for the others
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    set_timing(False)
    xch_on[0] = False
    S._gather = plain_gather
    xch_ms = None
    if xch_events:
        xch_ms = sum(e0.elapsed_time(e1) for e0, e1 in xch_events) / len(xch_events)
    ranks = None
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        # every rank's own step time and exchange time, and what RCCL says the
        # communicator holds: the line proves how many ranks exchanged
        ranks = rank_block(dist, world, backend, own_elapsed / args.steps * 1e3, xch_ms,
                           S._rccl.count() if S._rccl else None, dev)

    # the dominant kernel's device time over the timed region
    shard = events[0][1] if events else W // 2   # walkers per launch
    dom_ms, ncalls = kernel_ms([KERNELS[dom]])
    for evs in pool:  # unused sets of the timed region
        for i in range(NEV):
            if evs[i]:
                L.lfg_event_destroy(evs[i])
    pool.clear()
    emu = None
    if args.emu:
        # the same ensemble on one GPU through the fused single-process path
        S1 = sampler.EnsembleSampler(W, tree.ndim, ev, seed=args.seed)
        S1.set_state(init)
        for _ in range(args.warmup):
            S1.step()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(args.steps):
            S1.step()
        torch.cuda.synchronize()
        el1 = time.perf_counter() - t1
        S1.close()
        k, n = args.emu
        emu = {"rank": k, "nranks": n, "walkers_held": W, "walkers_evaluated_per_half": shard,
               "ms_per_step_rank": elapsed / args.steps * 1e3, "ms_per_step_one_gpu_fused": el1 / args.steps * 1e3,
               "projected_speedup_1_to_n": el1 / elapsed,
               "note": "one rank's launches (shard kernels, a one-rank ncclAllGather of its shard, the acceptance "
                       "over the whole half) timed on one GPU; the other shards' ln_prob entries are -inf (their "
                       "walkers stay in the starting ball), so the chain is not a sample.  Projected: the N ranks run these concurrently; the exchange of a "
                       "real N-rank all_gather over xGMI is latency-bound (W/2 doubles) and not included beyond "
                       "the one-rank call"}
    avg_dom = float(dom_ms[0])
    E = tree.E
    npts = int(np.max(np.diff(tree.offsets)))
    value = line_value(W, args.steps, elapsed, args.emu)
    acc = float(np.mean(S.acceptance_fraction))

    # ---- FP64 roofline on the counted work of the executed algorithm (MODEL_SPEC 11)
    fl = flops_per_pair(args.config, npts, tree.nsub)
    fpp = fl["per_kernel"]
    pairs = shard * E
    dom_flops = fpp[kname] * pairs                      # the dominant kernel, per launch
    dom_tf = dom_flops / (avg_dom * 1e-3) / 1e12
    step_tf = value / world * E * fl["executed"] / 1e12   # per GPU, whole step
    direct_tf = value / world * E * fl["direct"] / 1e12
    kern = {}
    for n, m in calib.items():
        f = fpp[n] * pairs
        kern[n] = {"warmup_ms": m, "flops_per_launch": f,
                   "tflops": f / (m * 1e-3) / 1e12 if m > 0 else None,
                   "frac": f / (m * 1e-3) / 1e12 / FP64_PEAK_TFLOPS if m > 0 else None}

    # ---- HBM: SURVEY 8(d) algorithmic bytes per half-step; materialised tables apart
    half_s = elapsed / args.steps / 2.0
    hbm_bytes = shard * (8 * tree.ndim + 8) + 32 * npts * E
    hbm_gbs = hbm_bytes / half_s / 1e9
    mat = MATERIALISED_PER_PAIR[kname] * pairs

    # counter-derived traffic and executed FP64 FLOPs of the dominant kernel
    # (rocprofv3 --pmc passes, tools/pmc_profile.sh -> tools/pmc_traffic.py ->
    # profiles/r04/pmc_traffic_<config>.json); per-pair counters carry over only
    # to the workload they were collected on
    row, pmc_path = pmc_row(kname, args.config, npts, tree.nsub, pairs)
    traffic = fp64x = None
    if row:
        traffic = row.get("traffic_bytes")
        if "fp64_flops" in row:
            f = row["fp64_flops"]
            fp64x = {"executed_flops_per_launch": f, "tflops": f / (avg_dom * 1e-3) / 1e12,
                     "frac": f / (avg_dom * 1e-3) / 1e12 / FP64_PEAK_TFLOPS,
                     "counted_over_executed": dom_flops / f if f else None,
                     "source": pmc_path}

    cpu = {"cpu_baseline": None}
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline(tree, S.pos.cpu().numpy(), args)

    if rank == 0:
        cfg = CONFIGS[args.config]
        xch = ("one rank: no exchange" if dist is None
               else ("%s all_gather" % backend if backend != "nccl"
                     else ("ncclAllGather on the compute stream" if os.environ.get("LFG_RCCL_DIRECT", "1") != "0"
                           else "torch ProcessGroupNCCL")))
        line = {
            "metric": "walker ln_prob evals/sec (300-pt phase, complex BS) at 1/2/4/8 MI355X",
            "value": value,
            "unit": "walker ln_prob evals/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": cfg["scaling"],
            "vs_baseline": None,
            "dtype": "f64",
            "data": ("the reference's own light curves (test_data/lightcurves, tests/golden/ref_test_data)"
                     if args.config == "gp" else
                     "synthetic light curve (model at mcmc_input.dat eclipse-0 truth + N(0, 0.004))")
                    + "; walkers from the comp_scat ball of mcmcfit.py",
            "config": {"workload": cfg["desc"] % (args.npts if args.npts else "166-303", args.nsub, per_gpu),
                       "walkers_total": W, "walkers_per_gpu": per_gpu, "eclipses": E, "ndim": tree.ndim,
                       "parallelism": "walker shards x%d, replicated Philox RNG, one all_gather of ln_prob "
                                      "per half-step (%s)" % (world, xch)},
            "roofline": {
                "bound": "fp64_valu", "achieved": dom_tf, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                "frac": dom_tf / FP64_PEAK_TFLOPS, "traffic": traffic,
                "basis": "the dominant kernel (%s): its counted FP64 work per launch (MODEL_SPEC 11, %s x %d "
                         "pairs) / its average launch time over the timed region (HIP events on its stream)"
                         % (kname, fl["source"], pairs),
                "kernel": {"name": kname, "avg_launch_ms": avg_dom, "launches_timed": ncalls,
                           "pairs_per_launch": pairs, "flops_per_pair": fpp[kname],
                           "flops_per_launch": dom_flops, "executed_fp64": fp64x,
                           "traffic_bytes_per_launch": traffic},
                "whole_step": {"achieved": step_tf, "frac": step_tf / FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                               "flops_per_pair": fl["executed"],
                               "basis": "counted FP64 work of every kernel the step launches (k_elements incl. "
                                        "its speculative setup lanes, k_lnlike incl. the GP kernels) x E pairs x "
                                        "evals/s per GPU"},
                "direct_form_equivalent": {
                    "achieved": direct_tf, "flops_per_pair": fl["direct"], "unit": "TFLOP/s",
                    "note": "SURVEY 8(d)'s direct-form count (each element against each point and sub-phase); "
                            "the kernels form the same sums with an interval sweep, so this is a rate of "
                            "equivalent work, not a utilisation, and may exceed the peak"},
                "flops_per_pair": fpp,
                **({"flops_note": fl["note"]} if fl["note"] else {}),
                **({"long_note": "k_pair's LONG variant executes the same element work and per sub-phase model "
                                 "terms as k_elements + k_lnlike; its counted figure is theirs (the table lookups "
                                 "replace the sweep's integer scan, which the count does not include)"}
                   if layout == 2 else {}),
                "kernels_warmup": kern,
                "hbm": {"algorithmic_bytes_per_half_step": hbm_bytes, "achieved": hbm_gbs, "peak": HBM_PEAK_GBS,
                        "unit": "GB/s", "frac": hbm_gbs / HBM_PEAK_GBS,
                        "basis": "SURVEY 8(d): 8 ndim + 8 B per walker + 32 N B per eclipse per launch",
                        "materialised_bytes_per_launch": {"kernel": kname, "bytes": mat,
                                                          "note": "element tables the kernels hand each other "
                                                                  "(DESIGN.md 3): an intermediate, not 8(d) work"}},
            },
            "acceptance_fraction": acc,
            "kernel_layout": {1: "k_pair", 2: "k_pair (LONG: per-pair breakpoint tables in LDS, each wave a "
                                                "cost-balanced range of the points)"}.get(layout, "k_elements + k_lnlike"),
            **({"ranks": ranks} if ranks else {}),
            **({"exchange_ms_per_half_step": xch_ms} if (xch_ms is not None and not ranks) else {}),
            **({"emulation": emu, "emulated_rank": True} if emu else {}),
            **cpu,
        }
        print(json.dumps(line), file=json_out, flush=True)
    S.close()
    if dist:
        dist.destroy_process_group()
    return 0


def _usable_cpus():
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    try:  # a cgroup CPU quota caps what the threads can use
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            n = min(n, max(1, int(round(int(q) / int(p)))))
    except (OSError, ValueError):
        pass
    return n


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return ""


def _time_cpu(fn, batch, nthr, seconds):
    """evals/s of fn(batch) repeated for about `seconds` after one warm call"""
    fn(batch[:nthr])
    n, t0 = 0, time.perf_counter()
    while True:
        fn(batch)
        n += batch.shape[0]
        el = time.perf_counter() - t0
        if el >= seconds:
            return n, el


def cpu_baseline(tree, walkers, args):
    """Two CPU baselines on this host's cores, same tree and walkers, each
    bounded to about args.cpu_seconds of work (timed after the GPU region):
      * "cpu_baseline": the GPU path's own algorithm on the CPU
        (cpu_baseline/lfg_cpu.cpp: lfg_device.hpp's solvers compiled for the
        host, mirror symmetry, the interval sweep), OpenMP over walkers;
      * "cpu_baseline_oracle": the oracle (MODEL_SPEC restated with the
        nested solver and the direct element x point sum).
    GP trees: the port runs the serial Kalman filter, the oracle the dense
    GP likelihood."""
    import subprocess
    import tempfile
    from oracle import oracle as orc
    avail = _usable_cpus()
    nthr = args.cpu_threads if args.cpu_threads > 0 else avail
    batch = walkers[: max(nthr * 4, 64)]
    model, out = _cpu_model(), {}
    from cpu_baseline import cpu as cpuport
    path = os.path.join(tempfile.gettempdir(), "liblfg_cpu_native_%d.so" % os.getpid())
    try:
        cpuport.build(out=path, march="native")
    except (subprocess.CalledProcessError, FileNotFoundError):
        path = cpuport.LIB_PATH
    port = cpuport.CpuPort(path)
    used = [nthr]

    def run_port(b):
        used[0] = port.lnprob_batch(b, tree, nthreads=nthr)[1]
    n, el = _time_cpu(run_port, batch, nthr, args.cpu_seconds)
    out["cpu_baseline"] = {
        "value": n / el, "unit": "walker ln_prob evals/s", "cores": int(used[0]), "kind": "port",
        "sample": "%d ln_prob evals (%d-walker batches of the same tree and walkers) in %.1f s: the GPU path's "
                  "algorithm on the CPU (cpu_baseline/lfg_cpu.cpp, g++ -O3 -march=native, OpenMP over walkers): "
                  "lfg_device.hpp's setup, stream table and envelope-Newton element solver compiled for the "
                  "host, mirror symmetry, the interval sweep over sorted windows%s" % (
                      n, batch.shape[0], el, "; the serial 4-state Kalman filter of lfg_device.hpp" if tree.gp else ""),
        "cpu": model, "host_cpus": os.cpu_count(), "cpus_available": avail}
    path = os.path.join(tempfile.gettempdir(), "liblfg_oracle_native_%d.so" % os.getpid())
    try:
        orc.build(march="native", out=path)
    except (subprocess.CalledProcessError, FileNotFoundError):
        path = orc.LIB_PATH
    o = orc.Oracle(path)
    used = [nthr]

    def run_oracle(b):
        used[0] = o.lnprob_batch(b, tree, nsub=tree.nsub, nthreads=nthr)[2]
    n, el = _time_cpu(run_oracle, batch, nthr, args.cpu_seconds)
    out["cpu_baseline_oracle"] = {
        "value": n / el, "unit": "walker ln_prob evals/s", "cores": int(used[0]), "kind": "port",
        "sample": "%d ln_prob evals (%d-walker batches of the same tree and walkers) in %.1f s: oracle/lfg_oracle.c "
                  "-O3 -march=native, OpenMP over walkers; the oracle's algorithm, not the GPU's: nested ray-minimum "
                  "solver per element (MODEL_SPEC 4.3), all 1900 elements solved directly (no mirror symmetry), "
                  "direct element x point accumulation" % (n, batch.shape[0], el),
        "cpu": model, "host_cpus": os.cpu_count(), "cpus_available": avail}
    return out


if __name__ == "__main__":
    sys.exit(main())
