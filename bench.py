#!/usr/bin/env python3
"""Benchmark: walker ln_prob evaluations per second of the device-resident
emcee loop, on BASELINE.json's metric config (single eclipse, complex bright
spot, 300-point phase grid; config 2 = 1024 walkers per GPU).

A step is one emcee iteration of the whole ensemble: two half-steps of
propose -> batched ln_prob of the proposals (k_setup, k_elements, k_lnlike)
-> accept.  On one GPU a half-step is those three kernels alone
(lfg_stretch_step_half: the proposal formed in k_setup, the acceptance in
k_lnlike); with N ranks each proposes, evaluates its shard (lfg_lnprob),
all_gathers ln_prob, and every rank accepts.  value = walkers x steps /
time, max over ranks, inputs resident in HBM.  Per-GPU work is fixed (weak
scaling): --walkers per GPU, total = walkers x N.

Kernel timing: the last warmup step records HIP events around every kernel
(include/lfg.h LFG_NEV, on the caller stream all kernels run on) and picks
the dominant kernel; every ln_prob call of the timed region then records a
start/stop event pair around that kernel only.  (A timing event is a queue barrier: events around all kernels
cost ~20 % of the step, so they stay out of the timed region.)

  python bench.py [--gpus N --steps K --warmup W]
  torchrun --nproc-per-node N bench.py --gpus N ...
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# MI355X peaks (/opt/skills/guides/MI355X_MICROARCH.md; FP64 vector = spec)
HBM_PEAK_GBS = 8000.0
FP64_PEAK_TFLOPS = 78.6
PMC_FILE = os.path.join(ROOT, "profiles", "r01", "pmc_traffic.json")

NEV = 4  # LFG_NEV (include/lfg.h)
# (name as rocprofv3 prints it, start event, end event)
KERNELS = [("k_setup", 0, 1), ("k_elements", 1, 2), ("k_lnlike<1>", 2, 3)]

# Algorithmic HBM bytes per (walker, eclipse) pair of each kernel (DESIGN.md
# section 3): what the kernel must read and write, counted once.
NEL, U_DON, DON_STRIDE = 1500, 100, 5
GEO_SETUP, GEO_BSPOT, GEO_READ = 41, 5, 40   # geometry doubles written / read
WT_N = 124                                     # weight doubles per pair
PER_PAIR = {
    "k_setup": 18 * 8 + GEO_SETUP * 8 + 4 + 3 * 8 + GEO_BSPOT * 8 + 4,   # setup + stream lanes
    "k_elements": GEO_READ * 8 + 8 + NEL * 16 + U_DON * DON_STRIDE * 8 + WT_N * 8,
    "k_lnlike<1>": GEO_READ * 8 + 4 + NEL * 16 + U_DON * DON_STRIDE * 8 + WT_N * 8 + 8,
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)  # ~20 ms timed: one host hiccup stays small
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", type=int, default=2, choices=(2, 3, 5),
                    help="BASELINE.json config: 2 (the metric's, default), 3 (3-band x 4-eclipse tree, "
                         "2048 walkers), 5 (10000 points x 5 sub-samples, 4096 walkers)")
    ap.add_argument("--walkers", type=int, default=None, help="walkers per GPU (default: the config's)")
    ap.add_argument("--npts", type=int, default=None)
    ap.add_argument("--nsub", type=int, default=None)
    ap.add_argument("--shard-path", action="store_true",
                    help="run the multi-rank half-step (lfg_stretch_step_shard + accept_regen) on one rank")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--exchange-path", action="store_true",
                    help="one GPU: a one-rank RCCL group and the multi-rank code path with its real "
                         "exchange (shard kernels, ncclAllGather on the compute stream, k_accept_regen)")
    ap.add_argument("--seed", type=int, default=20261015)
    ap.add_argument("--time-every", type=int, default=4,
                    help="record the dominant kernel's event pair on every k-th ln_prob call of the timed region")
    args = ap.parse_args()
    dflt = {2: (1024, 300, 1), 3: (2048, 300, 1), 5: (4096, 10000, 5)}[args.config]
    args.walkers = args.walkers or dflt[0]
    args.npts = args.npts or dflt[1]
    args.nsub = args.nsub or dflt[2]
    return args


def algo_bytes(kernel, pairs, walkers, ndim, E, npts):
    b = PER_PAIR[kernel] * pairs
    if kernel == "k_setup":
        b += walkers * (ndim * 8 + 8)          # per-walker prior lane
    if kernel == "k_lnlike<1>":
        b += E * npts * 4 * 8                   # x, y, ye, w once per launch
        b += walkers * (8 * 2 + E * 8 * 2)      # fused combine: prior, lnp; 2 Roche priors per eclipse
    return b


def pmc_row(kernel):
    """Counter-derived bytes / FLOPs per launch of `kernel` (profiles/), or None."""
    try:
        d = json.load(open(PMC_FILE))
    except (OSError, ValueError):
        return None, None
    row = d.get("kernels", {}).get(kernel)
    return row, d.get("meta", {})


def main():
    args = parse()
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
        os.environ.setdefault("MASTER_PORT", "29541")
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

    from lfit_python_amd import _native, batch, sampler, synthetic
    from lfit_python_amd.lfit import flux_batch
    _native.require_gpu()
    L = _native.lib()

    def flux_fn(pars, x, w, nsub):
        f, st = flux_batch(np.asarray(pars)[None, :], x, w, nsub=nsub, device=dev)
        assert int(st[0].item()) == 0
        return f[0].cpu().numpy()

    if args.config == 3:
        model = synthetic.config_tree(4, args.npts, flux_fn=flux_fn, nsub=args.nsub)
    else:
        model = synthetic.config_single(npts=args.npts, flux_fn=flux_fn, nsub=args.nsub)
    tree = batch.compile_tree(model, nsub=args.nsub)
    ev = batch.LnProbEvaluator(tree, device=dev, max_walkers=args.walkers * world)
    W = args.walkers * world
    p0 = np.array(model.dynasty_par_vals)
    scat = sampler.comp_scatter(model.dynasty_par_names, 0.1)
    init = sampler.initialise_walkers(
        p0, scat, W, lambda p: ev(torch.as_tensor(p, device=dev)).cpu().numpy(), seed=args.seed)
    S = sampler.EnsembleSampler(W, tree.ndim, ev, seed=args.seed)
    S.force_shard = args.shard_path
    S.force_exchange = args.exchange_path
    S.set_state(init)

    # HIP events around kernels of lfg_lnprob calls (include/lfg.h LFG_NEV)
    events = []
    want = [True] * NEV  # which events to record
    every = [1]          # record on every k-th call
    ncall = [0]

    def sampled():
        ncall[0] += 1
        return (ncall[0] - 1) % every[0] == 0

    def make_evs():
        evs = (ctypes.c_void_p * NEV)()
        for i in range(NEV):
            if want[i]:
                h = ctypes.c_void_p()
                _native.check(L.lfg_event_create(ctypes.byref(h)), "lfg_event_create")
                evs[i] = h.value
        return evs

    def timed_half(pos, lnp, half, a, seed, step, q, zfac, naccept, lnp_new=None):
        """the single-process path: lfg_stretch_step_half with the events"""
        evs = None
        if sampled():
            evs = make_evs()
            events.append((evs, q.shape[0]))
        ev.step_half(pos, lnp, half, a, seed, step, q, zfac, naccept, lnp_new=lnp_new, events=evs)

    def timed_shard(pos, half, a, seed, step, lo, q, zfac, lnp_sh):
        """the multi-rank path: this rank's lfg_stretch_step_shard with the events"""
        evs = None
        if sampled():
            evs = make_evs()
            events.append((evs, lnp_sh.shape[0]))
        ev.step_shard(pos, half, a, seed, step, lo, q, zfac, lnp_sh, events=evs)

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
    dom = 2  # k_lnlike unless calibrated
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
    set_timing(True)

    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        S.step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    set_timing(False)
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # the dominant kernel's device time over the timed region
    shard = events[0][1] if events else W // 2
    dom_ms, ncalls = kernel_ms([KERNELS[dom]])
    avg_dom = float(dom_ms[0])
    E = tree.E
    npts = int(np.max(np.diff(tree.offsets)))
    algo = algo_bytes(kname, shard * E, shard, tree.ndim, E, npts)
    achieved = algo / (avg_dom * 1e-3) / 1e9
    value = W * args.steps / elapsed
    acc = float(np.mean(S.acceptance_fraction))

    # counter-derived traffic and executed FP64 FLOPs of the same kernel
    # (rocprofv3 --pmc passes, tools/pmc_profile.sh -> profiles/r01/pmc_traffic.json)
    # the committed PMC pass is of the default workload (config 2, 300 points,
    # nsub 1); per-pair counters do not carry over to other point counts
    row, meta = pmc_row(kname) if (args.config == 2 and args.npts == 300 and args.nsub == 1) else (None, None)
    traffic = fp64 = None
    if row and meta:
        scale = shard * E / float(meta.get("pairs_per_launch", shard * E))
        if "traffic_bytes" in row:
            traffic = row["traffic_bytes"] * scale
        if "fp64_flops" in row:
            f = row["fp64_flops"] * scale
            tf = f / (avg_dom * 1e-3) / 1e12
            fp64 = {"executed_flops": f, "achieved": tf, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                    "frac": tf / FP64_PEAK_TFLOPS, "source": os.path.relpath(PMC_FILE, ROOT)}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline(tree, S.pos.cpu().numpy(), args)

    if rank == 0:
        line = {
            "metric": "walker ln_prob evals/sec (300-pt phase, complex BS) at 1/2/4/8 MI355X",
            "value": value,
            "unit": "walker ln_prob evals/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic light curve (model at mcmc_input.dat eclipse-0 truth + N(0, 0.004)); "
                    "walkers from the comp_scat ball of mcmcfit.py",
            "config": {"workload": "config %d: %s, complex 18-par bright spot, "
                                   "%d phase pts, nsub %d, %d walkers/GPU, emcee stretch move"
                                   % (args.config, "3-band x 4-eclipse tree" if args.config == 3
                                      else "single eclipse", args.npts, args.nsub, args.walkers),
                       "walkers_total": W, "eclipses": E, "ndim": tree.ndim,
                       "parallelism": "walker shards x%d, replicated Philox RNG, "
                                      "all_gather of ln_prob per half-step (%s)" % (
                                          world, "one rank: no exchange" if dist is None
                                          else ("%s all_gather" % backend if backend != "nccl"
                                                else ("ncclAllGather on the compute stream"
                                                      if os.environ.get("LFG_RCCL_DIRECT", "1") != "0"
                                                      else "torch ProcessGroupNCCL"))),
                       },
            "roofline": {"bound": "hbm", "kernel": kname, "achieved": achieved,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                         "traffic": traffic, "algo_bytes_per_launch": algo,
                         "avg_launch_ms": float(avg_dom),
                         "fp64_valu": fp64,
                         "note": "FP64-VALU bound root finding (DESIGN.md 3); HBM fraction reported per contract; "
                                 "traffic = FETCH_SIZE x2 + WRITE_SIZE per launch from the committed PMC pass"},
            "kernel_ms_per_launch_warmup": calib,
            "launches_timed": ncalls,
            "acceptance_fraction": acc,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line))
    S.close()
    if dist:
        dist.destroy_process_group()


def cpu_baseline(tree, walkers, args):
    """The C oracle (OpenMP over walkers) on this host's cores, same tree and
    walkers, bounded to about args.cpu_seconds of work."""
    import subprocess
    import tempfile
    from oracle import oracle as orc
    path = os.path.join(tempfile.gettempdir(), "liblfg_oracle_native_%d.so" % os.getpid())
    try:
        orc.build(march="native", out=path)
    except (subprocess.CalledProcessError, FileNotFoundError):
        path = orc.LIB_PATH
    o = orc.Oracle(path)
    nthr = max(1, min(args.cpu_threads, os.cpu_count() or 1))
    batch = walkers[: max(nthr * 4, 64)]
    o.lnprob_batch(batch[:nthr], tree, nsub=args.nsub, nthreads=nthr)  # warm
    n, t0 = 0, time.perf_counter()
    used = nthr
    while True:
        _, _, used = o.lnprob_batch(batch, tree, nsub=args.nsub, nthreads=nthr)
        n += batch.shape[0]
        el = time.perf_counter() - t0
        if el >= args.cpu_seconds:
            break
    model = ""
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"value": n / el, "unit": "walker ln_prob evals/s", "cores": int(used), "kind": "port",
            "sample": "%d ln_prob evals (%d-walker batches of the same tree) in %.1f s, "
                      "oracle/lfg_oracle.c -O3 -march=native OpenMP" % (n, batch.shape[0], el),
            "cpu": model}


if __name__ == "__main__":
    main()
