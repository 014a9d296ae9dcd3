#!/usr/bin/env python3
"""Benchmark: walker ln_prob evaluations per second of the device-resident
emcee loop, on BASELINE.json's metric config (single eclipse, complex bright
spot, 300-point phase grid; config 2 = 1024 walkers per GPU).

A step is one emcee iteration of the whole ensemble: two half-steps of
propose -> batched ln_prob (lfg_lnprob: setup, elements, lnlike, combine
kernels) -> all_gather -> accept.  value = walkers x steps / time, max over
ranks, inputs resident in HBM.  Per-GPU work is fixed (weak scaling):
--walkers per GPU, total = walkers x N.

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


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--walkers", type=int, default=1024, help="walkers per GPU")
    ap.add_argument("--npts", type=int, default=300)
    ap.add_argument("--nsub", type=int, default=1)
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--seed", type=int, default=20261015)
    return ap.parse_args()


def main():
    args = parse()
    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=dev)

    from lfit_python_amd import _native, batch, sampler, synthetic
    from lfit_python_amd.lfit import flux_batch
    _native.require_gpu()
    L = _native.lib()

    def flux_fn(pars, x, w, nsub):
        f, st = flux_batch(np.asarray(pars)[None, :], x, w, nsub=nsub, device=dev)
        assert int(st[0].item()) == 0
        return f[0].cpu().numpy()

    model = synthetic.config_single(npts=args.npts, flux_fn=flux_fn, nsub=args.nsub)
    tree = batch.compile_tree(model, nsub=args.nsub)
    ev = batch.LnProbEvaluator(tree, device=dev, max_walkers=args.walkers * world)
    W = args.walkers * world
    p0 = np.array(model.dynasty_par_vals)
    scat = sampler.comp_scatter(model.dynasty_par_names, 0.1)
    init = sampler.initialise_walkers(
        p0, scat, W, lambda p: ev(torch.as_tensor(p, device=dev)).cpu().numpy(), seed=args.seed)
    S = sampler.EnsembleSampler(W, tree.ndim, ev, seed=args.seed)
    S.set_state(init)

    # kernel timing: HIP events around each kernel of every lfg_lnprob call
    # in the timed region, on the stream the kernels run on
    events, pending = [], []

    def make_evs():
        evs = (ctypes.c_void_p * 5)()
        for i in range(5):
            h = ctypes.c_void_p()
            _native.check(L.lfg_event_create(ctypes.byref(h)), "lfg_event_create")
            evs[i] = h.value
        return evs

    def timed_eval(x, out=None):
        if out is None:
            out = torch.empty(x.shape[0], dtype=torch.float64, device=dev)
        ev._ensure(x.shape[0])
        evs = pending.pop() if pending else make_evs()
        events.append((evs, x.shape[0]))
        rc = L.lfg_lnprob_timed(ctypes.c_void_p(x.data_ptr()), x.shape[0], ctypes.byref(ev.ctree),
                                ctypes.c_void_p(out.data_ptr()), None, ctypes.c_void_p(ev._ws.data_ptr()),
                                ev._ws.numel(), _native.stream_ptr(dev), evs)
        _native.check(rc, "lfg_lnprob_timed")
        return out

    for _ in range(args.warmup):
        S.step()
    torch.cuda.synchronize()
    S.timer = timed_eval
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
    S.timer = None
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # per-kernel device time over the timed region
    names = ["k_setup", "k_elements", "k_lnlike", "k_combine"]
    tot = np.zeros(4)
    fms = ctypes.c_float()
    for evs, n in events:
        for k in range(4):
            _native.check(L.lfg_event_elapsed_ms(evs[k], evs[k + 1], ctypes.byref(fms)), "elapsed")
            tot[k] += fms.value
    ncalls = len(events)
    avg_ms = tot / max(ncalls, 1)
    for evs, _ in events:
        for i in range(5):
            L.lfg_event_destroy(evs[i])
    dom = int(np.argmax(tot))
    shard = events[0][1] if events else W // 2
    E = tree.E
    # algorithmic HBM bytes per launch
    NEL, NDON, NGEO = 1500, 400, 48
    npts = int(np.max(np.diff(tree.offsets)))
    bytes_per_pair = {
        "k_setup": 18 * 8 + (NGEO * 8 + 4),
        "k_elements": NGEO * 8 + 4 + NEL * 3 * 8 + NDON * 3 * 8,
        "k_lnlike": NGEO * 8 + 4 + NEL * 3 * 8 + NDON * 3 * 8 + npts * 4 * 8 + 8,
        "k_combine": 8 * 3,
    }
    algo_bytes = bytes_per_pair[names[dom]] * shard * E
    achieved = algo_bytes / (avg_ms[dom] * 1e-3) / 1e9
    value = W * args.steps / elapsed
    acc = float(np.mean(S.acceptance_fraction))

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
            "config": {"workload": "config 2: single eclipse, complex 18-par bright spot, "
                                   "%d phase pts, nsub %d, %d walkers/GPU, emcee stretch move"
                                   % (args.npts, args.nsub, args.walkers),
                       "walkers_total": W, "eclipses": E, "ndim": tree.ndim,
                       "parallelism": "walker shards x%d, replicated Philox RNG, "
                                      "all_gather of ln_prob per half-step" % world},
            "roofline": {"bound": "hbm", "kernel": names[dom], "achieved": achieved,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                         "traffic": None, "algo_bytes_per_launch": algo_bytes,
                         "avg_launch_ms": float(avg_ms[dom]),
                         "note": "path is FP64-VALU bound (DESIGN.md 4); HBM fraction reported per contract"},
            "kernel_ms_per_launch": {n: float(m) for n, m in zip(names, avg_ms)},
            "launches_timed": ncalls,
            "acceptance_fraction": acc,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line))
    if dist:
        dist.destroy_process_group()


def cpu_baseline(tree, walkers, args):
    """The C oracle (OpenMP over walkers) on this host's cores, same tree and
    walkers, bounded to about args.cpu_seconds of work."""
    import subprocess
    import tempfile
    sys.path.insert(0, ROOT)
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
