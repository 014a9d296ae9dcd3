"""Device-resident affine-invariant ensemble sampler.

Stands in for emcee.EnsembleSampler(nwalkers, ndim, ln_prob, args=(model,),
pool=pool) as the reference drives it (mcmcfit.py:272-343,
mcmc_utils.py:46-183): the walker ensemble lives in HBM, each emcee step is
two half-steps (red/blue halves, emcee 2.x fixed split) of
  propose (HIP, Philox) -> ln_prob of the proposals (one batched lfg_lnprob
  on this rank's shard) -> all_gather of the new ln_prob -> accept (HIP)
and nothing crosses PCIe inside the loop.  With torch.distributed
initialised, every rank holds the full ensemble and draws identical random
numbers (counter-based Philox keyed by the seed), evaluates only its shard of
each half and exchanges W/2 doubles per half-step; the accept step is then
identical on every rank, so positions never travel.
"""
import ctypes
import os

import numpy as np

from . import _native

# comp_scat scatter factors (mcmcfit.py:208-232)
SCATTER_FACTORS = {
    'ln_ampin_gp': 5.0, 'ln_ampout_gp': 5.0, 'ln_tau_gp': 5.0,
    'q': 1, 'rwd': 1, 'dphi': 0.2, 'dFlux': 1, 'sFlux': 1, 'wdFlux': 1, 'rsFlux': 1,
    'rdisc': 1, 'ulimb': 1e-6, 'scale': 1, 'fis': 1, 'dexp': 1, 'phi0': 1, 'az': 1,
    'exp1': 1, 'exp2': 1, 'yaw': 1, 'tilt': 1,
}


def comp_scatter(names, scatter):
    """Per-parameter scatter vector of mcmcfit.py:204-246."""
    from .tree import extract_par_and_key
    out = np.full(len(names), float(scatter))
    for i, n in enumerate(names):
        key, _ = extract_par_and_key(n)
        if key.startswith('ln'):
            continue
        out[i] *= SCATTER_FACTORS[key]
    return out


def _host(t):
    """a host copy of a tensor (never a view of device-side or live state)"""
    return t.cpu().numpy() if t.device.type != "cpu" else t.numpy().copy()


class HipStretchOps:
    """The stretch move's two device kernels (include/lfg.h)."""

    def __init__(self, device):
        self.L = _native.lib()
        self.device = device

    @staticmethod
    def _vp(t):
        return ctypes.c_void_p(t.data_ptr())

    def propose(self, pos, half, a, seed, step, q, zfac):
        W, ndim = pos.shape
        rc = self.L.lfg_stretch_propose(self._vp(pos), W, ndim, half, a, seed, step, self._vp(q),
                                        self._vp(zfac), _native.stream_ptr(self.device))
        _native.check(rc, "lfg_stretch_propose")

    def accept(self, pos, lnp, half, q, zfac, lnp_new, seed, step, naccept):
        W, ndim = pos.shape
        rc = self.L.lfg_stretch_accept(self._vp(pos), self._vp(lnp), W, ndim, half, self._vp(q),
                                       self._vp(zfac), self._vp(lnp_new), seed, step,
                                       self._vp(naccept), _native.stream_ptr(self.device))
        _native.check(rc, "lfg_stretch_accept")

    # step counter in device memory (int64 tensor of one element): HIP-graph capturable
    def accept_regen(self, pos, lnp, half, a, lnp_new, seed, step, naccept):
        W, ndim = pos.shape
        rc = self.L.lfg_stretch_accept_regen(self._vp(pos), self._vp(lnp), W, ndim, half, a, seed, step,
                                             self._vp(lnp_new), self._vp(naccept), _native.stream_ptr(self.device))
        _native.check(rc, "lfg_stretch_accept_regen")

    def propose_dev(self, pos, half, a, seed, step_dev, q, zfac):
        W, ndim = pos.shape
        rc = self.L.lfg_stretch_propose_dev(self._vp(pos), W, ndim, half, a, seed, self._vp(step_dev),
                                            self._vp(q), self._vp(zfac), _native.stream_ptr(self.device))
        _native.check(rc, "lfg_stretch_propose_dev")

    def accept_dev(self, pos, lnp, half, q, zfac, lnp_new, seed, step_dev, naccept):
        W, ndim = pos.shape
        rc = self.L.lfg_stretch_accept_dev(self._vp(pos), self._vp(lnp), W, ndim, half, self._vp(q),
                                           self._vp(zfac), self._vp(lnp_new), seed, self._vp(step_dev),
                                           self._vp(naccept), _native.stream_ptr(self.device))
        _native.check(rc, "lfg_stretch_accept_dev")


class EnsembleSampler:
    """evaluator(x [n, ndim] tensor, out=None) -> ln_prob [n] on evaluator.device.
    ops: the propose/accept implementation (HipStretchOps by default; the
    CPU tests inject a host double to exercise the sharding logic)."""

    def __init__(self, nwalkers, ndim, evaluator, a=2.0, seed=0, group=None, ops=None):
        import torch
        if nwalkers % 2 or nwalkers < 4:
            raise ValueError("nwalkers must be even and >= 4")
        self.W, self.ndim, self.a = int(nwalkers), int(ndim), float(a)
        self.ev = evaluator
        self.dev = evaluator.device
        self.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
        self.ops = ops if ops is not None else HipStretchOps(self.dev)
        self.group = group
        dist = torch.distributed
        self.world = dist.get_world_size(group) if (dist.is_available() and dist.is_initialized()) else 1
        self.rank = dist.get_rank(group) if self.world > 1 else 0
        ns = self.W // 2
        if ns % self.world:
            raise ValueError("W/2 = %d walkers per half must divide over %d ranks" % (ns, self.world))
        self.shard = ns // self.world
        f64 = dict(dtype=torch.float64, device=self.dev)
        self._pos = torch.empty((self.W, self.ndim), **f64)
        self._lnp = torch.empty(self.W, **f64)
        self.q = torch.empty((ns, self.ndim), **f64)
        self.zfac = torch.empty(ns, **f64)
        self.lnp_new = torch.empty(ns, **f64)
        self._naccept = torch.zeros(self.W, dtype=torch.int32, device=self.dev)
        self.iteration = 0   # emcee's counter: reset() clears it (acceptance fractions)
        # Philox step counter of every draw: monotone over the sampler's life,
        # so the production run after reset() never replays burn-in draws
        # (the reference hands the burn-in RNG state on, mcmc_utils.py:135-183)
        self.rng_step = 0
        # stored chain: (chain [n, W, ndim], lnprob [n, W]) per stored run.  A run
        # fills a device chunk (the steps stay free of host syncs); when it ends
        # the chunk moves to host memory, as emcee keeps its chain in
        # RAM, so device memory holds one run's chunk at a time however long
        # the chain grows (offload = False keeps every chunk on the device)
        self._chunks = []
        self._cat = None
        self._last = None  # the most recent run's chunk (None: it stored nothing)
        self._active = None  # the chunk of a run in progress (sample() generator, run_mcmc)
        self.offload = True
        self.timer = None  # optional callable(walkers) -> lnp used instead of self.ev
        # one process, HIP moves, an evaluator with the fused entry: proposal,
        # ln_prob and acceptance in one launch sequence (lfg_stretch_step_half);
        # the optional half_timer replaces evaluator.step_half (bench timing)
        self.fuse = hasattr(evaluator, "step_half") and isinstance(self.ops, HipStretchOps)
        self.half_timer = None
        # speculative setup on the fused path (lfg_stretch_step_half_spec): each
        # half's k_elements also forms the next half's k_setup outputs for both
        # fates of every partner, so the next half skips k_setup (the evaluator
        # tracks whether its workspace holds valid candidates)
        self.spec = os.environ.get("LFG_SPEC", "1") != "0"
        # sharded fused path (N ranks, or forced on one for tests): proposal and
        # ln_prob of this rank's shard in three kernels (lfg_stretch_step_shard),
        # all_gather of ln_prob, acceptance re-forming the proposals
        # (lfg_stretch_accept_regen); shard_timer replaces evaluator.step_shard
        self.fuse_shard = hasattr(evaluator, "step_shard") and isinstance(self.ops, HipStretchOps)
        self.force_shard = False
        self.force_exchange = False  # one rank: still exchange through the collective (rehearsal)
        self.shard_timer = None
        self._q_sh = self._zf_sh = self._lnp_sh = None
        # deferred acceptance on the sharded path (lfg_stretch_step_shard_fold):
        # each half-step is ONE launch + the exchange; the launch applies the
        # other half's gathered verdicts of the half-step before.  _V: the
        # gathered verdicts per half (ln_prob where accepted, NaN); _pending:
        # (half, step) of verdicts not yet applied; _store_next: a chain record
        # of the step before, taken once its last verdicts are applied
        self.fold = os.environ.get("LFG_FOLD", "1") != "0"
        self._V = None
        self._v_sh = None
        self._pending = None
        self._store_next = None
        self._emu = None   # (rank, nranks) of emulate_rank()
        self._rccl = None  # direct RCCL all-gather (built at the first nccl exchange)
        # HIP-graph replay of whole iterations (single rank, HIP ops): the first
        # step() after enabling runs eagerly, the next captures, later ones replay
        self.use_graph = False
        self._graph = None
        self._graph_gen = None  # evaluator workspace generation the graph was captured on
        self._step_dev = None
        self._dev_iter = 0
        self._warm = False  # one eager iteration (allocations, side stream) before capture

    def _gather(self, out, mine):
        import torch.distributed as dist
        if dist.get_backend(self.group) == "nccl":
            # ncclAllGather on the kernels' own stream (comm.py); LFG_RCCL_DIRECT=0
            # keeps torch's ProcessGroupNCCL path (its stream hand-off ~6 us more)
            if self._rccl is None:
                direct = os.environ.get("LFG_RCCL_DIRECT", "1") != "0"
                if direct:
                    # every rank must take the same path (building the
                    # communicator is collective): agree first that each
                    # can load librccl, else all use ProcessGroupNCCL
                    from . import comm
                    try:
                        comm._load_rccl()
                        ok = 1
                    except (OSError, AttributeError):
                        ok = 0
                    import torch
                    flag = torch.tensor([ok], dtype=torch.int32, device=out.device)
                    dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=self.group)
                    direct = bool(flag.item())
                self._rccl = comm.RcclAllGather(self.group) if direct else False
            if self._rccl:
                self._rccl(out, mine)
                return
            dist.all_gather_into_tensor(out, mine, group=self.group)
        else:
            dist.all_gather(list(out.chunk(self.world)), mine, group=self.group)

    def _eval(self, x, out):
        return (self.timer or self.ev)(x, out=out)

    # the ensemble, brought up to date first: with the deferred acceptance the
    # last half-step's moves are applied by the next launch, or here
    @property
    def pos(self):
        self.sync()
        return self._pos

    @property
    def lnp(self):
        self.sync()
        return self._lnp

    @property
    def naccept(self):
        self.sync()
        return self._naccept

    def _flush(self):
        if self._pending is not None:
            half, step = self._pending
            self._pending = None
            self.ev.apply_verdicts(self._pos, self._lnp, half, self.a, self.seed, step, self._V[half],
                                   self._naccept)

    def sync(self):
        """Apply pending verdicts (lfg_stretch_apply_verdicts) and take a
        deferred chain record: afterwards pos / lnp / naccept are the state
        after the last step, as on the other paths."""
        self._flush()
        if self._store_next is not None:
            rec, self._store_next = self._store_next, None
            self._store(*rec)

    def _fold_ok(self):
        return (self.fold and self.spec and hasattr(self.ev, "step_shard_fold") and
                (self.shard_timer is None or getattr(self.shard_timer, "takes_fold", False)))

    def set_state(self, p0, lnp0=None):
        import torch
        if hasattr(self.ev, "invalidate_spec"):
            self.ev.invalidate_spec()  # the candidates were formed from the old positions
        self._pending = None   # verdicts of the old state are void
        self._store_next = None
        self._pos.copy_(torch.as_tensor(np.asarray(p0), dtype=torch.float64))
        if lnp0 is None:
            self._lnp.copy_(self.ln_prob(self._pos))
        else:
            self._lnp.copy_(torch.as_tensor(np.asarray(lnp0), dtype=torch.float64))
        self._naccept.zero_()

    def ln_prob(self, x):
        """ln_prob of walkers x [n, ndim], sharded over ranks when n divides."""
        import torch
        n = x.shape[0]
        if self.world == 1 or n % self.world:
            return self.ev(x)
        k = n // self.world
        mine = self.ev(x[self.rank * k:(self.rank + 1) * k].contiguous())
        out = torch.empty(n, dtype=torch.float64, device=self.dev)
        self._gather(out, mine)
        return out

    def _graphable(self):
        return (self.use_graph and self.timer is None and self._graph_ok())

    def _graph_ok(self):
        return self.world == 1 and isinstance(self.ops, HipStretchOps) and self.dev.type == "cuda"

    def _graph_body(self, ev):
        for half in (0, 1):
            self.ops.propose_dev(self._pos, half, self.a, self.seed, self._step_dev, self.q, self.zfac)
            ev(self.q, out=self.lnp_new)
            self.ops.accept_dev(self._pos, self._lnp, half, self.q, self.zfac, self.lnp_new, self.seed,
                                self._step_dev, self._naccept)
        self._step_dev.add_(1)

    def _sync_step_dev(self):
        import torch
        if self._step_dev is None:
            self._step_dev = torch.full((1,), self.rng_step, dtype=torch.int64, device=self.dev)
            self._dev_iter = self.rng_step
        elif self._dev_iter != self.rng_step:  # the counter was set from outside (set_rng_state)
            self._step_dev.fill_(self.rng_step)
            self._dev_iter = self.rng_step

    def capture_iteration(self, evaluator=None):
        """A HIP graph of one whole emcee iteration (single rank, HIP ops) that
        reads the step counter from device memory; `evaluator` (default: the
        sampler's) is the ln_prob call captured inside.  Replay with replay()."""
        import torch
        if not self._graph_ok():
            raise RuntimeError("graph capture needs a single rank and the HIP stretch kernels")
        self._sync_step_dev()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            self._graph_body(evaluator or self.ev)
        return g

    def replay(self, g):
        """One emcee iteration by replaying a graph from capture_iteration()."""
        self._sync_step_dev()
        g.replay()
        self.iteration += 1
        self.rng_step += 1
        self._dev_iter += 1

    def _graph_step(self):
        # the graph bakes in the evaluator's workspace pointer: re-capture when
        # the evaluator has reallocated it since (batch.LnProbEvaluator.generation)
        gen = getattr(self.ev, "generation", None)
        if self._graph is None or gen != self._graph_gen:
            self._graph = None
            self._graph = self.capture_iteration()
            self._graph_gen = gen
        self.replay(self._graph)

    def step(self):
        """One emcee iteration: both halves, in place.

        On the sharded fold path (lfg_stretch_step_shard_fold) the last
        half-step's acceptance stays pending after step() returns: it is
        applied by the next step's first launch.  The ensemble is current
        through the pos / lnp / naccept / naccepted / acceptance_fraction
        properties, or after sync() or close(); the raw _pos / _lnp tensors
        lag one half-step until then."""
        if self._pending is not None and not (
                (self.world > 1 or self.force_shard) and self.fuse_shard and self.timer is None and self._fold_ok()):
            self.sync()  # a path without the deferred acceptance follows
        if self._graphable() and self._warm:
            self._graph_step()
            return
        self._warm = True
        for half in (0, 1):
            if self.world == 1 and self.fuse and self.timer is None and not self.force_shard:
                f = self.half_timer or self.ev.step_half
                # a replacement step_half (bench timing, tests) takes spec only if it says so
                kw = dict(spec=True) if self.spec and (self.half_timer is None or
                                                       getattr(self.half_timer, "takes_spec", False)) else {}
                f(self._pos, self._lnp, half, self.a, self.seed, self.rng_step, self.q, self.zfac, self._naccept,
                  lnp_new=self.lnp_new, **kw)
                continue
            if (self.world > 1 or self.force_shard) and self.fuse_shard and self.timer is None:
                self._shard_half(half)
                continue
            self.ops.propose(self._pos, half, self.a, self.seed, self.rng_step, self.q, self.zfac)
            if self.world == 1:
                self._eval(self.q, self.lnp_new)
            else:
                lo = self.rank * self.shard
                mine = self._eval(self.q[lo:lo + self.shard], None)
                self._gather(self.lnp_new, mine)
            self.ops.accept(self._pos, self._lnp, half, self.q, self.zfac, self.lnp_new, self.seed,
                            self.rng_step, self._naccept)
        self.iteration += 1
        self.rng_step += 1

    def emulate_rank(self, k, nranks):
        """Timing rehearsal of one rank of an nranks-GPU run on this one
        process: each half-step evaluates only walkers k*n .. (k+1)*n - 1 of
        the half (n = W / 2 / nranks) through the multi-rank kernels, the
        exchange moves that shard alone (a one-rank group's all_gather with
        force_exchange), and the acceptance runs over the whole half as on
        every rank.  The other shards' entries of the gathered ln_prob stay
        -inf, so their walkers never move (they stay in the valid starting
        ball and keep rank k's partners realistic); the chain is NOT a valid
        sample, but the launches are exactly rank k's (bench.py --emulate-rank)."""
        ns = self.W // 2
        if ns % nranks or not (0 <= k < nranks):
            raise ValueError("W/2 = %d does not shard over %d ranks" % (ns, nranks))
        self.force_shard = True
        self.shard = ns // nranks
        self._emu = (int(k), int(nranks))
        self._q_sh = self._zf_sh = self._lnp_sh = None
        self.lnp_new.fill_(float("-inf"))
        self.sync()
        self._V = self._v_sh = None

    def _shard_half(self, half):
        import torch
        if self._lnp_sh is None:
            f64 = dict(dtype=torch.float64, device=self.dev)
            self._q_sh = torch.empty((self.shard, self.ndim), **f64)
            self._zf_sh = torch.empty(self.shard, **f64)
            self._lnp_sh = torch.empty(self.shard, **f64)
        lo = (self._emu[0] if self._emu else self.rank) * self.shard
        if self._fold_ok():
            self._fold_half(half, lo)
            return
        self._flush()
        f = self.shard_timer or self.ev.step_shard
        spec = self.spec and hasattr(self.ev, "accept_regen") and (
            self.shard_timer is None or getattr(self.shard_timer, "takes_spec", False))
        f(self._pos, half, self.a, self.seed, self.rng_step, lo, self._q_sh, self._zf_sh,
          self._lnp_sh, **(dict(spec=True) if spec else {}))
        dst = self.lnp_new[lo:lo + self.shard] if self._emu else self.lnp_new
        if self.world > 1 or self.force_exchange:
            self._gather(dst, self._lnp_sh)
        else:
            dst.copy_(self._lnp_sh)
        if spec:  # records the acceptances for the next half's speculative setup
            self.ev.accept_regen(self._pos, self._lnp, half, self.a, self.seed, self.rng_step, self.lnp_new,
                                 self._naccept, self.shard)
        else:
            self.ops.accept_regen(self._pos, self._lnp, half, self.a, self.lnp_new, self.seed, self.rng_step,
                                  self._naccept)

    def _fold_half(self, half, lo):
        import torch
        if self._V is None:
            f64 = dict(dtype=torch.float64, device=self.dev)
            # NaN: no move accepted (the other shards' entries when emulating one rank)
            self._V = [torch.full((self.W // 2,), float("nan"), **f64) for _ in range(2)]
            self._v_sh = torch.empty(self.shard, **f64)
        want = (1 - half, self.rng_step - 1 if half == 0 else self.rng_step)
        if self._pending is not None and self._pending != want:
            self._flush()   # not the half-step just before: apply on its own
        vprev = self._V[1 - half] if self._pending is not None else None
        f = self.shard_timer or self.ev.step_shard
        f(self._pos, half, self.a, self.seed, self.rng_step, lo, self._q_sh, self._zf_sh, self._lnp_sh, spec=True,
          fold=(self._lnp, vprev, self._v_sh, self._naccept))
        self._pending = None
        if half == 0 and self._store_next is not None:
            # the launch applied the previous step's last verdicts and none of
            # this step's yet: the ensemble is the previous step's state
            rec, self._store_next = self._store_next, None
            self._store(*rec)
        dst = self._V[half][lo:lo + self.shard] if self._emu else self._V[half]
        if self.world > 1 or self.force_exchange:
            self._gather(dst, self._v_sh)
        else:
            dst.copy_(self._v_sh)
        self._pending = (half, self.rng_step)

    def close(self):
        """Release the direct RCCL communicator (every rank, before the
        process group is destroyed); pending verdicts are applied first."""
        self.sync()
        if self._rccl:
            self._rccl.close()
        self._rccl = None

    # ---- emcee 2.x surface (EnsembleSampler.sample / run_mcmc / chain /
    # lnprobability / flatchain / reset), as the reference drives it:
    # mcmc_utils.py:114-183 (sample generators), mcmcfit.py:313-341 (reset,
    # chain as (nwalkers, nsteps, npars) into utils.flatchain(..., thin=10))
    def _begin(self, p0, lnprob0, rstate0, iterations, thin, store):
        """common start of sample() / run_mcmc(): state, RNG counter, and a
        device chunk [iterations // thin, W, ndim] appended to the chain"""
        import torch
        if rstate0 is not None:
            self.random_state = rstate0
        if p0 is not None:
            self.set_state(p0, lnprob0)
        thin = max(1, int(thin))
        if not store:
            self._last = None
            return None, thin
        n = -(-int(iterations) // thin)  # steps i with i % thin == 0 (emcee 2.x stores those)
        buf = (torch.empty((n, self.W, self.ndim), dtype=torch.float64, device=self.dev),
               torch.empty((n, self.W), dtype=torch.float64, device=self.dev))
        self._chunks.append(buf)
        self._last = buf
        self._active = buf   # written step by step until _end()
        self._cat = None
        return buf, thin

    def _end(self, buf, rows=None):
        """end of a stored run: its device chunk moves to host memory
        (offload); rows: the chunk's rows actually written (a sample()
        generator left early), the rest is dropped"""
        if buf is not None and self._active is buf:
            self._active = None
        if buf is not None and rows is not None and rows < buf[0].shape[0]:
            cut = (buf[0][:rows], buf[1][:rows])
            self._chunks = [cut if c is buf else c for c in self._chunks]
            if self._last is buf:
                self._last = cut
            self._cat = None
            buf = cut
        if buf is None or not self.offload or self.dev.type != "cuda":
            return
        host = tuple(t.cpu() for t in buf)
        self._chunks = [host if c is buf else c for c in self._chunks]
        self._last = host
        self._cat = None

    def _record(self, buf, i, thin):
        """the chain record of step i: at once, or (verdicts pending) when
        the next step's first launch has applied them (sync() at the end)"""
        if self._pending is not None and buf is not None and i % thin == 0:
            self._store_next = (buf, i, thin)
        else:
            self._store(buf, i, thin)

    def _store(self, buf, i, thin):
        if buf is not None and i % thin == 0:
            buf[0][i // thin].copy_(self._pos)
            buf[1][i // thin].copy_(self._lnp)
            self._cat = None   # a concatenation taken mid-run is a copy: re-take it

    def sample(self, p0=None, lnprob0=None, rstate0=None, blobs0=None, iterations=1, thin=1,
               storechain=True, store=None, skip_initial_state_check=False, **kwargs):
        """emcee 2.x EnsembleSampler.sample: a generator over `iterations`
        steps yielding (pos [W, ndim], lnprob [W], state) as host arrays after
        each step (mcmc_utils.py:121-126, 151-164).  `p0` None continues from
        the current state; `rstate0` sets the RNG counter (random_state);
        storechain (emcee 2.x) / store (emcee 3) append every thin-th step to
        the chain.  Each yield copies the ensemble to the host: the bulk,
        sync-free path is run_mcmc()."""
        buf, thin = self._begin(p0, lnprob0, rstate0, iterations,
                                thin, storechain if store is None else store)
        done = 0
        try:
            for i in range(int(iterations)):
                self.step()
                self.sync()
                self._store(buf, i, thin)
                done = i + 1
                if i == int(iterations) - 1:
                    self._end(buf)
                    buf = None
                yield _host(self._pos), _host(self._lnp), self.random_state
        finally:
            # a caller that leaves the generator early (break, GeneratorExit)
            # keeps the steps it ran, offloaded
            if buf is not None:
                self._end(buf, rows=-(-done // thin))

    def run_mcmc(self, pos0, N, rstate0=None, lnprob0=None, storechain=True, store=None, thin=1, **kwargs):
        """emcee 2.x run_mcmc: N steps from pos0 (None: the current state);
        returns (pos, lnprob, state) of the last step as host arrays.  The
        steps are launched back to back and the stored chain stays on the
        device (chain_dev) until it is read."""
        buf, thin = self._begin(pos0, lnprob0, rstate0, N, thin, storechain if store is None else store)
        for i in range(int(N)):
            self.step()
            self._record(buf, i, thin)
        self.sync()
        self._end(buf)
        return _host(self._pos), _host(self._lnp), self.random_state

    def _concat(self):
        """the stored chain as one (chain, lnprob) pair, wherever the chunks
        live (host after offload).  Host chunks are replaced by their
        concatenation (one host copy of the chain), and the last
        run's chunk becomes a view into it"""
        import torch
        if self._cat is None:
            if not self._chunks:
                self._cat = (torch.empty((0, self.W, self.ndim), dtype=torch.float64),
                             torch.empty((0, self.W), dtype=torch.float64))
            elif len(self._chunks) == 1:
                self._cat = self._chunks[0]
            else:
                # a run still in progress keeps writing its chunk: only a
                # chain of finished host chunks collapses into one
                on_host = (all(c.device.type == "cpu" for c, _ in self._chunks) and
                           not any(c is self._active for c in self._chunks))
                last = self._chunks[-1]
                self._cat = (torch.cat([c.cpu() for c, _ in self._chunks]),
                             torch.cat([l.cpu() for _, l in self._chunks]))
                if on_host:
                    n = last[0].shape[0]
                    if self._last is last:
                        self._last = (self._cat[0][self._cat[0].shape[0] - n:],
                                      self._cat[1][self._cat[1].shape[0] - n:])
                    self._chunks = [self._cat]
        return self._cat

    @property
    def chain_dev(self):
        """the stored chain on the device, step-major [nsteps, W, ndim] (an
        upload of the host chunks when they were offloaded)"""
        return self._concat()[0].to(self.dev)

    @property
    def lnprob_dev(self):
        """the stored ln_prob on the device, [nsteps, W]"""
        return self._concat()[1].to(self.dev)

    def last_run(self):
        """(chain [n, W, ndim], lnprob [n, W]) of the most recent
        sample()/run_mcmc() call, None if that call stored nothing (bulk
        chain_prod.txt writes; host tensors once the run was offloaded)"""
        return self._last

    @property
    def chain(self):
        """emcee's chain: host array (nwalkers, nsteps, ndim)"""
        return _host(self._concat()[0].permute(1, 0, 2))

    @property
    def lnprobability(self):
        """emcee's lnprobability: host array (nwalkers, nsteps)"""
        return _host(self._concat()[1].t())

    @property
    def flatchain(self):
        return self.chain.reshape((-1, self.ndim))

    @property
    def flatlnprobability(self):
        return self.lnprobability.reshape(-1)

    @property
    def iterations(self):
        """emcee 2.x's step counter (cleared by reset())"""
        return self.iteration

    @property
    def naccepted(self):
        self.sync()   # the last half-step's verdicts may still be pending
        return self._naccept.cpu().numpy()

    @property
    def acceptance_fraction(self):
        self.sync()
        return (self._naccept.double() / max(self.iteration, 1)).cpu().numpy()

    def reset(self):
        """emcee's reset: clears the chain, the iteration count and the
        acceptance counters; the RNG stream carries on (rng_step is kept)."""
        self.sync()
        self.iteration = 0
        self._naccept.zero_()
        self._chunks = []
        self._cat = None
        self._last = None
        self._active = None

    @property
    def random_state(self):
        """The RNG state, emcee's `state` / `rstate0`: the Philox counter of
        the next iteration (the key is the seed)."""
        return self.rng_step

    @random_state.setter
    def random_state(self, step):
        self.rng_step = int(step)


def initialise_walkers(p, scatter, nwalkers, ln_prob_fn, seed=0, max_rounds=1000):
    """mcmc_utils.initialise_walkers (mcmc_utils.py:46-72): a Gaussian ball
    (emcee.utils.sample_ball) resampled until every walker has a finite
    ln_prior.  ln_prob_fn maps [n, ndim] numpy -> [n] numpy; -inf means invalid."""
    rng = np.random.default_rng(seed)
    p = np.asarray(p, dtype=np.float64)
    std = scatter * p
    p0 = p + std * rng.standard_normal((nwalkers, len(p)))
    for _ in range(max_rounds):
        ok = np.isfinite(ln_prob_fn(p0))
        nbad = int((~ok).sum())
        if nbad == 0:
            return p0
        good = p0[ok]
        if len(good) == 0:
            raise RuntimeError("no valid walker in the initial ball")
        rep = good[rng.integers(len(good), size=nbad)]
        rep = rep + 0.5 * rep * scatter * rng.standard_normal(rep.shape)
        p0[~ok] = rep
    raise RuntimeError("could not initialise walkers")


def write_chain(fname, names, chain, lnprob, mode="w"):
    """chain_prod.txt in the reference's format (mcmcfit.py:317,
    mcmc_utils.py:157-164): header `walker_no <names> ln_prob`, then one row
    per walker per step: '{k:4d} {repr(x) ...} {lnp:f}'."""
    chain = np.asarray(chain)
    lnprob = np.asarray(lnprob)
    with open(fname, mode) as fh:
        if mode == "w":
            fh.write("walker_no " + " ".join(names) + " ln_prob\n")
        for s in range(chain.shape[0]):
            rows = ["{0:4d} {1:s} {2:f}\n".format(k, " ".join(map(repr, map(float, chain[s, k]))),
                                                 float(lnprob[s, k]))
                    for k in range(chain.shape[1])]
            fh.write("".join(rows))


def read_chain(fname):
    """Inverse of write_chain -> chain [nwalkers, nsteps, npars + 1] like
    mcmc_utils.readchain (mcmc_utils.py:252-272); last column is ln_prob."""
    data = np.loadtxt(fname, skiprows=1)
    nw = int(data[:, 0].max()) + 1
    ns = data.shape[0] // nw
    chain = np.full((nw, ns, data.shape[1] - 1), np.nan)
    for i in range(nw):
        chain[i] = data[data[:, 0] == i, 1:]
    return chain
