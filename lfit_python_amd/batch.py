"""Compile a model tree once; evaluate ln_prob for whole walker ensembles on
the GPU in one batched launch sequence.

compile_tree() flattens the tree's routing (Node.__set_parameter_vector__
model.py:586-603 and ancestor_param_dict model.py:706-712) into an index map
gather[E, 18]: CV parameter k of eclipse e (lfit order, CVModel.py:384-388)
is walker[:, gather[e, k]] or, for isVar = 0 parameters, a constant.  The
prior of every variable parameter becomes a row of a small table.  The
result is plain numpy (no GPU needed to build or inspect it).

LnProbEvaluator uploads that description once and then maps a device tensor
walkers[W, ndim] to lnp[W] with lfg_lnprob (include/lfg.h): the batched
replacement of mcmcfit.ln_prob (mcmcfit.py:37-41) for every walker at once.
"""
import ctypes
from dataclasses import dataclass, field

import numpy as np

from . import _native
from .cvmodel import LCModel, SimpleEclipse, SimpleGPEclipse


@dataclass
class CompiledTree:
    E: int
    ndim: int
    names: list
    gather: np.ndarray      # [E, 18] int32
    npars: np.ndarray       # [E] int32
    consts: np.ndarray      # [nconst] f64
    offsets: np.ndarray     # [E + 1] int32
    x: np.ndarray
    y: np.ndarray
    ye: np.ndarray
    w: np.ndarray
    prior_type: np.ndarray  # [ndim] int32
    prior_p1: np.ndarray
    prior_p2: np.ndarray
    prior_norm: np.ndarray
    nsub: int = 1
    roche_priors: bool = True
    fixed_invalid: bool = False
    leaf_labels: list = field(default_factory=list)
    # GP likelihood (GPLCModel trees, CVModel.py:494-711)
    gp: bool = False
    gp_gather: np.ndarray = None   # [E, 3] int32: ln_ampin_gp, ln_ampout_gp, ln_tau_gp
    gp_base: np.ndarray = None     # [E, 4] f64: q, dphi, rwd of the changepoint cache; dist_cp (device-filled)
    gp_ecl: np.ndarray = None      # [E, 2] int32: first, last eclipse number of the changepoint list
    order: list = field(default_factory=list)  # per eclipse: data order used (GP trees sort by phase)

    @property
    def max_n(self):
        return int(np.max(np.diff(self.offsets))) if self.E else 0


def compile_tree(model, nsub=1):
    """Flatten `model` (an LCModel tree or a lone eclipse subtree)."""
    params = [p for p, _ in model.descendant_params()]
    var = [p for p in params if p.isVar]
    index = {id(p): i for i, p in enumerate(var)}
    leaves = [n for n in model.walk() if isinstance(n, SimpleEclipse)]
    if not leaves:
        raise ValueError("the tree has no eclipse leaves")
    gp = [isinstance(n, SimpleGPEclipse) for n in leaves]
    if any(gp) and not all(gp):
        raise ValueError("a tree mixes GP and chi^2 eclipses")
    gp = all(gp)
    consts, gather, npars = [], np.zeros((len(leaves), 18), np.int32), []
    gp_gather = np.zeros((len(leaves), 3), np.int32)
    gp_base = np.zeros((len(leaves), 4))
    gp_ecl = np.zeros((len(leaves), 2), np.int32)
    orders = []

    def slot(p):
        if p.isVar:
            return index[id(p)]
        consts.append(float(p.currVal))
        return -len(consts)

    xs, ys, yes, ws, offs = [], [], [], [], [0]
    for e, leaf in enumerate(leaves):
        d = leaf.ancestor_param_dict
        names = leaf.cv_parnames
        npars.append(len(names))
        for k, nm in enumerate(names):
            gather[e, k] = slot(d[nm])
        for k in range(len(names), 18):
            gather[e, k] = gather[e, 0]
        order = np.arange(leaf.lc.n_data)
        if gp:
            # the Kalman filter runs over phase-sorted points; the likelihood
            # does not depend on the order
            order = np.argsort(leaf.lc.x, kind="stable")
            for k, nm in enumerate(('ln_ampin_gp', 'ln_ampout_gp', 'ln_tau_gp')):
                gp_gather[e, k] = slot(d[nm])
            # the changepoint cache: what the leaf holds, else the current values
            # (the reference fills it at the first ln_like, mcmcfit.py:154)
            cached = leaf._oldq < 9e99
            gp_base[e, :3] = ((leaf._oldq, leaf._olddphi, leaf._oldrwd) if cached else
                              (d['q'].currVal, d['dphi'].currVal, d['rwd'].currVal))
            gp_base[e, 3] = leaf._dist_cp if cached else np.nan
            x = leaf.lc.x
            ecl = [k for k in range(int(np.floor(x.min())), int(np.ceil(x.max())) + 1)
                   if x.min() < k < 1 + x.max()] if len(x) else []
            gp_ecl[e] = (ecl[0], ecl[-1]) if ecl else (1, 0)
        orders.append(order)
        xs.append(leaf.lc.x[order]); ys.append(leaf.lc.y[order]); yes.append(leaf.lc.ye[order])
        ws.append(leaf.lc.w[order])
        offs.append(offs[-1] + leaf.lc.n_data)
    fixed_invalid = any((not p.isVar) and (not p.isValid) for p in params)
    cat = lambda a: np.ascontiguousarray(np.concatenate(a).astype(np.float64)) if a else np.zeros(0)
    return CompiledTree(
        E=len(leaves), ndim=len(var), names=model.dynasty_par_names,
        gather=gather, npars=np.asarray(npars, np.int32),
        consts=np.asarray(consts, np.float64), offsets=np.asarray(offs, np.int32),
        x=cat(xs), y=cat(ys), ye=cat(yes), w=cat(ws),
        prior_type=np.asarray([p.prior.code for p in var], np.int32),
        prior_p1=np.asarray([p.prior.p1 for p in var], np.float64),
        prior_p2=np.asarray([p.prior.p2 for p in var], np.float64),
        prior_norm=np.asarray([p.prior.normalise for p in var], np.float64),
        nsub=int(nsub), roche_priors=isinstance(model, LCModel),
        fixed_invalid=fixed_invalid, leaf_labels=[l.label for l in leaves],
        gp=gp, gp_gather=gp_gather, gp_base=gp_base, gp_ecl=gp_ecl, order=orders)


def prior_consts(tree):
    """[ndim, 2] constants of Prior.ln_prob (model.py:83-113; include/lfg.h
    lfg_tree.prior_c), so the device's prior lanes take one log per chunk of
    parameters instead of one per parameter."""
    t, p1, p2, nm = tree.prior_type, tree.prior_p1, tree.prior_p2, tree.prior_norm
    c = np.zeros((len(t), 2), np.float64)
    with np.errstate(divide="ignore", invalid="ignore"):
        gs = t <= 1
        c[gs, 0] = -np.log(np.sqrt(2.0 * np.pi) * p2[gs])
        c[gs, 1] = 1.0 / p2[gs]
        un = t == 2
        c[un, 0] = np.log(1.0 / np.abs(p1[un] - p2[un]))
        lg = t >= 3
        c[lg, 0] = -np.log(nm[lg])
    return c


class LnProbEvaluator:
    """Device-resident ln_prob for a compiled tree (one per GPU / stream)."""

    def __init__(self, tree, device=None, max_walkers=0):
        import torch
        _native.require_gpu()
        self.L = _native.lib()
        self.tree = tree
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        t = lambda a, dt: torch.as_tensor(np.ascontiguousarray(a), dtype=dt, device=self.device)
        f64, i32 = torch.float64, torch.int32
        self._buf = dict(
            gather=t(tree.gather.reshape(-1), i32), npars=t(tree.npars, i32),
            consts=t(tree.consts if len(tree.consts) else np.zeros(1), f64),
            off=t(tree.offsets, i32), x=t(tree.x, f64), y=t(tree.y, f64),
            ye=t(tree.ye, f64), w=t(tree.w, f64),
            prior_type=t(tree.prior_type, i32), prior_p1=t(tree.prior_p1, f64),
            prior_p2=t(tree.prior_p2, f64), prior_norm=t(tree.prior_norm, f64),
            prior_c=t(prior_consts(tree).reshape(-1), f64))
        if tree.gp:
            self._buf.update(gp_gather=t(tree.gp_gather.reshape(-1), i32),
                             gp_base=t(self._gp_base(tree), f64),
                             gp_ecl=t(tree.gp_ecl.reshape(-1), i32))
        b = self._buf
        p = lambda k: ctypes.c_void_p(b[k].data_ptr()) if k in b else None
        self.ctree = _native.LfgTree(
            tree.E, tree.ndim, tree.nsub, tree.max_n, p('gather'), p('npars'), p('consts'),
            p('off'), p('x'), p('y'), p('ye'), p('w'), p('prior_type'), p('prior_p1'),
            p('prior_p2'), p('prior_norm'), int(tree.roche_priors), int(tree.gp),
            p('gp_gather'), p('gp_base'), p('gp_ecl'), int(tree.fixed_invalid), p('prior_c'))
        self._ws = None
        self._ws_walkers = 0
        self._spec_key = None  # step_half(spec=True): what the workspace's candidates are for
        # bumped whenever the workspace is reallocated: a captured HIP graph
        # holds the old pointer (sampler.EnsembleSampler re-captures on change)
        self.generation = 0
        if max_walkers:
            self._ensure(max_walkers)

    def _gp_base(self, tree):
        """[E, 4] q, dphi, rwd, dist_cp of the changepoint cache; a cache the
        host never filled gets its dist_cp from the device (findi + wdphases,
        CVModel.py:561-570)."""
        from . import roche
        base = np.array(tree.gp_base, dtype=np.float64)
        todo = ~np.isfinite(base[:, 3])
        if todo.any():
            q, dphi, rwd = base[todo, 0], base[todo, 1], base[todo, 2]
            inc = roche.findi(q, dphi)
            p3, p4 = roche.wdphases(q, inc, rwd, 10)
            base[todo, 3] = (dphi + (p4 - p3)) / 2.0
        return base.reshape(-1)

    def _ensure(self, W):
        import torch
        if W > self._ws_walkers:
            nbytes = self.L.lfg_workspace_size_tree(W, ctypes.byref(self.ctree))
            self._ws = torch.empty(nbytes, dtype=torch.uint8, device=self.device)
            self._ws_walkers = W
            self.generation += 1

    def __call__(self, walkers, out=None, lnlike_e=None):
        """walkers: float64 device tensor [W, ndim] -> lnp [W] (same stream)."""
        import torch
        if walkers.dtype != torch.float64 or walkers.device != self.device or not walkers.is_contiguous():
            walkers = walkers.to(device=self.device, dtype=torch.float64).contiguous()
        W, nd = walkers.shape
        if nd != self.tree.ndim:
            raise ValueError("walker vectors have %d entries, the tree has %d" % (nd, self.tree.ndim))
        self._ensure(W)
        self._spec_key = None  # lfg_lnprob's workspace layout overlaps the candidates
        if out is None:
            out = torch.empty(W, dtype=torch.float64, device=self.device)
        rc = self.L.lfg_lnprob(ctypes.c_void_p(walkers.data_ptr()), W, ctypes.byref(self.ctree),
                               ctypes.c_void_p(out.data_ptr()),
                               ctypes.c_void_p(lnlike_e.data_ptr()) if lnlike_e is not None else None,
                               ctypes.c_void_p(self._ws.data_ptr()), self._ws.numel(),
                               _native.stream_ptr(self.device))
        _native.check(rc, "lfg_lnprob")  # fixed_invalid trees: -inf from k_setup's prior lanes
        return out


    def lnprob_accept(self, q, pos, lnp, half, zfac, seed, step, naccept, lnp_new=None, events=None):
        """ln_prob of the proposals q [W/2, ndim] with the stretch move's
        Metropolis step fused in (lfg_stretch_lnprob_accept): updates pos,
        lnp and naccept of half `half` in place."""
        W = pos.shape[0]
        self._ensure(W // 2)
        self._spec_key = None
        vp = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None
        rc = self.L.lfg_stretch_lnprob_accept(vp(pos), vp(lnp), W, half, vp(q), vp(zfac), ctypes.byref(self.ctree),
                                              seed, step, vp(naccept), vp(lnp_new), vp(self._ws), self._ws.numel(),
                                              _native.stream_ptr(self.device), events)
        _native.check(rc, "lfg_stretch_lnprob_accept")

    def step_half(self, pos, lnp, half, a, seed, step, q, zfac, naccept, lnp_new=None, events=None, spec=False):
        """A whole stretch-move half-step (lfg_stretch_step_half): propose half
        `half` into q / zfac, evaluate, accept; pos, lnp, naccept in place.
        spec=True (lfg_stretch_step_half_spec): this call also forms the next
        half's setup for both fates of each partner, and skips its own k_setup
        when the previous call on this evaluator left exactly this half's
        candidates (same ensemble tensors, seed, a, the preceding half, and no
        other entry point since; the caller clears it with invalidate_spec()
        when it changes pos / lnp itself)."""
        W = pos.shape[0]
        gen = self.generation
        self._ensure(W // 2)
        vp = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None
        if not spec:
            self._spec_key = None
            rc = self.L.lfg_stretch_step_half(vp(pos), vp(lnp), W, half, a, seed, step, vp(q), vp(zfac),
                                              ctypes.byref(self.ctree), vp(naccept), vp(lnp_new), vp(self._ws),
                                              self._ws.numel(), _native.stream_ptr(self.device), events)
            _native.check(rc, "lfg_stretch_step_half")
            return
        # the key includes torch's in-place version counters of pos and lnp: a
        # write to S.pos / S.lnp between steps (same pointers) bumps them and
        # drops the candidates (the kernels' own writes go through raw
        # pointers and leave the counters alone)
        ens = (W, pos.data_ptr(), lnp.data_ptr(), q.data_ptr(), zfac.data_ptr(), seed, float(a),
               pos._version, lnp._version)
        spec_in = gen == self.generation and self._spec_key == ens + (half, step)
        self._spec_key = None
        rc = self.L.lfg_stretch_step_half_spec(vp(pos), vp(lnp), W, half, a, seed, step, vp(q), vp(zfac),
                                               ctypes.byref(self.ctree), vp(naccept), vp(lnp_new),
                                               int(spec_in), 1, vp(self._ws), self._ws.numel(),
                                               _native.stream_ptr(self.device), events)
        _native.check(rc, "lfg_stretch_step_half_spec")
        self._spec_key = ens + (1 - half, step + half)

    def invalidate_spec(self):
        """Forget the speculative candidates (the ensemble was changed outside
        step_half)."""
        self._spec_key = None

    def step_shard(self, pos, half, a, seed, step, lo, q, zfac, lnp_new, events=None, spec=False, fold=None):
        """This rank's part of a sharded half-step (lfg_stretch_step_shard):
        the proposals of walkers lo .. lo + n - 1 of half `half` (n =
        lnp_new.numel()) into q / zfac and their ln_prob into lnp_new.
        spec=True (lfg_stretch_step_shard_spec): speculative setup as in
        step_half; pair it with accept_regen() on this evaluator.
        fold=(lnp, verdict_prev, verdict, naccept): the deferred acceptance
        instead (step_shard_fold)."""
        if fold is not None:
            lnp, vprev, verdict, naccept = fold
            return self.step_shard_fold(pos, lnp, half, a, seed, step, lo, q, zfac, lnp_new, vprev, verdict, naccept,
                                        events=events)
        W, n = pos.shape[0], lnp_new.shape[0]
        vp = lambda t: ctypes.c_void_p(t.data_ptr())
        if not spec:
            self._ensure(n)
            self._spec_key = None
            rc = self.L.lfg_stretch_step_shard(vp(pos), W, half, a, seed, step, lo, n, vp(q), vp(zfac),
                                               ctypes.byref(self.ctree), vp(lnp_new), vp(self._ws), self._ws.numel(),
                                               _native.stream_ptr(self.device), events)
            _native.check(rc, "lfg_stretch_step_shard")
            return
        gen = self.generation
        self._ensure(W // 2)  # the acceptances of the whole half live here
        ens = ("shard", W, pos.data_ptr(), q.data_ptr(), zfac.data_ptr(), seed, float(a), lo, n,
               pos._version)  # as in step_half: an in-place write to pos drops the candidates
        spec_in = gen == self.generation and self._spec_key == ens + (half, step, "accepted")
        self._spec_key = None
        rc = self.L.lfg_stretch_step_shard_spec(vp(pos), W, half, a, seed, step, lo, n, vp(q), vp(zfac),
                                                ctypes.byref(self.ctree), vp(lnp_new), int(spec_in), 1, vp(self._ws),
                                                self._ws.numel(), _native.stream_ptr(self.device), events)
        _native.check(rc, "lfg_stretch_step_shard_spec")
        self._spec_key = ens + (half, step, "pending")

    def step_shard_fold(self, pos, lnp, half, a, seed, step, lo, q, zfac, lnp_new, verdict_prev, verdict, naccept,
                        events=None):
        """This rank's part of a sharded half-step with the acceptance
        deferred (lfg_stretch_step_shard_fold): applies verdict_prev (the
        other half's gathered verdicts of the half-step before, or None),
        evaluates walkers lo .. lo + n - 1 of half `half` into q / zfac /
        lnp_new and leaves their verdicts (ln_prob where accepted, NaN) in
        verdict [n] for the exchange.  The speculative candidates are used
        when the previous call on this evaluator was the preceding fold
        half-step of the same ensemble."""
        W, n = pos.shape[0], lnp_new.shape[0]
        gen = self.generation
        self._ensure(W // 2)
        vp = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None
        ens = ("fold", W, pos.data_ptr(), lnp.data_ptr(), q.data_ptr(), zfac.data_ptr(), seed, float(a), lo, n,
               pos._version, lnp._version)
        spec_in = verdict_prev is not None and gen == self.generation and self._spec_key == ens + (half, step)
        self._spec_key = None
        rc = self.L.lfg_stretch_step_shard_fold(vp(pos), vp(lnp), W, half, a, seed, step, lo, n, vp(q), vp(zfac),
                                                ctypes.byref(self.ctree), vp(verdict_prev), vp(verdict), vp(lnp_new),
                                                vp(naccept), int(spec_in), 1, vp(self._ws), self._ws.numel(),
                                                _native.stream_ptr(self.device), events)
        _native.check(rc, "lfg_stretch_step_shard_fold")
        self._spec_key = ens + (1 - half, step + half)

    def apply_verdicts(self, pos, lnp, half, a, seed, step, verdict, naccept):
        """Apply half `half`'s pending verdicts (the proposals of `step`) to
        the ensemble (lfg_stretch_apply_verdicts): the flush of the deferred
        acceptance.  The next fold half-step starts without candidates."""
        W, ndim = pos.shape
        self._spec_key = None
        vp = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None
        rc = self.L.lfg_stretch_apply_verdicts(vp(pos), vp(lnp), W, ndim, half, a, seed, step, vp(verdict),
                                               vp(naccept), _native.stream_ptr(self.device))
        _native.check(rc, "lfg_stretch_apply_verdicts")

    def accept_regen(self, pos, lnp, half, a, seed, step, lnp_new, naccept, n):
        """Metropolis step of the whole half after the gather
        (lfg_stretch_accept_regen_spec), recording the acceptances for the
        next step_shard(spec=True) of this rank (shard size n)."""
        W = pos.shape[0]
        self._ensure(W // 2)
        key, self._spec_key = self._spec_key, None
        vp = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None
        rc = self.L.lfg_stretch_accept_regen_spec(vp(pos), vp(lnp), W, half, a, seed, step, vp(lnp_new),
                                                  vp(naccept), ctypes.byref(self.ctree), n, vp(self._ws),
                                                  self._ws.numel(), _native.stream_ptr(self.device))
        _native.check(rc, "lfg_stretch_accept_regen_spec")
        if (key is not None and key[-3:] == (half, step, "pending") and key[2] == pos.data_ptr() and key[8] == n
                and key[9] == pos._version):
            self._spec_key = key[:-3] + (1 - half, step + half, "accepted")

    def ln_prior(self, walkers, out=None):
        """ln_prior alone (mcmcfit.ln_prior, mcmcfit.py:30-34) of walkers [W, ndim]."""
        import torch
        if walkers.dtype != torch.float64 or walkers.device != self.device or not walkers.is_contiguous():
            walkers = walkers.to(device=self.device, dtype=torch.float64).contiguous()
        W = walkers.shape[0]
        self._ensure(W)
        self._spec_key = None
        if out is None:
            out = torch.empty(W, dtype=torch.float64, device=self.device)
        rc = self.L.lfg_lnprior(ctypes.c_void_p(walkers.data_ptr()), W, ctypes.byref(self.ctree),
                                ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(self._ws.data_ptr()),
                                self._ws.numel(), _native.stream_ptr(self.device))
        _native.check(rc, "lfg_lnprior")
        return out


def ln_prob_batch(model, walkers, nsub=1):
    """Convenience: compile `model` and evaluate walkers [W, ndim] (numpy)."""
    import torch
    ev = LnProbEvaluator(compile_tree(model, nsub=nsub))
    return ev(torch.as_tensor(np.asarray(walkers, dtype=np.float64))).cpu().numpy()
