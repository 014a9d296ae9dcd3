"""Hierarchical parameter tree: Prior, Param and Node.

Behavioural mirror of the reference's model.py (Prior model.py:40-113, Param
model.py:116-141, Node model.py:144-844) for the parts the ln_prob hot path
touches: parameter routing between the flat emcee vector and the tree,
prior evaluation with the reference's quirks, and the recursive
ln_prior / ln_like / ln_prob sums.  Plotting, networkx diagrams and the
per-PID debug log are not part of the hot path and are left out.

The recursive evaluation here is the scalar, one-walker-at-a-time API.  The
production path compiles the tree once (lfit_python_amd.batch) and evaluates
whole walker ensembles on the GPU.
"""
import math
import warnings

import numpy as np

TINY = -np.inf
PRIOR_TYPES = ('gauss', 'gaussPos', 'uniform', 'log_uniform', 'mod_jeff')


def extract_par_and_key(key):
    """'wdFlux_long_label' -> ('wdFlux', 'long_label'); 'ln_tau_gp_core' ->
    ('ln_tau_gp', 'core') (model.py:22-37)."""
    if key.startswith("ln_"):
        parts = key.split("_")
        return "_".join(parts[:3]), "_".join(parts[3:])
    head, _, tail = key.partition("_")
    return head, tail


def _gauss_lnpdf(val, mean, sd):
    # log(scipy.stats.norm(loc, scale).pdf(val)); underflow -> -inf (model.py:85-89)
    z = (val - mean) / sd
    pdf = math.exp(-z * z / 2.0) / math.sqrt(2.0 * math.pi) / sd
    return math.log(pdf) if pdf > 0 else TINY


class Prior:
    """Prior('gauss'|'gaussPos'|'uniform'|'log_uniform'|'mod_jeff', p1, p2)."""

    def __init__(self, type, p1, p2):
        if type not in PRIOR_TYPES:
            raise AssertionError("unknown prior type %r" % type)
        self.type = type
        self.p1 = float(p1)
        self.p2 = float(p2)
        self.normalise = 1.0
        if type == 'log_uniform':
            if self.p1 < 1.0e-30:
                warnings.warn('lower limit on log_uniform prior rescaled from %f to 1.0e-30' % self.p1)
                self.p1 = 1.0e-30
            # model.py:77-79 integrates the *log*-density ln(1/v) over [p1, p2];
            # closed form of that integral: [v - v ln v] from p1 to p2.
            a, b = self.p1, self.p2
            self.normalise = abs((b - b * math.log(b)) - (a - a * math.log(a)))
        elif type == 'mod_jeff':
            self.normalise = math.log((self.p1 + self.p2) / self.p1)

    @property
    def code(self):
        return PRIOR_TYPES.index(self.type)

    def ln_prob(self, val):
        t, p1, p2 = self.type, self.p1, self.p2
        if t == 'gauss':
            return _gauss_lnpdf(val, p1, p2)
        if t == 'gaussPos':
            return TINY if val <= 0.0 else _gauss_lnpdf(val, p1, p2)
        if t == 'uniform':
            return math.log(1.0 / abs(p1 - p2)) if p1 < val < p2 else TINY
        if t == 'log_uniform':
            return math.log(1.0 / self.normalise / val) if p1 < val < p2 else TINY
        # mod_jeff
        return math.log(1.0 / self.normalise / (val + p1)) if 0 < val < p2 else TINY


class Param:
    """A named value with a prior and an isVar flag (model.py:116-141)."""

    def __init__(self, name, startVal, prior, isVar=True):
        self.name = name
        self.startVal = startVal
        self.currVal = startVal
        self.prior = prior
        self.isVar = isVar

    @classmethod
    def fromString(cls, name, parString):
        """'value prior p1 p2 [isVar]' (model.py:126-137)."""
        f = parString.split()
        isVar = bool(int(f[4])) if len(f) == 5 else True
        return cls(name, float(f[0]), Prior(f[1].strip(), float(f[2]), float(f[3])), isVar)

    @property
    def isValid(self):
        return bool(np.isfinite(self.prior.ln_prob(self.currVal)))

    def __repr__(self):
        return "Param(%s=%r, %s, isVar=%s)" % (self.name, self.currVal, self.prior.type, self.isVar)


class Node:
    """Tree node holding Params; leaves evaluate the model (model.py:144-844)."""

    node_par_names = ()

    def __init__(self, label, parameter_objects, parent=None, children=None, DEBUG=None):
        if not isinstance(label, str):
            raise TypeError("Label must be a string, not {}".format(type(label)))
        params = list(parameter_objects)
        if len(params) != len(self.node_par_names):
            raise TypeError('I recieved the wrong number of parameters! Expect: \n{}\nGot:\n{}'.format(
                self.node_par_names, [p.name for p in params]))
        self.label = label
        self._children = []
        self._parent = None
        for par in params:
            setattr(self, par.name, par)
        self.DEBUG = bool(DEBUG) if DEBUG is not None else (parent.DEBUG if parent is not None else False)
        if children:
            self.children = children
        self.parent = parent

    # -- family ---------------------------------------------------------
    @property
    def name(self):
        return "{}_{}".format(type(self).__name__, self.label)

    @property
    def parent(self):
        return self._parent

    @parent.setter
    def parent(self, parent):
        self._parent = parent
        if parent is not None:
            parent.add_child(self)

    @property
    def children(self):
        return self._children

    @children.setter
    def children(self, children):
        self._children = list(children)
        for child in self._children:
            child._parent = self

    def add_child(self, children):
        if not isinstance(children, list):
            children = [children]
        self._children.extend(children)

    @property
    def is_root(self):
        return self._parent is None

    @property
    def is_leaf(self):
        return len(self._children) == 0

    # -- searching ------------------------------------------------------
    def walk(self):
        """Pre-order traversal (the order of the emcee vector)."""
        yield self
        for child in self._children:
            yield from child.walk()

    def search_par(self, label, name):
        for node in self.walk():
            if node.label == label:
                return getattr(node, name)
        return None

    def search_Node(self, class_type, label):
        target = "{}_{}".format(class_type, label)
        for node in self.walk():
            if node.name == target:
                return node
        return None

    def search_node_type(self, class_type, nodes=None):
        found = set() if nodes is None else set(nodes)
        found.update(n for n in self.walk() if class_type in type(n).__name__)
        return found

    def leaves(self):
        return [n for n in self.walk() if n.is_leaf]

    def __getitem__(self, index):
        name, label = extract_par_and_key(index)
        return self.search_par(label, name)

    def __setitem__(self, index, value):
        name, label = extract_par_and_key(index)
        self.search_par(label, name).currVal = value

    # -- parameter routing ------------------------------------------------
    @property
    def node_params(self):
        return [getattr(self, n) for n in self.node_par_names]

    @property
    def node_varpars(self):
        return [p.name for p in self.node_params if p.isVar]

    def descendant_params(self):
        """(Param, owning label) pairs at or below this node, pre-order."""
        out = []
        for node in self.walk():
            out.extend((p, node.label) for p in node.node_params)
        return out

    @property
    def dynasty_par_names(self):
        return ["{}_{}".format(p.name, lab) for p, lab in self.descendant_params() if p.isVar]

    @property
    def dynasty_par_vals(self):
        return [p.currVal for p, _ in self.descendant_params() if p.isVar]

    @dynasty_par_vals.setter
    def dynasty_par_vals(self, values):
        var = [p for p, _ in self.descendant_params() if p.isVar]
        values = list(values)
        if len(values) != len(var):
            raise ValueError('Wrong vector length on {} - Expected {}, got {}'.format(
                self.name, len(var), len(values)))
        for p, v in zip(var, values):
            p.currVal = v

    @property
    def dynasty_par_dict(self):
        return dict(zip(self.dynasty_par_names, self.dynasty_par_vals))

    @dynasty_par_dict.setter
    def dynasty_par_dict(self, par_dict):
        for key, value in par_dict.items():
            par = self[key]
            if par is not None:
                par.currVal = value

    def ancestors(self):
        node = self
        while node is not None:
            yield node
            node = node._parent

    @property
    def ancestor_par_names(self):
        return [n for node in self.ancestors() for n in node.node_par_names]

    @property
    def ancestor_param_dict(self):
        """Params at and above this node (model.py:706-712).  As in the
        reference's dict(zip(...)), a name repeated higher up the tree
        overrides the nearer one."""
        d = {}
        for node in self.ancestors():
            for name in node.node_par_names:
                d[name] = getattr(node, name)
        return d

    # -- evaluation -------------------------------------------------------
    def _sum_children(self, fname, *args, **kwargs):
        if self.is_leaf:
            raise NotImplementedError('must overwrite {} on leaf nodes of model'.format(fname))
        total = 0.0
        for child in self._children:
            total += getattr(child, fname)(*args, **kwargs)
            if np.isinf(total):
                return total
        return total

    def chisq(self, *args, **kwargs):
        return self._sum_children('chisq', *args, **kwargs)

    def ln_like(self, *args, **kwargs):
        return self._sum_children('ln_like', *args, **kwargs)

    def ln_prior(self, verbose=False):
        lnp = 0.0
        for par in self.node_params:
            if not par.isValid:
                if verbose:
                    print("Param {} in {} is invalid!".format(par.name, self.name))
                return TINY
            if par.isVar:
                lnp += par.prior.ln_prob(par.currVal)
        for child in self._children:
            lnp += child.ln_prior(verbose=verbose)
            if np.isinf(lnp):
                return lnp
        return lnp

    def ln_prob(self, verbose=False):
        lnp = self.ln_prior(verbose=verbose)
        if not np.isfinite(lnp):
            return lnp
        try:
            return lnp + self.ln_like()
        except Exception:
            if verbose:
                print("Failed to evaluate ln_like at {}".format(self.name))
            return TINY

    def log(self, *args, **kwargs):
        """The reference's per-PID debug log (model.py:763-793) is not kept."""
        return None
