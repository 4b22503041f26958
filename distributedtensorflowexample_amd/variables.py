"""Variable registry: TF 1.x collections, ``variable_scope`` and ``get_vars``.

The reference finds its variables by collection query rather than by hand-written lists:
``get_vars(scope, trainable)`` (utils.py:3-8) is ``tf.get_collection(TRAINABLE_VARIABLES or
GLOBAL_VARIABLES, scope)``, and it drives the ps variables, the gradient pairing
``zip(get_vars('global'), gvs)`` (worker.py:73-79), the parameter pull (worker.py:81-85), the
init ops (worker.py:98-100) and the saver's var list (worker.py:102-103).  This module keeps
the same contract without a graph: models *declare* their variables (name, shape, dtype,
trainable, initializer) into a registry, under ``variable_scope``s, with ``tf.layers``-style
unique layer names (``dense``, ``dense_1``, ...); consumers query them back in creation
order.  The values live wherever the strategy puts them (ps tasks, GPU store, replicas).

    reg = VariableRegistry()
    with reg.as_default(), variable_scope("global"):
        model.build_variables()          # global/dense/kernel, global/dense/bias, ...
        create_global_step()             # global/global_step (int64, not trainable)
    get_vars("global", False)            # every global variable, creation order
    get_vars("global")                   # the trainable ones

Scope filtering follows ``tf.get_collection``: ``re.match(scope, name)`` (a prefix match for
plain names).
"""
from __future__ import annotations

import contextlib
import dataclasses
import re
from typing import Callable, Optional, Tuple

import torch

GLOBAL_VARIABLES = "variables"
TRAINABLE_VARIABLES = "trainable_variables"


@dataclasses.dataclass(frozen=True)
class Variable:
    name: str                       # full name, e.g. "global/dense/kernel"
    shape: Tuple[int, ...]
    dtype: str                      # "float32" | "int64"
    trainable: bool
    initializer: Optional[Callable] = dataclasses.field(default=None, compare=False,
                                                        repr=False)

    @property
    def spec(self):
        """(name, shape, dtype): the form ``PSVariableStore`` / ``variable_store`` take."""
        return (self.name, self.shape, self.dtype)

    @property
    def local_name(self):
        """Name without its outermost scope ("global/dense/kernel" -> "dense/kernel")."""
        return self.name.split("/", 1)[1] if "/" in self.name else self.name

    def initial_value(self, seed=0, index=0):
        """The initializer's value (CPU tensor); zeros when there is none."""
        if self.initializer is not None:
            return self.initializer(self.shape, seed, index)
        dt = torch.float32 if self.dtype == "float32" else torch.int64
        return torch.zeros(self.shape, dtype=dt)


class VariableRegistry:
    """Collections of declared variables (one per process, or one per ``as_default()``)."""

    def __init__(self):
        self._collections = {GLOBAL_VARIABLES: [], TRAINABLE_VARIABLES: []}
        self._by_name = {}
        self._scopes = []
        self._layer_counts = {}

    # -- declaration ---------------------------------------------------------
    def scope_name(self):
        return "/".join(self._scopes)

    def full_name(self, name):
        s = self.scope_name()
        return "%s/%s" % (s, name) if s else name

    @contextlib.contextmanager
    def variable_scope(self, name):
        self._scopes.append(str(name))
        try:
            yield self.scope_name()
        finally:
            self._scopes.pop()

    def unique_layer_name(self, base):
        """tf.layers naming inside the current scope: base, base_1, base_2, ..."""
        key = (self.scope_name(), base)
        n = self._layer_counts.get(key, 0)
        self._layer_counts[key] = n + 1
        return base if n == 0 else "%s_%d" % (base, n)

    def get_variable(self, name, shape, dtype="float32", trainable=True, initializer=None):
        full = self.full_name(name)
        if full in self._by_name:
            raise ValueError("Variable %s already exists" % full)
        v = Variable(full, tuple(int(d) for d in shape), str(dtype), bool(trainable), initializer)
        self._by_name[full] = v
        self._collections[GLOBAL_VARIABLES].append(v)
        if v.trainable:
            self._collections[TRAINABLE_VARIABLES].append(v)
        return v

    # -- queries -------------------------------------------------------------
    def get_collection(self, key, scope=None):
        items = self._collections.get(key, [])
        if scope is None:
            return list(items)
        pat = re.compile(scope)
        return [v for v in items if pat.match(v.name)]

    def get_vars(self, scope, trainable=True):
        """utils.py:3-8."""
        return self.get_collection(TRAINABLE_VARIABLES if trainable else GLOBAL_VARIABLES, scope)

    def __getitem__(self, name):
        return self._by_name[name]

    @contextlib.contextmanager
    def as_default(self):
        _STACK.append(self)
        try:
            yield self
        finally:
            _STACK.pop()


_STACK = [VariableRegistry()]


def get_default_registry():
    return _STACK[-1]


def reset_default_registry():
    _STACK[0] = VariableRegistry()


def variable_scope(name):
    return get_default_registry().variable_scope(name)


def get_variable(name, shape, dtype="float32", trainable=True, initializer=None):
    return get_default_registry().get_variable(name, shape, dtype, trainable, initializer)


def get_collection(key, scope=None):
    return get_default_registry().get_collection(key, scope)


def get_vars(scope, trainable=True):
    """``tf.get_collection(TRAINABLE_VARIABLES if trainable else GLOBAL_VARIABLES, scope)``
    (utils.py:3-8)."""
    return get_default_registry().get_vars(scope, trainable)


def create_global_step():
    """``tf.Variable(0, trainable=False, name='global_step')`` of worker.py:29-31."""
    return get_variable("global_step", (), "int64", trainable=False)


# -- initializers (deterministic per (seed, variable index): every process agrees) -------
def random_normal_initializer(mean=0.0, stddev=1.0):
    """tf.random_normal_initializer() (worker.py:51,53): N(mean, stddev)."""
    def init(shape, seed, index):
        g = torch.Generator().manual_seed(int(seed) * 1000003 + int(index))
        return torch.randn(shape, generator=g) * stddev + mean
    return init


def glorot_uniform_initializer():
    """tf.glorot_uniform_initializer (tf.layers.dense's default kernel init)."""
    def init(shape, seed, index):
        fan_in, fan_out = (shape[0], shape[-1]) if len(shape) >= 2 else (shape[0], shape[0])
        lim = (6.0 / (fan_in + fan_out)) ** 0.5
        g = torch.Generator().manual_seed(int(seed) * 1000003 + int(index))
        return (torch.rand(shape, generator=g) * 2 - 1) * lim
    return init


def zeros_initializer():
    def init(shape, seed, index):
        return torch.zeros(shape)
    return init
