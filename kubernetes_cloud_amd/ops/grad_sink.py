"""Per-parameter gradient sinks: ops that compute weight gradients themselves
(ops/fused_block.py) hand them to the owner of the parameter's gradient
storage -- the training engine's fp32 accumulation buffer -- instead of
materialising ``param.grad`` through autograd. Keyed by ``id(param)`` with a
weak reference guarding against id reuse, so parameters carry no attribute
(deepcopy / pickling of models stay unaffected)."""
from __future__ import annotations

import weakref

_SINKS: dict = {}


def register(param, fn) -> None:
    _SINKS[id(param)] = (weakref.ref(param), fn)


def unregister(param) -> None:
    ent = _SINKS.get(id(param))
    if ent is not None and ent[0]() is param:
        del _SINKS[id(param)]


def lookup(param):
    ent = _SINKS.get(id(param))
    if ent is None or ent[0]() is not param:
        return None
    return ent[1]
