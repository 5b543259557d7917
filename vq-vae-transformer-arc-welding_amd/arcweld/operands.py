"""Persistent GEMM operand copies of a model's weights (relayout + cast), kept current by the optimizer.

A forward needs each weight in the layout (and dtype) its GEMMs read: the centre tap of an encoder conv as [O][I],
a decoder conv as [O][3I] (forward) and [3O][I] (input gradient), the ConvT as [kO][I], the patch embed zero-padded
(aw_weight_relayout modes 0-5, 7).  An OperandSet allocates those copies once per (model, key) and

* refreshes them with ONE aw_weight_relayout_batch launch when a weight changed outside the optimizer (signature:
  data_ptr and version counter of every source parameter -- load_state_dict, .to(), manual edits), and
* otherwise leaves them alone when the flat RAdam maintains them (arcweld.optim.RAdam.attach_operands): its update
  kernel writes the cast copy of every updated element (aw_radam_step_ops), so a training step has no relayout
  launch at all.

A set that no optimizer maintains is refreshed on every use (the safe default).
"""
from __future__ import annotations

import torch

from . import kernels as K


class OperandJob:
    """One operand copy: `param` (the nn.Parameter whose flat segment feeds it), its relayout source and geometry
    (O, I, k, tap, mode, ldo) and the output tensor.  The source is derived from `param` at every use
    (``derive(param) -> (src, O, I, k, tap, mode)``; default: the parameter itself with the geometry given here), so a
    job built before the optimizer re-stores the parameter (flat buffer, tap-major or centre-tap views) reads the
    storage the parameter has now, never a view of a buffer it no longer uses."""
    __slots__ = ("name", "param", "derive", "O", "I", "k", "tap", "mode", "ldo", "out")

    def __init__(self, name, param, O, I, k, tap, mode, out, ldo=0, derive=None):
        self.name, self.param, self.derive = name, param, derive
        self.O, self.I, self.k, self.tap, self.mode, self.ldo, self.out = O, I, k, tap, mode, ldo, out

    def geometry(self):
        """(src, O, I, k, tap, mode) for the parameter's current storage."""
        if self.derive is not None:
            return self.derive(self.param)
        return (self.param, self.O, self.I, self.k, self.tap, self.mode)

    @property
    def src(self):
        return self.geometry()[0]

    def relayout_job(self):
        """(src, O, I, k, tap, mode, out, ldo) for the layout the source has NOW: a k = 3 conv weight the optimizer
        stores tap-major (arcweld.optim.RAdam.declare_tap_major: (O, 3, I) storage) turns the forward copy [O][3I]
        into a plain cast (mode 5 over O x 3I) and the input-gradient copy [3O][I] into mode 7."""
        s, O, I, k, tap, mode = self.geometry()
        if mode in (1, 2) and k == 3 and s.dim() == 3 and not s.is_contiguous() and s.stride() == (3 * I, 1, I):
            st = s.permute(0, 2, 1)       # the (O, 3, I) storage, contiguous
            if mode == 1:
                return (st, O, 3 * I, 1, 0, 5, self.out, self.ldo)
            return (st, O, I, 3, 0, 7, self.out, self.ldo)
        return (s, O, I, k, tap, mode, self.out, self.ldo)


class OperandSet:
    def __init__(self, jobs):
        self.jobs = list(jobs)
        self.out = {j.name: j.out for j in self.jobs}
        self.maintained = False     # set by the optimizer that writes the copies in its update kernel
        self._sig = None

    def _signature(self):
        return tuple((j.param.data_ptr(), j.param._version) for j in self.jobs)

    def invalidate(self):
        self._sig = None

    def refresh(self, force=False):
        """Relayout every copy unless they are known current (maintained and no outside change since)."""
        sig = self._signature()
        if not force and self.maintained and sig == self._sig:
            return self.out
        K.weight_relayout_batch([j.relayout_job() for j in self.jobs])
        self._sig = sig
        return self.out


def get(model, key, build):
    """The model's OperandSet for `key` (built by `build()` -> list of OperandJob on first use), refreshed."""
    cache = model.__dict__.setdefault("_operand_sets", {})
    st = cache.get(key)
    if st is None:
        st = OperandSet(build())
        cache[key] = st
    st.refresh()
    return st.out


def peek(model, key, build):
    """Like get() but without refreshing (the optimizer attaches to a set before the first forward)."""
    cache = model.__dict__.setdefault("_operand_sets", {})
    st = cache.get(key)
    if st is None:
        st = OperandSet(build())
        cache[key] = st
    return st


def invalidate(model):
    """Mark every operand set of `model` stale (weights changed behind the version counters, e.g. a broadcast into
    the optimizer's flat buffer)."""
    for st in model.__dict__.get("_operand_sets", {}).values():
        st.invalidate()
