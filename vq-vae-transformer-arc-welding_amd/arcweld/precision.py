"""Operand precision of the MFMA contractions (every conv / ConvT / Linear of the hot path).

The reference trains in fp32 (Lightning precision 32).  Its scripts call
``torch.set_float32_matmul_precision('medium')`` (train_reconstruction_embedding.py:253,
train_transformer_mtasks.py:245), but that flag does not lower Conv1d / ConvTranspose1d (MIOpen stays fp32) and
gfx950 has no xf32 for the Linears, so on MI355X the reference's numerics are exact fp32 throughout.  The default
here is therefore exact fp32 MFMA operands (``v_mfma_f32_16x16x4_f32``), independent of the torch flag.

bf16 operands with fp32 accumulation (``v_mfma_f32_16x16x32_bf16``; fp32 master weights, fp32 residual streams,
LayerNorm / softmax / losses / VQ distances in fp32) are an explicit opt-in:

* ``set_operand_dtype(torch.bfloat16)`` / ``operands(torch.bfloat16)`` (a context manager), or
* the environment variable ``ARCWELD_OPERANDS=bf16``, or
* the entry scripts' ``--precision bf16`` flag.

BASELINE.json configs[1] quotes the throughput metric in bf16, so bench.py opts in for that line and reports an
fp32 line beside it.  The VQ codebook indices are bit-exact against the reference only in fp32 mode: in bf16 mode
the encoder output z itself comes from bf16 contractions.
"""
from __future__ import annotations

import contextlib
import os

import torch

F32 = torch.float32
BF16 = torch.bfloat16
_NAMES = {"fp32": F32, "f32": F32, "float32": F32, "bf16": BF16, "bfloat16": BF16}
_dtype = None          # None: environment, then fp32


def _parse(v):
    if isinstance(v, torch.dtype):
        if v not in (F32, BF16):
            raise ValueError(f"operand dtype must be float32 or bfloat16, got {v}")
        return v
    key = str(v).lower()
    if key not in _NAMES:
        raise ValueError(f"unknown operand precision {v!r} (fp32 | bf16)")
    return _NAMES[key]


def set_operand_dtype(dt):
    """Process-wide operand dtype: torch.float32 / torch.bfloat16 / "fp32" / "bf16", or None for the default."""
    global _dtype
    _dtype = None if dt is None else _parse(dt)


def get_operand_dtype():
    if _dtype is not None:
        return _dtype
    env = os.environ.get("ARCWELD_OPERANDS")
    return _parse(env) if env else F32


@contextlib.contextmanager
def operands(dt):
    """with operands(torch.bfloat16): ... -- scoped opt-in (restores the previous setting)."""
    global _dtype
    old = _dtype
    set_operand_dtype(dt)
    try:
        yield
    finally:
        _dtype = old


def operand_dtype(override=None):
    """The dtype a forward runs its contraction operands in: an explicit per-call override, else the setting."""
    return _parse(override) if override is not None else get_operand_dtype()
