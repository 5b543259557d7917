"""CPU restatement (numpy, fp32 state) of the reference optimizer step semantics.

TEST INFRASTRUCTURE ONLY -- the checker, never the thing measured or shipped.

* ``torch.optim.RAdam`` as built by the reference: ``Autoencoder.configure_optimizers``
  (model/autencoder_lightning_base.py:122-124: one group, betas (0.9, 0.999), wd 0) and
  ``MyTransformerDecoder.configure_optimizers`` (model/transformer_decoder.py:64-114: Linear weights wd 0.1,
  everything else wd 0, betas (0.9, 0.95)); L2 weight decay (added to the gradient), eps 1e-8.
* Lightning ``gradient_clip_val`` = ``clip_grad_norm_`` with the L2 norm over all gradients
  (train_reconstruction_embedding.py:196 clip 0.7; train_transformer_mtasks.py:30 clip 0.8).

Pinned by ``tests/golden/radam.npz`` (torch's own RAdam/clip run in the fixture generator).
"""
from __future__ import annotations

import math

import numpy as np


class RAdamState:
    def __init__(self, shapes):
        self.step = 0
        self.m = [np.zeros(s, np.float32) for s in shapes]
        self.v = [np.zeros(s, np.float32) for s in shapes]


def radam_step(params, grads, state: RAdamState, lr, betas, eps, wds):
    """In-place update of ``params`` (list of fp32 arrays)."""
    b1, b2 = betas
    state.step += 1
    t = state.step
    bc1 = 1 - b1 ** t
    bc2 = 1 - b2 ** t
    rho_inf = 2 / (1 - b2) - 1
    rho_t = rho_inf - 2 * t * (b2 ** t) / bc2
    for p, g, m, v, wd in zip(params, grads, state.m, state.v, wds):
        g = g.astype(np.float32)
        if wd != 0:
            g = (g + np.float32(wd) * p).astype(np.float32)
        m += np.float32(1 - b1) * (g - m)
        v *= np.float32(b2)
        v += np.float32(1 - b2) * g * g
        mhat = m / np.float32(bc1)
        if rho_t > 5.0:
            rect = math.sqrt((rho_t - 4) * (rho_t - 2) * rho_inf / ((rho_inf - 4) * (rho_inf - 2) * rho_t))
            adaptive = np.float32(math.sqrt(bc2)) / (np.sqrt(v) + np.float32(eps))
            p -= mhat * np.float32(lr) * adaptive * np.float32(rect)
        else:
            p -= mhat * np.float32(lr)


def clip_grad_norm(grads, max_norm):
    """Returns the pre-clip total norm and scales grads in place (clip_coef clamped to 1)."""
    norms = np.array([np.linalg.norm(g.astype(np.float32).ravel()) for g in grads], np.float32)
    total = np.float32(np.linalg.norm(norms))
    coef = min(np.float32(max_norm) / (total + np.float32(1e-6)), np.float32(1.0))
    for g in grads:
        g *= np.float32(coef)
    return total
