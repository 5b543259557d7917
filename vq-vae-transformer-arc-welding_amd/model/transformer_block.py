"""minGPT pre-LN block -- drop-in for model/transformer_block.py of the reference (same module tree and keys:
ln_1, attn.{c_attn, c_proj, bias}, ln_2, mlp.{c_fc, c_proj}).  Training runs through the fused decoder path
(arcweld.decoder); a Block used on its own runs the same kernels, with its own autograd node."""
import math

import torch
from torch import nn, Tensor

from arcweld import modules


class NewGELUActivation(nn.Module):
    """tanh-approximate GELU (reference :8-15); computed inside the c_fc GEMM epilogue on the HIP path."""

    def forward(self, input: Tensor) -> Tensor:
        return 0.5 * input * (1.0 + torch.tanh(math.sqrt(2.0 / math.pi) * (input + 0.044715 * torch.pow(input, 3.0))))


class CausalSelfAttention(nn.Module):
    def __init__(self, d_model, seq_len, n_head, attn_pdrop, resid_pdrop):
        super().__init__()
        assert d_model % n_head == 0
        self.c_attn = nn.Linear(d_model, 3 * d_model)
        self.c_proj = nn.Linear(d_model, d_model)
        self.attn_dropout = nn.Dropout(attn_pdrop)
        self.resid_dropout = nn.Dropout(resid_pdrop)
        self.register_buffer("bias", torch.tril(torch.ones(seq_len, seq_len)).view(1, 1, seq_len, seq_len))
        self.n_head = n_head
        self.n_embd = d_model
        # the probability dropout runs inside the flash attention kernels (aw_attn_fwd_dropout): a counter-based
        # mask per (b, h, i, j) the backward regenerates; p > 0 takes the runtime-size VALU kernels
        self.attn_pdrop = float(attn_pdrop)

    def forward(self, x):
        """(B, T, d) -> resid_dropout(c_proj(attention)) (reference :40-63), an autograd node of its own."""
        return modules.causal_self_attention(self, x)


class Block(nn.Module):
    """x + attn(ln_1(x)); x + mlp(ln_2(x)) (reference :66-88)."""

    def __init__(self, d_model, seq_len, n_head, res_dropout, att_dropout):
        super().__init__()
        self.ln_1 = nn.LayerNorm(d_model)
        self.attn = CausalSelfAttention(d_model, seq_len, n_head, att_dropout, res_dropout)
        self.ln_2 = nn.LayerNorm(d_model)
        self.mlp = nn.ModuleDict(dict(
            c_fc=nn.Linear(d_model, 4 * d_model),
            c_proj=nn.Linear(4 * d_model, d_model),
            act=NewGELUActivation(),
            dropout=nn.Dropout(res_dropout),
        ))
        self.res_dropout = res_dropout
        m = self.mlp
        self.mlpf = lambda x: modules.mlp(m, x)   # MLP forward (reference :81-83), an autograd node of its own

    def forward(self, x):
        """(B, T, d) -> (B, T, d); dropout active in training mode.  An autograd node of its own when anything
        requires grad (arcweld.modules.block: the fused decoder's per-block kernels)."""
        return modules.block(self, x)
