"""Token + positional embeddings -- drop-in for model/embedding.py of the reference (same buffers/parameters)."""
import math

import torch
from torch import nn

from arcweld import modules


class PositionalEmbedding(nn.Module):
    """Fixed sinusoidal table (reference :6-24): buffer 'pe' (1, max_len, d_model) with
    pe[p, 2i] = sin(p * w_i), pe[p, 2i+1] = cos(p * w_i), w_i = exp(2i * -(ln 10000 / d_model)), evaluated in fp32
    exactly as the reference does (same operations, same rounding), so the buffer is bit-identical."""

    def __init__(self, d_model, max_len=5000):
        super().__init__()
        inv_freq = (torch.arange(0, d_model, 2).float() * -(math.log(10000.0) / d_model)).exp()
        angle = torch.arange(max_len, dtype=torch.float32)[:, None] * inv_freq[None, :]
        table = torch.stack((angle.sin(), angle.cos()), dim=-1).reshape(max_len, -1)[:, :d_model]
        self.register_buffer('pe', table.contiguous().unsqueeze(0))

    def forward(self, x):
        return self.pe[:, :x.size(1)]


class LatentEmbeddingCond(nn.Module):
    """Reference :27-43 (unused by the entry points): token + positional + per-window condition embedding."""

    def __init__(self, input_size: int, d_model: int, cond_size: int) -> None:
        super().__init__()
        self.positional_embedding = PositionalEmbedding(d_model=d_model, max_len=input_size)
        self.latent_embedding = nn.Embedding(num_embeddings=input_size, embedding_dim=d_model)
        self.cond_embedding = nn.Embedding(num_embeddings=cond_size, embedding_dim=d_model)

    def forward(self, x, cond):
        """latent_embedding(x) + pe[:T] + cond_embedding(cond) on every position (reference :38-43)."""
        return modules.latent_embedding(self, x, cond.contiguous(), self.cond_embedding.weight)


class LatentEmbedding(nn.Module):
    """latent_embedding(ids) + pe[:T] (reference :45-59); the PE table has seq_len rows (the decoder passes 512,
    reference model/transformer_decoder.py:22-23, unless its pe_len opt-in asks for more)."""

    def __init__(self, input_size: int, d_model: int, seq_len: int = 512) -> None:
        super().__init__()
        self.positional_embedding = PositionalEmbedding(d_model=d_model, max_len=seq_len)
        self.latent_embedding = nn.Embedding(num_embeddings=input_size, embedding_dim=d_model)
        self.input_size = input_size
        self.d_model = d_model
        self.seq_len = seq_len

    def forward(self, x):
        """latent_embedding(x) + pe[:T] (reference :57-59); trainable on its own (scatter-add backward)."""
        return modules.latent_embedding(self, x)
