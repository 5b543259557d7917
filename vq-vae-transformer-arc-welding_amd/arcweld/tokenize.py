"""GPU-resident latent tokenization for the Transformer stage.

Reference: LatentSpaceDataLoader.get_latent_space_IDs / create_latent_space_dataset_VQ_VAE_IDs
(dataloader/latentspace_dataloader.py:154-161, 205-250) and MyLatentAutoregressiveDataset
(dataloader/base_dataloader.py:74-110).  The reference loops over the n_cycles windows of each sequence, copies
every window's ids to the host and grows a numpy array with np.append; here all windows of a batch go through one
fused encoder + VQ pass (arcweld.vqvae.encode) and the (B, n_cycles*S) id tensor never leaves HBM.
"""
from __future__ import annotations

import numpy as np
import torch

from . import vqvae as engine


@torch.no_grad()
def encode_ids(vqvae, x, window_size=None, dtype=torch.float32):
    """x (B, n_cycles*window_size, C) f32 windows -> ids (B, n_cycles*S) int64.

    Window i of a sequence is x[:, i*window_size:(i+1)*window_size] and its S ids follow those of window i-1,
    exactly the order of the reference's per-window loop + swapaxes + reshape (:233-240, :261).
    """
    L = int(window_size or vqvae.seq_len)
    B, LT, C = x.shape
    if LT % L:
        raise ValueError(f"sequence length {LT} is not a multiple of the window size {L}")
    nc = LT // L
    idx, _ = engine.encode(vqvae, x.reshape(B * nc, L, C), dtype=dtype)
    return idx.view(B, -1)


def autoregressive_pairs(ids, start_token=None):
    """[start, ids] -> [ids, end] (base_dataloader.py:84-97).  start = max id + 1 and end = max id + 2 over the
    whole id set (data-dependent, like the reference) unless ``start_token`` is given.
    Returns (x (B, T+1), y (B, T+1), num_classes)."""
    if start_token is None:
        start_token = int(ids.max().item()) + 1
    B = ids.shape[0]
    col = torch.full((B, 1), start_token, dtype=ids.dtype, device=ids.device)
    x = torch.cat([col, ids], dim=1)
    y = torch.cat([ids, col + 1], dim=1)
    return x, y, start_token + 2


class MyLatentAutoregressiveDataset(torch.utils.data.Dataset):
    """Same items as the reference dataset: (x int64 (T+1,), cond int64 () or zeros((1,)), y int64 (T+1,))."""

    def __init__(self, data, y=None):
        data = (data if isinstance(data, torch.Tensor) else torch.as_tensor(np.asarray(data))).long()
        self.data, self.data_shifted, self.num_classes = autoregressive_pairs(data)
        if y is not None:
            y = (y if isinstance(y, torch.Tensor) else torch.as_tensor(np.asarray(y))).long().to(data.device)
        self.labels = y

    def __len__(self):
        return len(self.data)

    def __getitem__(self, idx):
        cond = self.labels[idx] if self.labels is not None else torch.zeros((1,), dtype=torch.long)
        return self.data[idx], cond, self.data_shifted[idx]
