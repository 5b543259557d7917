"""HBM-resident data plumbing for the two training stages.

The reference feeds host DataLoaders (ASIMoWDataModule for reconstruction, dataloader/asimow_dataloader.py; and
LatentPredDataModule over tokenized sequences, dataloader/latentspace_dataloader.py) and, under DDP, a
DistributedSampler per rank.  Here a whole split is resident in HBM (1024 windows x 200 x 2 f32 = 1.6 MB; a
288 GB device holds the full ASIMoW set many times over) and a batch is an index-gather on the device:

* DeviceBatches -- DataLoader(shuffle, drop_last=False) x DistributedSampler(rank, world) semantics: per-epoch
  permutation seeded by (seed + epoch), padded to a multiple of world, rank r takes positions r, r+world, ...
* synthetic_windows -- N(0, 1) 200x2 windows (the StandardScaler'd ASIMoW distribution); the real
  dataset is not available offline.
* ReconstructionDataModule / LatentPredDataModule -- the datamodule surface the entry scripts use.
"""
from __future__ import annotations

import math

import torch

from . import tokenize


def _rank_world():
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


class DeviceBatches:
    def __init__(self, tensors, batch_size, shuffle=True, seed=0, rank=None, world=None, drop_last=False):
        self.tensors = tensors if isinstance(tensors, (list, tuple)) else (tensors,)
        self.single = not isinstance(tensors, (list, tuple))
        self.n = len(self.tensors[0])
        self.batch_size = int(batch_size)
        self.shuffle = shuffle
        self.seed = seed
        r, w = _rank_world()
        self.rank = r if rank is None else rank
        self.world = w if world is None else world
        self.drop_last = drop_last
        self.epoch = 0

    def set_epoch(self, epoch):
        self.epoch = epoch

    def indices(self):
        """This rank's sample indices for the current epoch (torch DistributedSampler arithmetic)."""
        if self.shuffle:
            g = torch.Generator()
            g.manual_seed(self.seed + self.epoch)
            order = torch.randperm(self.n, generator=g)
        else:
            order = torch.arange(self.n)
        per_rank = math.ceil(self.n / self.world)
        total = per_rank * self.world
        if total > self.n:
            order = torch.cat([order, order[:total - self.n]])
        return order[self.rank:total:self.world]

    def __len__(self):
        per_rank = math.ceil(self.n / self.world)
        return per_rank // self.batch_size if self.drop_last else math.ceil(per_rank / self.batch_size)

    def __iter__(self):
        idx = self.indices().to(self.tensors[0].device)
        for b in range(len(self)):
            sel = idx[b * self.batch_size:(b + 1) * self.batch_size]
            out = tuple(t.index_select(0, sel) for t in self.tensors)
            yield out[0] if self.single else out


def synthetic_windows(n, n_cycles=1, seed=0, device="cuda", window=200, channels=2):
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    return torch.randn(n, window * n_cycles, channels, device=device, generator=g)


def synthetic_labels(n, seed=0, device="cuda"):
    g = torch.Generator(device=device)
    g.manual_seed(seed + 7)
    return torch.randint(0, 2, (n,), device=device, generator=g)


class ReconstructionDataModule:
    """ASIMoWDataModule(task="reconstruction", n_cycles=1) surface over synthetic windows (or given tensors)."""

    def __init__(self, batch_size=1024, n_train=8192, n_val=1024, n_test=1024, seed=0, device="cuda", data=None):
        self.batch_size, self.seed, self.device = batch_size, seed, device
        self.sizes = (n_train, n_val, n_test)
        self.data = data
        self.train_ds = self.val_ds = self.test_ds = None

    def setup(self, stage=None):
        if self.train_ds is not None:
            return
        if self.data is not None:
            self.train_ds, self.val_ds, self.test_ds = self.data
        else:
            self.train_ds, self.val_ds, self.test_ds = (synthetic_windows(n, 1, self.seed + 101 * i, self.device)
                                                        for i, n in enumerate(self.sizes))

    def train_dataloader(self):
        return DeviceBatches(self.train_ds, self.batch_size, shuffle=True, seed=self.seed)

    def val_dataloader(self):
        return DeviceBatches(self.val_ds, self.batch_size, shuffle=False)

    def test_dataloader(self):
        return DeviceBatches(self.test_ds, self.batch_size, shuffle=False, rank=0, world=1)


class LatentPredDataModule:
    """Tokenized sequences for the Transformer (latentspace_dataloader.py:23-135, task "autoregressive_ids" /
    "autoregressive_ids_classification"): every split's windows (n, n_cycles*200, 2) are encoded by the frozen
    VQ-VAE in one fused pass and wrapped in MyLatentAutoregressiveDataset (start/end tokens)."""

    def __init__(self, vqvae, splits, batch_size=16, task="autoregressive_ids", seed=0, encode_dtype=torch.float32,
                 tokenized=None):
        self.vqvae, self.splits, self.batch_size, self.task, self.seed = vqvae, splits, batch_size, task, seed
        self.encode_dtype = encode_dtype
        self.tokenized = tokenized          # optional [(ids, labels)] per split, shared between the two tasks
        self.ds = None

    def tokenize(self):
        if self.tokenized is None:
            self.tokenized = [(tokenize.encode_ids(self.vqvae, x, dtype=self.encode_dtype), y)
                              for x, y in self.splits]
        return self.tokenized

    def setup(self, stage=None):
        if self.ds is not None:
            return
        self.ds = []
        for ids, y in self.tokenize():
            labels = None if self.task == "autoregressive_ids" else y
            self.ds.append(tokenize.MyLatentAutoregressiveDataset(ids, labels))
        self.train_ds, self.val_ds, self.test_ds = self.ds

    def _batches(self, ds, shuffle, **kw):
        cond = ds.labels if ds.labels is not None else torch.zeros(len(ds), 1, dtype=torch.long,
                                                                   device=ds.data.device)
        return DeviceBatches((ds.data, cond, ds.data_shifted), self.batch_size, shuffle=shuffle, seed=self.seed, **kw)

    def train_dataloader(self):
        return self._batches(self.train_ds, True)

    def val_dataloader(self):
        return self._batches(self.val_ds, False)

    def test_dataloader(self):
        return self._batches(self.test_ds, False, rank=0, world=1)
