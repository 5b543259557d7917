"""Data-parallel plumbing on CPU with world_size 2 over gloo: bucketed SUM all-reduce of the flat
gradient buffer, the 1/(accumulate*world) loss scale (= Lightning DDP gradient mean), parameter broadcast,
DistributedSampler-identical sharding, rank-averaged validation metrics.  The HIP optimizer is replaced by a
flat SGD stand-in here (no GPU); its update rule is irrelevant to what is being checked."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
from torch import nn


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class FlatSGD:
    """Same surface the Trainer drives (flatten / set_active / flat_grad / clip / step / zero_grad)."""

    def __init__(self, params, lr):
        self.params, self.lr = list(params), lr
        self.active = None

    def flatten(self):
        n = sum(p.numel() for p in self.params)
        self.g = torch.zeros(n)
        o = 0
        for p in self.params:
            p.grad = self.g[o:o + p.numel()].view_as(p)
            o += p.numel()

    def set_active(self, ps):
        self.active = ps

    @property
    def flat_grad(self):
        return self.g

    def clip_grad_norm_(self, m):
        return torch.nn.utils.clip_grad_norm_(self.params, m)

    def step(self):
        with torch.no_grad():
            for p in self.params:
                p -= self.lr * p.grad

    def zero_grad(self):
        self.g.zero_()


class TinyModel(nn.Module):
    def __init__(self):
        super().__init__()
        torch.manual_seed(0)
        self.lin = nn.Linear(4, 3)

    def configure_optimizers(self):
        return FlatSGD(self.parameters(), lr=0.1)

    def training_step(self, batch, i):
        x, y = batch
        return ((self.lin(x) - y) ** 2).mean()

    def validation_step(self, batch, i):
        self._logged = {"val/loss": self.training_step(batch, i).detach()}

    @property
    def logged(self):
        return self._logged


def _data(n=24):
    g = torch.Generator().manual_seed(5)
    return torch.randn(n, 4, generator=g), torch.randn(n, 3, generator=g)


def _worker(rank, world, port, out, accumulate):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from arcweld import trainer as T
    from arcweld.data import DeviceBatches
    try:
        # bucketed all-reduce: several buckets, ragged tail
        flat = torch.arange(10, dtype=torch.float32) * (rank + 1)
        T.allreduce_flat(flat, bucket=3)
        assert torch.equal(flat, torch.arange(10, dtype=torch.float32) * 3)
        # region all-reduce as the split step graph issues it: [cut, n) first (async), then [0, cut)
        flat = torch.arange(10, dtype=torch.float32) * (rank + 1)
        works = T.allreduce_flat(flat, bucket=3, lo=6, wait=False)
        assert len(works) == 2
        works += T.allreduce_flat(flat, bucket=4, hi=6, wait=False)
        for w in works:
            w.wait()
        assert torch.equal(flat, torch.arange(10, dtype=torch.float32) * 3)
        # broadcast: rank 1 starts from different weights and receives rank 0's
        m = TinyModel()
        if rank == 1:
            with torch.no_grad():
                m.lin.weight.add_(1.0)
        tr = T.Trainer(gradient_clip_val=None, accumulate_grad_batches=accumulate)
        tr.setup_optimizer(m)
        x, y = _data()
        loader = DeviceBatches((x, y), batch_size=4, shuffle=False)
        tr.fit(m, train_dataloaders=loader, val_dataloaders=DeviceBatches((x, y), 4, shuffle=False))
        out[rank] = {"w": m.lin.weight.detach().clone(), "b": m.lin.bias.detach().clone(),
                     "val": tr.logged_metrics["val/loss"], "steps": tr.global_step}
    finally:
        dist.destroy_process_group()


def _reference_single_process(accumulate, world):
    """What DDP(world) + accumulate means: per optimizer step, gradient of the mean loss over the
    accumulate*world micro-batches of that step (sharded like DistributedSampler(shuffle=False))."""
    torch.manual_seed(0)
    m = TinyModel()
    opt = torch.optim.SGD(m.parameters(), lr=0.1)
    x, y = _data()
    per_rank = [list(range(r, 24, world)) for r in range(world)]
    nb = len(per_rank[0]) // 4
    steps = 0
    for s in range(0, nb, accumulate):
        opt.zero_grad()
        mb = list(range(s, min(s + accumulate, nb)))
        loss = 0
        for r in range(world):
            for b in mb:
                idx = per_rank[r][b * 4:(b + 1) * 4]
                loss = loss + ((m.lin(x[idx]) - y[idx]) ** 2).mean()
        (loss / (accumulate * world)).backward()
        opt.step()
        steps += 1
    return m, steps


@pytest.mark.parametrize("accumulate", [1, 2])
def test_ddp_gloo_world2_matches_global_batch_semantics(accumulate):
    port = _free_port()
    out = mp.Manager().dict()
    mp.spawn(_worker, args=(2, port, out, accumulate), nprocs=2, join=True)
    ref, steps = _reference_single_process(accumulate, 2)
    for r in range(2):
        assert out[r]["steps"] == steps
        torch.testing.assert_close(out[r]["w"], ref.lin.weight.detach(), rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(out[r]["b"], ref.lin.bias.detach(), rtol=1e-5, atol=1e-6)
    # validation metric is averaged over both ranks' shards = the full split
    x, y = _data()
    with torch.no_grad():
        full = ((ref.lin(x) - y) ** 2).mean(dim=1)
    assert abs(out[0]["val"] - out[1]["val"]) < 1e-7
    assert abs(out[0]["val"] - full.mean().item()) < 1e-5


@pytest.mark.parametrize("n,world,shuffle", [(24, 2, True), (23, 2, True), (10, 4, False), (7, 3, True)])
def test_device_batches_shard_like_distributed_sampler(n, world, shuffle):
    from torch.utils.data import DistributedSampler
    from arcweld.data import DeviceBatches
    t = torch.arange(n)
    for epoch in (0, 3):
        for r in range(world):
            ds = DistributedSampler(list(range(n)), num_replicas=world, rank=r, shuffle=shuffle, seed=7)
            ds.set_epoch(epoch)
            db = DeviceBatches(t, 4, shuffle=shuffle, seed=7, rank=r, world=world)
            db.set_epoch(epoch)
            assert db.indices().tolist() == list(ds)
            got = torch.cat(list(db)).tolist()
            assert got == list(ds)


def _worker_devices1(rank, world, port, out):
    """Trainer(devices=1) inside an initialised world-2 group: the rank trains alone on the whole split (no
    broadcast, no sharding, no all-reduce), as Lightning's Trainer(devices=1) does."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from arcweld import trainer as T
    from arcweld.data import DeviceBatches
    try:
        m = TinyModel()
        tr = T.Trainer(devices=1, gradient_clip_val=None)
        x, y = _data()
        tr.fit(m, train_dataloaders=DeviceBatches((x, y), batch_size=4, shuffle=False))
        out[rank] = {"w": m.lin.weight.detach().clone(), "steps": tr.global_step}
    finally:
        dist.destroy_process_group()


def test_trainer_devices1_under_a_process_group_trains_alone():
    port = _free_port()
    out = mp.Manager().dict()
    mp.spawn(_worker_devices1, args=(2, port, out), nprocs=2, join=True)
    ref, steps = _reference_single_process(1, 1)
    for r in range(2):
        assert out[r]["steps"] == steps == 6
        torch.testing.assert_close(out[r]["w"], ref.lin.weight.detach(), rtol=1e-5, atol=1e-6)
