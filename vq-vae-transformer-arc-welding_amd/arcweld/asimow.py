"""ASIMoW on-disk format -> device-resident welding windows.

Restates the reference's CSV path (dataloader/asimow_dataloader.py, dataloader/utils.py) with the same
semantics, minus its pickle cache:

* ``processed_asimow_dataset.csv``: columns ``experiment, welding_run, labels, V_0..V_199, I_0..I_199``; one row
  per welding cycle (asimow_dataloader.py:40-43,229-246).  Columns 3:203 are the voltage cycle, 203: the
  current cycle; a window is (200, 2) = [V, I] per sample.
* split by (experiment, welding_run) ids into train / val / test (:56-90); the classification tasks drop the
  rows labelled -1, reconstruction keeps them.
* windows: ``[window_offset, window_offset + window_size)`` of each cycle, or ``cycle_seq_number`` consecutive
  cycles concatenated (``create_sequence_ds`` :185-206: n - seq_len sequences, label of the cycle after).
* per-channel StandardScaler fitted on train, applied to all splits (utils.py MyScaler :81-98; population std,
  a zero-variance channel scaled by 1, as sklearn).
* shuffle after scaling with numpy's legacy global RNG seeded once (base_dataloader.py:134, utils.py:10-15):
  :class:`ASIMoWData` replays the same sequence of ``shuffle`` calls (train, val, test) on a
  ``RandomState(seed)``, so the order is the reference's.
* classification sampling weights (asimow_dataloader.py:107-121).

The reference caches the parsed frame as ``dataset.pickle``; pickles are not loaded here (they execute code on
load).  :func:`save_cache` / :func:`load_cache` keep the parsed cycles in an ``.npz`` instead.
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import numpy as np
import torch

N_SAMPLES = 200


@dataclass(frozen=True)
class DataSplitId:
    """(experiment, welding_run) selecting validation / test runs (asimow_dataloader.py:15-25)."""
    experiment: int
    welding_run: int


# get_val_test_ids() (dataloader/utils.py:46-68): the fixed validation / test runs the entry scripts use
REFERENCE_SPLIT_IDS = {
    "test_ids": [DataSplitId(e, r) for e, r in ((3, 32), (3, 18), (1, 27), (3, 19), (3, 17), (2, 21), (1, 20),
                                                (1, 11))],
    "val_ids": [DataSplitId(e, r) for e, r in ((3, 3), (2, 10), (1, 24), (3, 24), (1, 32), (2, 1), (1, 10),
                                               (1, 16))],
}


@dataclass
class Cycles:
    vi: np.ndarray            # (n, 200, 2) float64: [V, I]
    labels: np.ndarray        # (n,) int64 (-1: unlabelled)
    experiment: np.ndarray    # (n,) int64
    welding_run: np.ndarray   # (n,) int64


def read_csv(path: str) -> Cycles:
    """Parse ``processed_asimow_dataset.csv`` (convert_to_cycle_np_array, asimow_dataloader.py:229-246)."""
    import pandas as pd
    df = pd.read_csv(path)
    if df.shape[1] != 3 + 2 * N_SAMPLES:
        raise ValueError(f"{path}: expected {3 + 2 * N_SAMPLES} columns (experiment, welding_run, labels, V_0..V_199, "
                         f"I_0..I_199), got {df.shape[1]}")
    v = df.iloc[:, 3:3 + N_SAMPLES].to_numpy(dtype=np.float64)
    i = df.iloc[:, 3 + N_SAMPLES:].to_numpy(dtype=np.float64)
    vi = np.concatenate([v.reshape(-1, N_SAMPLES, 1), i.reshape(-1, N_SAMPLES, 1)], axis=2)
    return Cycles(vi=vi, labels=df["labels"].to_numpy().astype(np.int64),
                  experiment=df["experiment"].to_numpy().astype(np.int64),
                  welding_run=df["welding_run"].to_numpy().astype(np.int64))


def save_cache(c: Cycles, path: str) -> None:
    os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
    np.savez(path, vi=c.vi, labels=c.labels, experiment=c.experiment, welding_run=c.welding_run)


def load_cache(path: str) -> Cycles:
    with np.load(path, allow_pickle=False) as z:
        return Cycles(vi=z["vi"], labels=z["labels"], experiment=z["experiment"], welding_run=z["welding_run"])


class ChannelScaler:
    """Per-channel standardisation over all samples and time steps (MyScaler, utils.py:81-98)."""

    def fit(self, x: np.ndarray):
        flat = x.reshape(-1, x.shape[-1])
        self.mean_ = flat.mean(axis=0)
        var = flat.var(axis=0)                       # population variance, as StandardScaler
        self.scale_ = np.where(var > 0, np.sqrt(var), 1.0)
        return self

    def transform(self, x: np.ndarray) -> np.ndarray:
        return ((x.reshape(-1, x.shape[-1]) - self.mean_) / self.scale_).reshape(x.shape)

    def inverse_transform(self, x: np.ndarray) -> np.ndarray:
        return (x.reshape(-1, x.shape[-1]) * self.scale_ + self.mean_).reshape(x.shape)


def sampling_weights(labels: np.ndarray) -> np.ndarray:
    """WeightedRandomSampler weights balancing labels 0 / 1 (asimow_dataloader.py:107-121)."""
    ratio = np.mean(labels == 0)
    w = np.zeros_like(labels, dtype=np.float32)
    w[labels == 0] = 1 - ratio
    w[labels == 1] = ratio
    return w


def sequences(x: np.ndarray, y: np.ndarray, seq_len: int, window_size: int = 200, window_offset: int = 0):
    """``create_sequence_ds`` (asimow_dataloader.py:185-206): sample i = cycles i..i+seq_len-1 (each cut to the
    window) concatenated along time, label = y[i + seq_len]; n - seq_len samples."""
    n = x.shape[0] - seq_len
    if n <= 0:
        return np.zeros((0, window_size * seq_len, x.shape[2])), np.zeros((0,))
    w = x[:, window_offset:window_offset + window_size, :]
    idx = np.arange(n)[:, None] + np.arange(seq_len)[None, :]
    return w[idx].reshape(n, seq_len * window_size, x.shape[2]), y[seq_len:seq_len + n].astype(np.float64)


class ASIMoWData:
    """Train / val / test arrays exactly as ASIMoWDataLoader.get_dataset builds them (scaled, shuffled)."""

    TASKS = ("classification", "reconstruction")

    def __init__(self, cycles: Cycles, val_ids, test_ids, task: str = "reconstruction", cycle_seq_number: int = 1,
                 seed: int = 42, window_size: int = 200, window_offset: int = 0, shuffle: bool = True):
        if task not in self.TASKS:
            raise NotImplementedError(f"Task {task} not implemented")
        self.task, self.cycle_seq_number = task, int(cycle_seq_number)
        self.window_size, self.window_offset, self.shuffle = int(window_size), int(window_offset), shuffle
        self.scaler = ChannelScaler()
        self.rng = np.random.RandomState(seed)    # the reference seeds numpy's global RNG once and shuffles
        c = cycles

        def mask(ids):
            m = np.zeros(len(c.labels), dtype=bool)
            for s in ids:
                m |= (c.experiment == s.experiment) & (c.welding_run == s.welding_run)
            return m

        mv, mt = mask(val_ids), mask(test_ids)
        parts = {"train": ~(mv | mt), "val": mv, "test": mt}
        self.splits = {}
        for name in ("train", "val", "test"):        # the reference's call order (fit on train first)
            m = parts[name]
            if task == "classification":
                m = m & (c.labels != -1)
            self.splits[name] = self._scale_and_shuffle(c.vi[m], c.labels[m], name)

    def _scale_and_shuffle(self, x, y, ds_type):
        if self.cycle_seq_number > 1:
            x, y = sequences(x, y, self.cycle_seq_number, self.window_size, self.window_offset)
        else:
            x = x[:, self.window_offset:self.window_offset + self.window_size, :]
        if ds_type == "train":
            self.scaler.fit(x)
        x = self.scaler.transform(x)
        if self.shuffle:
            idx = np.arange(len(y))
            self.rng.shuffle(idx)
            x, y = x[idx], y[idx]
        return x, y

    def tensors(self, split: str, device="cuda"):
        """(windows float32 (n, L, 2), labels int64 (n,)) on ``device`` (MyClassificationDataset /
        MyReconstructionDataset dtypes, base_dataloader.py:14-72)."""
        x, y = self.splits[split]
        return (torch.tensor(x, dtype=torch.float32, device=device),
                torch.tensor(np.asarray(y), dtype=torch.long, device=device))


def load(data_dir: str, val_ids, test_ids, task: str = "reconstruction", cache: bool = True, **kw) -> ASIMoWData:
    """``<data_dir>/processed_asimow_dataset.csv`` -> :class:`ASIMoWData`; the parsed cycles are cached as
    ``<data_dir>/quality_prediction_data/asimow/dataset.npz`` (the reference's dataset_path, npz not pickle)."""
    cache_path = os.path.join(data_dir, "quality_prediction_data", "asimow", "dataset.npz")
    if cache and os.path.exists(cache_path):
        cycles = load_cache(cache_path)
    else:
        cycles = read_csv(os.path.join(data_dir, "processed_asimow_dataset.csv"))
        if cache:
            save_cache(cycles, cache_path)
    return ASIMoWData(cycles, val_ids, test_ids, task=task, **kw)
