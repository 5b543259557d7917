"""ASIMoW CSV format: parse, split, scale, sequence and shuffle exactly like the reference's
ASIMoWDataLoader (dataloader/asimow_dataloader.py, dataloader/utils.py).  The dataset itself is not available
offline; the CSV here is synthetic in the reference's column layout.  The scaler is pinned against
sklearn.preprocessing.StandardScaler (what the reference's MyScaler wraps) and the shuffle against numpy's
global-RNG calls in the reference's order."""
import numpy as np
import pandas as pd
import pytest

from arcweld import asimow as A


def _frame(n=60, seed=0):
    rng = np.random.default_rng(seed)
    exp = rng.integers(1, 4, n)
    run = rng.integers(1, 6, n)
    lab = rng.choice([-1, 0, 1], n)
    v = rng.normal(20, 3, (n, 200))
    i = rng.normal(150, 30, (n, 200))
    cols = {"experiment": exp, "welding_run": run, "labels": lab}
    cols.update({f"V_{k}": v[:, k] for k in range(200)})
    cols.update({f"I_{k}": i[:, k] for k in range(200)})
    return pd.DataFrame(cols), v, i


@pytest.fixture
def csv(tmp_path):
    df, v, i = _frame()
    p = tmp_path / "processed_asimow_dataset.csv"
    df.to_csv(p, index=False)
    return tmp_path, df, v, i


VAL = [A.DataSplitId(1, 2), A.DataSplitId(3, 1)]
TEST = [A.DataSplitId(2, 3)]


def test_read_csv_column_layout(csv):
    d, df, v, i = csv
    c = A.read_csv(str(d / "processed_asimow_dataset.csv"))
    assert c.vi.shape == (len(df), 200, 2)
    np.testing.assert_allclose(c.vi[:, :, 0], v)
    np.testing.assert_allclose(c.vi[:, :, 1], i)
    assert np.array_equal(c.labels, df.labels.to_numpy())


def test_scaler_matches_sklearn():
    from sklearn.preprocessing import StandardScaler
    x = np.random.default_rng(1).normal(3, 2, (40, 200, 2))
    x[:, :, 1] = 5.0          # zero-variance channel
    ref = StandardScaler().fit(x.reshape(-1, 2))
    s = A.ChannelScaler().fit(x)
    np.testing.assert_allclose(s.transform(x).reshape(-1, 2), ref.transform(x.reshape(-1, 2)), rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(s.inverse_transform(s.transform(x)), x, rtol=1e-12)


def _reference_split(df, task, seed, seq=1):
    """The reference's split + scale + shuffle, restated with its own numpy calls (global RNG)."""
    from sklearn.preprocessing import StandardScaler
    np.random.seed(seed)
    vcond = np.any([(df.welding_run == s.welding_run) & (df.experiment == s.experiment) for s in VAL], axis=0)
    tcond = np.any([(df.welding_run == s.welding_run) & (df.experiment == s.experiment) for s in TEST], axis=0)
    parts = [df[~(vcond | tcond)], df[vcond], df[tcond]]
    if task == "classification":
        parts = [p[p.labels != -1] for p in parts]
    scaler = StandardScaler()
    out = []
    for k, p in enumerate(parts):
        x = np.concatenate([p.iloc[:, 3:203].to_numpy().reshape(-1, 200, 1),
                            p.iloc[:, 203:].to_numpy().reshape(-1, 200, 1)], axis=2)
        y = p.labels.to_numpy()
        if seq > 1:
            nx = np.zeros((x.shape[0] - seq, 200 * seq, 2))
            ny = np.zeros(x.shape[0] - seq)
            for j in range(x.shape[0] - seq):
                nx[j] = x[j:j + seq].reshape(-1, 2)
                ny[j] = y[j + seq]
            x, y = nx, ny
        if k == 0:
            scaler.fit(x.reshape(-1, 2))
        x = scaler.transform(x.reshape(-1, 2)).reshape(x.shape)
        idx = np.arange(len(y))
        np.random.shuffle(idx)
        out.append((x[idx], y[idx]))
    return out


@pytest.mark.parametrize("task,seq", [("reconstruction", 1), ("classification", 1), ("classification", 3)])
def test_split_scale_shuffle_match_reference(csv, task, seq):
    d, df, _, _ = csv
    data = A.load(str(d), VAL, TEST, task=task, cycle_seq_number=seq, seed=7)
    ref = _reference_split(df, task, 7, seq)
    for name, (rx, ry) in zip(("train", "val", "test"), ref):
        x, y = data.splits[name]
        assert x.shape == rx.shape, name
        np.testing.assert_allclose(x, rx, rtol=1e-12, atol=1e-12, err_msg=name)
        np.testing.assert_array_equal(np.asarray(y, dtype=np.float64), np.asarray(ry, dtype=np.float64))
    if task == "classification":
        assert all((data.splits[s][1] != -1).all() for s in ("train", "val", "test"))


def test_npz_cache_round_trip(csv):
    d, df, _, _ = csv
    a = A.load(str(d), VAL, TEST, seed=3)
    cache = d / "quality_prediction_data" / "asimow" / "dataset.npz"
    assert cache.exists()
    (d / "processed_asimow_dataset.csv").unlink()          # the second load reads the cache only
    b = A.load(str(d), VAL, TEST, seed=3)
    for s in ("train", "val", "test"):
        np.testing.assert_array_equal(a.splits[s][0], b.splits[s][0])


def test_window_offset_and_weights(csv):
    d, df, v, _ = csv
    data = A.ASIMoWData(A.read_csv(str(d / "processed_asimow_dataset.csv")), VAL, TEST, window_size=100,
                        window_offset=50, shuffle=False)
    assert data.splits["train"][0].shape[1:] == (100, 2)
    y = np.array([0, 0, 1, 1, 1, -1])
    w = A.sampling_weights(y)
    np.testing.assert_allclose(w, [2 / 3, 2 / 3, 1 / 3, 1 / 3, 1 / 3, 0.0], rtol=1e-6)   # ratio = P(label 0)
    x, lab = data.tensors("val", device="cpu")
    assert x.dtype.is_floating_point and x.dtype.itemsize == 4 and lab.dtype.itemsize == 8


def test_reference_loader_fixture(tmp_path):
    """Against the reference's own ASIMoWDataLoader (tests/golden/asimow_split.npz, written by
    tests/golden/make_golden.py from the same synthetic CSV): every split's windows and labels, for
    reconstruction, classification and 3-cycle classification sequences (asimow_dataloader.py:56-206)."""
    import os
    import sys
    from conftest import golden
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
    import make_golden as mg
    mg.asimow_frame().to_csv(tmp_path / "processed_asimow_dataset.csv", index=False)
    g = golden("asimow_split.npz")
    val = [A.DataSplitId(e, r) for e, r in mg.ASIMOW_VAL]
    test = [A.DataSplitId(e, r) for e, r in mg.ASIMOW_TEST]
    for task, seq in mg.ASIMOW_CASES:
        data = A.load(str(tmp_path), val, test, task=task, cycle_seq_number=seq, seed=7, cache=False)
        for name in ("train", "val", "test"):
            x, y = data.splits[name]
            rx = g[f"{task}_{seq}/{name}/x"]
            assert x.shape == rx.shape, (task, seq, name)
            np.testing.assert_allclose(x, rx, rtol=1e-12, atol=1e-12, err_msg=f"{task} {seq} {name}")
            key = f"{task}_{seq}/{name}/y"
            if key in g.files:
                np.testing.assert_array_equal(np.asarray(y, dtype=np.float64), g[key])
