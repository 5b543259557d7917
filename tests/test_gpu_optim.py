"""Flat-buffer RAdam + clip-norm kernels against the reference's torch.optim.RAdam / clip_grad_norm_ golden
trajectories (tests/golden/radam.npz: both parameter-group setups the reference builds), plus the
find_unused_parameters semantics (inactive segments are neither clipped nor updated)."""
import numpy as np
import pytest
import torch

from conftest import golden
from oracle import gen

pytestmark = pytest.mark.gpu
SHAPES = [(33, 7), (7,), (5, 3, 2)]


@pytest.mark.parametrize("tag,betas,groups", [
    ("vqvae", (0.9, 0.999), [(0.0, [0, 1, 2])]),
    ("decoder", (0.9, 0.95), [(0.1, [0, 2]), (0.0, [1])]),
])
def test_radam_clip_trajectory_matches_reference(tag, betas, groups):
    from arcweld.optim import RAdam
    g = golden("radam.npz")
    params = [torch.nn.Parameter(torch.tensor(gen.normal(500 + i, s, 0.3), device="cuda"))
              for i, s in enumerate(SHAPES)]
    opt = RAdam([{"params": [params[i] for i in idx], "weight_decay": wd} for wd, idx in groups], lr=1e-3,
                betas=betas)
    opt.flatten()
    for step in range(8):
        for i, p in enumerate(params):
            p.grad.copy_(torch.tensor(gen.normal(600 + 17 * step + i, p.shape, 1.0)))
        norm = opt.clip_grad_norm_(0.7)
        np.testing.assert_allclose(norm.item(), g[f"{tag}/prenorm_{step}"], rtol=2e-6)
        opt.step()
        opt.zero_grad()
        for i, p in enumerate(params):
            np.testing.assert_allclose(p.detach().cpu().numpy(), g[f"{tag}/p{i}_step{step}"], rtol=2e-6, atol=2e-7,
                                       err_msg=f"step {step} param {i}")


def test_inactive_segments_untouched():
    from arcweld.optim import RAdam
    params = [torch.nn.Parameter(torch.randn(s, device="cuda")) for s in [(300,), (17, 5), (64,)]]
    before = [p.detach().clone() for p in params]
    opt = RAdam(params, lr=1e-2, weight_decay=0.1)
    opt.flatten()
    opt.set_active([params[0], params[2]])
    for p in params:
        p.grad.fill_(1.0)
    norm = opt.clip_grad_norm_(1e9)
    assert abs(norm.item() - (300 + 64) ** 0.5) < 1e-3          # the inactive segment is not in the norm
    opt.step()
    assert torch.equal(params[1].detach(), before[1])
    assert not torch.equal(params[0].detach(), before[0]) and not torch.equal(params[2].detach(), before[2])


def test_centre_tap_layout_matches_dense_layout():
    """declare_centre_tap: (O, I, 3) weights become tap-major strided views, their dead side taps leave the
    norm / update / all-reduce spans, and the trajectory equals the dense layout's when those taps get zero
    gradient (the per-token encoder convs)."""
    from arcweld.optim import RAdam
    shapes = [(6, 5, 3), (6,), (6, 5, 3), (4, 7), (6, 5, 3)]
    centre = [0, 2, 4]
    runs = []
    for declare in (False, True):
        params = [torch.nn.Parameter(torch.tensor(gen.normal(800 + i, s, 0.3), device="cuda"))
                  for i, s in enumerate(shapes)]
        init = [p.detach().clone() for p in params]
        opt = RAdam(params, lr=1e-2)
        if declare:
            opt.declare_centre_tap([params[i] for i in centre])
        opt.flatten()
        for i, p in enumerate(params):
            assert p.shape == init[i].shape and torch.equal(p.detach(), init[i])
            assert p.is_contiguous() == (not declare or i not in centre)
        norms = []
        for step in range(5):
            for i, p in enumerate(params):
                g = torch.tensor(gen.normal(900 + 7 * step + i, p.shape, 1.0), device="cuda")
                if i in centre:
                    g[:, :, 0] = 0
                    g[:, :, 2] = 0
                p.grad.copy_(g)
            norms.append(opt.clip_grad_norm_(0.5).item())
            opt.step()
            opt.zero_grad()
        if declare:
            spans = opt.live_spans()
            covered = sum(b - a for a, b in spans)
            assert covered < opt.flatten()[0].numel() - 2 * 3 * 30     # both dead tap blocks are outside
            for i in centre:
                assert torch.equal(params[i].detach()[:, :, 0], init[i][:, :, 0])
                assert torch.equal(params[i].detach()[:, :, 2], init[i][:, :, 2])
                assert params[i].grad[:, :, 1].is_contiguous()
        runs.append(([p.detach().clone() for p in params], norms))
    (p0, n0), (p1, n1) = runs
    np.testing.assert_allclose(n1, n0, rtol=1e-6)
    for a, b in zip(p0, p1):
        torch.testing.assert_close(b, a, rtol=1e-6, atol=1e-7)


def test_state_dict_round_trip_resumes_the_trajectory():
    """state_dict() / load_state_dict(): a fresh optimizer loaded mid-run (flat moments + device step counter)
    continues exactly as the uninterrupted one -- the bias corrections depend on the restored step."""
    from arcweld.optim import RAdam

    def make():
        ps = [torch.nn.Parameter(torch.tensor(gen.normal(950 + i, s, 0.3), device="cuda"))
              for i, s in enumerate(SHAPES)]
        return ps, RAdam([{"params": ps[:2], "weight_decay": 0.1}, {"params": ps[2:], "weight_decay": 0.0}],
                         lr=1e-3, betas=(0.9, 0.95))

    def grads(ps, step):
        for i, p in enumerate(ps):
            p.grad.copy_(torch.tensor(gen.normal(960 + 13 * step + i, p.shape, 1.0)))

    ps, opt = make()
    opt.flatten()
    for step in range(6):
        grads(ps, step)
        opt.clip_grad_norm_(0.8)
        opt.step()
        opt.zero_grad()
        if step == 2:
            sd = opt.state_dict()
            snap = [p.detach().clone() for p in ps]
    assert sd["arcweld_flat"]["step"] == 3
    qs, opt2 = make()
    with torch.no_grad():
        for q, s in zip(qs, snap):
            q.copy_(s)
    opt2.load_state_dict(sd)
    for step in range(3, 6):
        grads(qs, step)
        opt2.clip_grad_norm_(0.8)
        opt2.step()
        opt2.zero_grad()
    for p, q in zip(ps, qs):
        assert torch.equal(p.detach(), q.detach())
    bad = dict(sd)
    bad["arcweld_flat"] = dict(sd["arcweld_flat"], m=sd["arcweld_flat"]["m"][:-64], v=sd["arcweld_flat"]["v"][:-64])
    _, opt3 = make()
    with pytest.raises(ValueError):
        opt3.load_state_dict(bad)
