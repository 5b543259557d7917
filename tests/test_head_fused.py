"""The fused training-step head (aw_unpatch_head_fwd_bwd1: forward + MSE value / gradient + backward pass 1 in one read
of the ConvT output) against the separate passes it replaces (aw_unpatch_head_fwd_ex, aw_mse_fwd, aw_mse_bwd,
aw_unpatch_head_bwd1_ex) on the same inputs; model/vq_vae_patch_embedd.py:27-30,52-57 and
autencoder_lightning_base.py:80-97 define the math both follow."""
import pytest
import torch

from arcweld import kernels as K

pytestmark = pytest.mark.gpu

H, Q = 512, 80


def _inputs(R, ydt, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    dev = "cuda"
    st = torch.cat([torch.randn(H, device=dev, generator=g) * 0.2, torch.rand(H, device=dev, generator=g) + 0.5,
                    torch.rand(H, device=dev, generator=g) + 0.5, torch.randn(H, device=dev, generator=g) * 0.2])
    w2 = torch.randn(H, 5, device=dev, generator=g) * 0.05
    b2 = torch.randn(1, device=dev, generator=g)
    y = (torch.randn(R, H, device=dev, generator=g) * 1.5 + 0.3).to(ydt)
    x = torch.randn(R // Q, 200, 2, device=dev, generator=g)
    return st, w2, b2, y, x


@pytest.mark.parametrize("R,ydt", [(80 * 37, torch.float32), (80 * 37, torch.bfloat16), (80 * 1024, torch.float32),
                                   (80, torch.bfloat16)])
def test_fused_head_matches_separate_passes(R, ydt):
    st, w2, b2, y, x = _inputs(R, ydt, 5)
    gscale = torch.tensor([0.75], device="cuda")
    z = lambda *s, dt=torch.float32: torch.zeros(*s, device="cuda", dtype=dt)  # noqa: E731
    # separate passes
    xh_a, gx_a, sq_a = torch.empty_like(x), torch.empty_like(x), z(1, dt=torch.float64)
    gs_a, gw_a, gb_a, gg_a, gbe_a = z(2 * H, dt=torch.float64), z(H, 5), z(1), z(H), z(H)
    K.unpatch_head_fwd(y, Q, st, w2, b2, xh_a)
    K.mse_fwd(xh_a, x, sq_a)
    K.mse_bwd(xh_a, x, gscale, gx_a)
    K.unpatch_head_bwd1(y, Q, st, w2, gx_a, gs_a, gw_a, gb_a, gg_a, gbe_a)
    # fused
    xh_b, gx_b, sq_b = torch.empty_like(x), torch.empty_like(x), z(1, dt=torch.float64)
    gs_b, gw_b, gb_b, gg_b, gbe_b = z(2 * H, dt=torch.float64), z(H, 5), z(1), z(H), z(H)
    K.unpatch_head_fwd_bwd1(y, Q, st, w2, b2, x, gscale, xh_b, gx_b, sq_b, gs_b, gw_b, gb_b, gg_b, gbe_b)
    torch.cuda.synchronize()
    torch.testing.assert_close(xh_b, xh_a, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(gx_b, gx_a, rtol=1e-4, atol=1e-9)
    torch.testing.assert_close(sq_b, sq_a, rtol=1e-5, atol=0)
    for b, a in ((gs_b, gs_a), (gw_b, gw_a), (gb_b, gb_a), (gg_b, gg_a), (gbe_b, gbe_a)):
        scale = a.abs().max().item()
        torch.testing.assert_close(b, a, rtol=2e-4, atol=2e-5 * scale)
