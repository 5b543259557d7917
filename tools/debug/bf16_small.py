"""Debug: the bf16-operand VQ-VAE forward on the small golden case, fp32 vs bf16 residual streams: x_hat error
against the fp32 golden and codebook-index agreement (tests/test_vqvae_module.py::test_vqvae_bf16_mode_tracks_fp32)."""
import os
import sys

sys.path.insert(0, "vq-vae-transformer-arc-welding_amd")
sys.path.insert(0, ".")
sys.path.insert(0, "tests")
import numpy as np
import torch

from conftest import golden
from oracle import gen
from test_vqvae_module import CASES, make_model


def main():
    from arcweld.precision import operands
    kw, B, wseed, xseed = CASES["vqvae_small.npz"]
    g = golden("vqvae_small.npz")
    for rf in ("1", "0"):
        os.environ["ARCWELD_RESID_F32"] = rf
        with operands(torch.bfloat16):
            m = make_model(kw, wseed, "cuda")
            x = torch.tensor(gen.windows(xseed, B), device="cuda")
            emb, x_hat, perp = m(x)
            xh = x_hat.detach().cpu().numpy()
            idx = m._last_indices.cpu().numpy()
        err = np.abs(xh - g["x_hat"])
        agree = (idx == g["idx"]).mean()
        tok = err.reshape(B, -1)
        print(f"resid_f32={rf}: max err {err.max():.4f} (bound {0.05 * np.abs(g['x_hat']).max():.4f}), "
              f"index agreement {agree:.4f}, err by window {np.round(tok.max(1), 3)}", flush=True)


if __name__ == "__main__":
    main()
