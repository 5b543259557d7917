import sys; sys.path[:0] = ['.', 'vq-vae-transformer-arc-welding_amd']
import torch, numpy as np
from oracle import gen, vqvae as ov
from model.vq_vae_patch_embedd import VQVAEPatch
from arcweld import vqvae as eng
torch.set_float32_matmul_precision("highest")
kw = dict(hidden_dim=512, num_embeddings=512, embedding_dim=64, n_resblocks=8, patch_size=25)
m = VQVAEPatch(input_dim=2, learning_rate=1e-3, dropout_p=0.0, batch_norm=False, **kw)
sd = ov.det_state_dict(ov.VQVAEConfig(**kw), 309)
m.load_state_dict({k: torch.tensor(v) for k, v in sd.items()})
m = m.cuda().train()
x = torch.tensor(gen.windows(310, 4), device="cuda")
_, _, _, idx_f, sv = eng.forward(m, x, True, True)
idx_e, z_e = eng.encode(m, x)
print("z diff", (sv.z - z_e).abs().max().item(), "idx eq", torch.equal(idx_f, idx_e))
for r in range(3):
    print(r, "xs", None if sv.xs[r] is None else sv.xs[r].abs().max().item())
m.eval()
idx_e2, z_e2 = eng.encode(m, x)
print("eval z diff", (sv.z - z_e2).abs().max().item())
