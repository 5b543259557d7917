"""Where the fused encoder chain and the per-conv launches disagree (debug aid): R = 1, dropout 0.1, N = 16384;
prints the first mismatching elements of a[0] with the x' value both paths stored."""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "vq-vae-transformer-arc-welding_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, REPO)
from test_enc_chain import _rand, _weights, _unfused_fwd, H, BF  # noqa: E402
from arcweld import kernels as K  # noqa: E402

N, R, p = 16384, 2, 0.1
x0, a0 = _rand((N, H), 11), _rand((N, H), 12)
w1, w2, b1, b2 = _weights(R, 100)
seeds = [0x1234 + 77 * r for r in range(R)]
ctr = torch.tensor([5], device="cuda", dtype=torch.int64)
ref = _unfused_fwd(a0, x0, w1, w2, b1, b2, p, seeds, ctr)
e = lambda: torch.full((N, H), float("nan"), device="cuda", dtype=BF)  # noqa: E731
h, a1, x, a = [e() for _ in range(R)], [e() for _ in range(R)], [e() if r < R - 1 else None for r in range(R)], \
    [e() for _ in range(R)]
pk = [torch.empty(H, H, device="cuda", dtype=BF) for _ in range(2 * R)]
K.enc_pack_weights(w1 + w2, pk)
K.enc_chain_fwd(a0, x0, pk[:R], pk[R:], b1, b2, h, a1, x, a, drop=(p, seeds), seed_ptr=ctr)
torch.cuda.synchronize()
print("x equal:", torch.equal(x[0], ref[2][0]), "h1 equal:", torch.equal(h[1], ref[0][1]))
d = (a[0].view(torch.int16) != ref[3][0].view(torch.int16)).nonzero()
print("a[0] mismatches:", d.shape[0])
for rr, cc in d[:12].tolist():
    xv = x[0][rr, cc].float().item()
    print(rr, cc, "x'", xv, "chain", a[0][rr, cc].float().item(), "unfused", ref[3][0][rr, cc].float().item(),
          "gelu(x') f32", torch.nn.functional.gelu(torch.tensor(xv)).item())
rows, cols = d[:, 0], d[:, 1]
print("WGs:", sorted(set((rows // 64).tolist())))
print("tokens in WG:", sorted(set((rows % 64).tolist())))
print("waves (col//64):", sorted(set((cols // 64).tolist())), "chunk-in-slice:", sorted(set(((cols % 64) // 8).tolist())),
      "elem-in-chunk:", sorted(set((cols % 8).tolist())))
a1c = (a1[0].view(torch.int16) != ref[1][0].view(torch.int16)).sum().item()
print("a1[0] mismatches", a1c, "a[1] mismatches", (a[1].view(torch.int16) != ref[3][1].view(torch.int16)).sum().item())
