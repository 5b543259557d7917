"""Debug: where does the one-rank RCCL run of the VQ-VAE step differ from the plain run (ConvT2 bias)?"""
import os
import sys

sys.path.insert(0, "vq-vae-transformer-arc-welding_amd")
sys.path.insert(0, ".")
import torch
import torch.distributed as dist

from oracle import gen
from oracle import vqvae as ov

KW = dict(hidden_dim=512, num_embeddings=512, embedding_dim=64, n_resblocks=8, patch_size=25)


def make():
    from model.vq_vae_patch_embedd import VQVAEPatch
    m = VQVAEPatch(input_dim=2, learning_rate=1e-3, dropout_p=0.0, batch_norm=False, **KW)
    sd = ov.det_state_dict(ov.VQVAEConfig(**KW), 2101)
    m.load_state_dict({k: torch.tensor(v) for k, v in sd.items()})
    return m.cuda().train()


def run(scale, mode):
    from arcweld.precision import operands
    from arcweld.trainer import Trainer
    out = []
    with operands(torch.float32):
        m = make()
        tr = Trainer(gradient_clip_val=0.7)
        tr.setup_optimizer(m)
        opt = tr.optimizer
        b2 = m.reverse_patch_embed.proj[3].bias
        segs = {id(p): (o, n) for p, o, n, _, _ in opt._flat["segs"]}
        o2 = segs[id(b2)][0]
        if mode == "rccl" and not out:
            late = opt.param_spans(m.backward_late_parameters())
            early = opt.live_spans_excluding(late)
            inl = [s for s in late if s[0] <= o2 < s[1]]
            ine = [s for s in early if s[0] <= o2 < s[1]]
            print("b2 offset", o2, "in late", inl, "in early", ine, flush=True)
        orig = tr._update
        snaps = []

        def upd(model, _o=orig):
            if not torch.cuda.is_current_stream_capturing():    # eager steps only (graphs capture _update once)
                snaps.append(float(opt.flat_grad[o2]))
            return _o(model)
        tr._update = upd
        for s in range(5):
            b = torch.tensor(gen.windows(2110 + s, 128)).cuda()
            if s == 0:
                tr.micro_step(m, b, 0, scale)
                tr.optimizer_step(m)
            else:
                tr.graphed_step(m, b, scale)
            torch.cuda.synchronize()
            out.append((float(b2.detach()), float(opt.flat_grad[o2])))
        print(mode, "b2 after each step", out, "grad at eager updates", snaps, flush=True)


def main():
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT="29555", ARCWELD_FORCE_COLLECTIVES="1")
    torch.cuda.set_device(0)
    run(1.0, "plain")
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    orig = dist.all_reduce
    premul = dist._make_nccl_premul_sum(2.0)

    def doubling(t, op=dist.ReduceOp.SUM, group=None, async_op=False):
        return orig(t, op=premul, group=group, async_op=async_op)
    dist.all_reduce = doubling
    run(0.5, "rccl")
    dist.all_reduce = orig
    run(0.5, "half_no_collective")
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
