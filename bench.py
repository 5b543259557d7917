"""Benchmark: welding windows/sec of the VQ-VAE-Patch reconstruction TRAIN step (BASELINE.json configs[1]:
batch 1024 windows of 200x2 per GPU, codebook 512x64, H=512, 8 ResBlocks, patch 25, dropout 0.1, bf16 MFMA
operands with fp32 accumulation / fp32 master weights).

One step = forward + backward of loss = mse(x_hat, x) + vq_loss, global-norm clip 0.7 and the RAdam update
(train_reconstruction_embedding.py:190-199) over one batch of synthetic standardised windows that is resident
in HBM before the timed region.  Multi-GPU: one process per GPU (torch.distributed.run), RCCL all-reduce of the
flat gradient buffer every step, per-rank batch fixed (weak scaling).

Prints ONE JSON line (rank 0) with the roofline of the dominant kernel (the MFMA GEMM family, timed live with
HIP events on its launch stream over the timed region) and a CPU baseline (the oracle port on the host cores,
bounded sample, rank 0 at N=1 only).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "vq-vae-transformer-arc-welding_amd"))
sys.path.insert(0, REPO)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "welding windows/sec (train) VQ-VAE+8-blk Transformer at 1/2/4/8 MI355X"
BF16_PEAK_TFLOPS = 2500.0     # MI355X dense bf16 MFMA (MI355X_MICROARCH.md: ~2.5 PF dense)
HBM_PEAK_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=1024, help="windows per GPU")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-profile", action="store_true", help="skip the live per-GEMM event timing")
    ap.add_argument("--no-graph", action="store_true", help="eager launches instead of the captured step graph")
    ap.add_argument("--no-transformer", action="store_true",
                    help="skip the secondary configs[2] line item (tokenize + 8-block Transformer train step)")
    ap.add_argument("--seqs", type=int, default=51, help="Transformer sequences per GPU per step (configs[2])")
    ap.add_argument("--n-cycles", type=int, default=20)
    ap.add_argument("--gemm-tile", type=int, default=0, choices=[0, 128, 256],
                    help="GEMM tile policy (aw_gemm_set_tile): 0 = automatic")
    return ap.parse_args()


def build_model(dev):
    from model.vq_vae_patch_embedd import VQVAEPatch
    torch.manual_seed(1)
    m = VQVAEPatch(hidden_dim=512, input_dim=2, num_embeddings=512, embedding_dim=64, n_resblocks=8,
                   learning_rate=1e-3, dropout_p=0.1, patch_size=25, seq_len=200, batch_norm=False)
    return m.to(dev).train()


def transformer_workload(dev, rank, world, args):
    """configs[2]: per step the frozen VQ-VAE encoder tokenizes seqs x n_cycles windows (fused encoder + VQ, exact
    fp32 operands), then one train step of the 8-block/8-head d512 decoder on the generation task
    (T = 16*n_cycles + 1 = 321, V = 514, accumulate 1, clip 0.8, RAdam betas (0.9, 0.95) wd 0.1 on Linear weights).
    Returns windows/s over all ranks and ms/step."""
    from arcweld import tokenize
    from arcweld.trainer import Trainer
    from model.transformer_decoder import MyTransformerDecoder
    vq = build_model(dev).eval()
    nc = args.n_cycles
    torch.manual_seed(2)
    dec = MyTransformerDecoder(d_model=512, n_classes=514, seq_len=16 * nc + 1, n_blocks=8, n_head=8,
                               res_dropout=0.1).to(dev).train()
    tr = Trainer(gradient_clip_val=0.8)
    tr.setup_optimizer(dec)
    g = torch.Generator(device=dev)
    g.manual_seed(2000 + rank)
    wins = [torch.randn(args.seqs, 200 * nc, 2, device=dev, generator=g) for _ in range(2)]
    cond = torch.zeros(args.seqs, dtype=torch.long, device=dev)

    use_graph = not args.no_graph
    static_w = wins[0].clone()

    def train(w):
        ids = tokenize.encode_ids(vq, w)
        x, y, _ = tokenize.autoregressive_pairs(ids, start_token=512)
        return (x, cond, y)

    def step(i):
        if use_graph:
            # tokenization is captured with the step: the static window buffer feeds the encoder inside g1
            static_w.copy_(wins[i % 2])
            tr.graphed_step(dec, static_w, 1.0 / world)
        else:
            tr.micro_step(dec, train(wins[i % 2]), i, 1.0 / world)
            tr.optimizer_step(dec)

    if use_graph:
        orig = dec.training_step
        dec.training_step = lambda w, i: orig(train(w), i)

    for i in range(max(args.warmup, 1 if use_graph else 0)):
        step(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    t = torch.tensor([el], device=dev, dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    el = float(t.item())
    windows = world * args.seqs * nc * args.steps
    flops_seq = 3 * (8 * (24 * 512 * 512 * (16 * nc + 1) + 2 * 512 * (16 * nc + 1) * (16 * nc + 2))
                     + 2 * 512 * 514 * (16 * nc + 1))
    return {"value": round(windows / el, 2), "unit": "windows/s", "ms_per_step": round(el * 1e3 / args.steps, 3),
            "config": {"workload": "tokenize (frozen VQ-VAE encoder, fp32 exact) + Transformer train step "
                                   "(configs[2])", "seqs_per_gpu": args.seqs, "n_cycles": nc, "T": 16 * nc + 1,
                       "d_model": 512, "n_blocks": 8, "n_head": 8, "V": 514, "global_batch_windows": windows //
                       args.steps},
            "transformer_tflops": round(flops_seq * args.seqs * world * args.steps / el / 1e12, 2)}


def gemm_traffic():
    """HBM bytes per launch of the GEMM family from the committed rocprofv3 PMC passes (FETCH_SIZE and WRITE_SIZE in
    separate runs, FETCH_SIZE doubled on gfx950; tools/pmc_traffic.py) of this same workload: counters cannot be
    read from inside the timed run."""
    import glob
    files = sorted(glob.glob(os.path.join(REPO, "profiles", "*", "*", "pmc_gemm_traffic.json")) +
                   glob.glob(os.path.join(REPO, "profiles", "*", "pmc_gemm_traffic.json")))
    if not files:
        return None, None
    with open(files[-1]) as f:
        d = json.load(f)
    return round(d["avg_bytes_per_launch"]), os.path.relpath(files[-1], REPO)


def cpu_baseline(seconds):
    """Oracle port (oracle/vqvae.py, torch CPU fp32, all host threads) on a bounded sample of the same workload:
    full-size model, B=32 windows per step, fwd+bwd+RAdam; windows/s."""
    import numpy as np
    from oracle import gen
    from oracle import optim as oo
    from oracle import vqvae as ov
    threads = min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    cfg = ov.VQVAEConfig(dropout_p=0.0)
    sd = ov.det_state_dict(cfg, 1)
    names = [k for k in sd if not (k.endswith("running_mean") or k.endswith("running_var") or
                                   k.endswith("num_batches_tracked"))]
    st = oo.RAdamState([sd[k].shape for k in names])
    B = 32
    x = gen.windows(0, B)
    steps, t0 = 0, None
    while True:
        out, grads, state = ov.vqvae_train_step_grads(sd, x, cfg)
        gl = [grads[k].copy() for k in names]
        oo.clip_grad_norm(gl, 0.7)
        ps = [sd[k] for k in names]
        oo.radam_step(ps, gl, st, 1e-3, (0.9, 0.999), 1e-8, [0.0] * len(ps))
        if t0 is None:            # first step is warm-up
            t0 = time.time()
            continue
        steps += 1
        if time.time() - t0 > seconds:
            break
    el = time.time() - t0
    return {"value": round(B * steps / el, 2), "unit": "windows/s", "cores": threads, "kind": "port",
            "sample": f"oracle/vqvae.py full-size VQ-VAE (H512 R8 K512xD64) fp32 train step, B={B} windows, "
                      f"{steps} timed steps ({el:.1f} s) after 1 warm-up, torch CPU {threads} threads"}


def main():
    args = parse()
    distributed = int(os.environ.get("WORLD_SIZE", "1")) > 1
    if distributed:
        # ARCWELD_DIST_BACKEND=gloo rehearses N ranks on one GPU (RCCL refuses two ranks per device); the
        # measured multi-GPU path is "nccl" (= RCCL over xGMI)
        dist.init_process_group(os.environ.get("ARCWELD_DIST_BACKEND", "nccl"))
        rank, world = dist.get_rank(), dist.get_world_size()
        local = int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count())
    else:
        rank, world, local = 0, 1, 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    torch.set_float32_matmul_precision("medium")    # as train_reconstruction_embedding.py:253 -> bf16 MFMA

    from arcweld import _native, kernels
    from arcweld.trainer import Trainer
    _native.call("aw_gemm_set_tile", args.gemm_tile)

    model = build_model(dev)
    trainer = Trainer(gradient_clip_val=0.7)
    trainer.setup_optimizer(model)
    scale = 1.0 / world
    gen_ = torch.Generator(device=dev)
    gen_.manual_seed(1000 + rank)
    batches = [torch.randn(args.batch, 200, 2, device=dev, generator=gen_) for _ in range(4)]

    use_graph = not args.no_graph

    def eager_step(i):
        trainer.micro_step(model, batches[i % len(batches)], i, scale)
        trainer.optimizer_step(model)

    def step(i):
        if use_graph:
            trainer.graphed_step(model, batches[i % len(batches)], scale)
        else:
            eager_step(i)

    for i in range(max(args.warmup, 1 if use_graph else 0)):
        step(i)
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(i)
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    # per-GEMM HIP events cannot sit inside a captured graph: the kernel durations for the roofline come from a
    # profiled eager pass over the same workload right after the timed region (GPU-side durations are the
    # same; rocprofv3 in profiles/ cross-checks them against the graph replays)
    prof = None
    if not args.no_profile:
        n_prof = min(args.steps, 10)
        kernels.PROFILE = []
        t1 = time.perf_counter()
        for i in range(n_prof):
            eager_step(i)
        torch.cuda.synchronize()
        prof_elapsed, prof_steps = time.perf_counter() - t1, n_prof
        prof = kernels.PROFILE
        kernels.PROFILE = None
    t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
    if distributed:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    value = world * args.batch * args.steps / elapsed

    roofline = None
    traffic, traffic_src = gemm_traffic()
    if prof:
        ms = sum(e0.elapsed_time(e1) for e0, e1, _ in prof)
        flops = sum(f for _, _, f in prof)
        n = len(prof)
        achieved = flops / (ms * 1e-3) / 1e12
        roofline = {"bound": "mfma", "achieved": round(achieved, 2), "peak": BF16_PEAK_TFLOPS, "unit": "TFLOP/s",
                    "frac": round(achieved / BF16_PEAK_TFLOPS, 4), "traffic": traffic, "traffic_unit": "bytes/launch",
                    "traffic_source": traffic_src,
                    "kernel": "gemm_kernel<bf16> (aw_gemm)", "launches_per_step": n // prof_steps,
                    "avg_launch_us": round(ms * 1e3 / n, 2), "avg_algorithmic_gflop_per_launch": round(flops / n / 1e9, 4),
                    "gemm_ms_per_step": round(ms / prof_steps, 3),
                    "gemm_share_of_step": round(ms / prof_steps / (elapsed * 1e3 / args.steps), 4),
                    "measured_over": f"{prof_steps} eager steps after the timed region (HIP events per launch)",
                    "eager_ms_per_step_with_events": round(prof_elapsed * 1e3 / prof_steps, 3)}

    secondary = None
    if not args.no_transformer:
        secondary = transformer_workload(dev, rank, world, args)

    if rank == 0:
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(args.cpu_seconds)
        line = {"metric": METRIC, "value": round(value, 2), "unit": "windows/s", "n_gpus": world,
                "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed * 1e3 / args.steps, 3),
                "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "bf16",
                "data": "synthetic N(0,1) standardised 200x2 welding windows, random-init weights",
                "config": {"workload": "VQ-VAE-Patch reconstruction train step (configs[1])",
                           "global_batch": world * args.batch, "per_gpu_batch": args.batch, "seq_len": 200,
                           "codebook": "512x64", "hidden": 512, "n_resblocks": 8, "patch": 25,
                           "parallelism": f"dp{world}", "clip": 0.7, "optimizer": "RAdam(lr 1e-3)"},
                "roofline": roofline, "cpu_baseline": cpu, "transformer": secondary,
                "launch": "hip-graph" if use_graph else "eager"}
        print(json.dumps(line), flush=True)
    if distributed:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
