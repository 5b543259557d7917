"""The multitask training regime (train_transformer_mtasks.py:23-33, 178-190) against a trajectory
of the REFERENCE module (tests/golden/training_regime.npz, tests/golden/make_golden.py case_training_regime): a
generate stage of 3 optimizer steps, then a classification stage of 2, each with a new Trainer -- and so a new
RAdam (the module's configure_optimizers: betas (0.9, 0.95), wd 0.1 on Linear weights) --, accumulate_grad_batches
5 (each micro-batch loss / 5), gradient_clip_val 0.8, and the head the stage does not use left with grad None
(neither clipped, stepped nor decayed: find_unused_parameters=True).  Parameters after each stage and the
pre-clip gradient norms must match."""
import os
import sys

import numpy as np
import pytest
import torch

from conftest import golden
from oracle import decoder as od

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
import make_golden as mg  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("graphs", [False, True])
def test_accumulate5_clip08_two_stage_trajectory_matches_reference(graphs):
    """graphs: Trainer(hip_graphs=True) -- the first two accumulation groups of a stage run eagerly (warm-up), the
    third is captured and replayed (the group's five micro-batches as ONE forward/backward with a loss mean per
    micro-batch, arcweld/graphs.py grouped accumulation, then the captured clip + RAdam), so stage 0's last optimizer
    step comes from the graphs; the captured clip reports no norm to Python."""
    from arcweld.precision import operands
    from arcweld.trainer import Trainer
    from model.transformer_decoder import MyTransformerDecoder
    g = golden("training_regime.npz")
    kw = dict(mg.REGIME_KW)
    m = MyTransformerDecoder(**kw)
    sd = od.det_state_dict(1001, **{k: kw[k] for k in ("d_model", "n_classes", "seq_len", "n_blocks")})
    m.load_state_dict({k: torch.tensor(v) for k, v in sd.items()})
    m = m.cuda().train()
    with operands(torch.float32):
        for si, (task, nsteps) in enumerate(mg.REGIME_STAGES):
            (m.switch_to_generate if task == "generate" else m.switch_to_classification)()
            batches = [tuple(t.cuda() for t in mg.regime_batch(si, step, micro))
                       for step in range(nsteps) for micro in range(5)]
            tr = Trainer(gradient_clip_val=0.8, accumulate_grad_batches=5, max_epochs=1, log_every_n_steps=1,
                         hip_graphs=graphs)
            norms = []
            setup = tr.setup_optimizer

            def setup_and_watch(model, _setup=setup):
                opt = _setup(model)
                clip = opt.clip_grad_norm_

                def watched(max_norm):
                    n = clip(max_norm)
                    if not torch.cuda.is_current_stream_capturing():   # the captured clip has no host value
                        norms.append(float(n))
                    return n
                opt.clip_grad_norm_ = watched
                return opt
            tr.setup_optimizer = setup_and_watch
            tr.fit(m, train_dataloaders=batches)
            assert tr.global_step == nsteps
            assert len(norms) == (min(nsteps, 2) if graphs else nsteps)
            np.testing.assert_allclose(norms, [float(g[f"s{si}/gradnorm_{s}"]) for s in range(len(norms))], rtol=1e-5)
            for n, p in m.named_parameters():
                np.testing.assert_allclose(p.detach().cpu().numpy(), g[f"s{si}/param/{n}"], rtol=1e-5, atol=1e-6,
                                           err_msg=f"stage {si} {n}")


@pytest.mark.parametrize("n_batches", [13, 11])
def test_graphed_fit_with_short_last_group_matches_eager(n_batches):
    """An epoch whose length is not a multiple of accumulate_grad_batches ends on a short group (Lightning steps on
    the epoch's last batch): 13 micro-batches = 5 + 5 + 3, 11 = 5 + 5 + 1.  The captured step replays groups of five
    as one batch (arcweld/graphs.py), so the short group must run eagerly on the same gradients and optimizer state,
    in every epoch, before and after the capture, and must never become the captured group size.  Three epochs of a
    graphed fit (steps 1-2 warm up, epoch 1's short group eager before any capture, epoch 2 captures, replays and
    steps its short group eagerly, epoch 3 replays after an eager step) against the same fit without graphs; fp32
    operands, no dropout: only the weight-gradient reduction order differs."""
    from arcweld.precision import operands
    from arcweld.trainer import Trainer
    from model.transformer_decoder import MyTransformerDecoder
    kw = dict(d_model=128, n_classes=40, seq_len=33, n_blocks=2, n_head=4, res_dropout=0.0, att_dropout=0.0)
    g = torch.Generator(device="cpu").manual_seed(11)
    batches = []
    for j in range(n_batches):
        x = torch.randint(0, 38, (6, 33), generator=g)
        y = torch.randint(0, 38, (6, 33), generator=g)
        batches.append((x.cuda(), torch.zeros(6, dtype=torch.long).cuda(), y.cuda()))
    params, steps = [], []
    for graphs in (False, True):
        torch.manual_seed(0)
        m = MyTransformerDecoder(**kw).cuda().train()
        m.switch_to_generate()
        tr = Trainer(gradient_clip_val=0.8, accumulate_grad_batches=5, max_epochs=3, log_every_n_steps=1,
                     hip_graphs=graphs)
        with operands(torch.float32):
            tr.fit(m, train_dataloaders=batches)
        torch.cuda.synchronize()
        steps.append(tr.global_step)
        params.append({n: p.detach().clone() for n, p in m.named_parameters()})
    assert steps == [9, 9]
    assert tr._graphs.G == 5 and tr._graphs.static is not None
    for n, p0 in params[0].items():
        torch.testing.assert_close(params[1][n], p0, rtol=1e-4, atol=1e-6, msg=n)


@pytest.mark.parametrize("task", ["generate", "classification"])
def test_grouped_accumulation_equals_micro_batch_sum(task):
    """fused_train_step(groups=5) on the five micro-batches side by side (arcweld/decoder.py fused_step, what the
    captured accumulation step runs) == five fused_train_step calls accumulating into the same gradients, each
    micro-batch with its own valid-token count (ignore_index rows differ per micro-batch here); fp32 operands,
    no dropout: the same per-token math, only the weight-gradient reduction order differs."""
    from arcweld.precision import operands
    from model.transformer_decoder import MyTransformerDecoder
    torch.manual_seed(0)
    kw = dict(d_model=128, n_classes=40, seq_len=33, n_blocks=2, n_head=4, res_dropout=0.0, att_dropout=0.0)
    m = MyTransformerDecoder(**kw).cuda().train()
    (m.switch_to_generate if task == "generate" else m.switch_to_classification)()
    g = torch.Generator(device="cpu").manual_seed(5)
    mbs = []
    for j in range(5):
        x = torch.randint(0, 38, (6, 33), generator=g)
        y = torch.randint(0, 38, (6, 33), generator=g)
        y[:, 33 - 3 * j:] = -1                       # a different number of ignored targets per micro-batch
        cond = torch.randint(0, 2, (6,), generator=g)
        if task == "classification":
            cond[: j % 3] = -100
        mbs.append((x.cuda(), cond.cuda(), y.cuda()))
    grads, losses = [], []
    with operands(torch.float32):
        for grouped in (False, True):
            m.zero_grad(set_to_none=True)
            if grouped:
                cat = tuple(torch.cat([b[i] for b in mbs], 0) for i in range(3))
                losses.append(float(m.fused_train_step(cat, 0.2, groups=5)))
            else:
                losses.append(sum(float(m.fused_train_step(b, 0.2)) for b in mbs) / 5)
            torch.cuda.synchronize()
            grads.append({n: p.grad.detach().clone() for n, p in m.named_parameters() if p.grad is not None})
    assert abs(losses[0] - losses[1]) <= 1e-5 * abs(losses[0])
    assert grads[0].keys() == grads[1].keys()
    for n, g0 in grads[0].items():
        torch.testing.assert_close(grads[1][n], g0, rtol=1e-5, atol=1e-7, msg=n)
