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
    third is captured and replayed (the forward/backward graph once per micro-batch, then the captured clip + RAdam),
    so stage 0's last optimizer step comes from the graphs; the captured clip reports no norm to Python."""
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
