"""Persistent weight operands kept current by the optimizer (arcweld/operands.py, aw_radam_step_ops): the update
kernel's cast copies equal a fresh aw_weight_relayout_batch of the updated weights (every relayout mode the step
uses, bf16 and fp32 operands, H = 64 and the configs[1] width H = 512), training with them follows the per-forward
relayout trajectory (to the run-to-run noise of the weight-gradient atomics), and a maintained step issues no relayout launch."""
import pytest
import torch

from oracle import gen
from test_vqvae_module import make_model

pytestmark = pytest.mark.gpu
KW = dict(hidden_dim=64, num_embeddings=64, embedding_dim=16, n_resblocks=2, patch_size=25)


def _train(attach, T, steps=3, monkeypatch=None):
    from arcweld import kernels as K
    from arcweld.precision import operands as prec
    from arcweld.trainer import Trainer
    from arcweld.optim import RAdam
    m = make_model(KW, 331, "cuda", dropout=0.1).train()
    if not attach:
        monkeypatch.setattr(RAdam, "attach_operands", lambda self, opset: False)
    calls = []
    orig = K.weight_relayout_batch
    monkeypatch.setattr(K, "weight_relayout_batch", lambda jobs, **kw: calls.append(len(jobs)) or orig(jobs, **kw))
    with prec(T):
        tr = Trainer(gradient_clip_val=0.7)
        tr.setup_optimizer(m)
        for i in range(steps):
            x = torch.tensor(gen.windows(340 + i, 16), device="cuda")
            tr.micro_step(m, x, 0, 1.0)
            tr.optimizer_step(m)
    return m, calls


@pytest.mark.parametrize("T", [torch.bfloat16, torch.float32])
def test_maintained_operands_follow_the_relayout_trajectory(T, monkeypatch):
    m0, calls0 = _train(False, T, monkeypatch=monkeypatch)
    monkeypatch.undo()
    m1, calls1 = _train(True, T, monkeypatch=monkeypatch)
    s0, s1 = m0.state_dict(), m1.state_dict()
    for k in s0:   # same arithmetic; the weight-gradient atomics (<= 2 adders) make runs differ in the last bits
        torch.testing.assert_close(s1[k].float(), s0[k].float(), rtol=1e-5, atol=1e-6, msg=k)
    assert len(calls0) >= 3            # unmaintained: one relayout per forward
    assert len(calls1) == 1            # maintained: only the first forward (flatten moved the weights)


@pytest.mark.parametrize("T,H", [(torch.bfloat16, 64), (torch.float32, 64), (torch.bfloat16, 512)])
def test_update_kernel_copies_equal_a_fresh_relayout(T, H):
    from arcweld import kernels as K
    from arcweld import operands
    from arcweld.precision import operands as prec
    from arcweld.trainer import Trainer
    from model.vq_vae_patch_embedd import VQVAEPatch
    kw = dict(KW, hidden_dim=H)
    m = VQVAEPatch(input_dim=2, learning_rate=1e-3, dropout_p=0.0, batch_norm=False, **kw).cuda().train()
    with prec(T):
        tr = Trainer(gradient_clip_val=0.7)
        tr.setup_optimizer(m)
        st = m.operand_set()
        assert st.maintained
        for i in range(2):
            x = torch.tensor(gen.windows(350 + i, 8), device="cuda")
            tr.micro_step(m, x, 0, 1.0)
            tr.optimizer_step(m)
        torch.cuda.synchronize()
        names = [j.name for j in st.jobs]
        assert sum(n.startswith("enc") for n in names) == 2 * KW["n_resblocks"]
        fresh = [operands.OperandJob(j.name, j.param, j.O, j.I, j.k, j.tap, j.mode, torch.zeros_like(j.out),
                                     j.ldo, derive=j.derive) for j in st.jobs]
        K.weight_relayout_batch([j.relayout_job() for j in fresh])
        for j, f in zip(st.jobs, fresh):
            assert torch.equal(j.out, f.out), (j.name, j.mode)
        # the decoder convs are stored tap-major by the Trainer: check their copies against torch permutes of the
        # parameter itself (independent of both the relayout and the update kernel's index maps)
        dec = [j for j in st.jobs if j.name.startswith(("dec", "dgw"))]
        assert dec and all(not j.param.is_contiguous() for j in dec)
        for j in dec:
            W = j.param.detach()
            want = W.permute(0, 2, 1).reshape(j.O, 3 * j.I) if j.name.startswith("dec") else \
                W.permute(2, 0, 1).reshape(3 * j.O, j.I)
            assert torch.equal(j.out, want.to(j.out.dtype)), j.name


def test_outside_weight_change_triggers_a_refresh():
    from arcweld import kernels as K
    from arcweld.trainer import Trainer
    m = make_model(KW, 332, "cuda").train()
    tr = Trainer(gradient_clip_val=0.7)
    tr.setup_optimizer(m)
    x = torch.tensor(gen.windows(360, 8), device="cuda")
    tr.micro_step(m, x, 0, 1.0)
    tr.optimizer_step(m)
    st = m.operand_set()
    with torch.no_grad():
        m.decoder[0].weight.mul_(0.5)          # bumps the version counter
    n = []
    orig = K.weight_relayout_batch
    K.weight_relayout_batch = lambda jobs, **kw: n.append(1) or orig(jobs, **kw)
    try:
        tr.micro_step(m, x, 0, 1.0)
    finally:
        K.weight_relayout_batch = orig
    assert n == [1]
    w = st.out["Wd0"]
    torch.testing.assert_close(w.float(), m.decoder[0].weight[:, :, 0].float().to(w.dtype).float())


@pytest.mark.parametrize("T", [torch.bfloat16, torch.float32])
def test_forward_before_optimizer_then_fit_then_load_state_dict(T):
    """An operand set built by a forward BEFORE the optimizer re-stores the weights (flat buffer, centre-tap and
    tap-major views) follows the parameters' new storage: forward -> Trainer steps -> forward equals a fresh model
    with the trained weights, and a load_state_dict afterwards is picked up too (arcweld/operands.py derive)."""
    from arcweld.precision import operands as prec
    from arcweld.trainer import Trainer
    with prec(T):
        m = make_model(KW, 333, "cuda").train()
        x = torch.tensor(gen.windows(370, 8), device="cuda")
        with torch.no_grad():
            m.eval()
            m(x)                                     # builds the operand set on the reference layouts
            m.train()
        tr = Trainer(gradient_clip_val=0.7)
        tr.setup_optimizer(m)
        for i in range(2):
            tr.micro_step(m, torch.tensor(gen.windows(371 + i, 8), device="cuda"), 0, 1.0)
            tr.optimizer_step(m)

        def eval_out(model):
            with torch.no_grad():
                model.eval()
                out = model(x)[1]
                model.train()
            return out

        ref = make_model(KW, 333, "cuda")
        ref.load_state_dict(m.state_dict())
        torch.testing.assert_close(eval_out(m), eval_out(ref), rtol=0, atol=0)
        other = make_model(KW, 334, "cuda")
        m.load_state_dict(other.state_dict())
        torch.testing.assert_close(eval_out(m), eval_out(other), rtol=0, atol=0)
