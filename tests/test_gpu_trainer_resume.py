"""The generator has ONE AdamW state across the Trainer's step paths and across a resume
(reference: one torch.optim.AdamW for the whole run, trainer.py:217-221, saved and restored
with the discriminator and its optimizer, trainer.py:701-760).

Fused L1 engine steps (epoch 0), then stage-3 GAN steps on the module path (epoch >= 1), a
checkpoint, and a resume into a fresh Trainer whose first step is a GAN step (and, in a second
resume, a fused step): after every step the generator's parameters equal a single torch AdamW
(float64, clip_grad_norm_ semantics) fed the same gradients -- read from the trainer's gradient
buffers just before each update -- so the moments and the step count carry from one path to
the other and through the checkpoint."""
import copy

import pytest
import torch
import torch.nn as nn

pytestmark = pytest.mark.gpu
DEV = "cuda"
LR, WD, CLIP = 2e-3, 1e-2, 0.5


def _gen(seed):
    from src.models import FaceEnhanceNet
    torch.manual_seed(seed)
    m = FaceEnhanceNet(num_channels=64, num_groups=1, blocks_per_group=2, precision="fp32")
    with torch.no_grad():
        m.conv_last.weight.mul_(30.0)
    return m


def _trainer(m, D, tmp_path, gan_start):
    from src.models import GANLoss
    from src.training import Trainer, TrainerConfig
    cfg = TrainerConfig(learning_rate=LR, weight_decay=WD, gradient_clip=CLIP, gan_weight=0.05, gan_start_epoch=gan_start,
                        d_learning_rate=1e-4, d_weight_decay=0.0, use_wandb=False, scheduler_type="none",
                        checkpoint_dir=str(tmp_path))
    return Trainer(m, [], None, loss_fn=nn.L1Loss(), config=cfg, discriminator=D, gan_loss=GANLoss("vanilla"))


class Recorder:
    """The gradient each update consumes, read from the buffer it reads (in stream order)."""

    def __init__(self, monkeypatch):
        from src.training import optim
        self.grads = []
        orig = optim.FusedAdamW.step

        def step(opt):
            self.grads.append(("module", opt.flat_g.detach().clone()))
            return orig(opt)
        monkeypatch.setattr(optim.FusedAdamW, "step", step)

    def watch(self, eng):
        run = eng.upd.run

        def upd_run(*a):
            self.grads.append(("fused", eng.flat_g.detach().clone()))
            return run(*a)
        eng.upd.run = upd_run


class TorchAdamW:
    """The reference optimizer over the flat arena in float64 (clip_grad_norm_ then AdamW)."""

    def __init__(self, flat):
        self.p = nn.Parameter(flat.detach().double().cpu().clone())
        self.opt = torch.optim.AdamW([self.p], lr=LR, weight_decay=WD, eps=1e-8)

    def step(self, g):
        g = g.double().cpu()
        coef = min(CLIP / (float(g.norm()) + 1e-6), 1.0)
        self.p.grad = g * coef
        self.opt.step()


def _batches(n, seed):
    gen = torch.Generator().manual_seed(seed)
    return [{"hr": torch.rand(2, 3, 128, 128, generator=gen)} for _ in range(n)]


def _close(flat, ref, what):
    d = float((flat.double().cpu() - ref.p.detach()).abs().max())
    assert d <= 2e-6, (what, d)


def test_fused_then_gan_then_resume_is_one_adamw(tmp_path, monkeypatch):
    from src.models import VGGStyleDiscriminator
    rec = Recorder(monkeypatch)
    torch.manual_seed(3)
    D = VGGStyleDiscriminator(input_size=128, precision="fp32")
    D0 = copy.deepcopy(D.state_dict())
    tr = _trainer(_gen(1), D, tmp_path, gan_start=1)
    ref = TorchAdamW(tr.model._fen_flat)
    rec.watch(tr.engine(2, 128, 128))
    # epoch 0: two fused engine steps; epoch 1: two GAN steps on the module path
    for epoch, seed in ((0, 10), (1, 11)):
        tr.current_epoch = epoch
        tr.train_loader = _batches(2, seed)
        tr._train_epoch()
        torch.cuda.synchronize()
    assert [k for k, _ in rec.grads] == ["fused", "fused", "module", "module"]
    for _, g in rec.grads:
        ref.step(g)
    _close(tr.model._fen_flat, ref, "after fused + GAN steps")
    osd = tr._optimizer_state()
    assert int(osd["state"][0]["step"]) == 4
    tr._save_checkpoint("ck.pth")
    ck = torch.load(tmp_path / "ck.pth", map_location="cpu", weights_only=True)
    assert "discriminator_state_dict" in ck and "optimizer_d_state_dict" in ck
    d_sd = {k: v.detach().cpu().clone() for k, v in tr.discriminator.state_dict().items()}
    assert any(not torch.equal(d_sd[k], D0[k]) for k in d_sd)       # D was trained
    ref_state = copy.deepcopy(ref.opt.state_dict()), ref.p.detach().clone()

    for first, gan_start in (("module", 0), ("fused", 100)):
        rec.grads.clear()
        torch.manual_seed(4)
        D2 = VGGStyleDiscriminator(input_size=128, precision="fp32")
        tr2 = _trainer(_gen(7), D2, tmp_path, gan_start=gan_start)      # different init: all of it comes from ck
        tr2.load_checkpoint(str(tmp_path / "ck.pth"))
        for k, v in tr2.discriminator.state_dict().items():
            assert torch.equal(v.cpu(), d_sd[k]), k
        assert tr2.optimizer_d.state_dict()["state"][0]["step"] == tr.optimizer_d.state_dict()["state"][0]["step"]
        r2 = TorchAdamW(tr2.model._fen_flat)
        _close(tr2.model._fen_flat, ref, "resumed weights")
        r2.opt.load_state_dict(copy.deepcopy(ref_state[0]))   # load_state_dict keeps the tensors
        if first == "fused":
            rec.watch(tr2.engine(2, 128, 128))
        tr2.current_epoch = 2
        tr2.train_loader = _batches(1, 12)
        tr2._train_epoch()
        torch.cuda.synchronize()
        assert [k for k, _ in rec.grads] == [first]
        r2.step(rec.grads[0][1])
        _close(tr2.model._fen_flat, r2, f"first step after resume ({first})")
        assert int(tr2._optimizer_state()["state"][0]["step"]) == 5


def test_gan_capture_after_resume_from_noncapturable_optimizer_d(tmp_path):
    """A stage-3 checkpoint whose optimizer_d was saved with capturable=False and CPU step counts
    (the reference trainer's, a DP run's or a capture_gan_step=False run's) resumes into a
    capturing trainer: the restored param groups are made capturable again, so the third GAN
    iteration after the resume captures optimizer_d.step() and the later ones replay it."""
    from src.models import VGGStyleDiscriminator
    torch.manual_seed(3)
    D = VGGStyleDiscriminator(input_size=128, precision="fp32")
    tr = _trainer(_gen(1), D, tmp_path, gan_start=0)
    tr.config.capture_gan_step = False
    for g in tr.optimizer_d.param_groups:
        g["capturable"] = False
    tr.train_loader = _batches(1, 20)
    tr._train_epoch()
    torch.cuda.synchronize()
    osd = tr.optimizer_d.state_dict()
    assert not osd["param_groups"][0]["capturable"]
    tr._save_checkpoint("noncap.pth")
    torch.manual_seed(4)
    tr2 = _trainer(_gen(7), VGGStyleDiscriminator(input_size=128, precision="fp32"), tmp_path, gan_start=0)
    tr2.load_checkpoint(str(tmp_path / "noncap.pth"))
    assert all(g["capturable"] for g in tr2.optimizer_d.param_groups)
    assert all(st["step"].is_cuda for st in tr2.optimizer_d.state.values())
    tr2.train_loader = _batches(4, 21)          # 2 eager, then capture, then a replay
    tr2._train_epoch()
    torch.cuda.synchronize()
    assert tr2._gan_graph is not None
    flat = tr2.model._fen_flat
    assert bool(torch.isfinite(flat).all())
