"""The stage-3 GAN iteration replayed from a captured hipGraph (TrainerConfig.capture_gan_step)
equals the eager iteration bit for bit: losses, generator arena, discriminator parameters and
BatchNorm running statistics, across the two eager warm-ups, the capture, replays, and a
re-capture after a learning-rate change (reference iteration: trainer.py:424-485)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _trainer(capture, tmp_path):
    from src.models import FaceEnhanceNet, GANLoss, VGGStyleDiscriminator
    from src.training import Trainer, TrainerConfig
    torch.manual_seed(1)
    G = FaceEnhanceNet(num_channels=64, num_groups=1, blocks_per_group=2, precision="bf16")
    torch.manual_seed(2)
    D = VGGStyleDiscriminator(input_size=128, precision="bf16")
    cfg = TrainerConfig(learning_rate=2e-4, weight_decay=1e-2, gradient_clip=0.5, gan_weight=0.05,
                        d_learning_rate=1e-4, use_wandb=False, scheduler_type="none",
                        checkpoint_dir=str(tmp_path), capture_gan_step=capture)
    tr = Trainer(G, [], None, loss_fn=torch.nn.L1Loss(), config=cfg, discriminator=D, gan_loss=GANLoss("vanilla"))
    # the same AdamW form on both sides (capturable keeps its step count on the device and
    # orders the bias-correction arithmetic differently from the host-step form)
    for g in tr.optimizer_d.param_groups:
        g["capturable"] = True
    return tr


def _state(tr):
    return ([tr.model._fen_flat.clone()] + [p.detach().clone() for p in tr.discriminator.parameters()]
            + [b.clone() for b in tr.discriminator.buffers()])


def test_captured_gan_iteration_matches_eager(tmp_path):
    eager, cap = _trainer(False, tmp_path / "e"), _trainer(True, tmp_path / "c")
    gen = torch.Generator().manual_seed(5)
    batches = [torch.rand(2, 3, 128, 128, generator=gen).to(DEV) for _ in range(7)]
    for i, hr in enumerate(batches):
        if i == 5:                       # a new learning rate: the captured iteration is re-captured
            for tr in (eager, cap):
                for g in tr.optimizer.param_groups:
                    g["lr"] = 1e-4
        le = float(eager._gan_iteration(hr))
        lc = float(cap._gan_iteration(hr))
        assert le == lc, (i, le, lc)
        for a, b in zip(_state(eager), _state(cap)):
            assert torch.equal(a, b), i
    assert cap._gan_graph is not None and eager._gan_graph is None
    # the module path afterwards runs on the replayed updates (version counters bumped)
    x = torch.rand(2, 3, 32, 32, device=DEV)
    with torch.no_grad():
        cap.model.eval()
        eager.model.eval()
        assert torch.equal(cap.model(x), eager.model(x))


def test_frozen_d_in_g_step_same_updates(tmp_path):
    """TrainerConfig.freeze_d_in_g_step (default): the generator step's pass through D computes
    only D's data gradients -- the reference also computes D's parameter gradients there and never
    uses them (optimizer_d has stepped; its next zero_grad drops them).  Every update is the
    same bit for bit as with the dead work done, eager and captured; D's .grad after an
    iteration holds the D step's gradients alone."""
    ref = _trainer(False, tmp_path / "r")
    ref.config.freeze_d_in_g_step = False
    frz, cap = _trainer(False, tmp_path / "f"), _trainer(True, tmp_path / "c")
    gen = torch.Generator().manual_seed(9)
    for i in range(5):
        hr = torch.rand(2, 3, 128, 128, generator=gen).to(DEV)
        losses = [float(tr._gan_iteration(hr)) for tr in (ref, frz, cap)]
        assert losses[0] == losses[1] == losses[2], (i, losses)
        for a, b, c in zip(_state(ref), _state(frz), _state(cap)):
            assert torch.equal(a, b) and torch.equal(a, c), i
    assert all(p.requires_grad for p in frz.discriminator.parameters())


def test_reused_g_forward_same_updates(tmp_path):
    """TrainerConfig.reuse_g_forward (default): the iteration's generator forward runs once and
    the D step takes it detached -- the reference runs the same forward twice (no_grad for the D
    step, with grad for the G step: same LR batch, same weights).  The training forward's output
    equals the no-grad forward's bit for bit, so every update is the same as with both passes."""
    a, b = _trainer(False, tmp_path / "a"), _trainer(False, tmp_path / "b")
    a.config.reuse_g_forward = False
    gen = torch.Generator().manual_seed(11)
    hr0 = torch.rand(2, 3, 128, 128, generator=gen).to(DEV)
    from src.training.trainer import bicubic_down4
    lr = bicubic_down4(hr0)
    with torch.no_grad():
        y0 = a.model(lr)
    y1 = a.model(lr)
    torch.cuda.synchronize()
    assert torch.equal(y0, y1.detach())
    for i in range(4):
        hr = torch.rand(2, 3, 128, 128, generator=gen).to(DEV)
        la, lb = float(a._gan_iteration(hr)), float(b._gan_iteration(hr))
        assert la == lb, (i, la, lb)
        for x, y in zip(_state(a), _state(b)):
            assert torch.equal(x, y), i
