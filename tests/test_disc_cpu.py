"""Discriminator host surface on CPU: seeded init identical to the reference (pinned by
tests/golden/g8_disc.npz statistics), module tree / keys, GANLoss values, no CPU path."""
import numpy as np
import pytest
import torch


def test_disc_init_and_gan_loss(golden):
    from src.models import GANLoss, VGGStyleDiscriminator, create_discriminator
    g = golden("g8_disc.npz")
    torch.manual_seed(0)
    d = VGGStyleDiscriminator(input_size=64)
    sd = d.state_dict()
    assert list(sd.keys()) == list(g["stat_names"])
    for n, s1, s2 in zip(g["stat_names"], g["stat_sum"], g["stat_sumsq"]):
        t = sd[n].double()
        assert abs(float(t.sum()) - s1) <= 1e-9 * max(1, abs(s1)) and abs(float((t * t).sum()) - s2) <= 1e-9 * max(1, s2), n
    assert create_discriminator().get_model_info()["total_params"] == 42_964_353
    o = torch.from_numpy(g["out_train"])
    assert abs(float(GANLoss("vanilla")(o, True)) - float(g["gan_vanilla_real"])) <= 1e-6
    assert abs(float(GANLoss("vanilla")(o, False)) - float(g["gan_vanilla_fake"])) <= 1e-6
    assert abs(float(GANLoss("lsgan")(o, True)) - float(g["gan_lsgan_real"])) <= 1e-6
    with pytest.raises(RuntimeError, match="no CPU path"):
        d(torch.rand(1, 3, 64, 64))


def test_oracle_disc_forward_pinned(golden):
    """oracle.disc_forward (the functional restatement the D256 gradient replay runs with the HIP
    discriminator's LeakyReLU branches) against the reference's own outputs in g8_disc.npz:
    train-mode scores in fp32 and float64, d(input), and every parameter gradient's norm and
    noise projection of sum(out * R) in float64."""
    from oracle import fen_oracle as O
    from src.models import VGGStyleDiscriminator
    g = golden("g8_disc.npz")
    torch.manual_seed(0)
    p = {k: v for k, v in VGGStyleDiscriminator(input_size=64).state_dict().items() if "running" not in k
         and "num_batches" not in k}
    x, r = torch.from_numpy(g["x"]), torch.from_numpy(g["r"])
    out32 = O.disc_forward(p, x)
    np.testing.assert_allclose(out32.detach().numpy(), g["out_train"], rtol=0, atol=2e-5)
    leaves = {k: v.double().requires_grad_(True) for k, v in p.items()}
    x64 = x.double().requires_grad_(True)
    rec = []
    o64 = O.disc_forward(leaves, x64, record=rec)
    np.testing.assert_allclose(o64.detach().numpy(), g["f64/out_train"], rtol=1e-10, atol=1e-12)
    (o64 * r.double()).sum().backward()
    np.testing.assert_allclose(x64.grad.numpy(), g["f64/gx"], rtol=1e-9, atol=1e-12)
    for k, v in leaves.items():
        assert abs(float(v.grad.norm()) - float(g["f64/gn/" + k])) <= 1e-9 * float(g["f64/gn/" + k]), k
        proj = float((v.grad * torch.randn(v.shape, generator=torch.Generator().manual_seed(7)).double()).sum())
        assert abs(proj - float(g["f64/gp/" + k])) <= 1e-8 * max(1.0, float(g["f64/gn/" + k])), k
    # replaying with the masks this run took is the same function
    o64m = O.disc_forward({k: v.detach() for k, v in leaves.items()}, x.double(), masks=rec)
    assert torch.equal(o64m, o64.detach())
