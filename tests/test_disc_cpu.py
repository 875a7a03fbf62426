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
