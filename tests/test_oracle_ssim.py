"""The oracle's SSIM / MS-SSIM restatement against the reference's own values
(tests/golden/g7_ssim.npz, made by importing src/losses/ssim_loss.py), on CPU."""
import numpy as np
import torch

from oracle import fen_oracle as O


def test_ssim_oracle_matches_reference(golden):
    g = golden("g7_ssim.npz")
    p, t = torch.from_numpy(g["pred"]), torch.from_numpy(g["target"])
    assert np.allclose(O.gaussian_window().numpy(), g["window"], rtol=0, atol=1e-9)
    assert abs(float(O.ssim(p, t)) - float(g["ssim_mean"])) <= 1e-6
    assert np.allclose(O.ssim(p, t, size_average=False).numpy(), g["ssim_per_img"], atol=1e-6)
    assert abs(float(O.ssim(p, p)) - float(g["ssim_same"])) <= 1e-6
    pr = p.clone().requires_grad_(True)
    loss = 1 - O.ssim(pr, t)
    loss.backward()
    assert abs(float(loss) - float(g["loss"])) <= 1e-6
    assert np.abs(pr.grad.numpy() - g["dpred"]).max() <= 1e-9 + 1e-5 * np.abs(g["dpred"]).max()
    p64, t64 = torch.from_numpy(g["pred64"]), torch.from_numpy(g["target64"])
    assert abs(float(O.ms_ssim(p64, t64)) - float(g["msssim"])) <= 1e-6
