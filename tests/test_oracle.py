"""Pin the CPU oracle (oracle/fen_oracle.py) against the reference's own outputs.

The fixtures were produced by importing the reference (tests/golden/make_golden.py);
the oracle is an independent restatement, so agreement here is what licenses using it
as the checker for the HIP path.
"""
import numpy as np
import pytest
import torch

from oracle import fen_oracle as O

pytestmark = pytest.mark.filterwarnings("ignore::UserWarning")


def _params(d, prefix="p/"):
    return {k[len(prefix):]: torch.from_numpy(v) for k, v in d.items() if k.startswith(prefix)}


def test_bicubic_up_kat(golden):
    g = golden("g3_kat.npz")
    x = torch.from_numpy(g["up_in"])
    for s in (2, 4, 8):
        y = O.bicubic(x.double(), s).float()
        np.testing.assert_allclose(y.numpy(), g[f"up_x{s}"], rtol=0, atol=2e-6)


def test_bicubic_down_kat(golden):
    g = golden("g3_kat.npz")
    y = O.lr_from_hr(torch.from_numpy(g["down_in"]).double()).float()
    np.testing.assert_allclose(y.numpy(), g["down_x4"], rtol=0, atol=2e-6)


def test_pixel_shuffle_kat(golden):
    g = golden("g3_kat.npz")
    y = O.pixel_shuffle(torch.from_numpy(g["ps_in"]), 2)
    np.testing.assert_array_equal(y.numpy(), g["ps_out"])


def test_rcab_fwd_bwd(golden):
    g = golden("g2_rcab.npz")
    p = _params(g)
    out, dx, gp = O.rcab_with_grads(p, torch.from_numpy(g["x"]), torch.from_numpy(g["r"]))
    np.testing.assert_allclose(out.numpy(), g["out"], rtol=0, atol=1e-5)
    np.testing.assert_allclose(dx.numpy(), g["dx"], rtol=0, atol=1e-4)
    for k, v in gp.items():
        ref = g["g/" + k]
        np.testing.assert_allclose(v.numpy(), ref, rtol=1e-4, atol=1e-4 * np.abs(ref).max())


def test_config1_forward(golden):
    g = golden("g1_config1.npz")
    p = _params(g)
    shape = O.NetShape(64, 1, 2, 4, 4, 0.2)
    lr = torch.from_numpy(g["lr"])
    np.testing.assert_allclose(O.lr_from_hr(torch.from_numpy(g["hr"])).numpy(), g["lr"], atol=2e-6)
    attn = {}
    out_t = O.forward(p, lr, shape, training=True)
    out_e = O.forward(p, lr, shape, training=False, attn=attn)
    np.testing.assert_allclose(out_t.numpy(), g["out_train"], rtol=0, atol=1e-5)
    np.testing.assert_allclose(out_e.numpy(), g["out_eval"], rtol=0, atol=1e-5)
    for k, v in attn.items():
        np.testing.assert_allclose(v.numpy(), g["attn/" + k], rtol=0, atol=1e-6)


def test_config1_grads_and_step(golden):
    g = golden("g1_config1.npz")
    p = _params(g)
    shape = O.NetShape(64, 1, 2, 4, 4, 0.2)
    hr = torch.from_numpy(g["hr"])
    loss, grads = O.l1_grads(p, hr, shape)
    assert abs(loss - float(g["l1_loss"])) < 1e-6
    for k, v in grads.items():
        ref = g["g/" + k]
        scale = max(np.abs(ref).max(), 1e-12)
        np.testing.assert_allclose(v.numpy(), ref, rtol=0, atol=1e-4 * scale, err_msg=k)
    loss2, newp = O.train_step(p, hr, shape, lr=1e-4, clip=0.5)
    assert abs(loss2 - float(g["step_loss"])) < 1e-6
    for k, v in newp.items():
        np.testing.assert_allclose(v.numpy(), g["s/" + k], rtol=0, atol=2e-7, err_msg=k)


def test_g9_north_star_shape(golden):
    """The oracle at the north-star shape (6x10, 64x64 -> 256x256, B=2, smooth HR) vs the
    reference's own fp32 outputs and its float64 PSNR."""
    import math
    from src_models_seed import seeded_full_params
    g = golden("g9_full64.npz")
    p = seeded_full_params(g)
    shape = O.NetShape(64, 6, 10, 4, 4, 0.2)
    hr = torch.from_numpy(g["hr_u8"].astype(np.float32) / np.float32(255.0))
    lr = O.lr_from_hr(hr)
    np.testing.assert_allclose(lr.numpy(), g["lr"], rtol=0, atol=2e-6)
    out_e = O.forward(p, torch.from_numpy(g["lr"]), shape, training=False)
    out_t = O.forward(p, torch.from_numpy(g["lr"]), shape, training=True)
    np.testing.assert_allclose(out_e.numpy(), g["out_eval"], rtol=0, atol=1e-5)
    np.testing.assert_allclose(out_t.numpy(), g["out_train"], rtol=0, atol=1e-5)
    assert math.isclose(O.psnr(out_e, hr), float(g["psnr_eval_f64"]), abs_tol=1e-4)


def test_bf16_weight_rounding_alone_exceeds_001db(golden):
    """Why bf16 cannot carry the north star's 0.01 dB on this network:
    on g9 (6x10, 64x64 -> 256x256, HR target) rounding ONLY the conv / FC weights (>= 2-D) to
    bf16, activations and arithmetic fp32, already moves the reference network's PSNR by more
    than 0.01 dB; the same rounding to fp16 moves it by less than 0.002 dB -- so fp16 is the
    parity precision and the bf16 gate is 0.02 dB (test_gpu_northstar.py)."""
    from src_models_seed import seeded_full_params
    g = golden("g9_full64.npz")
    p = seeded_full_params(g)
    lr = torch.from_numpy(g["lr"])
    hr = torch.from_numpy(g["hr_u8"].astype(np.float32) / np.float32(255.0))
    shape = O.NetShape(64, 6, 10, 4, 4, 0.2)
    with torch.no_grad():
        base = O.psnr(O.forward(p, lr, shape, training=False), hr)
        d = {}
        for name, dt in (("bf16", torch.bfloat16), ("fp16", torch.float16)):
            pr = {k: (v.to(dt).float() if v.dim() >= 2 else v) for k, v in p.items()}
            d[name] = O.psnr(O.forward(pr, lr, shape, training=False), hr) - base
    print(d)
    assert abs(d["bf16"]) > 0.01, d
    assert abs(d["fp16"]) < 0.002, d
