"""Full-network parity at the north-star shape (BASELINE.json: 64x64 -> 256x256, 6x10 RCAB,
64 ch), against the reference's own outputs (tests/golden/g9_full64.npz, made by importing the
reference: smooth uint8 HR, LR = the reference's bicubic /4).

  * fp32: max per-pixel |d| <= 1e-3 against the reference (north_star), eval and train mode;
  * 16-bit: PSNR against the same HR (trainer.py:621-628) within 0.01 dB of the
    reference's;
  * both on the module path (src.models, autograd Functions) and on the graph-replayed engine
    at the bench's batch (B=32: the golden's 2 images tiled 16x), so the persistent kernels run
    at the bench's tile counts.
"""
import numpy as np
import pytest
import torch

from oracle import fen_oracle as O
from src_models_seed import full_ctor, seeded_model

pytestmark = pytest.mark.gpu
DEV = "cuda"
PSNR_TOL_DB = 0.01           # north_star: PSNR parity to reference within 0.01 dB (fp16, the parity mode)
PIX_TOL_FP32 = 1e-3          # north_star: |d| <= 1e-3 fp32 per pixel
# bf16: 0.02 dB.  bf16's 8-bit mantissa cannot hold 0.01 dB on this network whatever the kernels
# do: rounding only the WEIGHTS to bf16 (activations fp32) already moves the reference's own
# PSNR by -0.0187 dB here (fp16: -0.0009; tests/test_oracle.py::
# test_bf16_weight_rounding_alone_exceeds_001db); the kernels measure -0.0125 dB.  fp16
# (3 more mantissa bits, same MFMA rate) lands at -0.0016 dB and carries the 0.01 dB gate.
PSNR_TOL_BF16_DB = 0.02

DTYPES = {"bf16": torch.bfloat16, "fp16": torch.float16, "fp32": torch.float32}


@pytest.fixture(scope="module")
def g9(golden):
    return golden("g9_full64.npz")


def _hr(g):
    return torch.from_numpy(g["hr_u8"].astype(np.float32) / np.float32(255.0))


def _check(out_e, g, precision, out_t=None):
    ref_e = torch.from_numpy(g["out_eval"])
    hr = _hr(g)
    B = ref_e.shape[0]
    out_e = out_e.cpu()
    if precision == "fp32":
        assert float((out_e - ref_e).abs().max()) <= PIX_TOL_FP32
        if out_t is not None:
            assert float((out_t.cpu() - torch.from_numpy(g["out_train"])).abs().max()) <= PIX_TOL_FP32
    else:
        d = O.psnr(out_e, hr[:B]) - O.psnr(ref_e, hr[:B])
        print(f"{precision}: dPSNR {d:+.5f} dB, max|d| {float((out_e - ref_e).abs().max()):.2e}")
        assert abs(d) <= (PSNR_TOL_BF16_DB if precision == "bf16" else PSNR_TOL_DB), d


@pytest.mark.parametrize("precision", ["fp32", "bf16", "fp16"])
def test_g9_module(g9, precision):
    m = seeded_model(full_ctor(precision), g9).to(DEV)
    lr = torch.from_numpy(g9["lr"]).to(DEV)
    with torch.no_grad():
        m.eval()
        out_e = m(lr).clone()
        m.train()
        out_t = m(lr).clone()
    _check(out_e, g9, precision, out_t)


@pytest.mark.parametrize("precision", ["fp32", "bf16", "fp16"])
def test_g9_engine_batch32(g9, precision):
    """The graph-replayed inference engine at the bench's batch: 32 images = the golden's 2
    images x 16; every copy must match the reference (and all copies are bit-identical)."""
    from src.hip.engine import FENEngine
    m = seeded_model(full_ctor(precision), g9).to(DEV).eval()
    lr = torch.from_numpy(g9["lr"])
    eng = FENEngine(m, batch=32, lr_hw=(64, 64), dtype=DTYPES[precision], train=False)
    eng.x.copy_(lr.repeat(16, 1, 1, 1).to(DEV))
    eng.capture()
    eng.replay()
    eng.replay()
    torch.cuda.synchronize()
    out = eng.out.cpu()
    for i in range(16):
        assert torch.equal(out[2 * i:2 * i + 2], out[:2]), i
    _check(out[:2], g9, precision)


@pytest.mark.parametrize("chunk", [8, 4])
def test_g9_engine_tail_chunks(g9, chunk, monkeypatch):
    """FEN_TAIL_CHUNK: the inference upsampler + conv_last over the batch in chunks (the
    activations stay in the Infinity Cache).  Images are independent, so the chunked engine's
    output is bit-identical to the one-pass engine's at B=32 (fp16), and still matches the
    reference."""
    from src.hip import net
    from src.hip.engine import FENEngine
    m = seeded_model(full_ctor("fp16"), g9).to(DEV).eval()
    x = torch.from_numpy(g9["lr"]).repeat(16, 1, 1, 1).to(DEV)
    outs = {}
    for c in (0, chunk):
        monkeypatch.setattr(net, "TAIL_CHUNK", c)
        eng = FENEngine(m, batch=32, lr_hw=(64, 64), dtype=torch.float16, train=False)
        ncv = sum(op[0] == "conv3x3" for op in eng.ctx.ops)
        outs.setdefault("ncv", []).append(ncv)
        eng.x.copy_(x)
        eng.capture()
        eng.replay()
        torch.cuda.synchronize()
        outs[c] = eng.out.cpu()
        del eng
    assert outs["ncv"][1] - outs["ncv"][0] == 3 * (32 // chunk - 1)   # 2 upsampler stages + conv_last per chunk
    assert torch.equal(outs[chunk], outs[0])
    _check(outs[chunk][:2], g9, "fp16")
