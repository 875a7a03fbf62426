"""Data-parallel host logic on CPU (gloo, world size 2) -- SURVEY.md §8e.

The engine's DP step is: per-rank shard -> loss gradient pre-scaled by 1/world ->
bucketed async SUM all-reduce of the flat gradient arena in backward order
(src/training/dp.py) -> clip + AdamW on identical data.  Here the per-rank gradients come
from the CPU oracle (the checker; the GPU kernels are covered by the -m gpu tests), the
exchange is the product's own BucketExchange over gloo, and the result must equal the
reference's single-process step on the global batch (golden g1: reference
Trainer._train_epoch, B=2, AdamW lr 1e-4, clip 0.5).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import fen_oracle as O
from src.training.dp import BucketExchange, broadcast_arena, bucket_plan, model_bucket_plan

pytestmark = pytest.mark.filterwarnings("ignore::UserWarning")
SHAPE1 = O.NetShape(64, 1, 2, 4, 4, 0.2)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _golden_params(g):
    return {k[2:]: torch.from_numpy(v) for k, v in g.items() if k.startswith("p/")}


# ------------------------------------------------------------------ plan (no processes)
@pytest.mark.parametrize("kw", [dict(num_groups=6, blocks_per_group=10), dict(num_groups=1, blocks_per_group=2),
                                dict(num_groups=3, blocks_per_group=4, scale_factor=8)])
def test_bucket_plan_tiles_arena(kw):
    from src.models import FaceEnhanceNet
    m = FaceEnhanceNet(**kw)
    plan = model_bucket_plan(m)
    G = kw["num_groups"]
    assert [t for t, _, _ in plan] == ["tail"] + [f"rg{g}" for g in reversed(range(G))] + ["head"]
    spans = sorted((lo, hi) for _, lo, hi in plan)
    assert spans[0][0] == 0 and spans[-1][1] == sum(p.numel() for p in m.parameters())
    assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
    # every parameter lands in the bucket of its own layer
    off = 0
    where = {t: (lo, hi) for t, lo, hi in plan}
    for name, p in m.named_parameters():
        tag = "head" if name.startswith("conv_first") else (
            "rg" + name.split(".")[1] if name.startswith("residual_groups") else "tail")
        lo, hi = where[tag]
        assert lo <= off and off + p.numel() <= hi, name
        off += p.numel()


def test_bucket_plan_rejects_interleaved_order():
    with pytest.raises(ValueError):
        bucket_plan([("conv_first.weight", 4), ("residual_groups.0.conv.weight", 4), ("conv_last.weight", 2),
                     ("residual_groups.0.conv.bias", 1)], 1)
    with pytest.raises(ValueError):
        bucket_plan([("conv_first.weight", 4), ("conv_last.weight", 2)], 1)


def test_exchange_is_noop_single_process():
    flat = torch.arange(10.0)
    ex = BucketExchange(flat, [("tail", 0, 4), ("rg0", 4, 8), ("head", 8, 10)])
    for t in ("tail", "rg0", "head"):
        ex.launch(t)
    ex.wait()
    assert torch.equal(flat, torch.arange(10.0))


# ------------------------------------------------------------------ gloo, world size 2
def _worker(rank, world, port, g, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(2)
    try:
        p = _golden_params(g)
        names = list(p)  # npz order == the reference's named_parameters() order
        plan = bucket_plan(((n, p[n].numel()) for n in names), SHAPE1.num_groups)
        n_total = sum(p[n].numel() for n in names)

        # identical start: rank 1 holds garbage until rank 0's arena is broadcast
        flat_p = torch.cat([p[n].reshape(-1) for n in names]).clone()
        if rank:
            flat_p.normal_()
        broadcast_arena(flat_p, src=0)
        assert torch.equal(flat_p, torch.cat([p[n].reshape(-1) for n in names]))

        # this rank's shard of the global batch; loss grad pre-scaled by 1/world
        hr = torch.from_numpy(g["hr"]).chunk(world)[rank]
        loss, grads = O.l1_grads(p, hr, SHAPE1)
        flat_g = torch.cat([grads[n].reshape(-1) / world for n in names])
        assert flat_g.numel() == n_total
        ex = BucketExchange(flat_g, plan)
        for tag, _, _ in plan:  # backward order: tail, rg0, head
            ex.launch(tag)
        ex.wait()

        # clip + AdamW on the exchanged (identical) gradients
        off, gsum = 0, {}
        for n in names:
            k = p[n].numel()
            gsum[n] = flat_g[off:off + k].view_as(p[n])
            off += k
        c = O.clip_coef(gsum, 0.5)
        newp = {k: v.clone() for k, v in p.items()}
        m = {k: torch.zeros_like(v) for k, v in p.items()}
        v = {k: torch.zeros_like(t) for k, t in p.items()}
        O.adamw_step(newp, {k: t * c for k, t in gsum.items()}, m, v, 1, 1e-4)
        np.savez(os.path.join(out_dir, f"rank{rank}.npz"), flat_g=flat_g.numpy(),
                 newp=torch.cat([newp[n].reshape(-1) for n in names]).numpy(), loss=np.float64(loss))
    finally:
        dist.destroy_process_group()


def test_dp_step_world2_matches_reference_global_step(golden, tmp_path):
    g = golden("g1_config1.npz")
    mp.spawn(_worker, args=(2, _free_port(), g, str(tmp_path)), nprocs=2, join=True)
    r0, r1 = (np.load(tmp_path / f"rank{r}.npz") for r in (0, 1))
    # every rank ends the exchange with bit-identical gradients and parameters
    np.testing.assert_array_equal(r0["flat_g"], r1["flat_g"])
    np.testing.assert_array_equal(r0["newp"], r1["newp"])
    # the mean of the shard losses is the global-batch loss
    assert abs(0.5 * (float(r0["loss"]) + float(r1["loss"])) - float(g["l1_loss"])) < 1e-6
    # summed 1/world-scaled shard grads == the reference's global-batch grads
    p = _golden_params(g)
    ref_g = np.concatenate([g["g/" + n].reshape(-1) for n in p])
    np.testing.assert_allclose(r0["flat_g"], ref_g, rtol=0, atol=1e-4 * np.abs(ref_g).max())
    # and the step lands on the reference Trainer's post-step parameters
    ref_s = np.concatenate([g["s/" + n].reshape(-1) for n in p])
    np.testing.assert_allclose(r0["newp"], ref_s, rtol=0, atol=2e-7)


# ------------------------------------------------------------------ validation metrics under DP
def _val_worker(rank, world, port, out_dir):
    """Two ranks validate different shards (different batch counts and values); after the
    reduce both hold the global batch means, so EarlyStopping / plateau decide alike."""
    from src.training.trainer import EarlyStopping, reduce_val_metrics
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # per-epoch shard sums: rank 0 sees 3 batches, rank 1 sees 2; rank 1's PSNR improves, rank 0's does not
        shards = {0: [(3.0, 90.0, 2.4, 3), (3.0, 89.0, 2.4, 3), (3.0, 88.0, 2.4, 3), (3.0, 87.0, 2.4, 3)],
                  1: [(2.0, 50.0, 1.6, 2), (2.0, 56.0, 1.6, 2), (2.0, 62.0, 1.6, 2), (2.0, 68.0, 1.6, 2)]}
        es = EarlyStopping(patience=2, mode="max")
        stops, metrics = [], []
        for tl, tp, ts, n in shards[rank]:
            m = reduce_val_metrics(tl, tp, ts, n, world)
            metrics.append(m["psnr"])
            stops.append(bool(es(m["psnr"])))
        np.savez(os.path.join(out_dir, f"val{rank}.npz"), psnr=np.array(metrics), stops=np.array(stops))
    finally:
        dist.destroy_process_group()


def test_val_metrics_reduced_across_ranks(tmp_path):
    mp.spawn(_val_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    r0, r1 = (np.load(tmp_path / f"val{r}.npz") for r in (0, 1))
    np.testing.assert_array_equal(r0["psnr"], r1["psnr"])
    np.testing.assert_array_equal(r0["stops"], r1["stops"])
    # global mean over all 5 batches of each epoch: (90 + 50) / 5, ...
    np.testing.assert_allclose(r0["psnr"], [28.0, 29.0, 30.0, 31.0])


# ------------------------------------------------------------------ module-path exchange
def _pge_worker(rank, world, port, out_dir):
    """ParamGradExchange over gloo: each rank back-propagates its shard of a global batch with
    the loss pre-scaled by 1/world; the buckets' hooks copy and all-reduce as the backward
    completes them; after wait() the flat buffer (and, with copy_back, every .grad) holds the
    global-batch gradient.  An unarmed backward exchanges nothing."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from src.training.dp import ParamGradExchange, even_buckets
        torch.manual_seed(0)
        net = torch.nn.Sequential(torch.nn.Linear(6, 5), torch.nn.Tanh(), torch.nn.Linear(5, 4), torch.nn.Tanh(),
                                  torch.nn.Linear(4, 3))
        ps = list(net.parameters())
        flat = torch.zeros(sum(p.numel() for p in ps))
        ex = ParamGradExchange(ps, flat, even_buckets(len(ps), 3), copy_back=True)
        assert ex.active and ex.world == world and len(ex.ranges) == 3
        x = torch.randn(8, 6, generator=torch.Generator().manual_seed(1))
        y = torch.randn(8, 3, generator=torch.Generator().manual_seed(2))
        shard = slice(rank * 4, rank * 4 + 4)
        # unarmed: hooks see the grads but launch nothing; flat stays zero
        loss = torch.nn.functional.mse_loss(net(x[shard]), y[shard])
        (loss / world).backward()
        assert float(flat.abs().sum()) == 0.0
        ex.wait()                                     # a no-op when not armed
        for p in ps:
            p.grad = None
        ex.arm()
        loss = torch.nn.functional.mse_loss(net(x[shard]), y[shard])
        (loss / world).backward()
        ex.wait()
        got = [p.grad.clone() for p in ps]
        for p in ps:
            p.grad = None
        torch.nn.functional.mse_loss(net(x), y).backward()   # the global batch, one process
        ref = [p.grad for p in ps]
        err = max(float((a - b).abs().max()) for a, b in zip(got, ref))
        torch.save({"err": err, "flat_ok": bool(torch.allclose(flat, torch.cat([r.reshape(-1) for r in ref]),
                                                                atol=1e-6))}, os.path.join(out_dir, f"pge{rank}.pt"))
    finally:
        dist.destroy_process_group()


def test_param_grad_exchange_world2(tmp_path):
    mp.spawn(_pge_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    for r in range(2):
        d = torch.load(tmp_path / f"pge{r}.pt", weights_only=True)
        assert d["err"] <= 1e-6 and d["flat_ok"], d


def test_even_buckets():
    from src.training.dp import even_buckets
    assert even_buckets(10, 3) == [(0, 3), (3, 7), (7, 10)]
    assert even_buckets(2, 5) == [(0, 1), (1, 2)]
    assert even_buckets(7, 1) == [(0, 7)]
