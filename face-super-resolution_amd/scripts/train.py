#!/usr/bin/env python
"""Training entry point with the reference's CLI and YAML surface (scripts/train.py:84-391).

Single GPU:   python scripts/train.py --config configs/stages/stage1_psnr_config.yaml --perceptual-weight 0
8 GPUs:       python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \\
                  scripts/train.py --config ... --perceptual-weight 0
Every reference flag and YAML key is parsed; new flags: --precision {fp32,bf16} and
--synthetic N (N seeded random HR images instead of a data directory; without it a missing
--data-root is an error).  loss.gan.weight > 0 builds the discriminator and GANLoss (stage 3).
"""
import argparse
import os
import random
import sys
from pathlib import Path
from typing import Optional

PKG = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(PKG))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
import yaml  # noqa: E402

from src.data import get_dataloader  # noqa: E402
from src.losses import create_loss_function  # noqa: E402
from src.models import create_face_enhance_net  # noqa: E402
from src.models.discriminator import GANLoss, create_discriminator  # noqa: E402
from src.training import Trainer, TrainerConfig, overfit_test  # noqa: E402


def load_config(path: str) -> dict:
    with open(path) as f:
        return yaml.safe_load(f)


def set_seed(seed: int) -> None:
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed_all(seed)


def resolve_precision(cli: Optional[str], tr_cfg: dict) -> str:
    """The compute precision.  The reference's `training.mixed_precision` (default true,
    scripts/train.py:300) means torch.cuda.amp fp16 autocast + GradScaler (trainer.py:18,227,460),
    which the HIP path does not restate: with it set, the precision must be chosen explicitly
    (--precision fp32 | bf16) rather than silently training in a different arithmetic.  The
    stage configs set mixed_precision: false -> fp32, the reference's own arithmetic."""
    if cli is not None:
        return cli
    if tr_cfg.get("mixed_precision", True):
        raise ValueError("training.mixed_precision is true (the reference's fp16 autocast + GradScaler, not "
                         "restated on the HIP path): pass --precision fp32 or --precision bf16 explicitly")
    return "fp32"


def create_model(model_type: str, config: dict, precision: str):
    if model_type != "custom":
        raise ValueError(f"model type {model_type!r}: only 'custom' (FaceEnhanceNet) is built on this MI355X path")
    mc = config.get("model", {}).get("custom", {})
    return create_face_enhance_net(num_channels=mc.get("num_channels", 64), num_groups=mc.get("num_groups", 3),
                                   blocks_per_group=mc.get("blocks_per_group", 4),
                                   reduction_ratio=mc.get("reduction_ratio", 4),
                                   scale_factor=mc.get("upscale_factor", 4), res_scale=mc.get("res_scale", 0.2),
                                   precision=precision)


def create_gan(config: dict, precision: str):
    """Stage 3 (reference scripts/train.py:335-351): the discriminator and GANLoss when
    loss.gan.weight > 0, else (None, None)."""
    gan = config.get("loss", {}).get("gan", {})
    if not gan.get("weight", 0.0) > 0:
        return None, None
    d = create_discriminator(input_size=config.get("data", {}).get("hr_size", 256),
                             base_channels=gan.get("d_channels", 64), use_bn=gan.get("d_use_bn", True),
                             precision=precision)
    return d, GANLoss(gan_type=gan.get("type", "vanilla"))


def train_loader_kwargs(config: dict) -> dict:
    """The train loader's augmentation keywords from the YAML, with the reference CLI's defaults
    (scripts/train.py:174-191): augmentation.random_crop.hr_patch_size (128),
    horizontal_flip (0.5), random_rotate90 (0.0), color_jitter.{probability 0.3, brightness 0.1,
    contrast 0.1, saturation 0.0, hue 0.0}.  Every one reaches get_dataloader, which applies it
    or raises (src/data)."""
    aug = config.get("augmentation", {}) or {}
    cj = aug.get("color_jitter", {}) or {}
    known = {"horizontal_flip", "random_rotate90", "random_crop", "color_jitter"}
    extra = sorted(set(aug) - known)
    if extra:
        raise ValueError(f"augmentation keys {extra} are not read by the reference's train.py either "
                         "(scripts/train.py:174-191): remove them")
    return dict(hr_patch_size=(aug.get("random_crop", {}) or {}).get("hr_patch_size", 128),
                horizontal_flip=aug.get("horizontal_flip", 0.5), random_rotate90=aug.get("random_rotate90", 0.0),
                color_jitter_prob=cj.get("probability", 0.3), brightness=cj.get("brightness", 0.1),
                contrast=cj.get("contrast", 0.1), saturation=cj.get("saturation", 0.0), hue=cj.get("hue", 0.0))


def build_loaders(config: dict, data_root: str, batch_size: int, synthetic: int = 0):
    """Train / val loaders as the reference CLI builds them (scripts/train.py:171-198): the train
    loader with the YAML's augmentation, the val loader with FFHQDataset's defaults (val mode:
    full images, no augmentation)."""
    data_cfg = config.get("data", {}) or {}
    nw = data_cfg.get("num_workers", 4)
    kw = train_loader_kwargs(config)
    seed = (config.get("project", {}) or {}).get("seed", 42)
    train = get_dataloader(data_root, "train", batch_size, nw, synthetic=synthetic, seed=seed, **kw)
    val_syn = max(synthetic // 8, batch_size) if synthetic else 0
    val = get_dataloader(data_root, "val", batch_size, nw, synthetic=val_syn, seed=seed,
                         hr_patch_size=kw["hr_patch_size"] if synthetic else 128)
    return train, val


def main(argv=None):
    ap = argparse.ArgumentParser(description="Train Face Super-Resolution Model (MI355X)")
    ap.add_argument("--config", type=str, default="configs/config.yaml")
    ap.add_argument("--model", type=str, default=None, choices=["custom", "transfer", "esrgan"])
    ap.add_argument("--data-root", type=str, default="data/processed")
    ap.add_argument("--batch-size", type=int, default=None)
    ap.add_argument("--epochs", type=int, default=None)
    ap.add_argument("--lr", type=float, default=None)
    ap.add_argument("--gradient-clip", type=float, default=None)
    ap.add_argument("--perceptual-weight", type=float, default=None)
    ap.add_argument("--patience", type=int, default=None)
    ap.add_argument("--resume", type=str, default=None)
    ap.add_argument("--fine-tune", action="store_true")
    ap.add_argument("--overfit-test", action="store_true")
    ap.add_argument("--device", type=str, default="cuda")
    ap.add_argument("--no-wandb", action="store_true")
    ap.add_argument("--precision", type=str, default=None, choices=["fp32", "bf16"])
    ap.add_argument("--synthetic", type=int, default=0)
    args = ap.parse_args(argv)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1 and not dist.is_initialized():
        local = int(os.environ.get("LOCAL_RANK", "0"))
        torch.cuda.set_device(local)
        from src.training.dp import init_rccl
        init_rccl(torch.device("cuda", local))
    rank = dist.get_rank() if dist.is_initialized() else 0

    config = load_config(args.config) if Path(args.config).exists() else {}
    project, data_cfg = config.get("project", {}), config.get("data", {})
    tr_cfg, loss_cfg = config.get("training", {}), config.get("loss", {})
    ck_cfg, log_cfg = config.get("checkpoint", {}), config.get("logging", {})
    set_seed(project.get("seed", 42))

    batch_size = args.batch_size or data_cfg.get("batch_size", 16)
    epochs = args.epochs or tr_cfg.get("epochs", 50)
    lr = args.lr or tr_cfg.get("optimizer", {}).get("lr", 1e-4)
    data_root = args.data_root or data_cfg.get("data_root", "data/processed")
    model_type = args.model or config.get("model", {}).get("type", "custom")
    train_loader, val_loader = build_loaders(config, data_root, batch_size, args.synthetic)

    precision = resolve_precision(args.precision, tr_cfg)
    model = create_model(model_type, config, precision)
    discriminator, gan_loss = create_gan(config, precision)
    gan = loss_cfg.get("gan", {})
    pw = args.perceptual_weight if args.perceptual_weight is not None else loss_cfg.get("perceptual_weight", 0.01)
    loss_fn = create_loss_function(l1_weight=loss_cfg.get("l1_weight", 1.0), perceptual_weight=pw,
                                   ssim_weight=loss_cfg.get("ssim_weight", 0.1),
                                   use_charbonnier=loss_cfg.get("use_charbonnier", False),
                                   charbonnier_eps=loss_cfg.get("charbonnier_eps", 1e-3),
                                   perceptual_layers=loss_cfg.get("perceptual", {}).get("layers"))
    if args.overfit_test:
        res = overfit_test(model, train_loader, loss_fn, num_images=10, num_iterations=1000, device=args.device)
        if rank == 0:
            print(f"overfit test: final PSNR {res['final_psnr']:.2f} dB, converged={res['converged']}")

    sched = tr_cfg.get("scheduler", {})
    es = tr_cfg.get("early_stopping", {})
    tcfg = TrainerConfig(
        epochs=epochs, learning_rate=lr, weight_decay=tr_cfg.get("optimizer", {}).get("weight_decay", 0.0),
        gradient_clip=args.gradient_clip if args.gradient_clip is not None else tr_cfg.get("gradient_clip", 1.0),
        accumulation_steps=tr_cfg.get("accumulation_steps", 1), use_amp=tr_cfg.get("mixed_precision", True),
        scheduler_type=sched.get("type", "cosine"), scheduler_T_max=sched.get("T_max", epochs),
        scheduler_eta_min=sched.get("eta_min", 1e-7), scheduler_step_size=sched.get("step_size", 10),
        scheduler_gamma=sched.get("gamma", 0.5),
        early_stopping_patience=args.patience if args.patience is not None else es.get("patience", 10),
        early_stopping_metric=es.get("metric", "val_psnr"), early_stopping_mode=es.get("mode", "max"),
        checkpoint_dir=ck_cfg.get("save_dir", "checkpoints"), save_every=ck_cfg.get("save_every", 10),
        save_best=ck_cfg.get("save_best", True), log_every=log_cfg.get("console", {}).get("log_every", 100),
        use_wandb=False, device=args.device, gan_weight=gan.get("weight", 0.0), gan_type=gan.get("type", "vanilla"),
        d_learning_rate=gan.get("d_lr", 1e-4), d_weight_decay=gan.get("d_weight_decay", 0.0),
        d_updates_per_g=gan.get("d_updates_per_g", 1), gan_start_epoch=gan.get("start_epoch", 0))
    trainer = Trainer(model, train_loader, val_loader, loss_fn, tcfg, discriminator=discriminator, gan_loss=gan_loss)
    if args.resume:
        trainer.load_checkpoint(args.resume, weights_only=args.fine_tune)
    try:
        hist = trainer.train()
        if rank == 0:
            print(f"Training complete. Best PSNR: {max(hist['val_psnr']):.2f} dB")
    except KeyboardInterrupt:
        trainer._save_checkpoint("interrupted.pth")
    if dist.is_initialized():
        from src.training.dp import RcclComm
        RcclComm.destroy_all()          # before the group whose ranks they span goes away
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
