"""Training surface of the reference (src/training/__init__.py): Trainer, TrainerConfig,
EarlyStopping, overfit_test -- data-parallel over RCCL, fused HIP G-step."""
from .optim import FusedAdamW
from .trainer import EarlyStopping, Trainer, TrainerConfig, bicubic_down4, overfit_test

__all__ = ["Trainer", "TrainerConfig", "EarlyStopping", "overfit_test", "FusedAdamW", "bicubic_down4"]
