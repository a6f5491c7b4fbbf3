"""Training modules (reference: etpgt/train/__init__.py)."""

from etpgt.train.dataloader import DeviceSessionLoader, SessionDataset, collate_fn, create_dataloader
from etpgt.train.losses import BPRLoss, DualLoss, ListwiseLoss, SampledSoftmaxLoss, create_loss_function
from etpgt.train.trainer import Trainer

__all__ = [
    "SessionDataset",
    "collate_fn",
    "create_dataloader",
    "DeviceSessionLoader",
    "Trainer",
    "BPRLoss",
    "ListwiseLoss",
    "DualLoss",
    "SampledSoftmaxLoss",
    "create_loss_function",
]
