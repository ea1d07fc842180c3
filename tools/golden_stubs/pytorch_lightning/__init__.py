"""Arithmetic-free stand-in for pytorch_lightning 1.2.10 (not installed offline).

Only what the reference's `vqvae/model.py` and `utils/*` touch at import/construct
time: LightningModule is a plain nn.Module whose logging hooks are no-ops.
Used ONLY by tools/make_goldens.py to import the reference for fixture generation.
"""
import torch
from torch import nn


class LightningModule(nn.Module):
    def save_hyperparameters(self, *args, **kwargs):
        pass

    def log(self, *args, **kwargs):
        pass

    def log_dict(self, *args, **kwargs):
        pass

    @property
    def device(self):
        return next(self.parameters()).device


class LightningDataModule:
    pass


class _Trainer:
    @staticmethod
    def seed_everything(seed):
        torch.manual_seed(seed)


trainer = _Trainer()
