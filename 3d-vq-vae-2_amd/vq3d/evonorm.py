"""EvoNorm-S0 for 3-D volumes (reference vqvae/evonorm.py), on the libvq3d EvoNorm kernels."""
import torch
from torch import nn


def determine_num_groups(in_channels, preferred_channels_per_group=8):
    """evonorm.py:8-9"""
    return max(in_channels // preferred_channels_per_group, 1)


class EvoNorm3DS0(nn.Module):
    """Non-linear, affine EvoNorm S0 (evonorm.py:59-76):
    y = x * sigmoid(v * x) * gamma / group_std(x) + beta, unbiased variance over each group of
    max(C // 8, 1) channels and the whole volume.  Batch 1 only, as the reference."""

    def __init__(self, in_channels):
        super().__init__()
        self.v = nn.Parameter(torch.ones((in_channels, 1, 1, 1)))
        self.gamma = nn.Parameter(torch.zeros((in_channels, 1, 1, 1)))
        self.beta = nn.Parameter(torch.zeros((in_channels, 1, 1, 1)))

    def forward(self, x):
        assert x.dim() == 5
        from .functional import EvoNormFn
        return EvoNormFn.apply(x, self, self.v, self.gamma, self.beta)
