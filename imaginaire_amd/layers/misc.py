"""Small layers (reference layers/misc.py:9-47)."""
import torch
from torch import nn


class ApplyNoise(nn.Module):
    """Add Gaussian noise with a learned scale (misc.py:9-29)."""

    def __init__(self):
        super().__init__()
        self.weight = nn.Parameter(torch.zeros(1))

    def forward(self, x, noise=None):
        if noise is None:
            sz = x.size()
            noise = x.new_empty(sz[0], 1, *sz[2:]).normal_()
        return x + self.weight * noise


class PartialSequential(nn.Sequential):
    """Sequential of partial convs; the last input channel is the mask (misc.py:32-47)."""

    def forward(self, x):
        act = x[:, :-1]
        mask = x[:, -1].unsqueeze(1)
        for module in self:
            act, mask = module(act, mask_in=mask)
        return act
