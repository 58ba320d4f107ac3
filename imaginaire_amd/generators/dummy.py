"""Placeholder generator (reference generators/dummy.py:10-29)."""
import torch.nn as nn

from imaginaire_amd.layers import LinearBlock


class Generator(nn.Module):
    def __init__(self, gen_cfg, data_cfg):
        super().__init__()
        self.dummy_layer = LinearBlock(1, 1)

    def forward(self, data):
        return
