"""SAGAN self-attention block (reference layers/non_local.py:13-79).

θ/φ/g 1×1 convs, 2×2 max-pool on keys/values; the attention ``softmax(θᵀφ) g`` (no scaling,
matching the reference's raw softmax, reference layers/non_local.py:60-79) never materialises
the HW×HW/4 energy matrix in HBM: under bf16 autocast on the GPU it runs the k16 fused
attention kernel (ops/attention.py, csrc/attention.hip: online softmax on MFMA, LSE-recompute
backward) whenever the shapes fit it (HW % 256 == 0, C/8 <= 128); otherwise (fp32 compute,
CPU, other shapes) PyTorch's scaled-dot-product attention.
"""
from functools import partial

import torch
import torch.nn as nn
import torch.nn.functional as F

from .conv import Conv2dBlock
from imaginaire_amd.ops.attention import fused_attention, native_ok


def _k16_ok(q, k, v):
    """k16 computes in bf16: only for bf16-autocast callers (an fp32 step keeps fp32 attention)."""
    return q.is_cuda and torch.is_autocast_enabled('cuda') and \
        torch.get_autocast_dtype('cuda') == torch.bfloat16 and native_ok(q, k, v)


class NonLocal2dBlock(nn.Module):
    def __init__(self, in_channels, scale=True, clamp=False, weight_norm_type='none'):
        super().__init__()
        self.clamp = clamp
        self.gamma = nn.Parameter(torch.zeros(1)) if scale else 1.0
        self.in_channels = in_channels
        base_conv2d_block = partial(Conv2dBlock, kernel_size=1, stride=1, padding=0,
                                    weight_norm_type=weight_norm_type)
        self.theta = base_conv2d_block(in_channels, in_channels // 8)
        self.phi = base_conv2d_block(in_channels, in_channels // 8)
        self.g = base_conv2d_block(in_channels, in_channels // 2)
        self.out_conv = base_conv2d_block(in_channels // 2, in_channels)
        self.softmax = nn.Softmax(dim=-1)
        self.max_pool = nn.MaxPool2d(2)

    def forward(self, x):
        n, c, h, w = x.size()
        theta = self.theta(x).reshape(n, -1, h * w).permute(0, 2, 1)          # [n, hw, c/8]
        phi = self.max_pool(self.phi(x)).reshape(n, -1, h * w // 4).permute(0, 2, 1)  # [n, hw/4, c/8]
        g = self.max_pool(self.g(x)).reshape(n, -1, h * w // 4).permute(0, 2, 1)      # [n, hw/4, c/2]
        if _k16_ok(theta, phi, g):
            out = fused_attention(theta, phi, g, 1.0)                        # [n, hw, c/2]
        else:
            out = F.scaled_dot_product_attention(theta[:, None], phi[:, None], g[:, None],
                                                 scale=1.0)[:, 0]
        out = out.permute(0, 2, 1).reshape(n, c // 2, h, w)
        out = self.out_conv(out)
        if self.clamp:
            return self.gamma.clamp(-1, 1) * out + x
        return self.gamma * out + x
