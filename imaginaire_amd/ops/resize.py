"""Resampling that keeps the activation dtype under bf16 autocast.

torch.autocast runs ``upsample_*`` in fp32: every nearest/bilinear resize of a bf16 activation
becomes bf16->fp32 cast + fp32 resize + an fp32 tensor that the next fused norm kernel then
reads at twice the bytes (measured on MI355X: ~800 bf16->fp32 copy launches and fp32
``apply_fwd`` norm kernels per 3 SPADE steps, profiles/spade_step_k11v2_mi355x.txt). Nearest
resizing is exact in any dtype, so it runs on the input dtype with autocast disabled instead. Used by every resize on the
SPADE/pix2pixHD/vid2vid paths (reference: plain ``F.interpolate`` / ``nn.Upsample``).
"""
import torch
import torch.nn.functional as F
from torch import nn


def interpolate(x, size=None, scale_factor=None, mode='nearest', align_corners=None,
                recompute_scale_factor=None):
    # nearest only: the bf16 bilinear BACKWARD (atomic scatter) is 3x slower than fp32 on
    # MI355X (FPSE 2x upsample: 3.6 vs ~1 ms per step), so bilinear keeps autocast's fp32
    if mode == 'nearest' and x.is_cuda and x.dtype in (torch.bfloat16, torch.float16) and \
            torch.is_autocast_enabled('cuda'):
        with torch.autocast('cuda', enabled=False):
            return F.interpolate(x, size, scale_factor, mode, align_corners,
                                 recompute_scale_factor)
    return F.interpolate(x, size, scale_factor, mode, align_corners, recompute_scale_factor)


class Upsample(nn.Module):
    """Drop-in for ``nn.Upsample`` (no parameters, identical state dict)."""

    def __init__(self, size=None, scale_factor=None, mode='nearest', align_corners=None):
        super().__init__()
        self.size = size
        self.scale_factor = float(scale_factor) if scale_factor else None
        self.mode = mode
        self.align_corners = align_corners

    def forward(self, x):
        return interpolate(x, self.size, self.scale_factor, self.mode, self.align_corners)

    def extra_repr(self):
        return 'scale_factor={}, mode={}'.format(self.scale_factor, self.mode)
