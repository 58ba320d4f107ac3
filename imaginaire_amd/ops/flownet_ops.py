"""FlowNet2 native ops: Correlation (k6), Resample2d (k7), ChannelNorm (k8).

Autograd wrappers around ``csrc/correlation.hip`` / ``csrc/flow_warp.hip`` with
plain-PyTorch references of the same math (used on CPU and as the numerics
oracle in tests/test_kernels_gpu.py).

Reference semantics: third_party/correlation/correlation.py:8-104 +
correlation_cuda_kernel.cu:73-334; third_party/resample2d/resample2d.py +
resample2d_kernel.cu:15-203; third_party/channelnorm/channelnorm.py:7-39 +
channelnorm_kernel.cu:19-96.
"""
import math

import torch
import torch.nn.functional as F
from torch import nn

from imaginaire_amd.ops import _ext


# ---------------------------------------------------------------- correlation
def correlation_out_size(size, pad_size, kernel_size, max_displacement, stride1):
    border = (kernel_size - 1) // 2 + max_displacement
    return int(math.ceil((size + 2 * pad_size - 2 * border) / stride1))


def correlation_reference(input1, input2, pad_size=20, kernel_size=1, max_displacement=20,
                          stride1=1, stride2=2):
    """fp32 PyTorch correlation (same output layout/values as the HIP kernel)."""
    n, c, h, w = input1.shape
    a = F.pad(input1.float(), [pad_size] * 4)
    b = F.pad(input2.float(), [pad_size] * 4)
    kr = (kernel_size - 1) // 2
    rad = max_displacement // stride2
    oh = correlation_out_size(h, pad_size, kernel_size, max_displacement, stride1)
    ow = correlation_out_size(w, pad_size, kernel_size, max_displacement, stride1)
    ys = torch.arange(oh, device=a.device) * stride1 + max_displacement
    xs = torch.arange(ow, device=a.device) * stride1 + max_displacement
    outs = []
    for tj in range(-rad, rad + 1):
        for ti in range(-rad, rad + 1):
            acc = 0.
            for j in range(-kr, kr + 1):
                for i in range(-kr, kr + 1):
                    pa = a[:, :, ys + j][:, :, :, xs + i]
                    pb = b[:, :, ys + j + tj * stride2][:, :, :, xs + i + ti * stride2]
                    acc = acc + (pa * pb).sum(1)
            outs.append(acc / (kernel_size * kernel_size * c))
    return torch.stack(outs, 1).to(input1.dtype)


class _CorrelationFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, input1, input2, pad_size, kernel_size, max_displacement, stride1, stride2):
        ctx.save_for_backward(input1, input2)
        ctx.params = (pad_size, kernel_size, max_displacement, stride1, stride2)
        return _ext.ext().correlation_forward(input1, input2, *ctx.params)

    @staticmethod
    def backward(ctx, grad_out):
        input1, input2 = ctx.saved_tensors
        g1, g2 = _ext.ext().correlation_backward(input1, input2, grad_out, *ctx.params)
        return g1.to(input1.dtype), g2.to(input2.dtype), None, None, None, None, None


def correlation(input1, input2, pad_size=20, kernel_size=1, max_displacement=20, stride1=1,
                stride2=2):
    if _ext.use_native(input1):
        return _CorrelationFn.apply(input1, input2, pad_size, kernel_size, max_displacement,
                                    stride1, stride2)
    return correlation_reference(input1, input2, pad_size, kernel_size, max_displacement,
                                 stride1, stride2)


class Correlation(nn.Module):
    """Drop-in for the reference ``correlation.Correlation`` module."""

    def __init__(self, pad_size=0, kernel_size=0, max_displacement=0, stride1=1, stride2=2,
                 corr_multiply=1):
        super().__init__()
        self.pad_size = pad_size
        self.kernel_size = kernel_size
        self.max_displacement = max_displacement
        self.stride1 = stride1
        self.stride2 = stride2
        self.corr_multiply = corr_multiply

    def forward(self, input1, input2):
        return correlation(input1, input2, self.pad_size, self.kernel_size,
                           self.max_displacement, self.stride1, self.stride2)


# ----------------------------------------------------------------- resample2d
def resample2d_reference(input1, flow, kernel_size=1):
    """Bilinear warp with edge clamping (FlowNet2 Resample2d semantics)."""
    b, c, h, w = input1.shape
    x = input1.float()
    f = flow.float()
    gy, gx = torch.meshgrid(torch.arange(h, device=x.device, dtype=torch.float32),
                            torch.arange(w, device=x.device, dtype=torch.float32), indexing='ij')
    xf = gx[None] + f[:, 0]
    yf = gy[None] + f[:, 1]
    alpha = (xf - xf.floor())[:, None]
    beta = (yf - yf.floor())[:, None]
    x0 = xf.floor().long()
    y0 = yf.floor().long()
    out = 0.
    flat = x.reshape(b, c, h * w)

    def tap(yy, xx):
        idx = (yy.clamp(0, h - 1) * w + xx.clamp(0, w - 1)).reshape(b, 1, h * w).expand(b, c, -1)
        return flat.gather(2, idx).reshape(b, c, h, w)
    for fy in range(kernel_size):
        for fx in range(kernel_size):
            yt = y0.clamp(0, h - 1) + fy
            yb = (y0 + 1).clamp(0, h - 1) + fy
            xl = x0.clamp(0, w - 1) + fx
            xr = (x0 + 1).clamp(0, w - 1) + fx
            out = out + (1 - alpha) * (1 - beta) * tap(yt, xl) + alpha * (1 - beta) * tap(yt, xr) \
                + (1 - alpha) * beta * tap(yb, xl) + alpha * beta * tap(yb, xr)
    return out.to(input1.dtype)


class _Resample2dFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, input1, flow, kernel_size):
        ctx.save_for_backward(input1, flow)
        ctx.kernel_size = kernel_size
        return _ext.ext().resample2d_forward(input1, flow, kernel_size)

    @staticmethod
    def backward(ctx, grad_out):
        input1, flow = ctx.saved_tensors
        d1, d2 = _ext.ext().resample2d_backward(input1, flow, grad_out.contiguous(),
                                                ctx.kernel_size)
        return d1.to(input1.dtype), d2.to(flow.dtype), None


def resample2d(input1, flow, kernel_size=1):
    if _ext.use_native(input1):
        return _Resample2dFn.apply(input1, flow, kernel_size)
    return resample2d_reference(input1, flow, kernel_size)


class Resample2d(nn.Module):
    def __init__(self, kernel_size=1, bilinear=True):
        super().__init__()
        self.kernel_size = kernel_size
        self.bilinear = bilinear

    def forward(self, input1, input2):
        return resample2d(input1, input2, self.kernel_size)


# ---------------------------------------------------------------- channelnorm
def channelnorm_reference(x, norm_deg=2):
    return x.float().pow(2).sum(1, keepdim=True).sqrt().to(x.dtype)


class _ChannelNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        out = _ext.ext().channelnorm_forward(x)
        ctx.save_for_backward(x, out)
        return out

    @staticmethod
    def backward(ctx, grad_out):
        x, out = ctx.saved_tensors
        return _ext.ext().channelnorm_backward(x, out, grad_out)


def channelnorm(x, norm_deg=2):
    if _ext.use_native(x):
        return _ChannelNormFn.apply(x)
    return channelnorm_reference(x, norm_deg)


class ChannelNorm(nn.Module):
    def __init__(self, norm_deg=2):
        super().__init__()
        self.norm_deg = norm_deg

    def forward(self, input1):
        return channelnorm(input1, self.norm_deg)
