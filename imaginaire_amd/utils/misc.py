"""Misc helpers (reference utils/misc.py:17-236)."""
import collections.abc as container_abcs
from collections import OrderedDict

import numpy as np
import torch
import torch.nn.functional as F


def split_labels(labels, label_lengths):
    """Split a concatenated label tensor by the per-type channel counts."""
    assert isinstance(label_lengths, OrderedDict)
    start = 0
    outputs = {}
    for data_type, length in label_lengths.items():
        end = start + length
        if labels.dim() == 5:
            outputs[data_type] = labels[:, :, start:end]
        elif labels.dim() == 4:
            outputs[data_type] = labels[:, start:end]
        elif labels.dim() == 3:
            outputs[data_type] = labels[start:end]
        start = end
    return outputs


def requires_grad(model, require=True):
    for p in model.parameters():
        p.requires_grad = require


def to_device(data, device, non_blocking=False, memory_format=None):
    """Recursively move tensors to ``device`` ('cpu' / 'cuda' / torch.device)."""
    if isinstance(data, torch.Tensor):
        data = data.to(torch.device(device), non_blocking=non_blocking)
        if memory_format is not None and data.dim() == 4 and data.is_floating_point():
            data = data.contiguous(memory_format=memory_format)
        return data
    if isinstance(data, container_abcs.Mapping):
        return {k: to_device(v, device, non_blocking, memory_format) for k, v in data.items()}
    if isinstance(data, container_abcs.Sequence) and not isinstance(data, (str, bytes)):
        return [to_device(d, device, non_blocking, memory_format) for d in data]
    return data


def to_cuda(data):
    return to_device(data, 'cuda')


def to_cpu(data):
    return to_device(data, 'cpu')


def _cast(data, fn):
    if isinstance(data, torch.Tensor) and torch.is_floating_point(data):
        return fn(data)
    if isinstance(data, container_abcs.Mapping):
        return {k: _cast(v, fn) for k, v in data.items()}
    if isinstance(data, container_abcs.Sequence) and not isinstance(data, (str, bytes)):
        return [_cast(d, fn) for d in data]
    return data


def to_half(data):
    return _cast(data, lambda t: t.half())


def to_bfloat16(data):
    return _cast(data, lambda t: t.bfloat16())


def to_float(data):
    return _cast(data, lambda t: t.float())


def to_channels_last(data):
    """Recursively convert 4-D float tensors to channels_last (NHWC) layout."""
    return _cast(data, lambda t: t.contiguous(memory_format=torch.channels_last)
                 if t.dim() == 4 else t)


def get_and_setattr(cfg, name, default):
    if not hasattr(cfg, name) or name not in cfg.__dict__:
        setattr(cfg, name, default)
    return getattr(cfg, name)


def get_nested_attr(cfg, attr_name, default):
    atr = cfg
    for name in attr_name.split('.'):
        if not hasattr(atr, name):
            return default
        atr = getattr(atr, name)
    return atr


def gradient_norm(model):
    norms = [p.grad.norm(2) for p in model.parameters() if p.grad is not None]
    if not norms:
        return 0.0
    return float(torch.stack(norms).norm(2).item())


def random_shift(x, offset=0.05, mode='bilinear', padding_mode='reflection'):
    """Random translation by up to ``offset`` of the image size (misc.py:183-203)."""
    assert x.dim() == 4, "Input must be a 4D tensor."
    batch_size = x.size(0)
    theta = torch.eye(2, 3, device=x.device).unsqueeze(0).repeat(batch_size, 1, 1)
    theta[:, :, 2] = 2 * offset * torch.rand(batch_size, 2, device=x.device) - offset
    grid = F.affine_grid(theta, x.size(), align_corners=False)
    return F.grid_sample(x, grid.to(x.dtype), mode=mode, padding_mode=padding_mode,
                         align_corners=False)


def truncated_gaussian(threshold, size, seed=None, device=None):
    from scipy.stats import truncnorm
    state = None if seed is None else np.random.RandomState(seed)
    values = truncnorm.rvs(-threshold, threshold, size=size, random_state=state)
    return torch.tensor(values, device=device).float()


_IMNET_MEAN = (0.485, 0.456, 0.406, 0.5)
_IMNET_STD = (0.229, 0.224, 0.225, 0.225)
_IMNET_CACHE = {}


def apply_imagenet_normalization(input):
    """[-1, 1] → ImageNet-normalised. Supports 3- and 4-channel images.

    The reference fork hard-codes 4 channels (utils/misc.py:221-236); upstream
    uses 3. Here the statistics are sliced to the input's channel count.
    """
    c = input.shape[1]
    # ((x + 1) / 2 - mean) / std == x * (0.5 / std) + (0.5 - mean) / std: one fused
    # multiply-add with per-channel constants cached per (device, dtype) — created on
    # first use, so the op is also legal inside a hipGraph capture (no H2D copy there)
    key = (input.device, input.dtype, c)
    sc = _IMNET_CACHE.get(key)
    if sc is None:
        mean = torch.tensor(_IMNET_MEAN[:c], dtype=torch.float64)
        std = torch.tensor(_IMNET_STD[:c], dtype=torch.float64)
        scale = (0.5 / std).view(1, c, 1, 1).to(input.device, input.dtype)
        shift = ((0.5 - mean) / std).view(1, c, 1, 1).to(input.device, input.dtype)
        sc = _IMNET_CACHE[key] = (scale, shift)
    return torch.addcmul(sc[1], input, sc[0])
