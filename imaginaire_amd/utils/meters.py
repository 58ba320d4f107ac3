"""Meters and summary logging (reference utils/meters.py:19-159).

Uses ``torch.utils.tensorboard`` when tensorboard is installed, otherwise the
native event writer in ``utils/tb_writer.py``. Meters buffer device tensors
and only synchronise at ``flush`` (logging boundaries), so the training step
itself never blocks on ``loss.item()``.
"""
import math

import torch

from imaginaire_amd.utils.distributed import master_only
from imaginaire_amd.utils.distributed import master_only_print as print

LOG_WRITER = None
LOG_DIR = None


def _make_writer(log_dir):
    try:
        from torch.utils.tensorboard import SummaryWriter
        return SummaryWriter(log_dir=log_dir)
    except Exception:  # tensorboard not installed
        from imaginaire_amd.utils.tb_writer import SummaryWriter
        return SummaryWriter(log_dir)


@torch.no_grad()
def sn_reshape_weight_to_matrix(weight):
    return weight.reshape(weight.size(0), -1)


@torch.no_grad()
def get_weight_stats(mod, cfg=None, loss_id=None):
    """(grad-norm, weight-norm, sigma) of a spectral-normalised layer (meters.py:31-51)."""
    grad_norm = mod.weight_orig.grad.norm().item() if mod.weight_orig.grad is not None else 0.
    weight_norm = mod.weight_orig.data.norm().item()
    weight_mat = sn_reshape_weight_to_matrix(mod.weight_orig)
    sigma = torch.sum(mod.weight_u * torch.mv(weight_mat, mod.weight_v))
    return grad_norm, weight_norm, sigma


@master_only
def set_summary_writer(log_dir):
    global LOG_DIR, LOG_WRITER
    LOG_DIR = log_dir
    LOG_WRITER = _make_writer(log_dir)


def get_summary_writer():
    return LOG_WRITER


@master_only
def write_summary(name, summary, step, hist=False):
    lw = LOG_WRITER
    if lw is None:
        return
    if hist:
        lw.add_histogram(name, summary, step)
    else:
        lw.add_scalar(name, summary, step)


@master_only
def add_hparams(hparam_dict=None, metric_dict=None):
    if type(hparam_dict) is not dict or type(metric_dict) is not dict:
        raise TypeError('hparam_dict and metric_dict should be dictionary.')
    lw = LOG_WRITER
    if lw is None:
        return
    # both writers (torch's and the native one) emit the hparams plugin's experiment /
    # session-start / session-end summaries plus the metric scalars
    lw.add_hparams(hparam_dict, metric_dict)


class Meter(object):
    """Buffers values (floats or device tensors); averages finite ones on flush."""

    def __init__(self, name):
        self.name = name
        self.values = []

    def reset(self):
        self.values = []

    def write(self, value):
        self.values.append(value)

    def flush(self, step):
        vals = []
        for v in self.values:
            if isinstance(v, torch.Tensor):
                v = float(v.detach().float().mean().item())
            vals.append(float(v))
        if not all(math.isfinite(x) for x in vals):
            print("meter {} contained a nan or inf.".format(self.name))
        finite = [x for x in vals if math.isfinite(x)]
        if finite:
            write_summary(self.name, sum(finite) / len(finite), step)
        self.reset()
        return sum(finite) / len(finite) if finite else None

    def write_image(self, img_grid, step):
        lw = LOG_WRITER
        if lw is not None:
            lw.add_image("Visualizations", img_grid, step)
