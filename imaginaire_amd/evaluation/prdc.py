"""Precision / recall / density / coverage (reference evaluation/prdc.py:20-127).

Pairwise distances are computed with ``torch.cdist`` (GEMM-based, on the GPU
when available) instead of sklearn on the host.
"""
import numpy as np
import torch

from imaginaire_amd.utils.distributed import is_master
from imaginaire_amd.utils.distributed import master_only_print as print
from .common import get_activations

__all__ = ['compute_prdc', 'get_prdc']


def _dev():
    return torch.device('cuda') if torch.cuda.is_available() else torch.device('cpu')


def compute_pairwise_distance(data_x, data_y=None):
    x = torch.as_tensor(data_x, dtype=torch.float64, device=_dev())
    y = x if data_y is None else torch.as_tensor(data_y, dtype=torch.float64, device=_dev())
    return torch.cdist(x, y).cpu().numpy()


def get_kth_value(unsorted, k, axis=-1):
    indices = np.argpartition(unsorted, k, axis=axis)[..., :k]
    k_smallests = np.take_along_axis(unsorted, indices, axis=axis)
    return k_smallests.max(axis=axis)


def compute_nearest_neighbour_distances(input_features, nearest_k):
    distances = compute_pairwise_distance(input_features)
    return get_kth_value(distances, k=nearest_k + 1, axis=-1)


def get_prdc(real_features, fake_features, nearest_k):
    real_nn = compute_nearest_neighbour_distances(real_features, nearest_k)
    fake_nn = compute_nearest_neighbour_distances(fake_features, nearest_k)
    d_rf = compute_pairwise_distance(real_features, fake_features)
    precision = (d_rf < np.expand_dims(real_nn, axis=1)).any(axis=0).mean()
    recall = (d_rf < np.expand_dims(fake_nn, axis=0)).any(axis=1).mean()
    density = (1. / float(nearest_k)) * (d_rf < np.expand_dims(real_nn, axis=1)).sum(
        axis=0).mean()
    coverage = (d_rf.min(axis=1) < real_nn).mean()
    return dict(precision=precision, recall=recall, density=density, coverage=coverage)


def compute_prdc(cfg, data_loader, net_G, key_real='images', key_fake='fake_images', k=10):
    y_real = get_activations(data_loader, key_real, key_fake, generator=None)
    y_fake = get_activations(data_loader, key_real, key_fake, generator=net_G)
    if is_master():
        prdc_data = get_prdc(y_real, y_fake, k)
        return prdc_data['density'], prdc_data['coverage']
    return None, None
