"""Kernel Inception Distance (reference evaluation/kid.py:29-345).

Polynomial-kernel MMD² with the unbiased estimator and its variance; the
kernel matrices are GEMMs on the GPU (hipBLASLt), subsets drawn without
replacement.
"""
import os
import warnings

import numpy as np
import torch

from imaginaire_amd.evaluation.common import get_activations
from imaginaire_amd.utils.distributed import is_master
from imaginaire_amd.utils.distributed import master_only_print as print


def compute_kid(kid_path, data_loader, net_G, key_real='images', key_fake='fake_images',
                sample_size=None, preprocess=None, is_video=False, save_act=True,
                num_subsets=1, subset_size=None):
    print('Computing KID.')
    with torch.no_grad():
        fake_act = load_or_compute_activations(None, data_loader, key_real, key_fake, net_G,
                                               sample_size, preprocess, is_video)
        act_path = os.path.join(os.path.dirname(kid_path), 'activations.npy') \
            if save_act else None
        real_act = load_or_compute_activations(act_path, data_loader, key_real, key_fake, None,
                                               sample_size, preprocess, is_video)
    if is_master():
        mmd, _ = polynomial_mmd_averages(fake_act, real_act, num_subsets, subset_size,
                                         ret_var=True)
        return mmd.mean()
    return None


def compute_kid_data(kid_path, data_loader_a, data_loader_b, key_a='images', key_b='images',
                     sample_size=None, is_video=False, num_subsets=1, subset_size=None):
    if sample_size is None:
        sample_size = min(len(data_loader_a.dataset), len(data_loader_b.dataset))
    with torch.no_grad():
        path_a = os.path.join(os.path.dirname(kid_path), 'activations_a.npy')
        path_b = os.path.join(os.path.dirname(kid_path), 'activations_b.npy')
        act_a = load_or_compute_activations(path_a, data_loader_a, key_a, key_a,
                                            sample_size=sample_size, is_video=is_video)
        act_b = load_or_compute_activations(path_b, data_loader_b, key_b, key_b,
                                            sample_size=sample_size, is_video=is_video)
        if is_master():
            mmd, _ = polynomial_mmd_averages(act_a, act_b, num_subsets, subset_size,
                                             ret_var=True)
            return mmd.mean()
    return None


def load_or_compute_activations(act_path, data_loader, key_real, key_fake, generator=None,
                                sample_size=None, preprocess=None, is_video=False):
    if is_video:
        raise NotImplementedError("Video KID is not currently supported.")
    if act_path is not None and os.path.exists(act_path):
        return np.load(act_path)
    act = get_activations(data_loader, key_real, key_fake, generator, sample_size, preprocess)
    if act_path is not None and is_master():
        os.makedirs(os.path.dirname(act_path) or '.', exist_ok=True)
        np.save(act_path, act)
    return act


def polynomial_mmd_averages(codes_g, codes_r, n_subsets, subset_size, ret_var=True,
                            **kernel_args):
    dev = torch.device('cuda') if torch.cuda.is_available() else torch.device('cpu')
    codes_g = torch.as_tensor(codes_g, device=dev, dtype=torch.float64)
    codes_r = torch.as_tensor(codes_r, device=dev, dtype=torch.float64)
    mmds = np.zeros(n_subsets)
    mmd_vars = np.zeros(n_subsets)
    if subset_size is None:
        subset_size = min(len(codes_r), len(codes_g))
    if subset_size > len(codes_g) or subset_size > len(codes_r):
        subset_size = min(len(codes_r), len(codes_g))
        warnings.warn('Subset size is larger than the data size, using {}.'.format(subset_size))
    for i in range(n_subsets):
        g = codes_g[np.random.choice(len(codes_g), subset_size, replace=False)]
        r = codes_r[np.random.choice(len(codes_r), subset_size, replace=False)]
        o = polynomial_mmd(g, r, **kernel_args, ret_var=ret_var)
        if ret_var:
            mmds[i], mmd_vars[i] = o
        else:
            mmds[i] = o
    return (mmds, mmd_vars) if ret_var else mmds


def polynomial_kernel(X, Y=None, degree=3, gamma=None, coef0=1.):
    if gamma is None:
        gamma = 1.0 / X.shape[1]
    if Y is None:
        Y = X
    return (torch.matmul(X, Y.t()) * gamma + coef0) ** degree


def polynomial_mmd(codes_g, codes_r, degree=3, gamma=None, coef0=1, ret_var=True):
    K_XX = polynomial_kernel(codes_g, degree=degree, gamma=gamma, coef0=coef0)
    K_YY = polynomial_kernel(codes_r, degree=degree, gamma=gamma, coef0=coef0)
    K_XY = polynomial_kernel(codes_g, codes_r, degree=degree, gamma=gamma, coef0=coef0)
    return _mmd2_and_variance(K_XX, K_XY, K_YY, ret_var=ret_var)


def _sqn(arr):
    flat = arr.reshape(-1)
    return flat.dot(flat)


def _mmd2_and_variance(K_XX, K_XY, K_YY, unit_diagonal=False, mmd_est='unbiased',
                       ret_var=True):
    m = K_XX.shape[0]
    var_at_m = m
    if unit_diagonal:
        diag_X = diag_Y = 1
        sum_diag_X = sum_diag_Y = m
        sum_diag2_X = sum_diag2_Y = m
    else:
        diag_X = torch.diagonal(K_XX)
        diag_Y = torch.diagonal(K_YY)
        sum_diag_X = diag_X.sum()
        sum_diag_Y = diag_Y.sum()
        sum_diag2_X = _sqn(diag_X)
        sum_diag2_Y = _sqn(diag_Y)
    Kt_XX_sums = K_XX.sum(dim=1) - diag_X
    Kt_YY_sums = K_YY.sum(dim=1) - diag_Y
    K_XY_sums_0 = K_XY.sum(dim=0)
    K_XY_sums_1 = K_XY.sum(dim=1)
    Kt_XX_sum = Kt_XX_sums.sum()
    Kt_YY_sum = Kt_YY_sums.sum()
    K_XY_sum = K_XY_sums_0.sum()
    if mmd_est == 'biased':
        mmd2 = ((Kt_XX_sum + sum_diag_X) / (m * m) + (Kt_YY_sum + sum_diag_Y) / (m * m)
                - 2 * K_XY_sum / (m * m))
    else:
        mmd2 = (Kt_XX_sum + Kt_YY_sum) / (m * (m - 1))
        if mmd_est == 'unbiased':
            mmd2 = mmd2 - 2 * K_XY_sum / (m * m)
        else:
            mmd2 = mmd2 - 2 * (K_XY_sum - torch.trace(K_XY)) / (m * (m - 1))
    if not ret_var:
        return mmd2.cpu().numpy()
    Kt_XX_2_sum = _sqn(K_XX) - sum_diag2_X
    Kt_YY_2_sum = _sqn(K_YY) - sum_diag2_Y
    K_XY_2_sum = _sqn(K_XY)
    dot_XX_XY = Kt_XX_sums.dot(K_XY_sums_1)
    dot_YY_YX = Kt_YY_sums.dot(K_XY_sums_0)
    m1, m2 = m - 1, m - 2
    zeta1_est = (
        1 / (m * m1 * m2) * (_sqn(Kt_XX_sums) - Kt_XX_2_sum + _sqn(Kt_YY_sums) - Kt_YY_2_sum)
        - 1 / (m * m1) ** 2 * (Kt_XX_sum ** 2 + Kt_YY_sum ** 2)
        + 1 / (m * m * m1) * (_sqn(K_XY_sums_1) + _sqn(K_XY_sums_0) - 2 * K_XY_2_sum)
        - 2 / m ** 4 * K_XY_sum ** 2
        - 2 / (m * m * m1) * (dot_XX_XY + dot_YY_YX)
        + 2 / (m ** 3 * m1) * (Kt_XX_sum + Kt_YY_sum) * K_XY_sum)
    zeta2_est = (
        1 / (m * m1) * (Kt_XX_2_sum + Kt_YY_2_sum)
        - 1 / (m * m1) ** 2 * (Kt_XX_sum ** 2 + Kt_YY_sum ** 2)
        + 2 / (m * m) * K_XY_2_sum
        - 2 / m ** 4 * K_XY_sum ** 2
        - 4 / (m * m * m1) * (dot_XX_XY + dot_YY_YX)
        + 4 / (m ** 3 * m1) * (Kt_XX_sum + Kt_YY_sum) * K_XY_sum)
    var_est = (4 * (var_at_m - 2) / (var_at_m * (var_at_m - 1)) * zeta1_est
               + 2 / (var_at_m * (var_at_m - 1)) * zeta2_est)
    return mmd2.cpu().numpy(), var_est.cpu().numpy()
