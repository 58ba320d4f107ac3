"""Fréchet Inception Distance (reference evaluation/fid.py:16-226).

Statistics are cached as ``.npz`` (real stats in ``real_mean_cov.npz`` next
to the fake stats file). The matrix square root runs on the GPU in fp64 via
a symmetric eigendecomposition — tr(√(Σ₁Σ₂)) = Σ √λ(√Σ₁ Σ₂ √Σ₁) — instead of
``scipy.linalg.sqrtm`` on the host (which is kept as the CPU path).
"""
import os

import numpy as np
import torch

from imaginaire_amd.evaluation.common import get_activations, get_video_activations
from imaginaire_amd.utils.distributed import is_master
from imaginaire_amd.utils.distributed import master_only_print as print


def compute_fid(fid_path, data_loader, net_G, key_real='images', key_fake='fake_images',
                sample_size=None, preprocess=None, is_video=False, few_shot_video=False):
    print('Computing FID.')
    with torch.no_grad():
        fake_mean, fake_cov = load_or_compute_stats(fid_path, data_loader, key_real, key_fake,
                                                    net_G, sample_size, preprocess, is_video,
                                                    few_shot_video)
        mean_cov_path = os.path.join(os.path.dirname(fid_path), 'real_mean_cov.npz')
        real_mean, real_cov = load_or_compute_stats(mean_cov_path, data_loader, key_real,
                                                    key_fake, None, sample_size, preprocess,
                                                    is_video, few_shot_video)
    if is_master():
        return calculate_frechet_distance(real_mean, real_cov, fake_mean, fake_cov)
    return None


def compute_fid_data(fid_path, data_loader_a, data_loader_b, key_a='images', key_b='images',
                     sample_size=None, is_video=False, few_shot_video=False):
    if sample_size is None:
        sample_size = min(len(data_loader_a.dataset), len(data_loader_b.dataset))
    print('Computing FID using {} images from both distributions.'.format(sample_size))
    with torch.no_grad():
        path_a = os.path.join(os.path.dirname(fid_path), 'mean_cov_a.npz')
        path_b = os.path.join(os.path.dirname(fid_path), 'mean_cov_b.npz')
        mean_a, cov_a = load_or_compute_stats(path_a, data_loader_a, key_a, key_a,
                                              sample_size=sample_size, is_video=is_video)
        mean_b, cov_b = load_or_compute_stats(path_b, data_loader_b, key_b, key_b,
                                              sample_size=sample_size, is_video=is_video)
    if is_master():
        return calculate_frechet_distance(mean_b, cov_b, mean_a, cov_a)
    return None


def load_or_compute_stats(fid_path, data_loader, key_real, key_fake, generator=None,
                          sample_size=None, preprocess=None, is_video=False,
                          few_shot_video=False):
    if fid_path is not None and os.path.exists(fid_path):
        npz_file = np.load(fid_path)
        return npz_file['mean'], npz_file['cov']
    mean, cov = get_inception_mean_cov(data_loader, key_real, key_fake, generator, sample_size,
                                       preprocess, is_video, few_shot_video)
    if fid_path is not None and is_master():
        os.makedirs(os.path.dirname(fid_path) or '.', exist_ok=True)
        np.savez(fid_path, mean=mean, cov=cov)
    return mean, cov


def get_inception_mean_cov(data_loader, key_real, key_fake, generator, sample_size, preprocess,
                           is_video=False, few_shot_video=False):
    if is_video:
        y = get_video_activations(data_loader, key_real, key_fake, generator, sample_size,
                                  preprocess, few_shot_video)
    else:
        y = get_activations(data_loader, key_real, key_fake, generator, sample_size, preprocess)
    if is_master():
        if y.shape[0] < 2:  # covariance of a single sample is undefined
            return np.mean(y, axis=0), np.zeros((y.shape[1], y.shape[1]))
        return np.mean(y, axis=0), np.cov(y, rowvar=False)
    return None, None


def _sqrtm_trace(sigma1, sigma2, eps=1e-6):
    """tr(sqrt(S1 S2)) via two symmetric eigendecompositions in fp64:
    sqrt(S1) S2 sqrt(S1) is symmetric PSD with the same eigenvalues as S1 S2,
    so no non-symmetric sqrtm (and no complex round-off) is needed."""
    dev = torch.device('cuda', torch.cuda.current_device()) if torch.cuda.is_available() \
        else torch.device('cpu')
    s1 = torch.as_tensor(sigma1, dtype=torch.float64, device=dev)
    s2 = torch.as_tensor(sigma2, dtype=torch.float64, device=dev)
    eye = torch.eye(s1.shape[0], dtype=torch.float64, device=dev)
    for jitter in (0.0, eps, eps * 1e3):
        try:
            w, v = torch.linalg.eigh((s1 + s1.T) / 2 + jitter * eye)
            root1 = (v * w.clamp_min(0).sqrt()) @ v.T
            m = root1 @ (s2 + jitter * eye) @ root1
            ev = torch.linalg.eigvalsh((m + m.T) / 2)
            return float(ev.clamp_min(0).sqrt().sum().item())
        except RuntimeError:  # ill-conditioned (e.g. tiny sample sets): add jitter
            continue
    raise RuntimeError('FID: covariance eigendecomposition failed')


def calculate_frechet_distance(mu1, sigma1, mu2, sigma2, eps=1e-6):
    mu1 = np.atleast_1d(mu1)
    mu2 = np.atleast_1d(mu2)
    sigma1 = np.atleast_2d(sigma1)
    sigma2 = np.atleast_2d(sigma2)
    assert mu1.shape == mu2.shape, 'Training and test mean vectors have different lengths'
    assert sigma1.shape == sigma2.shape, 'Training and test covariances have different dimensions'
    diff = mu1 - mu2
    if not (np.isfinite(mu1).all() and np.isfinite(mu2).all() and np.isfinite(sigma1).all()
            and np.isfinite(sigma2).all()):
        print('FID: non-finite activation statistics (diverged generator?); returning nan')
        return float('nan')
    tr_covmean = _sqrtm_trace(sigma1, sigma2)
    return float(diff.dot(diff) + np.trace(sigma1) + np.trace(sigma2) - 2 * tr_covmean)
