"""Tensor → image helpers (reference utils/visualization/common.py:20-312).

Includes a native ``make_grid`` / ``save_image`` (torchvision is not a
dependency), label colourisation and optical-flow HSV rendering.
"""
import math
import os

import numpy as np
import torch
from PIL import Image


def make_grid(tensor, nrow=8, padding=2, normalize=False, pad_value=0.0):
    """Arrange a [B, C, H, W] batch into one [C, H', W'] grid image."""
    if tensor.dim() == 3:
        tensor = tensor.unsqueeze(0)
    tensor = tensor.detach().float().cpu()
    if normalize:
        lo, hi = float(tensor.min()), float(tensor.max())
        tensor = (tensor - lo) / max(hi - lo, 1e-5)
    b, c, h, w = tensor.shape
    if c == 1:
        tensor = tensor.repeat(1, 3, 1, 1)
        c = 3
    ncol = min(nrow, b)
    nrows = int(math.ceil(b / ncol))
    H, W = h + padding, w + padding
    grid = torch.full((c, nrows * H + padding, ncol * W + padding), pad_value)
    for k in range(b):
        r, col = k // ncol, k % ncol
        grid[:, r * H + padding:r * H + padding + h, col * W + padding:col * W + padding + w] = \
            tensor[k]
    return grid


def save_image_grid(tensor, path, nrow=8, padding=0, normalize=False):
    grid = make_grid(tensor, nrow=nrow, padding=padding, normalize=normalize)
    arr = (grid.clamp(0, 1) * 255 + 0.5).byte().permute(1, 2, 0).numpy()
    d = os.path.dirname(path)
    if d:
        os.makedirs(d, exist_ok=True)
    Image.fromarray(arr[:, :, :3] if arr.shape[2] >= 3 else arr[:, :, 0]).save(path)


def save_image(tensor, path, nrow=8, padding=2, normalize=False):
    save_image_grid(tensor, path, nrow=nrow, padding=padding, normalize=normalize)


def tensor2pilimage(image, width=None, height=None, minus1to1_normalized=False):
    if image.dim() == 4:
        image = image[0]
    if image.dim() == 3 and image.shape[0] > 3:
        image = image[:3]
    if minus1to1_normalized:
        image = (image + 1) / 2
    arr = (image.detach().float().clamp(0, 1).cpu() * 255 + 0.5).byte()
    arr = arr.permute(1, 2, 0).numpy()
    if arr.shape[2] == 1:
        arr = arr[:, :, 0]
    img = Image.fromarray(arr)
    if width is not None and height is not None:
        img = img.resize((width, height), Image.BICUBIC)
    return img


def tensor2im(image_tensor, imtype=np.uint8, normalize=True, three_channel_output=True):
    """Convert [-1,1] (or [0,1]) tensors (3/4/5-D) to uint8 HWC numpy arrays."""
    if image_tensor is None:
        return None
    if isinstance(image_tensor, list):
        return [tensor2im(x, imtype, normalize) for x in image_tensor]
    if image_tensor.dim() == 5 or image_tensor.dim() == 4:
        return [tensor2im(image_tensor[idx], imtype, normalize)
                for idx in range(image_tensor.size(0))]
    image_numpy = image_tensor.detach().float().cpu().numpy()
    if normalize:
        image_numpy = (np.transpose(image_numpy, (1, 2, 0)) + 1) / 2.0 * 255.0
    else:
        image_numpy = np.transpose(image_numpy, (1, 2, 0)) * 255.0
    image_numpy = np.clip(image_numpy, 0, 255)
    if image_numpy.shape[2] == 1 and three_channel_output:
        image_numpy = np.repeat(image_numpy, 3, axis=2)
    elif image_numpy.shape[2] > 3:
        image_numpy = image_numpy[:, :, :3]
    return image_numpy.astype(imtype)


# Cityscapes/GTA palettes of the reference (common.py:224-244): 35 train ids, 20 eval ids
_CITYSCAPES_35 = [(0, 0, 0)] * 5 + [
    (111, 74, 0), (81, 0, 81), (128, 64, 128), (244, 35, 232), (250, 170, 160),
    (230, 150, 140), (70, 70, 70), (102, 102, 156), (190, 153, 153), (180, 165, 180),
    (150, 100, 100), (150, 120, 90), (153, 153, 153), (153, 153, 153), (250, 170, 30),
    (220, 220, 0), (107, 142, 35), (152, 251, 152), (70, 130, 180), (220, 20, 60),
    (255, 0, 0), (0, 0, 142), (0, 0, 70), (0, 60, 100), (0, 0, 90), (0, 0, 110),
    (0, 80, 100), (0, 0, 230), (119, 11, 32), (0, 0, 142)]
_CITYSCAPES_20 = [
    (128, 64, 128), (244, 35, 232), (70, 70, 70), (102, 102, 156), (190, 153, 153),
    (153, 153, 153), (250, 170, 30), (220, 220, 0), (107, 142, 35), (152, 251, 152),
    (220, 20, 60), (255, 0, 0), (0, 0, 142), (0, 0, 70), (0, 60, 100), (0, 80, 100),
    (0, 0, 230), (119, 11, 32), (70, 130, 180), (0, 0, 0)]


def labelcolormap(N):
    """[N, 3] uint8 colours for label ids: Cityscapes palettes for N = 35 / 20, otherwise
    the bit-interleaved PASCAL-style palette (common.py:218-256)."""
    if N == 35:
        return np.array(_CITYSCAPES_35, dtype=np.uint8)
    if N == 20:
        return np.array(_CITYSCAPES_20, dtype=np.uint8)
    ids = np.arange(N)
    cmap = np.zeros((N, 3), dtype=np.int64)
    for j in range(8):
        for c in range(3):
            cmap[:, c] += ((ids >> (3 * j + c)) & 1) << (7 - j)
    return cmap.astype(np.uint8)


_label_colormap = labelcolormap


class Colorize(object):
    """Map integer label maps [1, H, W] to RGB [3, H, W] uint8 (common.py:259-290);
    one table gather instead of a per-label mask loop."""

    def __init__(self, n=35):
        self.cmap = torch.from_numpy(labelcolormap(n))

    def __call__(self, gray_image):
        idx = gray_image[0].long().cpu()
        valid = (idx >= 0) & (idx < len(self.cmap))
        color = self.cmap[idx.clamp(0, len(self.cmap) - 1)]
        color[~valid] = 0
        return color.permute(2, 0, 1).contiguous()


def tensor2label(segmap, n_label=None, imtype=np.uint8, colorize=True,
                 output_normalized_tensor=False):
    """One-hot (or index) label map → colour image (common.py:110-153).

    [C,H,W] → HxWx3 ``imtype`` array (HxW indices when ``colorize=False``); batched
    [N,C,H,W] / [N,T,C,H,W] inputs and lists give lists. ``output_normalized_tensor``
    returns a [3,H,W] float tensor in [-1, 1] on the input's device instead.
    """
    if segmap is None:
        return None
    if isinstance(segmap, list):
        return [tensor2label(x, n_label, imtype, colorize, output_normalized_tensor)
                for x in segmap]
    if segmap.dim() == 5 or segmap.dim() == 4:
        return [tensor2label(segmap[i], n_label, imtype, colorize, output_normalized_tensor)
                for i in range(segmap.size(0))]
    device = segmap.device
    segmap = segmap.detach().float().cpu()
    if n_label is None:
        n_label = segmap.size(0)
    if segmap.size(0) > 1:
        segmap = segmap.max(0, keepdim=True)[1]
    if output_normalized_tensor:
        out = Colorize(max(n_label, 2))(segmap).float() / 255.0
        return (out * 2 - 1).to(device)
    if colorize:
        return np.transpose(Colorize(max(n_label, 2))(segmap).numpy(), (1, 2, 0)).astype(imtype)
    return segmap.numpy().astype(imtype)


def tensor2flow(tensor, imtype=np.uint8):
    """Optical flow [2, H, W] → HSV-coded RGB uint8 (common.py:156-191)."""
    if tensor.dim() == 5 or tensor.dim() == 4:
        return [tensor2flow(tensor[b]) for b in range(tensor.size(0))]
    flow = tensor.detach().float().cpu().numpy().transpose(1, 2, 0)
    mag = np.sqrt(flow[..., 0] ** 2 + flow[..., 1] ** 2)
    ang = np.arctan2(flow[..., 1], flow[..., 0])
    hsv = np.zeros(flow.shape[:2] + (3,), dtype=np.uint8)
    hsv[..., 0] = ((ang + np.pi) * 180 / np.pi / 2).astype(np.uint8)
    hsv[..., 1] = 255
    mmax = mag.max() if mag.max() > 0 else 1.0
    hsv[..., 2] = np.clip(mag / mmax * 255, 0, 255).astype(np.uint8)
    return np.asarray(Image.fromarray(hsv, mode='HSV').convert('RGB'))


def plot_keypoints_on_black(resize_h, resize_w, crop_h, crop_w, is_flipped, cfgdata,
                            keypoints):
    """Keypoints ([N, 2] or [T, N, 2]) as green discs on black crop_h x crop_w RGB images,
    one per frame — a dataset ``vis::`` op (common.py:282-311)."""
    kp = np.asarray(keypoints)
    if kp.ndim == 2 and kp.shape[1] == 2:
        kp = kp[np.newaxis]
    return [plot_keypoints(np.zeros((crop_h, crop_w, 3), np.uint8), kp[t], radius=5)
            for t in range(kp.shape[0])]


def save_tensor_image(filename, image, minus1to1_normalized=False):
    """Save a [3, H, W] tensor in [0, 1] (or [-1, 1]) as an image file (common.py:14-40)."""
    if image.dim() != 3:
        raise ValueError('Image tensor dimension does not equal = 3.')
    if image.size(0) != 3:
        raise ValueError('Image has more than 3 channels.')
    if minus1to1_normalized:
        image = (image + 1) * 0.5
    dirname = os.path.dirname(filename)
    if dirname:
        os.makedirs(dirname, exist_ok=True)
    arr = (image.detach().float().clamp(0, 1).cpu().permute(1, 2, 0).numpy() * 255 + 0.5)
    Image.fromarray(arr.astype(np.uint8)).save(filename)


def plot_keypoints(image, keypoints, radius=4, color=(0, 255, 0)):
    """Draw (x, y) keypoints on an HWC uint8 image."""
    img = np.array(image, copy=True)
    h, w = img.shape[:2]
    for x, y in np.asarray(keypoints).reshape(-1, 2):
        if x < 0 or y < 0:
            continue
        x0, x1 = int(max(0, x - radius)), int(min(w, x + radius + 1))
        y0, y1 = int(max(0, y - radius)), int(min(h, y + radius + 1))
        img[y0:y1, x0:x1] = color
    return img
