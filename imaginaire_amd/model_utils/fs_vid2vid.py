"""Video-model utilities (reference model_utils/fs_vid2vid.py:14-865).

``resample`` (flow warp with bilinear sampling, border padding,
align_corners=True) runs on the HIP warp kernel (k9, ops/flow_warp.py) on
MI355X; the remaining helpers are small tensor manipulations.
"""
import random

import numpy as np
import torch
import torch.nn.functional as F

from imaginaire_amd.ops.flow_warp import flow_warp


def resample(image, flow):
    """Warp ``image`` by ``flow`` (pixels, [B,2,H,W]) — reference fs_vid2vid.py:14-38."""
    assert flow.shape[1] == 2
    return flow_warp(image, flow)


def get_grid(batchsize, size, minval=-1.0, maxval=1.0, device=None):
    if len(size) == 2:
        rows, cols = size
    elif len(size) == 3:
        deps, rows, cols = size
    else:
        raise ValueError('Dimension can only be 2 or 3.')
    x = torch.linspace(minval, maxval, cols, device=device).view(1, 1, 1, cols)
    x = x.expand(batchsize, 1, rows, cols)
    y = torch.linspace(minval, maxval, rows, device=device).view(1, 1, rows, 1)
    y = y.expand(batchsize, 1, rows, cols)
    t_grid = torch.cat([x, y], dim=1)
    if len(size) == 3:
        z = torch.linspace(minval, maxval, deps, device=device).view(1, 1, deps, 1, 1)
        z = z.expand(batchsize, 1, deps, rows, cols)
        t_grid = t_grid.unsqueeze(2).expand(batchsize, 2, deps, rows, cols)
        t_grid = torch.cat([t_grid, z], dim=1)
    return t_grid


def pick_image(images, idx):
    if type(images) == list:
        return [pick_image(r, idx) for r in images]
    if idx is None:
        return images[:, 0]
    if type(idx) == int:
        return images[:, idx]
    idx = idx.long().view(-1, 1, 1, 1, 1)
    return images.gather(1, idx.expand_as(images)[:, 0:1])[:, 0]


def concat_frames(prev, now, n_frames):
    """Append ``now`` to the sliding window ``prev`` keeping the last n_frames-1 entries."""
    now = now.unsqueeze(1)
    if prev is None:
        return now
    if prev.shape[1] == n_frames:
        prev = prev[:, 1:]
    return torch.cat([prev, now], dim=1)


def detach(output):
    if type(output) == dict:
        return {k: detach(v) for k, v in output.items()}
    if type(output) == list:
        return [detach(v) for v in output]
    if isinstance(output, torch.Tensor):
        return output.detach()
    return output


def crop_and_resize(img, coords, size=None, method='bilinear'):
    if isinstance(img, list):
        return [crop_and_resize(x, coords, size, method) for x in img]
    if img is None:
        return None
    min_y, max_y, min_x, max_x = coords
    img = img[..., min_y:max_y, min_x:max_x]
    if size is not None:
        if method == 'nearest':
            img = F.interpolate(img.reshape(-1, *img.shape[-3:]), size=size, mode='nearest')
        else:
            img = F.interpolate(img.reshape(-1, *img.shape[-3:]), size=size, mode='bilinear',
                                align_corners=False)
    return img


def random_roll(tensors):
    h = tensors[0].size(2)
    w = tensors[0].size(3)
    ny = np.random.choice([np.random.randint(h // 16), h - np.random.randint(h // 16)])
    nx = np.random.choice([np.random.randint(w // 16), w - np.random.randint(w // 16)])
    return [torch.roll(t, shifts=(int(ny), int(nx)), dims=(2, 3)) for t in tensors]


def select_object(data, obj_indices=None):
    """Keep only the selected object's instance in the label maps (fs_vid2vid.py:378-402)."""
    op_key = 'human_instance_maps'
    if op_key in data:
        for i in range(len(data[op_key])):
            people_map = data[op_key][i]
            if obj_indices is None:
                obj_idx = 0
            else:
                obj_idx = obj_indices[i] if i < len(obj_indices) else obj_indices[0]
            mask = (people_map == obj_idx + 1).astype(np.float32) if isinstance(people_map, np.ndarray) \
                else people_map
            for key in data:
                if key != op_key and key in ('pose_maps-densepose', 'poses-openpose'):
                    if isinstance(data[key][i], np.ndarray) and data[key][i].ndim == 3:
                        data[key][i] = data[key][i] * mask[..., :1] if mask.ndim == 3 else \
                            data[key][i] * mask[..., None]
    return data
