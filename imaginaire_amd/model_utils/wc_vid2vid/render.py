"""World-consistent vid2vid point-cloud splat renderer
(reference model_utils/wc_vid2vid/render.py:11-199).

The reference keeps the colour / seen-mask / first-seen-time arrays of the
3-D point cloud in host numpy and re-renders per frame on the CPU. Here the
arrays live on the device the frames live on (HBM on MI355X): updating the
cloud with a new frame and splatting it into a guidance image are two
index_put / gather launches, so guidance rendering never round-trips
through the host.

Semantics are unchanged: a point's colour is fixed the first time it is
seen; rendering writes the stored colour of every visible point and a 255
mask where the point has been seen. Duplicate targets (one point id listed
twice in a frame, two points projecting to one pixel) resolve as numpy's
fancy-index assignment does — the LAST row wins (reference render.py:87-97,
138) — by a scatter-max of row numbers that keeps only each target's winning
row before a duplicate-free index_put (a plain device index_put with duplicate
indices has an undefined write order).
"""
import json
import os

import numpy as np
import torch


def _last_rows(target, size):
    """Boolean mask of the rows of ``target`` (1-D long) that are the last occurrence of their
    value: numpy's last-write-wins order for ``a[target] = values``, made deterministic."""
    rows = torch.arange(target.numel(), device=target.device)
    last = torch.full((size,), -1, dtype=torch.long, device=target.device)
    last.scatter_reduce_(0, target, rows, reduce='amax')
    return last[target] == rows


class SplatRenderer(object):
    def __init__(self, device=None):
        self.device = device
        self.reset()

    def reset(self):
        self.seen_mask = None
        self.seen_time = None
        self.colors = None
        self.call_idx = 0

    def num_points(self):
        return 0 if self.seen_mask is None else int(self.seen_mask.sum())

    def _as_index(self, point_info, device):
        p = torch.as_tensor(np.asarray(point_info), device=device).long()
        return p[:, 0], p[:, 1], p[:, 2]

    def _resize_arrays(self, max_point_idx, device):
        old = 0 if self.colors is None else self.colors.shape[0]
        if max_point_idx > old:
            colors = torch.zeros(max_point_idx, 3, dtype=torch.uint8, device=device)
            seen = torch.zeros(max_point_idx, 1, dtype=torch.uint8, device=device)
            seen_t = torch.zeros(max_point_idx, 1, dtype=torch.int32, device=device)
            if old:
                colors[:old] = self.colors
                seen[:old] = self.seen_mask
                seen_t[:old] = self.seen_time
            self.colors, self.seen_mask, self.seen_time = colors, seen, seen_t

    def update_point_cloud(self, image, point_info):
        """image: HxWx3 uint8 (numpy or tensor); point_info: Nx3 (i, j, point id)."""
        if point_info is None or len(point_info) == 0:
            return
        image = torch.as_tensor(np.ascontiguousarray(image) if isinstance(image, np.ndarray)
                                else image)
        device = self.device or image.device
        image = image.to(device)
        self.call_idx += 1
        i, j, pid = self._as_index(point_info, device)
        self._resize_arrays(int(pid.max()) + 1, device)
        keep = _last_rows(pid, self.colors.shape[0])
        i, j, pid = i[keep], j[keep], pid[keep]
        seen = self.seen_mask[pid]
        self.colors[pid] = seen * self.colors[pid] + (1 - seen) * image[i, j].to(torch.uint8)
        self.seen_time[pid] = seen.int() * self.seen_time[pid] + \
            (1 - seen.int()) * self.call_idx
        self.seen_mask[pid] = 1

    def render_image(self, point_info, w, h, return_mask=False):
        device = self.device or (self.colors.device if self.colors is not None else 'cpu')
        output = torch.zeros(h, w, 3, dtype=torch.uint8, device=device)
        mask = torch.zeros(h, w, 1, dtype=torch.uint8, device=device)
        if point_info is not None and len(point_info) != 0:
            i, j, pid = self._as_index(point_info, device)
            self._resize_arrays(int(pid.max()) + 1, device)
            keep = _last_rows(i * w + j, h * w)
            i, j, pid = i[keep], j[keep], pid[keep]
            output[i, j] = self.colors[pid]
            mask[i, j] = 255 * self.seen_mask[pid]
        output, mask = output.cpu().numpy(), mask.cpu().numpy()
        return (output, mask) if return_mask else output


def _load_item(item):
    """Decode one serialized unprojection record: JSON (preferred) or, only
    when IMAGINAIRE_AMD_ALLOW_PICKLE=1, the reference's pickle format."""
    if isinstance(item, dict):
        return item
    if isinstance(item, (bytes, bytearray)):
        try:
            return json.loads(item.decode('utf-8'))
        except (UnicodeDecodeError, ValueError):
            if os.environ.get('IMAGINAIRE_AMD_ALLOW_PICKLE', '0') != '1':
                raise ValueError('unprojection record is not JSON; set '
                                 'IMAGINAIRE_AMD_ALLOW_PICKLE=1 to decode trusted pickles')
            import pickle
            return pickle.loads(item)  # noqa: S301 (explicit opt-in, trusted data)
    return json.loads(item)


def decode_unprojections(data):
    """List of per-frame {resolution: flat [i, j, id, ...]} records ->
    {resolution: [T, max_len + 1, 3] int array}; each row list is padded with
    -1 and ends with a sentinel row holding its length (render.py:150-199)."""
    per_res = {}
    for item in data:
        for resolution, value in _load_item(item).items():
            per_res.setdefault(resolution, []).append(list(value) if value else [])
    outputs = {}
    for resolution, values in per_res.items():
        max_len = max(len(v) for v in values)
        rows = []
        for v in values:
            assert len(v) % 3 == 0
            padded = v + [-1] * (max_len - len(v)) + [len(v) // 3] * 3
            rows.append(np.array(padded).reshape(-1, 3))
        outputs[resolution] = np.stack(rows, axis=0)
    return outputs
