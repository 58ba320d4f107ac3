"""Instance-wise segment mean (pix2pixHD encoder pooling).

Reference generators/pix2pixHD.py:323-349 loops in Python over instance ids
and batch entries with ``.nonzero()`` (a host sync per instance). Here the
(batch, instance-id) pairs are hashed to one key, mapped to dense segments
with a single device ``unique``, and per-segment channel means are computed
with ``index_add_`` (device atomics) and gathered back — one host sync total.
"""
import torch


def instance_mean(features, instance_map):
    """Replace every feature by the mean over its (sample, instance) region."""
    b, c, h, w = features.shape
    inst = instance_map.reshape(b, -1).long()
    key = inst + (torch.arange(b, device=inst.device).view(b, 1) << 32)
    uniq, inverse = torch.unique(key.reshape(-1), return_inverse=True)
    nseg = uniq.numel()
    feats = features.permute(0, 2, 3, 1).reshape(-1, c).float()
    sums = torch.zeros(nseg, c, device=features.device, dtype=torch.float32)
    sums.index_add_(0, inverse, feats)
    counts = torch.zeros(nseg, device=features.device, dtype=torch.float32)
    counts.index_add_(0, inverse, torch.ones_like(inverse, dtype=torch.float32))
    means = sums / counts.clamp_min(1).unsqueeze(1)
    out = means.index_select(0, inverse).reshape(b, h, w, c).permute(0, 3, 1, 2)
    return out.to(features.dtype).contiguous()


def get_edges(t):
    """4-neighbour instance boundary map (reference model_utils/pix2pixHD.py:137-154)."""
    edge = torch.zeros(t.size(), dtype=torch.bool, device=t.device)
    dx = t[:, :, :, 1:] != t[:, :, :, :-1]
    dy = t[:, :, 1:, :] != t[:, :, :-1, :]
    edge[:, :, :, 1:] |= dx
    edge[:, :, :, :-1] |= dx
    edge[:, :, 1:, :] |= dy
    edge[:, :, :-1, :] |= dy
    return edge.float()
