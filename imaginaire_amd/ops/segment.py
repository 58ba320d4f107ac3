"""Instance-wise segment mean (pix2pixHD encoder pooling).

Reference generators/pix2pixHD.py:323-349 loops in Python over instance ids and batch entries
with ``.nonzero()`` (a host sync per instance). Here the (batch, instance-id) pairs are hashed
to one key per pixel and SORTED (a static-shape device sort, no host sync — so the pooling
also runs inside a captured hipGraph, where ``torch.unique``'s data-dependent output size
cannot): run starts of the sorted keys give a dense segment id per pixel, per-segment channel
sums and counts go into a pixel-count-sized table with ``index_add_``, and the means are
gathered back.
"""
import torch


def instance_mean(features, instance_map):
    """Replace every feature by the mean over its (sample, instance) region."""
    b, c, h, w = features.shape
    inst = instance_map.reshape(b, -1).long()
    key = (inst + (torch.arange(b, device=inst.device).view(b, 1) << 32)).reshape(-1)
    n = key.numel()
    sk, perm = torch.sort(key)
    start = torch.ones_like(sk, dtype=torch.long)
    start[1:] = (sk[1:] != sk[:-1]).long()
    seg_sorted = torch.cumsum(start, 0) - 1          # dense segment id in sorted order
    seg = torch.empty_like(seg_sorted)
    seg[perm] = seg_sorted                           # segment id of every pixel
    feats = features.permute(0, 2, 3, 1).reshape(-1, c).float()
    sums = torch.zeros(n, c, device=features.device, dtype=torch.float32)
    sums.index_add_(0, seg, feats)
    counts = torch.zeros(n, device=features.device, dtype=torch.float32)
    counts.index_add_(0, seg, torch.ones_like(seg, dtype=torch.float32))
    means = sums / counts.clamp_min(1).unsqueeze(1)
    out = means.index_select(0, seg).reshape(b, h, w, c).permute(0, 3, 1, 2)
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
