"""Instance-wise segment mean (pix2pixHD encoder pooling).

Reference generators/pix2pixHD.py:323-349 loops in Python over instance ids and batch entries
with ``.nonzero()`` (a host sync per instance). Here the (batch, instance-id) pairs are hashed
to one key per pixel and SORTED (a static-shape device sort, no host sync — so the pooling
also runs inside a captured hipGraph, where ``torch.unique``'s data-dependent output size
cannot). In sorted order every segment is a contiguous run: its sum is the difference of an
fp64 running sum (cumsum) at the run's two ends and its count the run length, found with a
cummax / reversed cummax of the run boundaries. The averaging operator is symmetric, so the
backward is the same segment mean of the incoming gradient (an autograd Function: no
``index_add_`` scatter in either direction). No atomics anywhere: the earlier ``index_add_``
into a per-segment table serialised on the few large instances (~20 ms per pix2pixHD 512x1024
iteration, profiles/recipe_pix2pixhd512x1024_kernels_mi355x.txt).
"""
import torch


def _runs(key):
    """Sort order of ``key`` and, per sorted position, the first / last sorted position of its
    run of equal keys."""
    n = key.numel()
    sk, perm = torch.sort(key)
    pos = torch.arange(n, device=key.device)
    first = torch.ones(n, dtype=torch.bool, device=key.device)
    first[1:] = sk[1:] != sk[:-1]
    last = torch.ones(n, dtype=torch.bool, device=key.device)
    last[:-1] = first[1:]
    zero = torch.zeros_like(pos)
    s = torch.cummax(torch.where(first, pos, zero), 0)[0]
    e = (n - 1) - torch.cummax(torch.where(last, n - 1 - pos, zero).flip(0), 0)[0].flip(0)
    return perm, s, e


def _segment_mean(x, perm, s, e):
    """x [n, c] (pixel order) -> per-pixel mean over its run (same layout, fp32)."""
    c = x.shape[1]
    cs = torch.cumsum(x.index_select(0, perm).double(), 0)
    cs = torch.cat([cs.new_zeros((1, c)), cs], 0)        # cs[i] = sum of the first i sorted rows
    seg = cs.index_select(0, e + 1) - cs.index_select(0, s)
    means = (seg / (e - s + 1).unsqueeze(1).double()).to(torch.float32)
    out = torch.empty_like(means)
    out[perm] = means                                     # back to pixel order (a permutation)
    return out


class _SegmentMean(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, perm, s, e):
        ctx.save_for_backward(perm, s, e)
        return _segment_mean(x, perm, s, e)

    @staticmethod
    def backward(ctx, g):
        perm, s, e = ctx.saved_tensors
        return _segment_mean(g.float(), perm, s, e), None, None, None


def instance_mean(features, instance_map):
    """Replace every feature by the mean over its (sample, instance) region."""
    b, c, h, w = features.shape
    inst = instance_map.reshape(b, -1).long()
    key = (inst + (torch.arange(b, device=inst.device).view(b, 1) << 32)).reshape(-1)
    perm, s, e = _runs(key)
    feats = features.permute(0, 2, 3, 1).reshape(-1, c).float()
    out = _SegmentMean.apply(feats, perm, s, e)
    return out.reshape(b, h, w, c).permute(0, 3, 1, 2).to(features.dtype).contiguous()


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
