"""Instance-wise segment mean (pix2pixHD encoder pooling).

Reference generators/pix2pixHD.py:323-349 loops in Python over instance ids and batch entries
with ``.nonzero()`` (a host sync per instance). Here the (batch, instance-id) pairs are hashed
to one key per pixel and SORTED (a static-shape device sort, no host sync — so the pooling
also runs inside a captured hipGraph, where ``torch.unique``'s data-dependent output size
cannot). In sorted order every segment is a contiguous run, located per position by two binary
searches of its own key (``searchsorted`` left / right). Its sum is the difference of an fp64
running sum at the run's two ends — ONE flat 1-D cumsum over the channel-major [C, n] copy
(the device-wide scan; a cumsum along dim 0 of [n, C] ran as a near-serial outer-dim scan,
~150 ms at 1 M pixels) — and its count the run length. The averaging operator is symmetric, so
the backward is the same segment mean of the incoming gradient (an autograd Function: no
``index_add_`` scatter in either direction). No atomics anywhere: the earlier ``index_add_``
into a per-segment table serialised on the few large instances (~20 ms per pix2pixHD 512x1024
iteration, profiles/recipe_pix2pixhd512x1024_kernels_mi355x.txt).
"""
import torch


def _runs(key):
    """Sort order of ``key`` and, per sorted position, the first / last sorted position of its
    run of equal keys."""
    sk, perm = torch.sort(key)
    s = torch.searchsorted(sk, sk)
    e = torch.searchsorted(sk, sk, right=True) - 1
    return perm, s, e


def _segment_mean(x, perm, s, e):
    """x [n, c] (pixel order) -> per-pixel mean over its run (same layout, fp32)."""
    n, c = x.shape
    xs = x.index_select(0, perm).double().t().contiguous()          # [c, n], sorted order
    cs = torch.cumsum(xs.reshape(-1), 0)
    cs = torch.cat([cs.new_zeros(1), cs])                # cs[j] = sum of the first j flat items
    off = (torch.arange(c, device=x.device) * n).unsqueeze(1)      # channel row offsets
    seg = cs[off + (e + 1).unsqueeze(0)] - cs[off + s.unsqueeze(0)]
    means = (seg / (e - s + 1).unsqueeze(0).double()).to(torch.float32).t()
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
