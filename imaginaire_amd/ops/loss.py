"""Multi-tensor weighted L1 (k13) and GAN loss (k13b), ``csrc/loss.hip``.

``weighted_l1(as_, bs, weights) = sum_t weights[t] * mean(|as_[t] - bs[t]|)`` as one forward
and one backward launch over every pair (fp32 accumulation, bf16 features read in place,
deterministic fixed-order reduction). Used by the perceptual and feature-matching losses
(reference losses/perceptual.py:139-180, losses/feature_matching.py:19-38), which PyTorch
autocast would otherwise run as per-layer fp32 copies + l1_loss. CPU / unsupported inputs
use ``F.l1_loss`` with identical math.
"""
import torch
import torch.nn.functional as F

from imaginaire_amd.ops import _ext

_MAX_PAIRS = 16


class _MultiL1(torch.autograd.Function):
    @staticmethod
    def forward(ctx, weights, *ts):
        a, b = list(ts[0::2]), list(ts[1::2])
        ctx.weights = weights
        ctx.save_for_backward(*ts)
        return _ext.ext().mt_l1_loss(a, b, weights)

    @staticmethod
    def backward(ctx, g):
        ts = ctx.saved_tensors
        a, b = list(ts[0::2]), list(ts[1::2])
        need = ctx.needs_input_grad[1::2]
        grads = _ext.ext().mt_l1_loss_backward(a, b, ctx.weights, g) if any(need) else \
            [None] * len(a)
        out = [None]
        for ga, na in zip(grads, need):
            out += [ga if na else None, None]
        return tuple(out)


def _native_target(a, b):
    """``b`` (detached) in ``a``'s memory layout for the k13 kernel, or None when the pair stays
    on the PyTorch path. The targets of the feature-matching loss come from the real branch of a
    discriminator that still tracks grad, and may differ in layout or dtype from the fake
    features: re-laying them out is one pass, the fp32 ``l1_loss`` fallback was three (fp32
    copies of both operands + the difference; 1.4 GB per vid2vid recipe iteration). An fp32
    target of a bf16 input stays fp32 (the kernel reads it unrounded, as autocast's fp32
    ``l1_loss`` does); other dtypes are cast to ``a``'s."""
    if not (a.is_cuda and _ext.use_native(a) and a.dtype in (torch.bfloat16, torch.float32) and
            a.shape == b.shape and _ext.is_dense(a) and b.is_cuda):
        return None
    b = b.detach()
    dt = torch.float32 if b.dtype == torch.float32 else a.dtype
    if b.dtype == dt and b.stride() == a.stride():
        return b
    return torch.empty_like(a, dtype=dt).copy_(b)  # empty_like keeps a's (dense) strides


def weighted_l1(as_, bs, weights):
    """sum_t weights[t] * mean(|as_[t] - bs[t]|) as an fp32 scalar (``bs`` treated as
    constants, like the detached targets of both callers)."""
    as_, bs, weights = list(as_), list(bs), [float(w) for w in weights]
    total = None
    tg = [_native_target(a, b) for a, b in zip(as_, bs)]
    native = [i for i in range(len(as_)) if tg[i] is not None]
    # one launch per (input dtype, target dtype) class, at most _MAX_PAIRS pairs each
    groups = {}
    for i in native:
        groups.setdefault((as_[i].dtype, tg[i].dtype), []).append(i)
    chunks = [g[s:s + _MAX_PAIRS] for g in groups.values() for s in range(0, len(g), _MAX_PAIRS)]
    for idx in chunks:
        args = []
        for i in idx:
            args += [as_[i], tg[i]]
        v = _MultiL1.apply([weights[i] for i in idx], *args)
        total = v if total is None else total + v
    for i in sorted(set(range(len(as_))) - set(native)):
        v = weights[i] * F.l1_loss(as_[i], bs[i].detach()).float()
        total = v if total is None else total + v
    if total is None:
        raise ValueError('weighted_l1: empty input')
    return total


class _MultiGan(torch.autograd.Function):
    @staticmethod
    def forward(ctx, spec, *xs):
        ctx.spec = spec
        ctx.save_for_backward(*xs)
        return _ext.ext().mt_gan_loss(list(xs), *spec)

    @staticmethod
    def backward(ctx, g):
        xs = ctx.saved_tensors
        need = ctx.needs_input_grad[1:]
        grads = _ext.ext().mt_gan_loss_backward(list(xs), *ctx.spec, g) if any(need) else \
            [None] * len(xs)
        return (None,) + tuple(gr if n else None for gr, n in zip(grads, need))


# phi kinds of csrc/loss.hip k13b
GAN_RELU, GAN_LINEAR, GAN_BCE, GAN_LSQ = 0, 1, 2, 3


def _gan_phi_ref(kind, a, b, x):
    x = x.float()
    if kind == GAN_RELU:
        return F.relu(a + b * x).mean()
    if kind == GAN_LINEAR:
        return (b * x).mean()
    if kind == GAN_BCE:
        return F.binary_cross_entropy_with_logits(x, torch.full_like(x, a))
    return 0.5 * F.mse_loss(x, torch.full_like(x, a))


def gan_loss_multi(xs, kind, a=0.0, b=1.0, weight=1.0):
    """``weight * sum_t mean(phi(xs[t]))`` for one phi over every discriminator output, as one
    k13b forward + one backward launch (fp32 accumulation, fixed-order reduction). ``phi`` is
    relu(a + b x) (hinge D), b x (hinge G / wasserstein), BCE-with-logits against target a
    (non_saturated) or 0.5 (x - a)^2 (least squares). CPU / non-native inputs: same math in
    PyTorch ops."""
    xs = list(xs)
    native = len(xs) <= _MAX_PAIRS and all(
        x.is_cuda and _ext.use_native(x) and x.dtype in (torch.bfloat16, torch.float32) and
        x.dtype == xs[0].dtype and _ext.is_dense(x) for x in xs)
    if not native:
        total = None
        for x in xs:
            v = _gan_phi_ref(kind, a, b, x)
            total = v if total is None else total + v
        return weight * total
    n = len(xs)
    spec = ([kind] * n, [float(a)] * n, [float(b)] * n, [float(weight)] * n)
    return _MultiGan.apply(spec, *xs)
