"""Fused bias + activation epilogue (k2, ``csrc/bias_act.hip``).

Used after a bias-free MIOpen convolution / linear for the reference's
``CA``/``CNA``-without-norm block orders (layers/conv.py:59-91). The activation
is a leaky slope (0 = relu, 0.2 = leakyrelu, 1 = identity). The backward uses
the sign of the *output* (valid for slope > 0 and for relu), so the
pre-activation never has to be kept alive.
"""
import torch
import torch.nn.functional as F

from imaginaire_amd.ops import _ext


class _BiasActFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, bias, slope):
        out = _ext.ext().bias_act_fwd(x, bias, slope, False)
        ctx.slope = slope
        ctx.has_bias = bias is not None
        ctx.bias_dtype = bias.dtype if bias is not None else None
        ctx.save_for_backward(out)
        return out

    @staticmethod
    def backward(ctx, dy):
        (out,) = ctx.saved_tensors
        dx, db = _ext.ext().bias_act_bwd(out, dy, ctx.slope)
        return dx, (db.to(ctx.bias_dtype) if ctx.has_bias and ctx.needs_input_grad[1] else None), None


def bias_act(x, bias=None, slope=1.0):
    """``act(x + bias[c])`` with channel dim 1."""
    if _ext.use_native(x) and (x.dim() in (2, 4)):
        if not (x.is_contiguous() or x.is_contiguous(memory_format=torch.channels_last)):
            x = x.contiguous()
        if slope == 1.0 and bias is None:
            return x
        return _BiasActFn.apply(x, bias, float(slope))
    if bias is not None:
        shape = [1, -1] + [1] * (x.dim() - 2)
        x = x + bias.reshape(shape).to(x.dtype)
    if slope == 1.0:
        return x
    if slope == 0.0:
        return F.relu(x)
    return F.leaky_relu(x, slope)
