"""NHWC convolution entry points.

Every 2-D convolution issued by the framework's layers goes through here.

* **MFMA path (k10, ``csrc/conv_mfma.hip``).** bf16 (autocast or bf16 tensors), groups 1,
  Cout % 64 == 0, Cin a multiple of 64 after zero-padding (pad overhead ≤ 1/3), and enough
  output pixels to fill the chip: the forward runs the hand-written implicit-GEMM kernel
  (global_load_lds staging, v_mfma_f32_16x16x32_bf16, fused bias + leaky/relu epilogue);
  the stride-1 data gradient runs the SAME kernel on the flipped, transposed weight; the
  weight gradient runs the k11 kernel (``csrc/conv_wgrad_mfma.hip``: transposing LDS reads,
  split-K over pixels) or MIOpen's wrw, whichever was measured faster for the shape (first
  call). The activation backward + bias gradient is the k2 epilogue kernel.
* **MIOpen path.** Everything else. MIOpen's fast NHWC solvers require *packed* NHWC
  activations AND weights, otherwise they fall back to naive direct kernels (measured
  at >95% of a SPADE step on MI355X, profiles/spade_step_naive_conv_mi355x.txt), so both
  operands are made packed channels-last. Odd channel counts above 64 (185-channel label
  maps, 188-channel D inputs) are zero-padded to a multiple of 32 first: MIOpen's igemm
  kernels run 2.4-2.6x faster on 192 than on 185 channels
  (profiles/conv_pad_probe_mi355x.txt).

Reference: the reference's blocks call cuDNN through ``nn.Conv2d`` (layers/conv.py:59-91).
"""
import os

import torch
import torch.nn.functional as F

from imaginaire_amd.ops import _ext

_CL = torch.channels_last
# tiny grids (fewer 128-pixel x BN-channel tiles than this) stay on MIOpen; k10 splits K
# itself when its tile grid cannot fill the chip
_MFMA_MIN_BLOCKS = int(os.environ.get('IMAGINAIRE_AMD_MFMA_MIN_BLOCKS', '16'))
_MFMA_MIN_DGRAD_BLOCKS = int(os.environ.get('IMAGINAIRE_AMD_MFMA_MIN_DGRAD_BLOCKS', '16'))
# weight gradient: '1' = k11 (default: faster than MIOpen wrw on every SPADE/D/VGG shape in
# profiles/conv_mfma_probe_mi355x.txt, and it compiles nothing at first call), '0' = MIOpen,
# 'auto' = per-shape faster of the two (timed once; the choice is agreed across ranks)
_MFMA_WGRAD = os.environ.get('IMAGINAIRE_AMD_MFMA_WGRAD', '1')


# ---- per-call conv log (IMAGINAIRE_AMD_CONV_LOG=1 or enable_conv_log()): every k10 / k11 /
# MIOpen call of the steps that follow is timed with a pair of device events and recorded with
# its GEMM shape, so bench.py --conv-log can print time and TF/s per (kind, shape, kernel).
_CONV_LOG = [] if os.environ.get('IMAGINAIRE_AMD_CONV_LOG', '0') == '1' else None


def enable_conv_log(on=True):
    global _CONV_LOG
    _CONV_LOG = [] if on else None


class _Logged(object):
    """Context manager timing one conv kernel call into ``_CONV_LOG``."""
    __slots__ = ('rec',)

    def __init__(self, kind, path, flops, desc):
        self.rec = None
        if _CONV_LOG is not None and not torch.cuda.is_current_stream_capturing():
            self.rec = [kind, path, flops, desc, torch.cuda.Event(enable_timing=True),
                        torch.cuda.Event(enable_timing=True)]

    def __enter__(self):
        if self.rec is not None:
            self.rec[4].record()
        return self

    def __exit__(self, *exc):
        if self.rec is not None:
            self.rec[5].record()
            if self.rec[1].startswith('k10'):  # which k10 tile ran (csrc conv_last_variant)
                self.rec[1] += '/v%d' % _ext.ext().conv_last_variant()
            _CONV_LOG.append(self.rec)
        return False


def conv_log_summary(reset=True):
    """[(kind, path, desc, calls, ms, TF/s)] sorted by total time (synchronises)."""
    if _CONV_LOG is None:
        return []
    torch.cuda.synchronize()
    agg = {}
    for kind, path, flops, desc, e0, e1 in _CONV_LOG:
        a = agg.setdefault((kind, path, desc), [0, 0.0, 0.0])
        a[0] += 1
        a[1] += e0.elapsed_time(e1)
        a[2] += flops
    if reset:
        del _CONV_LOG[:]
    rows = [(k[0], k[1], k[2], v[0], v[1], v[2] / max(v[1], 1e-9) / 1e9) for k, v in agg.items()]
    rows.sort(key=lambda r: -r[4])
    return rows


def _gemm_desc(x, w, stride, padding):
    return '%s x %s s%s p%s' % (list(x.shape), list(w.shape), stride[0], padding[0])


def _mfma_enabled():
    return os.environ.get('IMAGINAIRE_AMD_MFMA_CONV', '1') == '1' and not _ext.force_eager()


def nhwc(t):
    """Packed channels-last view/copy of a 4-D CUDA tensor (identity otherwise)."""
    if t is not None and t.is_cuda and t.dim() == 4 and not t.is_contiguous(memory_format=_CL):
        return t.contiguous(memory_format=_CL)
    return t


def _pad_arg(padding):
    if isinstance(padding, int):
        return [padding] * 4
    ph, pw = padding
    return [pw, pw, ph, ph]


def _pair(v):
    return (v, v) if isinstance(v, int) else tuple(v)


def _round_up(c, m):
    return (c + m - 1) // m * m


def _out_pad(cout):
    """k10 output-channel padding (a multiple of 64: a 32-wide tile for the 3-channel RGB
    output measured slower than the 64-wide one — the A-operand stream, not the wasted MFMA
    columns, bounds those convs; profiles/spade_step_conv_log_mi355x.txt)."""
    return _round_up(cout, 64)


def _pad_channels(t, c, dtype=None):
    """Zero-pad dim 1 of a 4-D tensor to ``c`` channels (packed channels-last result), cast to
    ``dtype`` (default: t's). Outside autograd on the GPU this is ONE pass of the
    ``pad_channels_cast`` kernel (16-byte stores of whole padded pixels, any input layout);
    differentiable inputs keep the autograd-visible slice copy."""
    dtype = dtype or t.dtype
    one_pass = t.is_cuda and t.dim() == 4 and c % 8 == 0 and _ext.use_native(t) and \
        t.dtype in (torch.bfloat16, torch.float32) and \
        dtype in (torch.bfloat16, torch.float32) and \
        not (t.requires_grad and torch.is_grad_enabled())
    if t.shape[1] == c:
        # a cast of a non-channels-last tensor (an fp32 OIHW weight) is a cast pass plus a
        # layout pass through PyTorch: one pad_channels_cast pass instead
        if one_pass and t.dtype != dtype and not t.is_contiguous(memory_format=_CL):
            return _ext.ext().pad_channels_cast(t, c, dtype)
        return nhwc(t.to(dtype))
    if one_pass:
        return _ext.ext().pad_channels_cast(t, c, dtype)
    out = torch.empty((t.shape[0], c, t.shape[2], t.shape[3]), dtype=dtype, device=t.device,
                      memory_format=_CL)
    out[:, t.shape[1]:].zero_()
    out[:, :t.shape[1]] = t
    return out


class _StackNHWC(torch.autograd.Function):
    """Forward of :func:`stack_nhwc`; the backward hands every input the matching slice of the
    padded gradient (a view: no clone of the whole padded gradient and no per-slice copies,
    which autograd's CopySlices made — 2.2 GB per vid2vid recipe iteration for the 64-channel
    discriminator inputs)."""

    @staticmethod
    def forward(ctx, dtype, align, widths, n, *ts):
        first = ts[0]
        c = sum(widths)
        cp = _round_up(c, align)
        out = torch.empty((sum(n), cp) + tuple(first.shape[2:]), dtype=dtype,
                          device=first.device, memory_format=_CL)
        i = o = 0
        ctx.slices = []
        for k in n:
            ch = 0
            for wd in widths:
                out[o:o + k, ch:ch + wd] = ts[i]
                ctx.slices.append((o, k, ch, wd, ts[i].dtype))
                ch += wd
                i += 1
            o += k
        if cp > c:
            out[:, c:].zero_()
        return out

    @staticmethod
    def backward(ctx, g):
        grads = []
        for (o, k, ch, wd, dt), need in zip(ctx.slices, ctx.needs_input_grad[4:]):
            grads.append(g[o:o + k, ch:ch + wd].to(dt) if need else None)
        return (None, None, None, None) + tuple(grads)


def stack_nhwc(rows, dtype=None, align=64):
    """``cat([cat(row, 1) for row in rows], 0)`` written ONCE into a channel-padded NHWC
    buffer (channels rounded up to ``align``, zero tail marked for the convs): the
    discriminator inputs label|image for real and fake, without the two channel concats, the
    batch concat, the fp32 -> bf16 cast and the conv's own zero-padding copy. ``dtype``
    defaults to the autocast dtype (or the first tensor's). Every row holds tensors of the
    same channel widths."""
    first = rows[0][0]
    if dtype is None:
        dtype = torch.get_autocast_dtype('cuda') if (first.is_cuda and
                                                     torch.is_autocast_enabled('cuda')) \
            else first.dtype
    widths = [t.shape[1] for t in rows[0]]
    assert all([t.shape[1] for t in row] == widths for row in rows), 'stack_nhwc: row widths'
    n = [row[0].shape[0] for row in rows]
    out = _StackNHWC.apply(dtype, align, widths, n, *[t for row in rows for t in row])
    c = sum(widths)
    if _round_up(c, align) > c:
        mark_zero_tail(out, c)
    return out


def mark_zero_tail(t, valid_channels):
    """Declare channels ``[valid_channels:]`` of the NHWC tensor ``t`` to be zeros (a
    channel-padded buffer such as the 192-channel label|image discriminator input). A conv
    whose weight has ``valid_channels`` input channels then consumes ``t`` directly, its weight
    zero-padded to match (tiny), instead of slicing / re-padding the activation every call."""
    t._iamd_valid_channels = int(valid_channels)
    return t


def _match_channels(x, weight):
    cx, cw = x.shape[1], weight.shape[1]
    if cx == cw:
        return weight
    if cx > cw and getattr(x, '_iamd_valid_channels', None) == cw:
        if weight.dim() == 4 and weight.is_cuda:
            return _pad_channels(weight, cx)
        return torch.cat([weight, weight.new_zeros((weight.shape[0], cx - cw) +
                                                   tuple(weight.shape[2:]))], 1)
    raise RuntimeError('conv: input has {} channels, weight expects {}'.format(cx, cw))


def _compute_dtype(x, w):
    if x.is_cuda and torch.is_autocast_enabled('cuda'):
        return torch.get_autocast_dtype('cuda')
    return x.dtype if x.dtype == w.dtype else None


def _out_hw(H, W, k, stride, padding, dilation):
    return ((H + 2 * padding[0] - dilation[0] * (k[0] - 1) - 1) // stride[0] + 1,
            (W + 2 * padding[1] - dilation[1] * (k[1] - 1) - 1) // stride[1] + 1)


# > 0 inside utils.cuda_graph.graph_routing() (a graphed step's warm-up, its capture and
# eager comparisons against it): global, not thread-local — the backward runs on autograd's
# worker thread
_GRAPH_ROUTING = [0]


def _capturing():
    """True while a hipGraph is being captured on the current stream, or inside a graphed
    step's warm-up. MIOpen's backward solvers for small problems accumulate with atomics into
    buffers zeroed by calls that stream capture does not record, so under replay they add onto
    the previous replay's values (the pix2pixHD graph diverged to NaN in its 16 x 16 resblock
    weight gradients, scripts/probe/graph_stash_probe.py): there every conv k10 / k11 can run
    takes them, whatever its grid size."""
    return _GRAPH_ROUTING[0] > 0 or torch.cuda.is_current_stream_capturing()


def mfma_eligible(x, w, stride, padding, dilation, groups):
    """True if the k10 MFMA kernel runs this conv (see module docstring)."""
    if not (x.is_cuda and x.dim() == 4 and w.dim() == 4 and groups == 1 and _mfma_enabled()):
        return False
    if _compute_dtype(x, w) != torch.bfloat16:
        return False
    cout, cin = w.shape[0], w.shape[1]
    cp, op = _round_up(cin, 64), _out_pad(cout)
    # zero-padded channels cost MFMA work: allow ≤ 1/3 waste, except for the thin RGB-facing
    # convs (3-channel image in / out) where MIOpen's kernels run at ~1 TF/s and a 64-channel
    # padded MFMA tile is still an order of magnitude faster (profiles/spade_step_k10_k11)
    # up to 2x padding waste still runs k10 for the 32-channel full-resolution layers of the
    # video models (MIOpen's NHWC bf16 solvers reach only 35-150 TF/s on [2, 32, 512, 1024]
    # 1x1 / 3x3 convs, profiles/recipe_vid2vid512x1024_conv_log_mi355x.txt)
    if cp * op * 3 > cin * cout * 4 and min(cin, cout) > 16 and cp * op > 2 * cin * cout and \
            not _capturing():  # (in a graph: padded MFMA work rather than MIOpen's backward)
        return False
    ho, wo = _out_hw(x.shape[2], x.shape[3], w.shape[2:], stride, padding, dilation)
    if ho <= 0 or wo <= 0 or w.shape[2] * w.shape[3] > 64:  # k10 tap masks are 64-bit
        return False
    # 32-bit buffer byte offsets (k10 < 2 GiB operands, k11 < 1 GiB)
    if x.shape[0] * cp * x.shape[2] * x.shape[3] * 2 >= (1 << 30) or \
            x.shape[0] * op * ho * wo * 2 >= (1 << 30):
        return False
    blocks = -(-x.shape[0] * ho * wo // 128) * max(1, op // (128 if op % 128 == 0 else 64))
    # deterministic mode: tiny grids run k10 too (its split-K sums slabs in a fixed order);
    # MIOpen's immediate-mode solvers for them may split K with atomics
    # narrow outputs (flow / mask heads, FlowNet2's predict_flow on 1/64-scale maps): MIOpen
    # takes ~0.65 ms for a [2, 1056, 16, 32] -> 2-channel 3x3 conv; k10 splits K over the grid
    return blocks >= _MFMA_MIN_BLOCKS or cout <= 8 or \
        torch.are_deterministic_algorithms_enabled() or _capturing()


def _flip_t(w):
    """[Cout, Cin, KH, KW] -> [Cin, Cout, KH, KW] spatially flipped (dgrad-as-conv weight):
    one pass of the conv_aux.hip transpose kernel (PyTorch: flip + strided copy)."""
    if w.is_cuda and w.dtype == torch.bfloat16 and w.shape[0] % 8 == 0 and w.shape[1] % 8 == 0:
        return _ext.ext().conv_weight_flip_t(nhwc(w))
    return w.flip(2, 3).transpose(0, 1).contiguous(memory_format=_CL)


# flipped, transposed copies of conv weights for the stride-1 data gradient, made for many
# layers in one launch (``register_dgrad_weights``: the spectral-norm group right after its
# bf16 W / sigma launch) or cached for frozen weights (VGG in the perceptual loss):
# data_ptr -> (weight, flipped). The entry holds the weight itself, so its storage cannot be
# reused by another tensor while the entry lives.
_WFLIP = {}
_WFLIP_FROZEN = {}
_FROZEN_PREP = {}  # padded k10 operands of frozen weights / biases, see _frozen_prep
_GRAPH_KEEP = {}  # cached tensors a captured graph uses (kept for the process lifetime)


def register_dgrad_weights(weights, flipped, old_keys=()):
    """Record ``flipped[i]`` as the dgrad weight of ``weights[i]``; drops ``old_keys`` first.
    Returns the keys registered."""
    for k in old_keys:
        _WFLIP.pop(k, None)
    keys = []
    for w, f in zip(weights, flipped):
        k = w.data_ptr()
        _WFLIP[k] = (w, f)
        keys.append(k)
    return keys


def _dgrad_weight(wb):
    """The pre-flipped dgrad weight of ``wb`` (k10 bf16 weight), or None."""
    ent = _WFLIP.get(wb.data_ptr())
    if ent is not None and ent[0].shape == wb.shape and ent[0].stride() == wb.stride() and \
            ent[0].dtype == wb.dtype:
        return ent[1]
    if isinstance(wb, torch.nn.Parameter) and not wb.requires_grad and \
            wb.shape[0] % 8 == 0 and wb.shape[1] % 8 == 0:
        key = (wb.data_ptr(), wb._version, tuple(wb.shape))
        ent = _WFLIP_FROZEN.get(key)
        if ent is None:
            if len(_WFLIP_FROZEN) > 256:
                _WFLIP_FROZEN.clear()
            ent = _WFLIP_FROZEN[key] = (wb, _ext.ext().conv_weight_flip_t(wb, 1, 0, 0, 1))
        if torch.cuda.is_current_stream_capturing():
            # a captured graph reads this copy on every replay: never let an eviction free it
            _GRAPH_KEEP[id(ent[1])] = ent
        return ent[1]
    return None


def _frozen_prep(t, tag, fn):
    """``fn()`` — the padded / cast k10 operand made from ``t`` — cached when ``t`` is marked
    ``_iamd_frozen`` (never trained: the VGG-19 of the perceptual loss, FlowNet2's parameters
    and their bf16 casts), keyed on its storage and version counter, so the per-call pad / cast
    launches of those convs happen once. Not for parameters that are merely not requiring grad
    at the moment (a discriminator frozen for the G update): native optimizer steps change them
    without moving the version counter. Other tensors: ``fn()`` every call."""
    if t is None or t.requires_grad or not t.is_cuda or not getattr(t, '_iamd_frozen', False):
        return fn()
    key = (tag, t.data_ptr(), t._version, tuple(t.shape), t.dtype)
    ent = _FROZEN_PREP.get(key)
    if ent is None:
        if len(_FROZEN_PREP) > 1024:
            _FROZEN_PREP.clear()
        ent = _FROZEN_PREP[key] = (t, fn())
    if torch.cuda.is_current_stream_capturing():
        _GRAPH_KEEP[id(ent[1])] = ent  # a captured graph reads it on every replay
    return ent[1]


def _pad_rows(t, n):
    """Zero-pad dim 0 of a weight / bias to ``n`` rows."""
    if t is None or t.shape[0] == n:
        return t
    out = t.new_zeros((n,) + tuple(t.shape[1:]))
    out[:t.shape[0]] = t
    return out.contiguous(memory_format=_CL) if out.dim() == 4 else out


# stride-s data gradients as s*s phase convolutions on k10 (0: MIOpen backward-data)
_STRIDED_DGRAD = os.environ.get('IMAGINAIRE_AMD_STRIDED_DGRAD', '1') == '1'
_STRIDED_DGRAD_MIN_PIX = int(os.environ.get('IMAGINAIRE_AMD_STRIDED_DGRAD_MIN_PIX', 131072))


_STRIDED_ONE_LAUNCH = os.environ.get('IMAGINAIRE_AMD_STRIDED_ONE_LAUNCH', '1') == '1'


def _strided_dgrad(dy, wb, H, W, s, padding, wts=None, ncv=-1, ascale=None):
    """Data gradient of a stride-``s`` conv (weight ``wb`` [Cout, Cin, KH, KW], channels-last
    bf16) as s*s stride-1 phase convolutions on k10. Input row i = s*q + r receives
    dy[q + c0 - j] * w[kh0 + s*j] for kh0 = (r + p) mod s, c0 = (r + p - kh0) / s: a J-tap
    correlation of dy with the flipped phase sub-kernel (``conv_weight_flip_t(w, s, kh0, kw0)``),
    whose output rows [m0, m0 + Q) are scattered into the parity sub-grid of dx
    (``conv_phase_scatter``). Same FLOPs as the dense dgrad, no zero-insertion. ``ascale``: a
    device scalar the k10 epilogues divide by (spectral norm's sigma)."""
    X = _ext.ext()
    cout, cin, kh, kw = wb.shape
    ho, wo = dy.shape[2], dy.shape[3]
    ph, pw = padding
    if wts is None and _STRIDED_ONE_LAUNCH and cout % 64 == 0 and cin % 64 == 0 and \
            0 <= ph < kh and 0 <= pw < kw:
        # every phase in one launch, stored straight into its parity sub-grid of dx
        return X.conv2d_dgrad_strided(dy, wb, s, ph, pw, H, W, ncv, ascale)
    dx = None
    phases = []
    for ry in range(s):
        for rx in range(s):
            ky0, kx0 = (ry + ph) % s, (rx + pw) % s
            jy, jx = -(-(kh - ky0) // s), -(-(kw - kx0) // s)
            qy, qx = (H - ry + s - 1) // s, (W - rx + s - 1) // s
            phases.append((ry, rx, ky0, kx0, jy, jx, qy, qx))
    zero_fill = any(p[4] <= 0 or p[5] <= 0 for p in phases)
    dx = torch.empty((dy.shape[0], cin, H, W), dtype=torch.bfloat16, device=dy.device,
                     memory_format=_CL)
    if zero_fill:  # some parity sub-grid receives no filter taps
        dx.zero_()
    for ry, rx, ky0, kx0, jy, jx, qy, qx in phases:
        if jy <= 0 or jx <= 0 or qy <= 0 or qx <= 0:
            continue
        cy, cx = (ry + ph - ky0) // s, (rx + pw - kx0) // s
        py = max(0, jy - 1 - cy, qy + cy - ho)
        px = max(0, jx - 1 - cx, qx + cx - wo)
        wt = wts[(ry, rx)] if wts is not None else X.conv_weight_flip_t(wb, s, ky0, kx0, 1)
        out = X.conv2d_mfma(dy, wt, None, 1, 1, py, px, 1, 1, 1.0, 1, -1, None, ascale)
        X.conv_phase_scatter(out, dx, s, ry, rx, cy - (jy - 1) + py, cx - (jx - 1) + px, qy, qx)
    return dx


# Off by default: the SPADE step ran 2% SLOWER with the weight / bias gradients on a side
# stream (51.1-51.2 vs 52.2 images/s back to back, gpurun_out r4t) — the large dgrad and wgrad
# grids each fill the chip, and sharing it costs both more than the launch gaps it hides.
_OVERLAP_BWD = os.environ.get('IMAGINAIRE_AMD_CONV_BWD_OVERLAP', '0')  # '1' | 'bias' | '0'
# 'small[:P]': the weight gradient goes to the side stream only for convs of at most P output
# pixels (default 8192: SPADE's 16x32 / 32x64 layers at batch 4), whose split-K grids leave CUs
# idle, and only where its spectral-norm <G, W> comes from the k11 epilogue anyway
_OVERLAP_SMALL_PIX = int(_OVERLAP_BWD.split(':')[1]) if _OVERLAP_BWD.startswith('small:') \
    else 8192
if _OVERLAP_BWD.startswith('small'):
    _OVERLAP_BWD = 'small'
# spectral-norm weight gradient: <G, W> from the data gradient (sigma <dx, x>, one bandwidth
# pass over dx and x) when the input has at most this many times the weight's elements, else in
# the k11 epilogue (which re-reads W once per split-K slab). 0: always the epilogue.
_SN_DOT_RATIO = float(os.environ.get('IMAGINAIRE_AMD_SN_DOT_RATIO', '8'))
_BWD_SIDE = {}


def _bwd_side_stream():
    """The per-device side stream of the conv backward's weight gradients (None when off, in
    the conv log's timing mode, or under the eager reference path)."""
    if _OVERLAP_BWD not in ('1', 'bias', 'small') or _CONV_LOG is not None:
        return None
    dev = torch.cuda.current_device()
    st = _BWD_SIDE.get(dev)
    if st is None:
        st = _BWD_SIDE[dev] = torch.cuda.Stream(device=dev)
    return st


class _MfmaConv2d(torch.autograd.Function):
    """k10 forward / stride-1 dgrad, k11 wgrad, k2 activation + bias backward. Channel
    counts are zero-padded to multiples of 64 (input) / 64 (output) around the kernels.

    Spectral norm (``sw``: an :class:`SNWeight`; ``w`` is then its fp32 parameter W and the
    function is differentiable w.r.t. W, reference torch.nn.utils.spectral_norm):

    * forward: k10 on the bf16 shadow, ``y = act(conv(x, W) / sigma + b)`` — 1 / sigma in the
      epilogue, no bf16(W / sigma) copy per forward;
    * data gradient: k10 on the flipped shadow (the group flips every fused conv's shadow in
      one launch) or the strided data gradient, 1 / sigma in the epilogue;
    * weight gradient: k11 into fp32 split-K slabs whose epilogue also sums <G, W> per block;
      the pass that sums the slabs writes ``dW = G / sigma - (<G, W> / sigma^2) u v^T`` (the
      gradient of W / (u^T W v) with u, v constant, as torch's spectral_norm backward).
    """

    @staticmethod
    def forward(ctx, x, w, bias, stride, padding, dilation, slope, res=None, sw=None):
        cout, cin = w.shape[0], w.shape[1]
        cp, op = _round_up(cin, 64), _out_pad(cout)
        xb = _pad_channels(x, cp, torch.bfloat16)
        sig = None if sw is None else sw.sigma.reshape(1)
        if sw is None:
            wb = _frozen_prep(w, ('w', cp, op), lambda: _pad_rows(
                _pad_channels(w, cp, torch.bfloat16), op))
        else:
            wb = _pad_rows(_pad_channels(sw.shadow, cp, torch.bfloat16), op)
        ho, wo = _out_hw(x.shape[2], x.shape[3], w.shape[2:], stride, padding, dilation)
        # Cout % 8 == 0: k10 stores only the real output channels (no crop copy after it)
        ncv = cout if (op != cout and cout % 8 == 0) else op
        ctx.res_dtype = None if res is None else res.dtype
        with _Logged('fwd', 'k10', 2.0 * x.shape[0] * ho * wo * op * cp * w.shape[2] * w.shape[3],
                     _gemm_desc(xb, wb, stride, padding) + ('' if sw is None else ' sn')):
            bp = None if bias is None else _frozen_prep(bias, ('b', op),
                                                        lambda: _pad_rows(bias, op).float())
            y = _ext.ext().conv2d_mfma(xb, wb, bp, stride[0], stride[1],
                                       padding[0], padding[1], dilation[0], dilation[1],
                                       float(slope), 1, ncv, res, sig)
        ctx.conf = (stride, padding, dilation, float(slope), cin, cout, x.dtype, w.dtype,
                    None if bias is None else bias.dtype, x.shape[1])
        ctx.sn = None if sw is None else (sw.shadow, sw.u, sw.v, sig)
        # the weight-gradient destination is looked up on the leaf parameter (DDP bucket slice)
        ctx.wparam = w if (isinstance(w, torch.nn.Parameter) and w.dtype == torch.float32) else None
        ctx.wflip = _dgrad_weight(wb) if (stride == (1, 1) and dilation == (1, 1) and
                                          ctx.needs_input_grad[0]) else None
        # the output is needed only for a fused activation's mask: with slope 1 it is not
        # saved, so in-place ops on the conv output stay legal (as after a plain F.conv2d)
        ctx.save_for_backward(xb, wb, y if slope != 1.0 else None)
        if y.shape[1] == cout:
            return y
        # a fresh tensor, not a view of y: callers apply in-place activations (nn.ReLU(
        # inplace=True)) to conv outputs, which autograd forbids on a custom Function's view
        return y[:, :cout].contiguous(memory_format=_CL)

    @staticmethod
    def backward(ctx, dy):
        dy_in = dy  # the residual's gradient (added after the activation: identity)
        xb, wb, y = ctx.saved_tensors
        if _PS_CHECK:
            _ps_check('conv.dy', dy)
        stride, padding, dilation, slope, cin, cout, xdt, wdt, bdt, xc = ctx.conf
        need_x, need_w, need_b = ctx.needs_input_grad[:3]
        sn = ctx.sn
        sig = None if sn is None else sn[3]
        # the activation backward runs at the saved output's channel count (the real Cout when
        # k10 stored only those, else the padded one), then dy is padded for the GEMMs; without
        # an activation / bias gradient that is ONE pad-cast pass from any dy layout
        db = None
        # the weight (and, without an activation, the bias) gradient runs on a side stream,
        # concurrently with the data gradient: they are independent, and the small convs'
        # grids leave most CUs idle on their own
        side = _bwd_side_stream() if (need_x and (need_w or need_b)) else None
        if side is not None and _OVERLAP_BWD == 'small' and (
                dy.shape[0] * dy.shape[2] * dy.shape[3] > _OVERLAP_SMALL_PIX or not need_w or
                (sn is not None and _SN_DOT_RATIO > 0 and
                 xb.numel() <= _SN_DOT_RATIO * wb.numel())):
            side = None
        side_bias = side is not None and slope == 1.0 and need_b
        if slope != 1.0:
            dy = _pad_channels(dy, y.shape[1], torch.bfloat16)
            dy, db = _ext.ext().bias_act_bwd(y, dy, slope)
        elif need_b and not side_bias:
            dy = _pad_channels(dy, dy.shape[1], torch.bfloat16)
        dy_b = dy  # the bias gradient's operand (identity activation: computed last, below)
        dy = _pad_channels(dy, wb.shape[0], torch.bfloat16)
        dx = dw = None
        cap = _capturing()
        kh, kw = wb.shape[2], wb.shape[3]
        if cout <= 16 and stride == (1, 1) and dilation == (1, 1) and sn is None and \
                _TAPPACK and kh * kw > 1 and kh * kw * cout <= 512 and \
                0 <= padding[0] < kh and 0 <= padding[1] < kw and (need_x or need_w):
            # thin OUTPUT (the RGB heads): both gradients from ONE tap-packed operand of dy,
            # dycol[q][(t', co)] = dy[q + t' - (K - 1 - pad)] (t' = flipped tap): dx is the 1x1
            # GEMM of dycol with the flipped weight, dW the 1x1 k11 GEMM of (dycol, x) — no
            # 64-channel padding of dy, no KH*KW x 64 implicit-GEMM k loop over zero channels
            dx, dw = _thin_output_grads(dy[:, :cout], xb, wb, padding, cout, cin, xc, need_x,
                                        need_w, wdt)
            need_x_left, need_w_left = False, False
        else:
            need_x_left, need_w_left = need_x, need_w
        if side is not None:
            main = torch.cuda.current_stream()
            side.wait_stream(main)
            with torch.cuda.stream(side):
                if side_bias:  # bias gradient only: the k2 kernel reads dy, writes no dx
                    db = _ext.ext().bias_act_bwd(dy, dy, 1.0)[1]
                if need_w_left and _OVERLAP_BWD in ('1', 'small'):
                    dw = _wgrad(dy, xb, wb, stride, padding, dilation, cout, cin, wdt, sn)
        if need_x_left:
            pt = (dilation[0] * (kh - 1) - padding[0], dilation[1] * (kw - 1) - padding[1])
            cp = wb.shape[1]
            dblocks = -(-dy.shape[0] * xb.shape[2] * xb.shape[3] // 128) * \
                (cp // (128 if cp % 128 == 0 else 64))
            # the dgrad GEMM has N = Cin (few tiles, K = taps x Cout for the SPADE γ/β convs):
            # k10 splits K over the grid's y dimension for those
            fl = 2.0 * dy.shape[0] * dy.shape[2] * dy.shape[3] * wb.numel()
            big = dblocks >= _MFMA_MIN_DGRAD_BLOCKS or cap
            # dx keeps only the input's real channels when they are a multiple of 8
            ncv = xc if (cp != xc and xc % 8 == 0) else cp
            if stride == (1, 1) and dilation == (1, 1) and pt[0] >= 0 and pt[1] >= 0 and big:
                # the flipped weight (made for the whole network in one launch, or cached for a
                # frozen weight), else one flip_t pass of it here; then the k10 routing (v4 / v5
                # for stride-1 3x3-5x5 rows). IMAGINAIRE_AMD_DGRAD_BT=1 reads the forward weight
                # transposed in-kernel instead (csrc/conv_mfma.hip dgrad_bt_enabled)
                with _Logged('dgrad', 'k10', fl, _gemm_desc(dy, wb.transpose(0, 1), (1, 1), pt)):
                    if ctx.wflip is not None:
                        dx = _ext.ext().conv2d_mfma(dy, ctx.wflip, None, 1, 1, pt[0], pt[1], 1,
                                                    1, 1.0, 1, ncv, None, sig)
                    else:
                        dx = _ext.ext().conv2d_dgrad_mfma(dy, wb, padding[0], padding[1], ncv,
                                                          sig)
            elif stride == (1, 1) and pt[0] >= 0 and pt[1] >= 0 and big:
                wt = _flip_t(wb)
                with _Logged('dgrad', 'k10', fl, _gemm_desc(dy, wt, (1, 1), pt)):
                    dx = _ext.ext().conv2d_mfma(dy, wt, None, 1, 1, pt[0], pt[1],
                                                dilation[0], dilation[1], 1.0, 1, ncv, None, sig)
            elif _STRIDED_DGRAD and stride[0] == stride[1] and 2 <= stride[0] <= 4 and \
                    dilation == (1, 1) and (cap or (
                        dblocks >= _MFMA_MIN_DGRAD_BLOCKS * stride[0] ** 2 and
                        xb.shape[0] * xb.shape[2] * xb.shape[3] >= _STRIDED_DGRAD_MIN_PIX)):
                # large maps only: 1.3-1.6x MIOpen on the full-resolution PatchGAN layers, on par
                # or slower below ~128K dx pixels (profiles/strided_dgrad_probe_mi355x.txt)
                with _Logged('dgrad', 'k10s', fl, _gemm_desc(dy, wb, stride, padding)):
                    dx = _strided_dgrad(dy, wb, xb.shape[2], xb.shape[3], stride[0], padding,
                                        ncv=ncv, ascale=sig)
            else:
                with _Logged('dgrad', 'miopen', fl, _gemm_desc(dy, wb, stride, padding)):
                    dx = torch.ops.aten.convolution_backward(
                        dy, xb, wb, None, stride, padding, dilation, False, [0, 0], 1,
                        [True, False, False])[0]
                    if sig is not None:
                        dx = dx.div_(sig)  # one pass (fp32 divisor, no reciprocal / cast kernels)
            if sn is not None and need_w and dw is None and _SN_DOT_RATIO > 0 and \
                    xb.numel() <= _SN_DOT_RATIO * wb.numel() and dx.dtype == torch.bfloat16 and \
                    dx.shape[1] % 8 == 0 and dx.is_contiguous(memory_format=_CL):
                # <G, W> = sigma <dx, x> (the adjoint identity): for a low-resolution layer the
                # activation is smaller than the weight the k11 epilogue would re-read per split
                sn = tuple(sn) + (_ext.ext().sn_dot_partials(dx, xb, sig),)
            if dx.shape[1] != xc:
                dx = dx[:, :xc]
            dx = dx.to(xdt)
        elif dx is not None:  # (thin-output path)
            if dx.shape[1] != xc:
                dx = dx[:, :xc]
            dx = dx.to(xdt)
        if side is not None:
            main.wait_stream(side)
            for t in (dw, db):  # (allocated on the side stream, consumed on this one)
                if t is not None:
                    t.record_stream(main)
        if need_w:
            if dw is None:
                dest = _take_grad_dest(ctx.wparam, (cout, cin, wb.shape[2], wb.shape[3]))
                dw = _wgrad(dy, xb, wb, stride, padding, dilation, cout, cin, wdt, sn, dest)
            elif not need_w_left:  # (thin-output path: already cropped, in fp32)
                pass
            if dw.shape[0] != cout or dw.shape[1] != cin:
                dw = dw[:cout, :cin]
            dw = dw.to(wdt)
            if _TEST_FLIP_WGRAD[0]:
                dw = _test_flip_wgrad(dw)
        if slope == 1.0 and need_b and not side_bias:
            # identity activation: bias gradient only (the k2 kernel reads dy, writes no dx),
            # after the data and weight gradients
            db = _ext.ext().bias_act_bwd(dy_b, dy_b, 1.0)[1]
        if db is not None:
            db = db[:cout].to(bdt) if need_b else None
        if _PS_CHECK:
            for nm, t in (('conv.db', db), ('conv.dw', dw), ('conv.dx', dx)):
                if t is not None:
                    _ps_check(nm, t)
        dres = None
        if ctx.res_dtype is not None and ctx.needs_input_grad[7]:
            dres = dy_in if dy_in.dtype == ctx.res_dtype else dy_in.to(ctx.res_dtype)
        return dx, dw, db, None, None, None, None, dres, None


# Negative control of the model-parity gate (tests/test_model_parity_gpu.py): with
# ``_TEST_FLIP_WGRAD = [k, 0]`` (or IMAGINAIRE_AMD_TEST_FLIP_WGRAD=k at import) the k-th k10/k11
# conv weight gradient computed from then on is returned negated. Test use only.
_TEST_FLIP_WGRAD = [int(os.environ.get('IMAGINAIRE_AMD_TEST_FLIP_WGRAD', '0')), 0]


def _test_flip_wgrad(dw):
    _TEST_FLIP_WGRAD[1] += 1
    return -dw if _TEST_FLIP_WGRAD[1] == _TEST_FLIP_WGRAD[0] else dw


def _thin_output_grads(dy, xb, wb, padding, cout, cin, xc, need_x, need_w, wdt):
    """Data and weight gradients of a stride-1 conv with a thin output (Cout <= 16) from the
    tap-packed operand of its output gradient (see :class:`_MfmaConv2d` backward).
    dy [B, cout, Ho, Wo] (a view is fine), xb [B, cp, H, W] bf16, wb [op, cp, KH, KW] bf16.
    Returns (dx [B, xc or cp, H, W] bf16 or None, dW [cout, cin, KH, KW] fp32 or None)."""
    X = _ext.ext()
    kh, kw = wb.shape[2], wb.shape[3]
    cp = wb.shape[1]
    K = kh * kw * cout
    kp = _round_up(K, 64)
    dyc = X.im2col_pack(dy, kh, kw, 1, 1, kh - 1 - padding[0], kw - 1 - padding[1], 1, 1, kp)
    fl = 2.0 * dyc.shape[0] * dyc.shape[2] * dyc.shape[3] * kp * cp
    dx = dw = None
    if need_x:
        # Wd[ci][(t', co)] = w[co, ci, flip(t')]
        wd = torch.zeros((cp, kp), dtype=torch.bfloat16, device=wb.device)
        wd[:, :K] = wb[:cout].flip(2, 3).permute(1, 2, 3, 0).reshape(cp, K)
        ncv = xc if (cp != xc and xc % 8 == 0) else cp
        with _Logged('dgrad', 'k10p', fl, '%s thin-out' % list(dyc.shape)):
            dx = X.conv2d_mfma(dyc, wd.view(cp, kp, 1, 1), None, 1, 1, 0, 0, 1, 1, 1.0, 1, ncv,
                               None, None)
    if need_w:
        with _Logged('wgrad', 'k11', fl, '%s thin-out' % list(dyc.shape)):
            g = X.conv2d_wgrad_mfma(dyc, xb, 1, 1, 1, 1, 0, 0, 1, 1, K, cin, False, 1)
        # g[(t', co)][ci] -> dW[co, ci, t] with t = flip(t')
        dw = g.reshape(kh, kw, cout, cin).flip(0, 1).permute(2, 3, 0, 1)
        if _TEST_FLIP_WGRAD[0]:
            dw = _test_flip_wgrad(dw)
    return dx, dw


class SNWeight(object):
    """A spectrally normalised conv weight handed to :func:`conv2d` / :func:`conv2d_act`
    unmaterialised (layers/spectral_norm.py ``weight_ref``): the fp32 parameter ``W``, its bf16
    shadow (= bf16(W), written by the optimizer step), the power iteration's u / v snapshots
    and sigma (a device scalar). On the k10 / k11 path the conv runs on the shadow with
    1 / sigma in its epilogues and the SN backward in its weight gradient
    (:class:`_MfmaConv2d`); any other consumer calls :meth:`materialize` for the usual
    bf16(W / sigma) tensor (reference: torch.nn.utils.spectral_norm, W / (u^T W v)). After such
    a fused forward the module's ``weight`` attribute holds this object (not a stale tensor):
    ``module.weight.materialize()`` is the normalised weight that forward used."""

    __slots__ = ('W', 'shadow', 'u', 'v', 'sigma', 'hook', 'module')

    def __init__(self, W, shadow, u, v, sigma, hook, module):
        self.W, self.shadow, self.u, self.v, self.sigma = W, shadow, u, v, sigma
        self.hook, self.module = hook, module

    @property
    def shape(self):
        return self.W.shape

    def dim(self):
        return self.W.dim()

    def materialize(self):
        from imaginaire_amd.layers.spectral_norm import _SNScaleCast, materialize_scaled
        w16 = materialize_scaled(self.W, self.sigma, self.shadow)
        return _SNScaleCast.apply(self.W, self.u, self.v, self.sigma, w16, self.shadow)


def _sn_fused_ok(x, sw, stride, padding, dilation, residual=None):
    """The fused SN conv runs exactly where the plain k10 path would (no tap-split head).
    Decided on the weight's shape alone (a meta tensor: no padded copy of the shadow here)."""
    cx, cw = x.shape[1], sw.shadow.shape[1]
    if cx != cw and not (cx == _round_up(cw, 64) and
                         getattr(x, '_iamd_valid_channels', None) == cw):
        return False
    wm = torch.empty((sw.shadow.shape[0], cx) + tuple(sw.shadow.shape[2:]), dtype=torch.bfloat16,
                     device='meta')
    if tappack_eligible(_thin_view(x, cw), sw.shadow, stride, padding, dilation, 1) or \
            tapsplit_eligible(x, wm, stride, padding, dilation, 1) or \
            not mfma_eligible(x, wm, stride, padding, dilation, 1):
        return False
    return residual is None or _residual_fusible(residual, x, wm, stride, padding, dilation)


class _MfmaConvPerSample(torch.autograd.Function):
    """B independent convolutions with per-sample weights — the hyper convolutions of
    few-shot vid2vid (reference layers/conv.py:575-590 loops over the batch) — as ONE batched
    k10 launch (grid z = sample) forward, k10 on the per-sample flipped weights for the data
    gradient and one batched k11 launch for the weight gradients. x [B, Cin, H, W], w [B, Cout,
    Cin, KH, KW], bias [B, Cout]; stride 1, channels zero-padded to multiples of 64."""

    @staticmethod
    def forward(ctx, x, w, bias, padding, dilation):
        B, cout, cin, kh, kw = w.shape
        cp, op = _round_up(cin, 64), _round_up(cout, 64)
        xb = _pad_channels(x, cp, torch.bfloat16)
        # sample-major channels-last weights [B][op][kh][kw][cp], zero-padded
        wp = w.new_zeros((B, op, kh, kw, cp), dtype=torch.bfloat16)
        wp[:, :cout, :, :, :cin] = w.permute(0, 1, 3, 4, 2)
        wb = wp.view(B * op, kh, kw, cp).permute(0, 3, 1, 2)
        bb = None
        if bias is not None:
            bb = bias.new_zeros((B, op), dtype=torch.float32)
            bb[:, :cout] = bias
            bb = bb.view(-1)
        with _Logged('fwd', 'k10b', 2.0 * x.shape[2] * x.shape[3] * B * op * cp * kh * kw,
                     _gemm_desc(xb, wb, (1, 1), padding) + ' nb%d' % B):
            y = _ext.ext().conv2d_mfma(xb, wb, bb, 1, 1, padding[0], padding[1], dilation[0],
                                       dilation[1], 1.0, B)
        ctx.conf = (padding, dilation, cin, cout, x.dtype, w.dtype, x.shape[1],
                    None if bias is None else bias.dtype)
        ctx.save_for_backward(xb, wb)
        return y if op == cout else y[:, :cout].contiguous(memory_format=_CL)

    @staticmethod
    def backward(ctx, dy):
        xb, wb = ctx.saved_tensors
        padding, dilation, cin, cout, xdt, wdt, xc, bdt = ctx.conf
        if _PS_CHECK:
            _ps_check('dy', dy)
            _ps_check('xb', xb)
            _ps_check('wb', wb)
        B, cp = xb.shape[0], xb.shape[1]
        op = wb.shape[0] // B
        kh, kw = wb.shape[2], wb.shape[3]
        dy = _pad_channels(dy, op, torch.bfloat16)
        dx = dw = db = None
        dbg = _PS_DEBUG
        if dbg:  # bisection switch: bit 1 dx, bit 2 dw on PyTorch's reference ops
            xs = xb.float().detach()
            ws_ = wb.float().reshape(B, op, cp, kh, kw)
            if dbg & 1 and ctx.needs_input_grad[0]:
                dx = torch.cat([torch.nn.grad.conv2d_input(
                    (1,) + tuple(xs.shape[1:]), ws_[i], dy[i:i + 1].float(), 1, padding,
                    dilation) for i in range(B)])
                dx = (dx[:, :xc] if dx.shape[1] != xc else dx).to(xdt).contiguous(
                    memory_format=_CL)
            if dbg & 2 and ctx.needs_input_grad[1]:
                g = torch.stack([torch.nn.grad.conv2d_weight(
                    xs[i:i + 1], (op, cp, kh, kw), dy[i:i + 1].float(), 1, padding, dilation)
                    for i in range(B)])
                dw = g[:, :cout, :cin].to(wdt)
        if ctx.needs_input_grad[0] and dx is None:
            pt = (dilation[0] * (kh - 1) - padding[0], dilation[1] * (kw - 1) - padding[1])
            wt = _ext.ext().conv_weight_flip_t(wb, 1, 0, 0, B)
            dx = _ext.ext().conv2d_mfma(dy, wt, None, 1, 1, pt[0], pt[1], dilation[0],
                                        dilation[1], 1.0, B)
            dx = (dx[:, :xc] if dx.shape[1] != xc else dx).to(xdt)
        if ctx.needs_input_grad[1] and dw is None:
            g = _ext.ext().conv2d_wgrad_mfma(dy, xb, kh, kw, 1, 1, padding[0], padding[1],
                                             dilation[0], dilation[1], -1, -1, False, B)
            # [B * op, cp, kh, kw] (memory [B][op][kh][kw][cp]) -> [B, cout, cin, kh, kw]
            if _PS_CHECK:
                _ps_check('g', g)
            g = g.permute(0, 2, 3, 1).reshape(B, op, kh, kw, cp)[:, :cout, :, :, :cin]
            dw = g.permute(0, 1, 4, 2, 3).to(wdt)
            if _PS_CHECK:
                _ps_check('dw', dw)
        if ctx.needs_input_grad[2]:
            # per-sample bias gradients on the k2 column-sum kernel (one small launch per
            # sample): torch's dy.sum((2, 3)) came out non-finite from finite dy inside the
            # fs-vid2vid hipGraph replay (scripts/probe/graph_nan_probe.py, PS_CHECK)
            db = torch.stack([_ext.ext().bias_act_bwd(dy[i:i + 1], dy[i:i + 1], 1.0)[1]
                              for i in range(B)])[:, :cout].to(bdt)
            if _PS_CHECK:
                _ps_check('db', db)
        if _PS_CHECK and dx is not None:
            _ps_check('dx', dx)
        return dx, dw, db, None, None


_PER_SAMPLE = os.environ.get('IMAGINAIRE_AMD_PER_SAMPLE', '1') == '1'
_PS_DEBUG = int(os.environ.get('IMAGINAIRE_AMD_PS_DEBUG', '0'))
# IMAGINAIRE_AMD_PS_CHECK=1 (debugging): the per-sample backward records isfinite() of its
# operands and results into a device flag array (graph-capturable); read with ps_check_report()
_PS_CHECK = os.environ.get('IMAGINAIRE_AMD_PS_CHECK', '0') == '1'
_PS_FLAGS = {}


def _ps_check(name, t):
    st = _PS_FLAGS.setdefault('state', {'n': 0, 'labels': []})
    if 'flags' not in _PS_FLAGS:
        _PS_FLAGS['flags'] = torch.ones(4096, dtype=torch.bool, device=t.device)
    i = st['n'] % 4096
    st['n'] += 1
    st['labels'].append((name, tuple(t.shape), t.dtype))
    _PS_FLAGS['flags'][i:i + 1].copy_(torch.isfinite(t.detach()).all().reshape(1))


def ps_check_report(reset=True):
    """(label, finite) of every per-sample backward check recorded since the last reset."""
    st = _PS_FLAGS.get('state')
    if not st:
        return []
    f = _PS_FLAGS['flags'][:min(st['n'], 4096)].cpu().tolist()
    out = list(zip(st['labels'][:len(f)], f))
    if reset:
        _PS_FLAGS['flags'].fill_(True)
    return out


def per_sample_eligible(x, w, stride, groups):
    """k10/k11 batched path for HyperConv2d: bf16 compute, stride 1, groups 1, 4-D x and
    5-D per-sample weights, and enough pixels per sample to fill tiles."""
    if not (_PER_SAMPLE and x.is_cuda and x.dim() == 4 and w.dim() == 5 and groups == 1 and
            stride == 1 and _mfma_enabled() and w.shape[0] == x.shape[0]):
        return False
    if _compute_dtype(x, w) != torch.bfloat16:
        return False
    # no padding-waste limit here: the alternative is MIOpen's grouped convolution, whose
    # weight-gradient kernels ran at a few TF/s on the fs-vid2vid hyper layers (4.5 ms per call,
    # profiles/recipe_fsvid2vid512_kernels_mi355x.txt), far below a 4x-padded MFMA tile
    cin = w.shape[2]
    # (small maps go to MIOpen's grouped convolution eagerly, never inside a graph: its backward
    # solvers accumulate with atomics into buffers the capture does not re-zero)
    return (x.shape[2] * x.shape[3] >= 256 or _capturing()) and \
        x.numel() // x.shape[0] * _round_up(cin, 64) // max(cin, 1) * 2 < (1 << 30)


def conv2d_per_sample(x, w, bias, padding, dilation=1):
    """``y[b] = conv2d(x[b], w[b], bias[b])`` for every sample b in one batched MFMA launch."""
    return _MfmaConvPerSample.apply(x, w, bias, _pair(padding), _pair(dilation))


class _TapSplitConv2d(torch.autograd.Function):
    """Narrow-output (Cout <= 8) stride-1 convolutions — the RGB image heads — re-associated
    as a 1x1 MFMA GEMM into per-tap partial outputs Z[p, t*Cout + c] (k10, N = KH*KW*Cout
    padded to 64) followed by a tap-sum gather (csrc/conv_tapsplit.hip). Backward: per-tap
    gather of dy into dZ, then dx = k10 1x1 conv of dZ with the transposed Z weight and
    dW = k11 1x1 weight gradient of (dZ, x). Every input element is read once by a useful-width
    MFMA tile instead of streaming the KH*KW*Cin im2col operand for 3 outputs per pixel."""

    @staticmethod
    def forward(ctx, x, w, bias, padding, dilation):
        cout, cin, kh, kw = w.shape
        cp, cz = _round_up(cin, 64), _round_up(cout * kh * kw, 64)
        xb = _pad_channels(x, cp, torch.bfloat16)
        # Wz[t*cout + c, ci] = w[c, ci, t]
        wz = torch.zeros((cz, cp), dtype=torch.bfloat16, device=w.device)
        wz[:cout * kh * kw, :cin] = w.to(torch.bfloat16).permute(2, 3, 0, 1).reshape(-1, cin)
        wz = wz.view(cz, cp, 1, 1)
        ho, wo = _out_hw(x.shape[2], x.shape[3], (kh, kw), (1, 1), padding, dilation)
        with _Logged('fwd', 'k10t', 2.0 * x.shape[0] * x.shape[2] * x.shape[3] * cz * cp,
                     _gemm_desc(xb, w, (1, 1), padding) + ' tapsplit'):
            z = _ext.ext().conv2d_mfma(xb, wz, None, 1, 1, 0, 0, 1, 1, 1.0, 1)
            y = _ext.ext().conv_tap_sum(z, bias, cout, kh, kw, padding[0], padding[1],
                                        dilation[0], dilation[1])
        ctx.conf = (padding, dilation, cin, cout, kh, kw, x.dtype, w.dtype,
                    None if bias is None else bias.dtype, x.shape[1])
        ctx.save_for_backward(xb, wz)
        return y

    @staticmethod
    def backward(ctx, dy):
        xb, wz = ctx.saved_tensors
        padding, dilation, cin, cout, kh, kw, xdt, wdt, bdt, xc = ctx.conf
        cz, cp = wz.shape[0], wz.shape[1]
        dz = _ext.ext().conv_tap_gather(dy.to(torch.bfloat16), cz, kh, kw, padding[0], padding[1],
                                        dilation[0], dilation[1], xb.shape[2], xb.shape[3])
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            wzt = wz.view(cz, cp).t().contiguous().view(cp, cz, 1, 1)
            ncv = xc if (cp != xc and xc % 8 == 0) else cp  # only the real input channels
            dx = _ext.ext().conv2d_mfma(dz, wzt, None, 1, 1, 0, 0, 1, 1, 1.0, 1, ncv)
            dx = (dx[:, :xc] if dx.shape[1] != xc else dx).to(xdt)
        if ctx.needs_input_grad[1]:
            g = _ext.ext().conv2d_wgrad_mfma(dz, xb, 1, 1, 1, 1, 0, 0, 1, 1, cout * kh * kw, cin,
                                             False, 1)
            # [t*cout + c, ci] -> [c, ci, kh, kw]
            dw = g.reshape(kh, kw, cout, cin).permute(2, 3, 0, 1).to(wdt)
        if ctx.needs_input_grad[2]:  # the k2 column-sum kernel (no torch reduction)
            dyb = nhwc(dy if dy.dtype in (torch.bfloat16, torch.float32) else dy.float())
            db = _ext.ext().bias_act_bwd(dyb, dyb, 1.0)[1].to(bdt)
        return dx, dw, db, None, None


def _pack_taps(w, kp, op):
    """[Cout, Cin, KH, KW] -> the 1x1 GEMM weight [op, kp, 1, 1] (bf16) of a tap-packed conv:
    row n = w[n] in (ky, kx, ci) order, zero-padded to kp columns and op rows."""
    cout, cin, kh, kw = w.shape
    out = torch.zeros((op, kp), dtype=torch.bfloat16, device=w.device)
    out[:cout, :kh * kw * cin] = w.detach().to(torch.bfloat16).permute(0, 2, 3, 1).reshape(cout, -1)
    return out.view(op, kp, 1, 1)


class _TapPackConv2d(torch.autograd.Function):
    """Thin-input convolutions (Cin <= 16: RGB stems, image + mask inputs, flow inputs) with the
    filter taps packed into the GEMM's K dimension (csrc/im2col.hip): im2col_pack writes
    col[m][(ky, kx, ci)] once (K = KH*KW*Cin padded to 64, e.g. 147 -> 192 for a 7x7 RGB stem,
    instead of 49 taps x 64 zero-padded channels), the conv is a 1x1 k10 GEMM with the fused
    bias / activation epilogue, and the weight gradient a 1x1 k11 GEMM on the same operand; the
    data gradient (a thin-output conv of dy) runs on the k10 dgrad."""

    @staticmethod
    def forward(ctx, x, w, bias, stride, padding, dilation, slope):
        cout, cin, kh, kw = w.shape
        kp, op = _round_up(kh * kw * cin, 64), _out_pad(cout)
        X = _ext.ext()
        col = X.im2col_pack(x.detach(), kh, kw, stride[0], stride[1], padding[0], padding[1],
                            dilation[0], dilation[1], kp)
        wp = _frozen_prep(w, ('tp', kp, op), lambda: _pack_taps(w, kp, op))
        ncv = cout if (op != cout and cout % 8 == 0) else op
        with _Logged('fwd', 'k10p', 2.0 * col.shape[0] * col.shape[2] * col.shape[3] * op * kp,
                     _gemm_desc(x, w, stride, padding) + ' tappack'):
            bp = None if bias is None else _frozen_prep(bias, ('b', op),
                                                        lambda: _pad_rows(bias, op).float())
            y = X.conv2d_mfma(col, wp, bp, 1, 1, 0, 0, 1, 1, float(slope), 1, ncv, None, None)
        ctx.conf = (stride, padding, dilation, float(slope), cin, cout, kh, kw, x.shape[2],
                    x.shape[3], x.dtype, w.dtype, None if bias is None else bias.dtype)
        ctx.save_for_backward(col, wp, y if slope != 1.0 else None)
        if y.shape[1] == cout:
            return y
        return y[:, :cout].contiguous(memory_format=_CL)

    @staticmethod
    def backward(ctx, dy):
        col, wp, y = ctx.saved_tensors
        (stride, padding, dilation, slope, cin, cout, kh, kw, H, W, xdt, wdt, bdt) = ctx.conf
        need_x, need_w, need_b = ctx.needs_input_grad[:3]
        X = _ext.ext()
        op, kp = wp.shape[0], wp.shape[1]
        db = None
        if slope != 1.0:
            dy = _pad_channels(dy, y.shape[1], torch.bfloat16)
            dy, db = X.bias_act_bwd(y, dy, slope)
        elif need_b:
            dy = _pad_channels(dy, dy.shape[1], torch.bfloat16)
            db = X.bias_act_bwd(dy, dy, 1.0)[1]
        dy = _pad_channels(dy, op, torch.bfloat16)
        dx = dw = None
        if need_x:
            # the data gradient of a thin INPUT is a thin-output conv of dy: on the usual k10
            # dgrad (flipped weight, output channels padded to 64). (The adjoint of the packing —
            # a [M][Kp] dcol GEMM + col2im_pack gather — ran at ~12 TF/s: its 2-byte gathers
            # from KH*KW rows per pixel are the bottleneck; gpurun_out r6b, MUNIT / pix2pixHD.)
            K = kh * kw * cin
            wb = torch.empty((op, 64, kh, kw), dtype=torch.bfloat16, device=wp.device,
                             memory_format=_CL).zero_()
            wb[:cout, :cin] = wp.view(op, kp)[:cout, :K].view(cout, kh, kw, cin).permute(
                0, 3, 1, 2)
            fl = 2.0 * dy.shape[0] * dy.shape[2] * dy.shape[3] * wb.numel()
            ncv = cin if cin % 8 == 0 else 64
            if stride == (1, 1) and dilation == (1, 1):
                with _Logged('dgrad', 'k10', fl, _gemm_desc(dy, wb.transpose(0, 1), (1, 1),
                                                           padding) + ' tappack-in'):
                    dx = X.conv2d_dgrad_mfma(dy, wb, padding[0], padding[1], ncv, None)
            elif stride[0] == stride[1] and 2 <= stride[0] <= 4 and dilation == (1, 1) and \
                    0 <= padding[0] < kh and 0 <= padding[1] < kw:
                with _Logged('dgrad', 'k10s', fl, _gemm_desc(dy, wb, stride, padding) +
                             ' tappack-in'):
                    dx = _strided_dgrad(dy, wb, H, W, stride[0], padding, ncv=ncv)
            else:
                dx = torch.ops.aten.convolution_backward(
                    dy, torch.empty((dy.shape[0], 64, H, W), dtype=torch.bfloat16,
                                    device=dy.device, memory_format=_CL),
                    wb, None, stride, padding, dilation, False, [0, 0], 1,
                    [True, False, False])[0]
            dx = dx[:, :cin].to(xdt)
        if need_w:
            with _Logged('wgrad', 'k11', 2.0 * col.shape[0] * col.shape[2] * col.shape[3] * op *
                         kp, '%s tappack' % list(col.shape)):
                g = X.conv2d_wgrad_mfma(dy, col, 1, 1, 1, 1, 0, 0, 1, 1, cout, kh * kw * cin,
                                        False, 1)
            dw = g.reshape(cout, kh, kw, cin).permute(0, 3, 1, 2).to(wdt)
            if _TEST_FLIP_WGRAD[0]:
                dw = _test_flip_wgrad(dw)
        if db is not None:
            db = db[:cout].to(bdt) if need_b else None
        return dx, dw, db, None, None, None, None


_TAPPACK = os.environ.get('IMAGINAIRE_AMD_TAPPACK', '1') == '1'


def _thin_view(x, cin):
    """``x`` itself, or — for a channel-padded buffer whose zero tail starts at a thin weight's
    ``cin`` (``mark_zero_tail``) — the strided view of its real channels, which im2col_pack reads
    without a copy."""
    if x.dim() == 4 and x.shape[1] != cin and cin <= 16 and \
            getattr(x, '_iamd_valid_channels', None) == cin:
        return x[:, :cin]
    return x


def tappack_eligible(x, w, stride, padding, dilation, groups):
    """The tap-packed path (:class:`_TapPackConv2d`): bf16 compute, groups 1, a thin input
    (Cin <= 16) whose packed K = KH*KW*Cin fits 512, a spatial filter, and enough output pixels
    for the 1x1 GEMM (or inside a graph capture)."""
    if not (_TAPPACK and x.is_cuda and x.dim() == 4 and w.dim() == 4 and groups == 1 and
            _mfma_enabled() and x.dtype in (torch.float32, torch.bfloat16)):
        return False
    cout, cin, kh, kw = w.shape
    if cin > 16 or x.shape[1] != cin or kh * kw * cin > 512 or kh * kw == 1:
        return False
    if _compute_dtype(x, w) != torch.bfloat16:
        return False
    ho, wo = _out_hw(x.shape[2], x.shape[3], (kh, kw), stride, padding, dilation)
    if ho <= 0 or wo <= 0:
        return False
    m = x.shape[0] * ho * wo
    kp, op = _round_up(kh * kw * cin, 64), _out_pad(cout)
    # the packed operand is written once and read twice (forward, weight gradient): it pays
    # where it removes >= 8x of the implicit GEMM's zero-padded k loop (RGB / 1-6 channel
    # inputs). Cin 8 / 16 layers (pix2pixHD's instance encoder: 7x7x8 -> 448, 3x3x16 -> 192)
    # moved ~0.6 ms of operand traffic per call for a 3-7x smaller GEMM: no net gain
    # (gpurun_out r6ab)
    if kh * kw * 64 < 8 * kp:
        return False
    if m * kp * 2 >= (1 << 30) or m * op * 2 >= (1 << 30):
        return False
    return m >= _TAPPACK_MIN_PIX or _capturing()


_TAPPACK_MIN_PIX = int(os.environ.get('IMAGINAIRE_AMD_TAPPACK_MIN_PIX', 2048))


_TAPSPLIT = os.environ.get('IMAGINAIRE_AMD_TAPSPLIT', '1') == '1'


def tapsplit_eligible(x, w, stride, padding, dilation, groups):
    """The tap-split path (``_TapSplitConv2d``) for narrow RGB heads: bf16 compute, stride 1,
    groups 1, Cout <= 8 with a spatial filter, a wide input and enough pixels to fill the chip."""
    if not (_TAPSPLIT and x.is_cuda and x.dim() == 4 and w.dim() == 4 and groups == 1 and
            stride == (1, 1) and _mfma_enabled()):
        return False
    cout, cin, kh, kw = w.shape
    if not (cout <= 8 and kh * kw > 1 and cin >= 32 and kh * kw * cout <= 512):
        return False
    if _compute_dtype(x, w) != torch.bfloat16:
        return False
    ho, wo = _out_hw(x.shape[2], x.shape[3], (kh, kw), stride, padding, dilation)
    if (ho, wo) != (x.shape[2] + 2 * padding[0] - dilation[0] * (kh - 1),
                    x.shape[3] + 2 * padding[1] - dilation[1] * (kw - 1)) or ho <= 0 or wo <= 0:
        return False
    npix = x.shape[0] * x.shape[2] * x.shape[3]
    cp, cz = _round_up(cin, 64), _round_up(cout * kh * kw, 64)
    # the partials Z must not outweigh the input (MUNIT's 64 -> 3 7x7 head: 147 partial
    # channels per pixel ran slower than the direct 64-wide k10 tile,
    # profiles/recipe_munit256_conv_log_mi355x.txt); k10 / k11 32-bit buffer offsets
    return cz <= cp and npix >= 128 * 64 and npix * cp * 2 < (1 << 30) and \
        npix * cz * 2 < (1 << 30)


_WGRAD_CHOICE = {}
# shapes first seen inside a backward under IMAGINAIRE_AMD_MFMA_WGRAD=auto: they run k11 until
# tune_pending() (called by the trainer at rank-uniform iteration boundaries, never inside a
# backward) has timed both kernels and agreed the choice across ranks
_WGRAD_PENDING = {}


def _time_ms(fn, reps=3):
    fn()  # warm (MIOpen find / compile)
    start, end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    start.record()
    for _ in range(reps):
        fn()
    end.record()
    end.synchronize()
    return start.elapsed_time(end)


def _time_candidates(fns, reps=3, trials=3):
    """{name: ms} for {name: fn}: every candidate warmed, then ``trials`` rounds that time each
    one in turn (interleaved, so clock / power drift hits all alike), the minimum per candidate.
    (One back-to-back timing each picked different k11 variants for near-tied SPADE shapes from
    run to run: ±1-2% on the step.)"""
    for fn in fns.values():
        fn()
    best = {name: float('inf') for name in fns}
    start, end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(trials):
        for name, fn in fns.items():
            start.record()
            for _ in range(reps):
                fn()
            end.record()
            end.synchronize()
            best[name] = min(best[name], start.elapsed_time(end))
    return best


def _agree(times):
    """Sum per-candidate timings over ranks (every rank then takes the same argmin).
    ``times``: {key: {candidate: ms}} with identical keys and candidates on every rank."""
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1) or \
            not times:
        return times
    keys = sorted(times, key=repr)
    cands = [sorted(times[k]) for k in keys]
    flat = [times[k][c] for k, cs in zip(keys, cands) for c in cs]
    dev = 'cpu' if dist.get_backend() == 'gloo' else torch.device('cuda',
                                                                  torch.cuda.current_device())
    t = torch.tensor(flat, dtype=torch.float64, device=dev)
    dist.all_reduce(t)
    t = t.cpu().tolist()
    out, i = {}, 0
    for k, cs in zip(keys, cands):
        out[k] = {}
        for c in cs:
            out[k][c] = t[i]
            i += 1
    return out


def _wgrad_fns(dy, xb, wb, stride, padding, dilation, cout, cin, wdt, variant=0, sn=None,
               dest=None):
    def k11(v=variant):
        return _ext.ext().conv2d_wgrad_mfma(dy, xb, wb.shape[2], wb.shape[3], stride[0],
                                            stride[1], padding[0], padding[1], dilation[0],
                                            dilation[1], cout, cin, wdt == torch.bfloat16, 1, v,
                                            None if sn is None else list(sn), dest)

    def miopen():
        return torch.ops.aten.convolution_backward(
            dy, xb, wb, None, stride, padding, dilation, False, [0, 0], 1,
            [False, True, False])[1]
    return k11, miopen


def _k11_variants(dy, xb, wb, stride, dilation):
    """k11 kernel variants that can run this weight gradient: 'k11' (multi-tap / one-tap, two
    or three blocks per CU) and, where eligible, 'k11v2' (one block per CU, 64 x 64 x KW-tap
    accumulators per wave). Neither wins everywhere (profiles/wgrad_readahead_probe_mi355x.txt),
    so the autotuner times both per shape."""
    if _ext.ext().conv2d_wgrad_v2_eligible(dy, xb, wb.shape[2], wb.shape[3], stride[0],
                                           stride[1], dilation[0], dilation[1]):
        return ('k11', 'k11v2')
    return ('k11',)


def _take_grad_dest(p, shape):
    """The DDP bucket slice armed for parameter ``p``'s gradient (``parallel/ddp.py``
    ``begin()``: ``p._iamd_grad_dest = (flat, offset)``), handed out ONCE per backward and only
    while ``p`` has no gradient yet: k11 then writes the weight gradient straight into the
    bucket and autograd adopts that view as ``p.grad`` (no copy into the bucket). A second use
    of the weight in the same backward gets fresh memory (autograd sums the two)."""
    if p is None:
        return None
    d = getattr(p, '_iamd_grad_dest', None)
    if d is None or p.grad is not None or getattr(p, '_iamd_grad_dest_used', True):
        return None
    if tuple(p.shape) != tuple(shape) or p.dtype != torch.float32 or \
            not p.is_contiguous(memory_format=_CL):
        return None
    p._iamd_grad_dest_used = True
    flat, off = d
    return flat[off:off + p.numel()].as_strided(p.size(), p.stride())


def _wgrad(dy, xb, wb, stride, padding, dilation, cout=-1, cin=-1, wdt=torch.float32, sn=None,
           dest=None):
    """Weight gradient: k11 or MIOpen wrw (``IMAGINAIRE_AMD_MFMA_WGRAD`` = 1 | 0 | auto; auto =
    the faster of the two per shape, timed by :func:`tune_pending` outside the backward and
    agreed across ranks). k11 returns the gradient already cropped to (cout, cin) and in the
    weight's dtype (bf16 for the bf16 spectral-norm / autocast weights): the crop and cast ride
    in its split-K sum. ``sn`` = (bf16 shadow, u, v, sigma) of a spectrally normalised weight
    (:class:`_MfmaConv2d`): k11 only, returning the fp32 gradient w.r.t. W."""
    k11, miopen = _wgrad_fns(dy, xb, wb, stride, padding, dilation, cout, cin, wdt, sn=sn,
                             dest=dest)
    mode = _MFMA_WGRAD if sn is None else '1'  # (the SN backward rides in k11's split-K sum)
    fl = 2.0 * dy.shape[0] * dy.shape[2] * dy.shape[3] * wb.numel()
    desc = _gemm_desc(xb, wb, stride, padding)
    if mode == '0' and not _capturing():
        with _Logged('wgrad', 'miopen', fl, desc):
            return miopen()
    variants = _k11_variants(dy, xb, wb, stride, dilation)
    if mode == '1' and len(variants) == 1:
        with _Logged('wgrad', 'k11', fl, desc):
            return k11()
    # per-shape choice among the candidates (mode 1: the k11 variants; auto: those and MIOpen),
    # timed by tune_pending() between iterations; the default routing runs until then
    key = (tuple(dy.shape), tuple(xb.shape), tuple(wb.shape), stride, padding, dilation,
           cout, cin, wdt) + (() if sn is None else ('sn',) if len(sn) == 4 else ('sndx',))
    # ('sn': tuned with the k11 <G, W> epilogue; 'sndx': <G, W> came from the data gradient)
    choice = _WGRAD_CHOICE.get(key)
    if choice is None:
        _WGRAD_PENDING.setdefault(key, (dy.dtype, xb.dtype, wb.dtype))
        choice = 'k11'
    with _Logged('wgrad', choice, fl, desc):
        if choice == 'miopen' and sn is None and not _capturing():
            return miopen()
        if choice == 'k11v2':
            return k11(2)
        return k11(1 if len(variants) > 1 and key in _WGRAD_CHOICE else 0)


def routing_table():
    """The autotuned routing decisions so far (for logs / bench jsonl rows)."""
    return {'wgrad': {repr(k[:6]): v for k, v in _WGRAD_CHOICE.items()},
            'deconv': {repr(k): v for k, v in _DECONV_CHOICE.items()}}


def _pending_union():
    """Every rank's pending tuning keys, agreed: [(kind, key, dtypes)] sorted by repr, the same
    list on every rank. World size 1: the local keys. At world > 1 one fixed-size count
    all-reduce runs on EVERY call (a rank with nothing pending must still take part, or the
    ranks with new keys would wait in a collective it never joins), then the key lists are
    all-gathered only when some rank has one. A rank may miss keys a peer saw (per-rank shapes:
    the fs-vid2vid hand crops, ragged batches): the weight-gradient candidates are timed from the
    key's shapes alone, so every rank times the union."""
    import torch.distributed as dist
    local = [('w', k, v) for k, v in _WGRAD_PENDING.items()] + \
        [('d', k, None) for k in _DECONV_PENDING]
    if not (dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1):
        return sorted(local, key=lambda e: repr(e[:2]))
    dev = 'cpu' if dist.get_backend() == 'gloo' else torch.device('cuda',
                                                                  torch.cuda.current_device())
    n = torch.tensor([len(local)], dtype=torch.int64, device=dev)
    dist.all_reduce(n, op=dist.ReduceOp.MAX)
    if int(n.item()) == 0:
        return []
    gathered = [None] * dist.get_world_size()
    dist.all_gather_object(gathered, [(kind, k, v) for kind, k, v in local])
    union = {}
    for lst in gathered:
        for kind, k, v in lst:
            union.setdefault((kind, k), v)
    return sorted([(kind, k, v) for (kind, k), v in union.items()], key=lambda e: repr(e[:2]))


_TUNE_STATE = {'calls': 0, 'empty': 0}
# interleaved timing rounds per wgrad candidate set (the minimum over them decides; A/B knob)
_TUNE_TRIALS = max(1, int(os.environ.get('IMAGINAIRE_AMD_TUNE_TRIALS', '3')))
_TUNE_QUIET_PERIOD = 64


def tune_pending():
    """Resolve the per-shape kernel choices first seen since the last call (wgrad k11 variants /
    k11 vs MIOpen; FlowNet2 deconv k10 phases vs MIOpen): time each candidate on scratch tensors
    of the recorded shapes and agree across ranks (:func:`_pending_union`, :func:`_agree`). Call
    it at the same iteration on every rank, outside any forward / backward and outside graph
    capture (every rank skips it while capturing)."""
    if torch.cuda.is_available() and torch.cuda.is_current_stream_capturing():
        return 0
    import torch.distributed as dist
    multi = dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1
    if not multi and not (_WGRAD_PENDING or _DECONV_PENDING):
        return 0
    if multi:
        # the union is a collective + host sync: once it has come back empty a few calls in a
        # row, only every _TUNE_QUIET_PERIOD-th call runs it. Every rank makes the same calls
        # and sees the same union, so the schedule stays rank-uniform.
        _TUNE_STATE['calls'] += 1
        if _TUNE_STATE['empty'] >= 3 and _TUNE_STATE['calls'] % _TUNE_QUIET_PERIOD:
            return 0
    entries = _pending_union()
    if not entries:
        _TUNE_STATE['empty'] += 1
        return 0
    _TUNE_STATE['empty'] = 0
    times = {}
    dev = torch.device('cuda', torch.cuda.current_device())
    cl = torch.channels_last
    for kind, key, dts in entries:
        if kind == 'w':
            dyt, xt, wt = dts
            dys, xs, ws, stride, padding, dilation, cout, cin, wdt = key[:9]
            dy = torch.randn(dys, device=dev).to(dyt).contiguous(memory_format=cl)
            xb = torch.randn(xs, device=dev).to(xt).contiguous(memory_format=cl)
            wb = torch.randn(ws, device=dev).to(wt).contiguous(memory_format=cl)
            sn = None
            if len(key) > 9 and key[9] == 'sn':  # the k11 variants with their <G, W> epilogue
                kk = ws[2] * ws[3]
                sn = (torch.randn((cout, cin) + tuple(ws[2:]), device=dev).to(
                    torch.bfloat16).contiguous(memory_format=cl),
                    torch.randn(cout, device=dev), torch.randn(cin * kk, device=dev),
                    torch.ones(1, device=dev))
            k11, miopen = _wgrad_fns(dy, xb, wb, stride, padding, dilation, cout, cin, wdt,
                                     sn=sn)
            fns = {}
            if _MFMA_WGRAD != '1' and sn is None:
                fns['miopen'] = miopen
            if len(_k11_variants(dy, xb, wb, stride, dilation)) > 1:
                fns['k11'] = lambda: k11(1)
                fns['k11v2'] = lambda: k11(2)
            else:
                fns['k11'] = k11
            times[('w',) + key] = _time_candidates(fns, trials=_TUNE_TRIALS)
        else:
            # a deconv key names its weight, which only the ranks that saw it hold: those time
            # it, the others report 0 and the vote below averages over the ranks that timed
            fns = _DECONV_PENDING.get(key)
            cand = {'k10s': 0.0, 'miopen': 0.0, '#': 0.0}
            if fns is not None:
                cand = {name: _time_ms(fn) for name, fn in fns().items()}
                cand['#'] = 1.0
            times[('d',) + key] = cand
    times = _agree(times)
    for k, t in times.items():
        t = {c: v for c, v in t.items() if c != '#'}
        choice = min(t, key=t.get)
        if k[0] == 'w':
            _WGRAD_CHOICE[k[1:]] = choice
        else:
            _DECONV_CHOICE[k[1:]] = choice
    n = len(times)
    _WGRAD_PENDING.clear()
    _DECONV_PENDING.clear()
    return n


def conv2d_act(x, weight, bias=None, stride=1, padding=0, dilation=1, slope=1.0):
    """``act(conv2d(x, weight) + bias)`` with a leaky slope (1 = identity, 0 = relu);
    one k10 launch when eligible, otherwise MIOpen conv + k2 bias-act epilogue."""
    stride, padding, dilation = _pair(stride), _pair(padding), _pair(dilation)
    if isinstance(weight, SNWeight):
        if _sn_fused_ok(x, weight, stride, padding, dilation):
            return _MfmaConv2d.apply(x, weight.W, bias, stride, padding, dilation, slope, None,
                                     weight)
        weight = weight.materialize()
    xt = _thin_view(x, weight.shape[1])
    if tappack_eligible(xt, weight, stride, padding, dilation, 1):
        return _TapPackConv2d.apply(xt, weight, bias, stride, padding, dilation, slope)
    weight = _match_channels(x, weight)
    if slope == 1.0 and tapsplit_eligible(x, weight, stride, padding, dilation, 1):
        return _TapSplitConv2d.apply(x, weight, bias, padding, dilation)
    if mfma_eligible(x, weight, stride, padding, dilation, 1):
        return _MfmaConv2d.apply(x, weight, bias, stride, padding, dilation, slope)
    from imaginaire_amd.ops.bias_act import bias_act
    if slope == 1.0:
        return conv2d(x, weight, bias, stride, padding, dilation)
    return bias_act(conv2d(x, weight, None, stride, padding, dilation), bias, slope)


class _PadNHWC(torch.autograd.Function):
    """Reflect / replicate padding of NHWC activations (csrc/conv_aux.hip pad_nhwc_*)."""

    @staticmethod
    def forward(ctx, x, pad, mode):
        ctx.conf = (x.shape[2], x.shape[3], pad, mode)
        return _ext.ext().pad_nhwc_fwd(x, pad[0], pad[1], pad[2], pad[3], mode)

    @staticmethod
    def backward(ctx, dy):
        h, w, pad, mode = ctx.conf
        dy = dy.contiguous(memory_format=_CL)
        return _ext.ext().pad_nhwc_bwd(dy, h, w, pad[0], pad[1], pad[2], pad[3], mode), \
            None, None


_PAD_MODES = {'reflect': 0, 'replicate': 1}


def pad(x, pad_lrtb, mode):
    """``F.pad(x, pad_lrtb, mode)`` for 4-D inputs; reflect / replicate padding of packed NHWC
    activations (any channel count: 16-byte copies when it is a multiple of 8) runs the HIP
    gather kernels (forward and backward)."""
    m = _PAD_MODES.get(mode)
    if m is not None and x.dim() == 4 and \
            x.dtype in (torch.bfloat16, torch.float32) and _ext.use_native(x) and \
            x.is_contiguous(memory_format=_CL) and len(pad_lrtb) == 4 and min(pad_lrtb) >= 0 and \
            (m == 1 or (max(pad_lrtb[0], pad_lrtb[1]) < x.shape[3] and
                        max(pad_lrtb[2], pad_lrtb[3]) < x.shape[2])) and \
            (m == 0 or max(pad_lrtb) < 15):
        return _PadNHWC.apply(x, tuple(int(p) for p in pad_lrtb), m)
    return F.pad(x, pad_lrtb, mode=mode)


_RESIDUAL_EPILOGUE = os.environ.get('IMAGINAIRE_AMD_CONV_RESIDUAL', '1') == '1'


def _residual_fusible(res, x, weight, stride, padding, dilation):
    """The k10 epilogue can add ``res`` (a bf16 packed-NHWC tensor shaped like the conv output,
    whose channels k10 stores directly)."""
    if res is None or not _RESIDUAL_EPILOGUE or not (
            torch.is_tensor(res) and res.is_cuda and res.dtype == torch.bfloat16 and
            res.dim() == 4 and res.is_contiguous(memory_format=_CL)):
        return False
    cout = weight.shape[0]
    op = _out_pad(cout)
    ncv = cout if (op != cout and cout % 8 == 0) else op
    ho, wo = _out_hw(x.shape[2], x.shape[3], weight.shape[2:], stride, padding, dilation)
    return ncv == cout and tuple(res.shape) == (x.shape[0], cout, ho, wo)


def conv2d(x, weight, bias=None, stride=1, padding=0, dilation=1, groups=1,
           padding_mode='zeros', residual=None):
    """``F.conv2d`` (+ ``residual``, added to the output: on the k10 path inside its epilogue,
    otherwise as a separate add). ``weight`` may be an :class:`SNWeight`."""
    if isinstance(weight, SNWeight):
        st, pd, dl = _pair(stride), _pair(padding), _pair(dilation)
        if groups == 1 and x.is_cuda and x.dim() == 4:
            if padding_mode not in ('zeros', None):  # reflect / replicate: pad, then the conv
                vc = getattr(x, '_iamd_valid_channels', None)
                x = pad(nhwc(x), _pad_arg(padding), padding_mode)
                if vc is not None:
                    x._iamd_valid_channels = vc
                padding, pd, padding_mode = 0, (0, 0), 'zeros'
            if _sn_fused_ok(x, weight, st, pd, dl, residual):
                return _MfmaConv2d.apply(x, weight.W, bias, st, pd, dl, 1.0, residual, weight)
        weight = weight.materialize()
    if residual is not None:
        st, pd, dl = _pair(stride), _pair(padding), _pair(dilation)
        if groups == 1 and padding_mode in ('zeros', None) and x.is_cuda and x.dim() == 4:
            w = _match_channels(x, weight)
            if not tapsplit_eligible(x, w, st, pd, dl, groups) and \
                    mfma_eligible(x, w, st, pd, dl, groups) and \
                    _residual_fusible(residual, x, w, st, pd, dl):
                return _MfmaConv2d.apply(x, w, bias, st, pd, dl, 1.0, residual)
        return conv2d(x, weight, bias, stride, padding, dilation, groups, padding_mode) + residual
    if padding_mode != 'zeros' and padding_mode is not None:
        vc = getattr(x, '_iamd_valid_channels', None)
        x = pad(nhwc(x), _pad_arg(padding), padding_mode)
        if vc is not None:
            x._iamd_valid_channels = vc
        padding = 0
    if x.is_cuda and x.dim() == 4 and weight.dim() == 4:
        st, pd, dl = _pair(stride), _pair(padding), _pair(dilation)
        xt = _thin_view(x, weight.shape[1])
        if tappack_eligible(xt, weight, st, pd, dl, groups):
            return _TapPackConv2d.apply(xt, weight, bias, st, pd, dl, 1.0)
    if groups == 1:
        weight = _match_channels(x, weight)
    if x.is_cuda and x.dim() == 4:
        st, pd, dl = _pair(stride), _pair(padding), _pair(dilation)
        if tapsplit_eligible(x, weight, st, pd, dl, groups):
            return _TapSplitConv2d.apply(x, weight, bias, pd, dl)
        if mfma_eligible(x, weight, st, pd, dl, groups):
            return _MfmaConv2d.apply(x, weight, bias, st, pd, dl, 1.0)
        cin = weight.shape[1]
        if groups == 1 and cin > 64 and cin % 32:
            cp = _round_up(cin, 32)
            x = _pad_channels(x, cp)
            weight = _pad_channels(weight, cp)
        x = nhwc(x)
        weight = nhwc(weight)
        if _CONV_LOG is not None and weight.dim() == 4:
            ho, wo = _out_hw(x.shape[2], x.shape[3], weight.shape[2:], st, pd, dl)
            with _Logged('fwd', 'miopen', 2.0 * x.shape[0] * ho * wo * weight.numel(),
                         _gemm_desc(x, weight, st, pd)):
                return F.conv2d(x, weight, bias, stride, padding, dilation, groups)
    return F.conv2d(x, weight, bias, stride, padding, dilation, groups)


_DECONV_MIN_PIX = int(os.environ.get('IMAGINAIRE_AMD_DECONV_MIN_PIX', 4096))
_DECONV_CHOICE = {}
_DECONV_PENDING = {}
_DECONV_FORCE = os.environ.get('IMAGINAIRE_AMD_DECONV')  # 'k10s' / 'miopen': skip the tuning


def deconv_eligible(x, weight, stride, padding, output_padding, groups, dilation):
    """The phase-convolution path of :func:`conv_transpose2d`: inference (no autograd graph),
    bf16, square stride 2-4, no dilation / output padding / groups, >= 16 channels each side
    and an output map that is not tiny — inside a captured graph (``_capturing``) any channel
    count and map size (MIOpen's backward-data solvers never run in a graph: their workspace
    zeroing is not captured)."""
    if not (x.is_cuda and x.dim() == 4 and weight.dim() == 4 and groups == 1 and
            _STRIDED_DGRAD and _mfma_enabled() and _ext.use_native(x)):
        return False
    if torch.is_grad_enabled() and (x.requires_grad or weight.requires_grad):
        return False
    s, op, dl = stride, output_padding, dilation
    if not (s[0] == s[1] and 2 <= s[0] <= 4 and op == (0, 0) and dl == (1, 1)):
        return False
    if _compute_dtype(x, weight) != torch.bfloat16:
        return False
    cin, cout, kh, kw = weight.shape
    cap = _capturing()
    if (min(cin, cout) < 16 and not cap) or kh < s[0] or kw < s[1] or not (
            0 <= padding[0] < kh and 0 <= padding[1] < kw):
        return False
    ho = (x.shape[2] - 1) * s[0] - 2 * padding[0] + kh
    wo = (x.shape[3] - 1) * s[1] - 2 * padding[1] + kw
    return ho > 0 and wo > 0 and (cap or x.shape[0] * ho * wo >= _DECONV_MIN_PIX)


def _deconv_phase_weights(weight, s, padding, cp, op, phases=True):
    """The padded bf16 weight of a transposed conv and (``phases``) its s*s flipped phase
    sub-kernels. For a Parameter (FlowNet2's frozen decoders) they are cached on the Parameter
    itself, keyed on its storage and version counter, so the cache dies with the weight and an
    in-place update invalidates it."""
    key = (weight.data_ptr(), weight._version, s, tuple(padding), cp, op, phases)
    cached = getattr(weight, '_iamd_deconv', None)
    if cached is not None and cached[0] == key:
        return cached[1]
    wb = _pad_rows(_pad_channels(weight.detach(), op, torch.bfloat16), cp)
    wts = None
    if phases:
        wts = {}
        for ry in range(s):
            for rx in range(s):
                wts[(ry, rx)] = _ext.ext().conv_weight_flip_t(
                    wb, s, (ry + padding[0]) % s, (rx + padding[1]) % s, 1)
    if isinstance(weight, torch.nn.Parameter) or not weight.requires_grad:
        weight._iamd_deconv = (key, (wb, wts))  # (dies with the weight tensor)
    return wb, wts


def _deconv_phase(x, weight, bias, st, pd, ho, wo):
    """Transposed conv as the strided data gradient of :func:`_strided_dgrad`: the one-launch
    kernel (every phase stored straight into its parity sub-grid, no scatter pass) when
    ``IMAGINAIRE_AMD_STRIDED_ONE_LAUNCH`` is on, else the s*s k10 phase convolutions + scatter."""
    cin, cout, kh, kw = weight.shape
    cp, op = _round_up(cin, 64), _out_pad(cout)
    one = _STRIDED_ONE_LAUNCH and 0 <= pd[0] < kh and 0 <= pd[1] < kw
    wb, wts = _deconv_phase_weights(weight, st[0], pd, cp, op, phases=not one)
    # (one launch: Cout % 8 == 0 stores only the real output channels, no crop copy)
    ncv = cout if (one and op != cout and cout % 8 == 0) else -1
    y = _strided_dgrad(_pad_channels(x, cp, torch.bfloat16), wb, ho, wo, st[0], pd, wts,
                       ncv=ncv)
    y = y[:, :cout] if y.shape[1] != cout else y
    return y if bias is None else y + bias.to(y.dtype).view(1, -1, 1, 1)


def conv_transpose2d(x, weight, bias=None, stride=1, padding=0, output_padding=0, groups=1,
                     dilation=1):
    """``F.conv_transpose2d``. A strided transposed conv is the data gradient of the strided
    conv with the same weight ([Cin_t, Cout_t, KH, KW] read as [Cout, Cin, KH, KW]), so on
    eligible inference calls (FlowNet2's 4x4 / stride-2 decoders) it runs as the s*s k10
    phase convolutions of :func:`_strided_dgrad` instead of MIOpen's backward-data solvers."""
    st, pd = _pair(stride), _pair(padding)
    if deconv_eligible(x, weight, st, pd, _pair(output_padding), groups, _pair(dilation)):
        cin, cout, kh, kw = weight.shape
        cp, op = _round_up(cin, 64), _out_pad(cout)
        ho = (x.shape[2] - 1) * st[0] - 2 * pd[0] + kh
        wo = (x.shape[3] - 1) * st[1] - 2 * pd[1] + kw
        xn, wn = nhwc(x), nhwc(weight)

        def phase():
            return _deconv_phase(x, weight, bias, st, pd, ho, wo)

        def miopen():
            return F.conv_transpose2d(xn, wn, bias, st, pd)

        # per-shape choice: MIOpen's backward-data solvers range from ~20 to ~140 TF/s over
        # FlowNet2's decoder shapes, the phase path from ~40 to ~100
        # (profiles/deconv_probe_mi355x.txt). Unseen shapes run MIOpen until tune_pending()
        # times both at a rank-uniform point and agrees the choice across ranks (a per-rank
        # choice could give ranks different ground-truth flow at bf16 rounding level).
        key = (tuple(x.shape), tuple(weight.shape), st, pd)
        choice = 'k10s' if _capturing() else (_DECONV_FORCE or _DECONV_CHOICE.get(key))
        if choice is None:
            if key not in _DECONV_PENDING:
                shapes = (tuple(x.shape), x.dtype, weight.detach(), bias, st, pd)

                def fns(shapes=shapes):
                    xs, xdt, w, b, st_, pd_ = shapes
                    xt = torch.randn(xs, device=w.device).to(xdt)
                    cin_, cout_, kh_, kw_ = w.shape
                    ho_ = (xs[2] - 1) * st_[0] - 2 * pd_[0] + kh_
                    wo_ = (xs[3] - 1) * st_[1] - 2 * pd_[1] + kw_

                    def ph():
                        with torch.no_grad():
                            return _deconv_phase(xt, w, b, st_, pd_, ho_, wo_)

                    def mi():
                        with torch.no_grad():
                            return F.conv_transpose2d(nhwc(xt), nhwc(w), b, st_, pd_)
                    return {'k10s': ph, 'miopen': mi}
                _DECONV_PENDING[key] = fns
            choice = 'miopen'
        fl = 2.0 * x.shape[0] * x.shape[2] * x.shape[3] * weight.numel()
        with _Logged('deconv', choice, fl, _gemm_desc(x, weight, st, pd)):
            return phase() if choice == 'k10s' else miopen()
    if x.is_cuda:
        x = nhwc(x)
        weight = nhwc(weight)
    return F.conv_transpose2d(x, weight, bias, stride, padding, output_padding, groups, dilation)
