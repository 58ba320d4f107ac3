"""Activation normalisation layers (reference layers/activation_norm.py:22-432).

Every batch / sync-batch / instance norm here is a fused-norm module: its
``fused(x, gamma, beta, gb, act_slope)`` method runs statistics, affine,
(spatially) adaptive modulation and the following activation in the k1 HIP
kernels. Parameter / buffer names equal PyTorch's BatchNorm / InstanceNorm so
checkpoints match the reference's state dicts.

SPADE MI355X specifics (SpatiallyAdaptiveNorm):
  * with ``separate_projection`` the γ and β convolutions (two MIOpen calls on
    the same hidden map in the reference) are concatenated into ONE conv with
    2C output channels; its NHWC output is consumed directly by the fused
    kernel through strided views, and the backward writes dγ|dβ into one
    buffer (no slicing copies);
  * the nearest-neighbour resize of the label map is cached per resolution
    for the duration of one generator forward (``LabelMapCache``).
"""
import os
from types import SimpleNamespace

import torch

from imaginaire_amd.ops import conv as nhwc_conv
from torch import nn
from torch.nn import functional as F

from imaginaire_amd.ops.norm import defer_sync_bwd, fused_norm_act, prefetch_sync_stats
from imaginaire_amd.ops.resize import interpolate
from .conv import LinearBlock, Conv2dBlock, HyperConv2d, PartialConv2dBlock
from .misc import PartialSequential


class LabelMapCache(object):
    """Per-forward cache of resized conditional maps keyed by (id, size)."""

    _active = None

    def __init__(self):
        self.store = {}

    def __enter__(self):
        self._prev = LabelMapCache._active
        LabelMapCache._active = self
        return self

    def __exit__(self, *args):
        LabelMapCache._active = self._prev
        self.store = {}

    @staticmethod
    def resize(t, size, mode='nearest', conv_pad=False):
        """Resized conditional map, memoised per forward. ``conv_pad``: the consumer is a
        conv block — a CUDA NHWC map with an odd channel count (185-channel COCO-Stuff
        labels) is returned zero-padded to the conv kernels' channel granularity and marked
        (ops.conv.mark_zero_tail), so the padding happens once per resolution per forward
        instead of inside every SPADE layer's MLP conv."""
        cache = LabelMapCache._active
        same = tuple(t.shape[2:]) == tuple(size) and mode == 'nearest'
        pad = conv_pad and t.is_cuda and t.dim() == 4 and t.shape[1] > 64 and \
            t.shape[1] % 64 != 0
        if same and not pad:
            return t
        key = (id(t), t.data_ptr(), tuple(size), mode, pad)
        out = cache.store.get(key) if cache is not None else None
        if out is None:
            src = t
            if pad:
                # pad ONCE at the source resolution (cached), then resize the padded map: the
                # zero tail stays zero and the NHWC resize kernels need channels % 8 == 0
                pkey = (id(t), t.data_ptr(), 'padded')
                src = cache.store.get(pkey) if cache is not None else None
                if src is None:
                    c = t.shape[1]
                    src = nhwc_conv.mark_zero_tail(
                        nhwc_conv._pad_channels(t, (c + 63) // 64 * 64), c)
                    if cache is not None:
                        cache.store[pkey] = src
            out = src if same else interpolate(src, size=size, mode=mode)
            if cache is not None:
                cache.store[key] = out
        return out


class _FusedNormBase(nn.Module):
    """Shared machinery of the fused batch / instance norms."""

    supports_fused_act = True
    mode = 'batch'

    def __init__(self, num_features, eps=1e-5, momentum=0.1, affine=True,
                 track_running_stats=True):
        super().__init__()
        self.num_features = num_features
        self.eps = eps
        self.momentum = momentum
        self.affine = affine
        self.track_running_stats = track_running_stats
        if affine:
            self.weight = nn.Parameter(torch.ones(num_features))
            self.bias = nn.Parameter(torch.zeros(num_features))
        else:
            self.register_parameter('weight', None)
            self.register_parameter('bias', None)
        if track_running_stats:
            self.register_buffer('running_mean', torch.zeros(num_features))
            self.register_buffer('running_var', torch.ones(num_features))
            self.register_buffer('num_batches_tracked', torch.tensor(0, dtype=torch.long))
        else:
            self.register_buffer('running_mean', None)
            self.register_buffer('running_var', None)
            self.register_buffer('num_batches_tracked', None)
        self.process_group = None

    def reset_running_stats(self):
        if self.track_running_stats:
            self.running_mean.zero_()
            self.running_var.fill_(1)
            self.num_batches_tracked.zero_()

    def reset_parameters(self):
        self.reset_running_stats()
        if self.affine:
            nn.init.ones_(self.weight)
            nn.init.zeros_(self.bias)

    def _factor(self, defer_count=False):
        """Running-average factor of this call. With ``defer_count`` (and a fixed momentum)
        ``num_batches_tracked`` is NOT incremented here: the caller hands it to
        :func:`fused_norm_act`, whose statistics kernel increments it."""
        if not (self.training and self.track_running_stats):
            return 0.0
        if defer_count and self.momentum is not None:
            return self.momentum
        self.num_batches_tracked.add_(1)
        if self.momentum is None:
            return 1.0 / float(self.num_batches_tracked.item())
        return self.momentum

    def _deferred_count(self, use_batch):
        return self.num_batches_tracked if (
            use_batch and self.training and self.track_running_stats and
            self.momentum is not None) else None

    def _effective_mode(self):
        return self.mode

    def fused(self, x, gamma=None, beta=None, gb=None, act_slope=1.0, deferred=None):
        squeeze = None
        if x.dim() == 2:
            squeeze = x.shape
            x = x[:, :, None, None]
        elif x.dim() == 3:
            squeeze = x.shape
            x = x[:, :, :, None]
        elif x.dim() == 5:
            return self._fallback_nd(x, gamma, beta, act_slope)
        use_batch = self.training or not self.track_running_stats or \
            self._effective_mode() == 'instance'
        y = fused_norm_act(
            x, self._effective_mode(), self.weight, self.bias, gamma=gamma, beta=beta, gb=gb,
            running_mean=self.running_mean if self.track_running_stats else None,
            running_var=self.running_var if self.track_running_stats else None,
            training=use_batch, momentum=self._factor(True) if use_batch else 0.0, eps=self.eps,
            slope=act_slope, process_group=self.process_group, deferred=deferred,
            num_batches=self._deferred_count(use_batch))
        if squeeze is not None:
            y = y.reshape(squeeze)
        return y

    def _fallback_nd(self, x, gamma, beta, act_slope):
        if self._effective_mode() == 'instance':
            y = F.instance_norm(x, weight=self.weight, bias=self.bias, eps=self.eps)
        else:
            y = F.batch_norm(x, self.running_mean, self.running_var, self.weight, self.bias,
                             self.training or not self.track_running_stats,
                             self.momentum or 0.1, self.eps)
        if gamma is not None:
            y = y * (1 + gamma) + beta
        if act_slope != 1.0:
            y = F.leaky_relu(y, act_slope) if act_slope > 0 else F.relu(y)
        return y

    def forward(self, x, act_slope=1.0):
        return self.fused(x, act_slope=act_slope)

    def extra_repr(self):
        return '{num_features}, eps={eps}, momentum={momentum}, affine={affine}, ' \
               'track_running_stats={track_running_stats}'.format(**self.__dict__)


class BatchNorm2d(_FusedNormBase):
    """BatchNorm (1d/2d inputs) running on the fused HIP kernels."""
    mode = 'batch'


class SyncBatchNorm(_FusedNormBase):
    """Cross-replica BatchNorm: one all-gather (fwd) / all-reduce (bwd) per layer."""
    mode = 'sync_batch'

    def _effective_mode(self):
        from imaginaire_amd.ops.norm import sync_active
        if self.training and sync_active(self.process_group):
            return 'sync_batch'
        return 'batch'


class InstanceNorm2d(_FusedNormBase):
    """InstanceNorm (PyTorch defaults: no running stats)."""
    mode = 'instance'

    def __init__(self, num_features, eps=1e-5, momentum=0.1, affine=False,
                 track_running_stats=False):
        super().__init__(num_features, eps, momentum, affine, track_running_stats)


def fused_norm_or_none(norm, x, gamma=None, beta=None, gb=None, act_slope=1.0, deferred=None):
    """Apply ``norm`` (fused module, torch module or None) + modulation + activation."""
    if norm is None:
        return fused_norm_act(x, 'none', gamma=gamma, beta=beta, gb=gb, slope=act_slope)
    if isinstance(norm, _FusedNormBase):
        return norm.fused(x, gamma=gamma, beta=beta, gb=gb, act_slope=act_slope,
                          deferred=deferred)
    y = norm(x)
    if gb is not None:
        gamma, beta = gb.chunk(2, dim=1)
    if gamma is not None:
        if gamma.dim() == 2:
            gamma, beta = gamma[:, :, None, None], beta[:, :, None, None]
        y = y * (1 + gamma) + beta
    if act_slope != 1.0:
        y = F.leaky_relu(y, act_slope) if act_slope > 0 else F.relu(y)
    return y


def _modulate_more(out, gbs, act_slope):
    """Further SPADE modulations ``out·(1+γ_i) + β_i`` (multi-condition SPADE: label map +
    warped image / flow mask in vid2vid / fs-vid2vid), the last one followed by the activation:
    each is one pass of the k1 kernel in 'none' (identity-normalisation) mode, forward and
    backward, with γ|β read straight from the fused γ|β conv output — instead of separate
    add / mul / add / leaky-relu passes and their backward, plus two slice-gradient scatters."""
    if _MULTIMOD_FUSED:
        for i, gb in enumerate(gbs):
            out = fused_norm_act(out, 'none', gb=gb,
                                 slope=act_slope if i == len(gbs) - 1 else 1.0)
        return out
    for gb in gbs:  # A/B reference path (IMAGINAIRE_AMD_SPADE_MULTIMOD=0)
        g, b = gb.chunk(2, dim=1)
        out = out * (1 + g) + b
    if act_slope != 1.0:
        out = F.leaky_relu(out, act_slope) if act_slope > 0 else F.relu(out)
    return out


_MULTIMOD_FUSED = os.environ.get('IMAGINAIRE_AMD_SPADE_MULTIMOD', '1') == '1'
# sync-BN data gradient finished by a join node after the γ|β backward (0: synchronous)
_ASYNC_SYNCBN_BWD = os.environ.get('IMAGINAIRE_AMD_ASYNC_SYNCBN_BWD', '1') == '1'


class AdaptiveNorm(nn.Module):
    """AdaIN / conditional BN: ``norm(x)·(1+γ(y)) + β(y)`` (activation_norm.py:22-106)."""

    supports_fused_act = True

    def __init__(self, num_features, cond_dims, weight_norm_type='', projection=True,
                 separate_projection=False, input_dim=2, activation_norm_type='instance',
                 activation_norm_params=None):
        super().__init__()
        self.projection = projection
        self.separate_projection = separate_projection
        if activation_norm_params is None:
            activation_norm_params = SimpleNamespace(affine=False)
        self.norm = get_activation_norm_layer(num_features, activation_norm_type, input_dim,
                                              **vars(activation_norm_params))
        if self.projection:
            if self.separate_projection:
                self.fc_gamma = LinearBlock(cond_dims, num_features,
                                            weight_norm_type=weight_norm_type)
                self.fc_beta = LinearBlock(cond_dims, num_features,
                                           weight_norm_type=weight_norm_type)
            else:
                self.fc = LinearBlock(cond_dims, num_features * 2,
                                      weight_norm_type=weight_norm_type)
        self.conditional = True

    def forward(self, x, y, act_slope=1.0, **kwargs):
        if self.projection:
            if self.separate_projection:
                gamma = self.fc_gamma(y)
                beta = self.fc_beta(y)
            else:
                gamma, beta = self.fc(y).chunk(2, 1)
        else:
            gamma, beta = y.chunk(2, 1)
        if x.dim() == 4 and gamma.dim() == 2:
            return fused_norm_or_none(self.norm, x, gamma=gamma.contiguous(),
                                      beta=beta.contiguous(), act_slope=act_slope)
        for _ in range(x.dim() - gamma.dim()):
            gamma = gamma.unsqueeze(-1)
            beta = beta.unsqueeze(-1)
        out = self.norm(x) if self.norm is not None else x
        out = out * (1 + gamma) + beta
        if act_slope != 1.0:
            out = F.leaky_relu(out, act_slope) if act_slope > 0 else F.relu(out)
        return out


class _Cat0View(torch.autograd.Function):
    """``cat([a, b], 0)`` of two channels-last tensors that already sit back to back in one
    storage (the γ and β conv weights of a SPADE layer written consecutively into the k5c
    spectral-norm buffer): a view, no copy; the backward splits the gradient."""

    @staticmethod
    def forward(ctx, a, b):
        ctx.n = a.shape[0]
        shape = (a.shape[0] + b.shape[0],) + tuple(a.shape[1:])
        return a.as_strided(shape, a.stride(), a.storage_offset())

    @staticmethod
    def backward(ctx, g):
        return g[:ctx.n], g[ctx.n:]


def cat0(a, b):
    cl = torch.channels_last
    if a.is_cuda and a.dim() == 4 and b.dim() == 4 and a.dtype == b.dtype and \
            a.shape[1:] == b.shape[1:] and a.stride() == b.stride() and \
            a.is_contiguous(memory_format=cl) and b.is_contiguous(memory_format=cl) and \
            a.untyped_storage().data_ptr() == b.untyped_storage().data_ptr() and \
            b.storage_offset() == a.storage_offset() + a.numel():
        return _Cat0View.apply(a, b)
    return torch.cat([a, b], 0)


class SpatiallyAdaptiveNorm(nn.Module):
    """SPADE (activation_norm.py:109-234), fused on MI355X (see module docstring)."""

    supports_fused_act = True

    def __init__(self, num_features, cond_dims, num_filters=128, kernel_size=3,
                 weight_norm_type='', separate_projection=False,
                 activation_norm_type='sync_batch', activation_norm_params=None, partial=False):
        super().__init__()
        if activation_norm_params is None:
            activation_norm_params = SimpleNamespace(affine=False)
        padding = kernel_size // 2
        self.separate_projection = separate_projection
        self.mlps = nn.ModuleList()
        self.gammas = nn.ModuleList()
        self.betas = nn.ModuleList()
        self.num_features = num_features
        if type(cond_dims) != list:
            cond_dims = [cond_dims]
        if not isinstance(num_filters, list):
            num_filters = [num_filters] * len(cond_dims)
        if not isinstance(partial, list):
            partial = [partial] * len(cond_dims)
        self.partial = partial
        for i, cond_dim in enumerate(cond_dims):
            mlp = []
            conv_block = PartialConv2dBlock if partial[i] else Conv2dBlock
            sequential = PartialSequential if partial[i] else nn.Sequential
            if num_filters[i] > 0:
                mlp += [conv_block(cond_dim, num_filters[i], kernel_size, padding=padding,
                                   weight_norm_type=weight_norm_type, nonlinearity='relu')]
            mlp_ch = cond_dim if num_filters[i] == 0 else num_filters[i]
            if self.separate_projection:
                if partial[i]:
                    raise NotImplementedError(
                        'Separate projection not yet implemented for partial conv')
                self.mlps.append(nn.Sequential(*mlp))
                self.gammas.append(conv_block(mlp_ch, num_features, kernel_size, padding=padding,
                                              weight_norm_type=weight_norm_type))
                self.betas.append(conv_block(mlp_ch, num_features, kernel_size, padding=padding,
                                             weight_norm_type=weight_norm_type))
                # γ and β run as ONE conv over their concatenated weights (_gb): their spectral
                # norm group materialises bf16(W / sigma) for them back to back (zero-copy cat)
                for blk in (self.gammas[-1], self.betas[-1]):
                    blk.layers.conv._iamd_sn_materialize = True
            else:
                mlp += [conv_block(mlp_ch, num_features * 2, kernel_size, padding=padding,
                                   weight_norm_type=weight_norm_type)]
                self.mlps.append(sequential(*mlp))
        self.norm = get_activation_norm_layer(num_features, activation_norm_type, 2,
                                              **vars(activation_norm_params))
        self.conditional = True

    def _gb(self, i, label_map):
        """γ|β for condition i as one [N, 2C, H, W] tensor (first C = γ)."""
        if self.separate_projection:
            from .weight_norm import get_weight
            hidden = self.mlps[i](label_map)
            cg = self.gammas[i].layers.conv
            cb = self.betas[i].layers.conv
            w = cat0(get_weight(cg), get_weight(cb))
            b = torch.cat([cg.bias, cb.bias], 0) if cg.bias is not None else None
            return nhwc_conv.conv2d(hidden, w, b, cg.stride, cg.padding, cg.dilation, cg.groups,
                                    cg.padding_mode)
        return self.mlps[i](label_map)

    def forward(self, x, *cond_inputs, act_slope=1.0, **kwargs):
        active = [i for i in range(len(cond_inputs)) if cond_inputs[i] is not None]
        size = x.shape[2:]
        deferred = None
        if isinstance(self.norm, SyncBatchNorm) and self.training and \
                self.norm._effective_mode() == 'sync_batch':
            if not self.norm.affine:
                # start the cross-rank statistics exchange of x now: it rides xGMI while the
                # γ|β convolutions below (independent of it) run
                prefetch_sync_stats(x, self.norm.eps, self.norm.process_group)
            if _ASYNC_SYNCBN_BWD and active:
                # backward mirror: the norm's Σg, Σg·x̂ all-reduce runs while the γ|β / mlp
                # convolution backward runs; this join node (created before them) finishes dx
                x, deferred = defer_sync_bwd(x)
        gbs = []
        for i in active:
            label_map = LabelMapCache.resize(cond_inputs[i], size,
                                             conv_pad=not self.partial[i])
            gbs.append(self._gb(i, label_map))
        if len(gbs) == 0:
            return fused_norm_or_none(self.norm, x, act_slope=act_slope)
        if len(gbs) == 1:
            return fused_norm_or_none(self.norm, x, gb=gbs[0], act_slope=act_slope,
                                      deferred=deferred)
        return _modulate_more(fused_norm_or_none(self.norm, x, gb=gbs[0], act_slope=1.0,
                                                 deferred=deferred),
                              gbs[1:], act_slope)


class HyperSpatiallyAdaptiveNorm(nn.Module):
    """SPADE whose first MLP's weights are supplied at run time (activation_norm.py:237-326)."""

    supports_fused_act = True

    def __init__(self, num_features, cond_dims, num_filters=0, kernel_size=3,
                 weight_norm_type='', activation_norm_type='sync_batch', is_hyper=True):
        super().__init__()
        padding = kernel_size // 2
        self.mlps = nn.ModuleList()
        if type(cond_dims) != list:
            cond_dims = [cond_dims]
        for i, cond_dim in enumerate(cond_dims):
            mlp = []
            if not is_hyper or (i != 0):
                if num_filters > 0:
                    mlp += [Conv2dBlock(cond_dim, num_filters, kernel_size, padding=padding,
                                        weight_norm_type=weight_norm_type, nonlinearity='relu')]
                mlp_ch = cond_dim if num_filters == 0 else num_filters
                mlp += [Conv2dBlock(mlp_ch, num_features * 2, kernel_size, padding=padding,
                                    weight_norm_type=weight_norm_type)]
                mlp = nn.Sequential(*mlp)
            else:
                if num_filters > 0:
                    raise ValueError('Multi hyper layer not supported yet.')
                mlp = HyperConv2d(padding=padding)
            self.mlps.append(mlp)
        self.norm = get_activation_norm_layer(num_features, activation_norm_type, 2, affine=False)
        self.num_features = num_features
        self.conditional = True

    def forward(self, x, *cond_inputs, norm_weights=(None, None), act_slope=1.0, **kwargs):
        deferred = None
        if isinstance(self.norm, SyncBatchNorm) and self.training and _ASYNC_SYNCBN_BWD and \
                self.norm._effective_mode() == 'sync_batch' and \
                any(c is not None for c in cond_inputs):
            x, deferred = defer_sync_bwd(x)  # see SpatiallyAdaptiveNorm.forward
        gbs = []
        for i in range(len(cond_inputs)):
            if cond_inputs[i] is None:
                continue
            if type(cond_inputs[i]) == list:
                cond_input, mask = cond_inputs[i]
                mask = interpolate(mask, size=x.size()[2:], mode='bilinear',
                                     align_corners=False)
            else:
                cond_input = cond_inputs[i]
                mask = None
            label_map = LabelMapCache.resize(cond_input, x.size()[2:])
            if norm_weights is None or norm_weights[0] is None or i != 0:
                gb = self.mlps[i](label_map)
            else:
                gb = self.mlps[i](label_map, conv_weights=norm_weights)
            if mask is not None:
                # the mask (fp32 from the flow branch) must not promote the 2C-channel
                # modulation maps (and everything after them) to fp32
                gb = gb * (1 - mask.to(gb.dtype))
            gbs.append(gb)
        if len(gbs) == 0:
            return fused_norm_or_none(self.norm, x, act_slope=act_slope)
        if len(gbs) == 1:
            return fused_norm_or_none(self.norm, x, gb=gbs[0], act_slope=act_slope,
                                      deferred=deferred)
        return _modulate_more(fused_norm_or_none(self.norm, x, gb=gbs[0], act_slope=1.0,
                                                 deferred=deferred),
                              gbs[1:], act_slope)


class LayerNorm2d(nn.Module):
    """Per-sample mean/std normalisation over (C, H, W) (activation_norm.py:329-374)."""

    def __init__(self, num_features, eps=1e-5, affine=True):
        super().__init__()
        self.num_features = num_features
        self.affine = affine
        self.eps = eps
        if self.affine:
            self.gamma = nn.Parameter(torch.Tensor(num_features).uniform_())
            self.beta = nn.Parameter(torch.zeros(num_features))

    def forward(self, x):
        shape = [-1] + [1] * (x.dim() - 1)
        if x.size(0) == 1:
            mean = x.reshape(-1).mean().view(*shape)
            std = x.reshape(-1).std().view(*shape)
        else:
            mean = x.reshape(x.size(0), -1).mean(1).view(*shape)
            std = x.reshape(x.size(0), -1).std(1).view(*shape)
        x = (x - mean) / (std + self.eps)
        if self.affine:
            shape = [1, -1] + [1] * (x.dim() - 2)
            x = x * self.gamma.view(*shape) + self.beta.view(*shape)
        return x


def get_activation_norm_layer(num_features, norm_type, input_dim, **norm_params):
    """Activation-norm factory (activation_norm.py:377-432)."""
    input_dim = max(input_dim, 1)
    if norm_type == 'none' or norm_type == '':
        return None
    if norm_type == 'batch':
        if input_dim == 3:
            return nn.BatchNorm3d(num_features, **norm_params)
        return BatchNorm2d(num_features, **norm_params)
    if norm_type == 'instance':
        affine = norm_params.pop('affine', True)
        if input_dim == 3:
            return nn.InstanceNorm3d(num_features, affine=affine, **norm_params)
        return InstanceNorm2d(num_features, affine=affine, **norm_params)
    if norm_type == 'sync_batch':
        affine = norm_params.pop('affine', True)
        layer = SyncBatchNorm(num_features, affine=True, **norm_params)
        layer.weight.requires_grad = affine
        layer.bias.requires_grad = affine
        return layer
    if norm_type == 'layer':
        return nn.LayerNorm(num_features, **norm_params)
    if norm_type == 'layer_2d':
        return LayerNorm2d(num_features, **norm_params)
    if norm_type == 'group':
        return nn.GroupNorm(num_channels=num_features, **norm_params)
    if norm_type == 'adaptive':
        return AdaptiveNorm(num_features, **norm_params)
    if norm_type == 'spatially_adaptive':
        if input_dim != 2:
            raise ValueError('Spatially adaptive normalization layers only supports 2D input')
        return SpatiallyAdaptiveNorm(num_features, **norm_params)
    if norm_type == 'hyper_spatially_adaptive':
        if input_dim != 2:
            raise ValueError('Spatially adaptive normalization layers only supports 2D input')
        return HyperSpatiallyAdaptiveNorm(num_features, **norm_params)
    raise ValueError('Activation norm layer %s is not recognized' % norm_type)
