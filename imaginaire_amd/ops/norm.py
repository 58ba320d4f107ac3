"""Fused normalisation + (spatially) adaptive modulation + activation (k1).

One op serves every normalisation the reference builds in its blocks:

* ``SpatiallyAdaptiveNorm`` (SPADE; reference layers/activation_norm.py:109-234)
  ``out = act((norm(x)·a + b)·(1 + γ) + β)`` with γ, β ∈ [N, C, H, W];
* ``AdaptiveNorm`` (AdaIN / CBN; activation_norm.py:22-106) — same with γ, β
  ∈ [N, C] broadcast over pixels;
* plain batch / sync-batch / instance norm followed by the block's activation.

``mode`` is ``'batch'``, ``'sync_batch'``, ``'instance'`` or ``'none'``; the
activation is a leaky slope (1.0 = identity, 0.0 = relu, 0.2 = the reference's
``leakyrelu``). On GPU tensors the HIP kernels of ``csrc/spade_norm.hip`` run
(stats → finalize → apply; backward reduce → apply); on CPU the PyTorch
reference below runs. SyncBN exchanges per-rank (count, mean, var) with one
all-gather in forward and Σg, Σg·x̂ with one all-reduce in backward.
"""
import os

import torch
import torch.distributed as dist
import torch.nn.functional as F

from imaginaire_amd.ops import _ext


def _world(group):
    if not (dist.is_available() and dist.is_initialized()):
        return 1
    return dist.get_world_size(group)


def sync_active(group):
    """True when sync-BN exchanges statistics: more than one rank, or a process group of ANY
    size with ``IMAGINAIRE_AMD_FORCE_DIST=1`` (exercises the collective path — including
    under hipGraph capture — on a one-GPU RCCL world, tests/test_graph_gpu.py)."""
    if not (dist.is_available() and dist.is_initialized()):
        return False
    return dist.get_world_size(group) > 1 or os.environ.get('IMAGINAIRE_AMD_FORCE_DIST') == '1'


def _native(group):
    if not x_is_hip_group(group):
        return None
    from imaginaire_amd.parallel.rccl import native_comm_for
    return native_comm_for(group)


def x_is_hip_group(group):
    return dist.is_available() and dist.is_initialized() and dist.get_backend(group) == 'nccl'


def _all_reduce_sums(s, group, async_op=False):
    """Σ over ranks of the sync-BN gradient sums (native RCCL when enabled: capturable)."""
    nc = _native(group)
    if nc is not None:
        return nc.all_reduce(s, async_op=async_op)
    return dist.all_reduce(s, group=group, async_op=async_op)


def _gather_rows(allst, stacked, group, async_op=False):
    """``allst[r] = stacked`` of rank r. RCCL: ONE flat all-gather (native communicator when
    enabled, else all_gather_into_tensor); gloo (CPU tests) has no flat all-gather: list form
    plus a copy after the wait."""
    nc = _native(group)
    if nc is not None:
        return nc.all_gather(allst, stacked, async_op=async_op)
    if dist.get_backend(group) != 'gloo':
        return dist.all_gather_into_tensor(allst, stacked, group=group, async_op=async_op)
    bufs = list(allst.unbind(0))
    return dist.all_gather(bufs, stacked, group=group, async_op=async_op)


def _stats_rows(cnt, mean, var):
    """(count, mean, var) as one contiguous [3, C] tensor: the [3, 1, C] buffer norm_stats
    writes them into when they are its rows, else a stacked copy."""
    base = cnt._base
    if base is not None and base.dim() == 3 and base.shape[0] == 3 and base.shape[1] == 1 and \
            base.is_contiguous() and cnt.data_ptr() == base.data_ptr() and \
            mean.data_ptr() == base[1].data_ptr() and var.data_ptr() == base[2].data_ptr():
        return base.view(3, -1)
    return torch.stack([cnt.reshape(-1), mean.reshape(-1), var.reshape(-1)], 0).contiguous()


def _gather_local(cnt, mean, var, group):
    """This rank's (count, mean, var) [1, C] rows all-gathered into [W, 3, C] (one collective)."""
    stacked = _stats_rows(cnt, mean, var)
    allst = stacked.new_empty((_world(group),) + tuple(stacked.shape))
    _gather_rows(allst, stacked, group)
    return allst


def _merge_stats(cnt, mean, var, group):
    """All-gather per-rank (count, mean, var) [1, C] and merge (Chan)."""
    stacked = torch.stack([cnt.reshape(-1), mean.reshape(-1), var.reshape(-1)], 0).contiguous()
    world = _world(group)
    # one flat output tensor (not a list): a single collective, safe under hipGraph capture
    allst = stacked.new_empty((world,) + tuple(stacked.shape))
    _gather_rows(allst, stacked, group)  # [W, 3, C]
    n_i, m_i, v_i = allst[:, 0], allst[:, 1], allst[:, 2]
    n = n_i.sum(0)
    mean_g = (n_i * m_i).sum(0) / n.clamp_min(1)
    m2 = (n_i * (v_i + (m_i - mean_g) ** 2)).sum(0)
    var_g = m2 / n.clamp_min(1)
    return n.reshape(1, -1), mean_g.reshape(1, -1), var_g.reshape(1, -1)


# ---- per-tensor batch-statistics cache ---------------------------------------------------
# In a SPADE residual block norm_0 and norm_s normalise the SAME tensor with the same
# (param-free) settings: the second layer reuses the first one's statistics — for sync-BN that
# is one cross-rank exchange per block input instead of two. The cache lives on the tensor
# (freed with it) and is keyed by its version counter, eps and the process group. For sync-BN
# the exchange can also be started early (prefetch_sync_stats: launched before the SPADE γ|β
# convolutions, which do not depend on it, and joined when the norm applies).

def _stats_key(x, eps, group, sync):
    return (x._version, float(eps), id(group), bool(sync))


def _cached_stats(x, key):
    c = getattr(x, '_iamd_bn_stats', None)
    if c is None or c[0] != key:
        return None
    if c[1] == 'pending':
        work, allst, local = c[2], c[3], c[4]
        work.wait()
        if allst.is_cuda and _ext.available():
            # (count, mean, var, rstd, scale, shift) of the param-free norm in one launch
            stats = tuple(_ext.ext().sync_stats_merge(allst, key[1]))
        else:
            stats = _merge_gathered(allst, local)
        x._iamd_bn_stats = (key, 'done', stats)
        return stats
    return c[2]


def _merge_gathered(allst, local=None):
    """Chan merge of the gathered per-rank (count, mean, var) rows ``allst`` [W, 3, C]."""
    n_i, m_i, v_i = allst[:, 0], allst[:, 1], allst[:, 2]
    n = n_i.sum(0)
    mean_g = (n_i * m_i).sum(0) / n.clamp_min(1)
    m2 = (n_i * (v_i + (m_i - mean_g) ** 2)).sum(0)
    var_g = m2 / n.clamp_min(1)
    return n.reshape(1, -1), mean_g.reshape(1, -1), var_g.reshape(1, -1)


def prefetch_sync_stats(x, eps, group):
    """Compute this rank's batch statistics of ``x`` and START their all-gather (async); the
    sync-BN forward that later normalises ``x`` joins it. No-op unless the HIP path runs with
    more than one rank."""
    if not (_ext.use_native(x) and sync_active(group) and x.dim() == 4):
        return
    key = _stats_key(x, eps, group, True)
    if getattr(x, '_iamd_bn_stats', (None,))[0] == key:
        return
    count, mean, var = _ext.ext().norm_stats(x, False, eps, None, None, True)[:3]
    stacked = _stats_rows(count, mean, var)
    allst = stacked.new_empty((_world(group),) + tuple(stacked.shape))
    work = _gather_rows(allst, stacked, group, async_op=True)
    x._iamd_bn_stats = (key, 'pending', work, allst, stacked)


def _native_running(running_mean, running_var, cfg):
    """The running statistics can be updated by the k1 finalize kernel (fp32, contiguous)."""
    if running_mean is None:
        return cfg.num_batches is None or cfg.num_batches.dtype == torch.int64
    return (running_var is not None and running_mean.dtype == torch.float32 and
            running_var.dtype == torch.float32 and running_mean.is_contiguous() and
            running_var.is_contiguous() and
            (cfg.num_batches is None or cfg.num_batches.dtype == torch.int64))


def _update_running(running_mean, running_var, mean, var, count, factor):
    if running_mean is None:
        return
    with torch.no_grad():
        n = count.reshape(-1)
        unbiased = var.reshape(-1) * n / (n - 1).clamp_min(1)
        running_mean.mul_(1 - factor).add_(mean.reshape(-1).to(running_mean.dtype), alpha=factor)
        running_var.mul_(1 - factor).add_(unbiased.to(running_var.dtype), alpha=factor)


def _expand_mod(t, x):
    """[N, C] → stride-0 [N, C, H, W] view (dtype converted BEFORE expanding so
    the pixel stride stays 0 and the kernel sees a broadcast modulation)."""
    if t is None:
        return None
    if t.dtype != x.dtype:
        t = t.to(x.dtype)
    if t.dim() == 2:
        return t.contiguous()[:, :, None, None].expand(-1, -1, x.shape[2], x.shape[3])
    return t


class _NormCfg:
    __slots__ = ('mode', 'training', 'momentum', 'eps', 'slope', 'group', 'use_batch_stats',
                 'deferred', 'num_batches')

    def __init__(self, mode, training, momentum, eps, slope, group, deferred=None,
                 num_batches=None):
        self.num_batches = num_batches
        self.mode = mode
        self.training = training
        self.momentum = momentum
        self.eps = eps
        self.slope = slope
        self.group = group
        self.use_batch_stats = mode == 'instance' or (mode in ('batch', 'sync_batch') and training)
        self.deferred = deferred


# ---- asynchronous sync-BN backward -------------------------------------------------------
# The data gradient of a sync-BN layer needs the GLOBAL Σg and Σg·x̂; the γ|β gradient and the
# γ|β / mlp convolution backward do not. The norm's backward therefore starts the all-reduce
# of its local sums (async) and hands the rest of the data-gradient computation to a join node
# inserted on the norm's input BEFORE the γ|β convolutions in the forward
# (:func:`defer_sync_bwd`): autograd runs nodes in decreasing creation order, so the γ|β and
# mlp convolution backward run between the launch and the join, while the sums ride xGMI.

class DeferredSyncBwd(object):
    """Hand-off between a sync-BN norm's backward and its join node."""
    __slots__ = ('args', 'work', 'sums')
    completed = 0  # joins that finished a deferred data gradient (tests / diagnostics)

    def __init__(self):
        self.args = None
        self.work = None
        self.sums = None


class _SyncBwdJoin(torch.autograd.Function):
    """Identity on the norm input; its backward finishes the data gradient that the norm's
    backward deferred (waits for the all-reduce, then one ``norm_bwd_apply`` pass)."""

    @staticmethod
    def forward(ctx, x, holder):
        ctx.holder = holder
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        h = ctx.holder
        if h.args is None:  # the norm computed dx itself (no deferral happened)
            return g, None
        h.work.wait()
        x, dout, scale, shift, mean, rstd, k1, M, gamma_v, beta_v, slope = h.args
        k = h.sums / M
        k2, k3 = k[0:1], k[1:2]
        h.args = h.work = h.sums = None
        DeferredSyncBwd.completed += 1
        dx = _ext.ext().norm_bwd_apply(x, dout, scale, shift, mean, rstd, k1, k2, k3,
                                       gamma_v, beta_v, slope)
        # g is the norm's stride-0 zero placeholder plus whatever other consumers of x' sent
        # back: add it unless it is exactly that placeholder (no extra pass in the usual case)
        if g is not None and not (g.dim() == dx.dim() and all(st == 0 for st in g.stride())):
            dx = dx + g
        return dx, None


def defer_sync_bwd(x):
    """``(x', holder)``: x' is x behind a join node whose backward completes the sync-BN data
    gradient of the norm that consumes x' with ``deferred=holder``. Call it before building the
    norm's γ|β branch. Inactive (returns ``(x, None)``) off the HIP path or at one rank."""
    if not (_ext.use_native(x) and x.requires_grad and torch.is_grad_enabled() and
            x.dim() == 4):
        return x, None
    holder = DeferredSyncBwd()
    x1 = _SyncBwdJoin.apply(x, holder)
    st = getattr(x, '_iamd_bn_stats', None)
    if st is not None:  # the prefetched statistics exchange belongs to the same values
        x1._iamd_bn_stats = st
    return x1, holder


class _FusedNormActFn(torch.autograd.Function):
    """HIP path. ``gb`` (combined [N, 2C, H, W] γ|β tensor) or (γ, β)."""

    @staticmethod
    def forward(ctx, x, weight, bias, gamma, beta, gb, running_mean, running_var, cfg):
        C = x.shape[1]
        ext = _ext.ext()
        if gb is not None:
            gamma_v, beta_v = gb[:, :C], gb[:, C:]
        else:
            gamma_v, beta_v = _expand_mod(gamma, x), _expand_mod(beta, x)
        wf = weight.float() if weight is not None else None
        bf = bias.float() if bias is not None else None
        per_instance = cfg.mode == 'instance'
        updated = False
        if cfg.mode == 'none':
            mean = x.new_zeros((1, C), dtype=torch.float32)
            var = x.new_ones((1, C), dtype=torch.float32)
            rstd = torch.ones_like(var)
            scale = wf.reshape(1, C).contiguous() if wf is not None else torch.ones_like(var)
            shift = bf.reshape(1, C).contiguous() if bf is not None else torch.zeros_like(var)
            count = None
        elif cfg.use_batch_stats:
            sync = cfg.mode == 'sync_batch' and sync_active(cfg.group)
            shareable = not per_instance and wf is None and bf is None
            key = _stats_key(x, cfg.eps, cfg.group, sync)
            cached = _cached_stats(x, key) if shareable else None
            if cached is not None and len(cached) == 6:  # a previous layer's full result
                count, mean, var, rstd, scale, shift = cached
            else:
                if cached is not None:  # merged statistics of a prefetched exchange
                    count, mean, var = cached
                    scale = rstd = None
                else:
                    # without a cross-rank merge the finalize kernel also updates the running
                    # statistics and the batch counter in place
                    fold = (not sync and cfg.training and not per_instance and
                            _native_running(running_mean, running_var, cfg))
                    count, mean, var, scale, shift, rstd = ext.norm_stats(
                        x, per_instance, cfg.eps, wf, bf, sync,
                        running_mean if fold else None, running_var if fold else None,
                        cfg.num_batches if fold else None, float(cfg.momentum))
                    if fold:
                        updated = True
                    if sync:
                        # one gather, then ONE kernel: merge + rsqrt + scale / shift + running
                        # statistics and batch counter (ops that were ~25 PyTorch launches)
                        fold_r = cfg.training and not per_instance and \
                            _native_running(running_mean, running_var, cfg)
                        allst = _gather_local(count, mean, var, cfg.group)
                        count, mean, var, rstd, scale, shift = ext.sync_stats_merge(
                            allst, cfg.eps, wf, bf, running_mean if fold_r else None,
                            running_var if fold_r else None,
                            cfg.num_batches if fold_r else None, float(cfg.momentum))
                        updated = fold_r
                if rstd is None:
                    rstd = torch.rsqrt(var + cfg.eps)
                if scale is None:
                    a = wf.reshape(1, C) if wf is not None else 1.0
                    b = bf.reshape(1, C) if bf is not None else 0.0
                    scale = (rstd * a).contiguous()
                    shift = (b - mean * scale).contiguous()
                if shareable:
                    x._iamd_bn_stats = (key, 'done', (count, mean, var, rstd, scale, shift))
            if cfg.training and not per_instance and not updated:
                _update_running(running_mean, running_var, mean, var, count, cfg.momentum)
        else:  # eval with running statistics
            mean = running_mean.float().reshape(1, C)
            var = running_var.float().reshape(1, C)
            rstd = torch.rsqrt(var + cfg.eps)
            a = wf.reshape(1, C) if wf is not None else 1.0
            b = bf.reshape(1, C) if bf is not None else 0.0
            scale = (rstd * a).contiguous()
            shift = (b - mean * scale).contiguous()
            count = None
        if cfg.num_batches is not None and not updated:
            cfg.num_batches.add_(1)
        out = ext.norm_apply(x, scale, shift, gamma_v, beta_v, cfg.slope)
        ctx.cfg = cfg
        ctx.has_gb = gb is not None
        ctx.has_mod = gamma_v is not None
        ctx.mod_bcast = gb is None and gamma is not None and gamma.dim() == 2
        ctx.mod_dtypes = (gamma.dtype if gamma is not None else None,
                          beta.dtype if beta is not None else None)
        ctx.count = count
        ctx.save_for_backward(x, weight, gamma, beta, gb, scale, shift, mean, rstd)
        return out

    @staticmethod
    def backward(ctx, dout):
        x, weight, gamma, beta, gb, scale, shift, mean, rstd = ctx.saved_tensors
        cfg = ctx.cfg
        ext = _ext.ext()
        C = x.shape[1]
        fmt = torch.channels_last if (x.is_contiguous(memory_format=torch.channels_last)
                                      and not x.is_contiguous()) else torch.contiguous_format
        dout = dout.contiguous(memory_format=fmt)
        if dout.dtype != x.dtype:
            dout = dout.to(x.dtype)
        dgb = dgamma = dbeta = None
        if ctx.has_gb:
            gamma_v, beta_v = gb[:, :C], gb[:, C:]
            dgb = torch.empty_like(gb)
            dgam_v, dbet_v = dgb[:, :C], dgb[:, C:]
        elif ctx.has_mod:
            gamma_v, beta_v = _expand_mod(gamma, x), _expand_mod(beta, x)
            if ctx.mod_bcast:
                dgam_v = dbet_v = None
            else:
                dgam_v = torch.empty_like(gamma_v, memory_format=fmt)
                dbet_v = torch.empty_like(beta_v, memory_format=fmt)
        else:
            gamma_v = beta_v = dgam_v = dbet_v = None
        sums = ext.norm_bwd_reduce(x, dout, scale, shift, mean, rstd, gamma_v, beta_v,
                                   dgam_v, dbet_v, cfg.slope)
        S1, S2 = sums[0], sums[1]
        if ctx.has_mod and ctx.mod_bcast:
            dgamma = sums[2].to(ctx.mod_dtypes[0])
            dbeta = sums[3].to(ctx.mod_dtypes[1])
        elif ctx.has_mod and not ctx.has_gb:
            dgamma = dgam_v.to(ctx.mod_dtypes[0])
            dbeta = dbet_v.to(ctx.mod_dtypes[1])
        N, HW = x.shape[0], x.shape[2] * x.shape[3]
        sync = cfg.mode == 'sync_batch' and sync_active(cfg.group)
        need_dw = weight is not None and ctx.needs_input_grad[1]
        need_db = ctx.needs_input_grad[2]
        if cfg.use_batch_stats and cfg.mode != 'none' and not sync and \
                S1.dtype == torch.float32 and S1.is_contiguous() and S2.is_contiguous():
            # one launch for k1 / k2 / k3 and the affine gradients
            inst = cfg.mode == 'instance'
            k1, k2, k3, dw32, db32 = ext.norm_bwd_coeffs(
                S1, S2, rstd.contiguous(), weight, inst, 1.0 / float(HW if inst else N * HW),
                need_dw, need_db)
            dweight = dw32.to(weight.dtype) if need_dw else None
            dbias = db32.to(weight.dtype if weight is not None else torch.float32) \
                if need_db else None
            dx = ext.norm_bwd_apply(x, dout, scale, shift, mean, rstd, k1, k2, k3, gamma_v,
                                    beta_v, cfg.slope) if ctx.needs_input_grad[0] else None
            return dx, dweight, dbias, dgamma, dbeta, dgb, None, None, None
        batch_sums = cfg.mode not in ('none', 'instance') and cfg.use_batch_stats
        s_loc = None
        if need_dw or need_db or batch_sums:
            # [2, C] = (Σ_N S1, Σ_N S2): one reduction feeds dbias, dweight and k2 / k3
            base = S1._base  # norm_bwd_reduce returns rows of one [Q, N, C] buffer
            both = base[:2] if (base is not None and base.dim() == 3 and
                                base[1].data_ptr() == S2.data_ptr()) else torch.stack([S1, S2], 0)
            s_loc = both.sum(1)
        dweight = s_loc[1].to(weight.dtype) if need_dw else None
        dbias = s_loc[0].to(weight.dtype if weight is not None else torch.float32) \
            if need_db else None
        if cfg.mode == 'none' or not cfg.use_batch_stats:
            # no batch statistics in the graph: dx = g * scale
            k1 = scale.contiguous()
            k2 = torch.zeros_like(k1)
            k3 = k2
        elif cfg.mode == 'instance':
            k1 = (rstd * (weight.float().reshape(1, C) if weight is not None else 1.0))
            k1 = k1.expand(N, C).contiguous()
            k2 = (S1 / HW).contiguous()
            k3 = (S2 / HW).contiguous()
        else:
            # (the exchange is in place: keep the local sums dweight / dbias may alias)
            s = s_loc.clone() if sync else s_loc
            M = ctx.count.reshape(1, C) if sync else float(N * HW)
            k1 = (rstd * (weight.float().reshape(1, C) if weight is not None else 1.0)).contiguous()
            h = cfg.deferred
            if sync and h is not None and ctx.needs_input_grad[0]:
                # start the exchange and let the join node finish dx after the γ|β backward
                h.work = _all_reduce_sums(s, cfg.group, async_op=True)
                h.sums = s
                h.args = (x, dout, scale, shift, mean, rstd, k1, M, gamma_v, beta_v, cfg.slope)
                dx = x.new_zeros(()).expand_as(x)  # placeholder: the join ignores it
                return dx, dweight, dbias, dgamma, dbeta, dgb, None, None, None
            if sync:
                _all_reduce_sums(s, cfg.group)
            k = s / M
            k2, k3 = k[0:1], k[1:2]
        mean_b, rstd_b = mean, rstd
        dx = ext.norm_bwd_apply(x, dout, scale, shift, mean_b, rstd_b, k1, k2, k3,
                                gamma_v, beta_v, cfg.slope) if ctx.needs_input_grad[0] else None
        return dx, dweight, dbias, dgamma, dbeta, dgb, None, None, None


def _reference(x, mode, weight, bias, gamma, beta, gb, running_mean, running_var, cfg):
    C = x.shape[1]
    if mode == 'none':
        y = x
        if weight is not None:
            y = y * weight.reshape(1, C, 1, 1) + bias.reshape(1, C, 1, 1)
    elif mode == 'instance':
        y = F.instance_norm(x, weight=weight, bias=bias, eps=cfg.eps)
    else:
        sync = mode == 'sync_batch' and sync_active(cfg.group)
        if cfg.training:
            xf = x.float()
            dims = (0, 2, 3)
            if sync:
                cnt = torch.full((1, C), float(x.shape[0] * x.shape[2] * x.shape[3]),
                                 device=x.device)
                mean_l = xf.mean(dims).reshape(1, C)
                var_l = xf.var(dims, unbiased=False).reshape(1, C)
                cnt_g, mean_g, var_g = _SyncStats.apply(cnt, mean_l, var_l, cfg.group)
            else:
                mean_g = xf.mean(dims).reshape(1, C)
                var_g = xf.var(dims, unbiased=False).reshape(1, C)
                cnt_g = torch.full((1, C), float(x.shape[0] * x.shape[2] * x.shape[3]),
                                   device=x.device)
            _update_running(running_mean, running_var, mean_g.detach(), var_g.detach(),
                            cnt_g.detach(), cfg.momentum)
            y = (xf - mean_g.reshape(1, C, 1, 1)) * torch.rsqrt(var_g.reshape(1, C, 1, 1) + cfg.eps)
            y = y.to(x.dtype)
        else:
            y = (x - running_mean.reshape(1, C, 1, 1)) * torch.rsqrt(
                running_var.reshape(1, C, 1, 1) + cfg.eps)
        if weight is not None:
            y = y * weight.reshape(1, C, 1, 1) + bias.reshape(1, C, 1, 1)
    if gb is not None:
        gamma, beta = gb[:, :C], gb[:, C:]
    if gamma is not None:
        if gamma.dim() == 2:
            gamma, beta = gamma[:, :, None, None], beta[:, :, None, None]
        y = y * (1 + gamma) + beta
    if cfg.slope != 1.0:
        y = F.leaky_relu(y, cfg.slope) if cfg.slope > 0 else F.relu(y)
    return y


class _SyncStats(torch.autograd.Function):
    """Differentiable cross-rank merge of (count, mean, var) for the CPU reference."""

    @staticmethod
    def forward(ctx, cnt, mean, var, group):
        ctx.group = group
        ctx.save_for_backward(cnt)
        n, m, v = _merge_stats(cnt, mean, var, group)
        ctx.mark_non_differentiable(n)
        ctx.local = (cnt, mean, var, n, m)
        return n, m, v

    @staticmethod
    def backward(ctx, dn, dmean_g, dvar_g):
        cnt, mean_l, var_l, n, mean_g = ctx.local
        # the global statistics feed every rank's loss: sum their gradients
        g = torch.stack([dmean_g.reshape(-1), dvar_g.reshape(-1)], 0).contiguous()
        dist.all_reduce(g, group=ctx.group)
        dmean_g, dvar_g = g[0].reshape(dmean_g.shape), g[1].reshape(dvar_g.shape)
        # d mean_g / d mean_l = cnt/n ; d var_g / d var_l = cnt/n ;
        # d var_g / d mean_l = 2 cnt (mean_l - mean_g) / n
        w = cnt / n
        dmean_l = dmean_g * w + dvar_g * 2 * w * (mean_l - mean_g)
        dvar_l = dvar_g * w
        return None, dmean_l, dvar_l, None


def fused_norm_act(x, mode='batch', weight=None, bias=None, gamma=None, beta=None, gb=None,
                   running_mean=None, running_var=None, training=True, momentum=0.1,
                   eps=1e-5, slope=1.0, process_group=None, deferred=None, num_batches=None):
    """``act((norm(x)·w + b)·(1+γ) + β)`` — see module docstring.

    ``momentum`` is the already-resolved exponential-average factor. ``num_batches`` (the
    layer's ``num_batches_tracked``) is incremented when the running statistics are updated.
    ``gb`` is an alternative to (γ, β): one [N, 2C, H, W] tensor whose first C
    channels are γ and last C are β (output of a fused γ|β convolution).
    """
    if mode == 'sync_batch' and not training:
        mode_eff = 'batch'
    else:
        mode_eff = mode
    cfg = _NormCfg(mode_eff, training, momentum, eps, slope, process_group, deferred,
                   num_batches)
    if gamma is not None and gamma.dim() == 2 and x.shape[2] * x.shape[3] == 1:
        gamma = gamma.reshape(x.shape[0], x.shape[1], 1, 1)
        beta = beta.reshape(x.shape[0], x.shape[1], 1, 1)
    if _ext.use_native(x):
        fmt = torch.channels_last if x.is_contiguous(memory_format=torch.channels_last) \
            else torch.contiguous_format
        if not x.is_contiguous(memory_format=fmt):
            x = x.contiguous()
        if gb is not None and gb.dtype != x.dtype:
            gb = gb.to(x.dtype)
        if gb is not None and not gb.is_contiguous(memory_format=fmt):
            gb = gb.contiguous(memory_format=fmt)
        if gamma is not None and gamma.dim() == 4 and not gamma.is_contiguous(memory_format=fmt):
            gamma = gamma.contiguous(memory_format=fmt)
            beta = beta.contiguous(memory_format=fmt)
        return _FusedNormActFn.apply(x, weight, bias, gamma, beta, gb, running_mean,
                                     running_var, cfg)
    if num_batches is not None:
        num_batches.add_(1)
    return _reference(x, mode_eff, weight, bias, gamma, beta, gb, running_mean, running_var, cfg)
