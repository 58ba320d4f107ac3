"""Spectral normalisation, MI355X execution (reference layers/weight_norm.py:84-85,
which wraps ``torch.nn.utils.spectral_norm``).

Same parametrisation and state-dict layout as PyTorch's ``spectral_norm``
(``weight_orig`` / ``weight_u`` / ``weight_v``, the same hooks), so
checkpoints interchange with the reference. Two changes in how it runs:

* **fp32, outside autocast.** Under bf16 autocast PyTorch's power iteration
  runs its GEMVs in bf16 through hipBLASLt (with a host-side heuristic query
  per call) — numerically worse and measured as the dominant host cost of a
  SPADE forward on MI355X (profiles/spade_step_phases_mi355x.txt).
* **Batched per network.** ``install_batched_spectral_norm(net)`` registers a
  forward pre-hook on the network that runs ONE power iteration for every SN
  layer of the network with the k5b HIP kernels (``mt_sn_power``: 4 launches
  in total instead of ~10 per layer) and hands each layer its σ; the layer
  then forms ``W / σ`` with an autograd function whose backward is exactly
  the gradient of PyTorch's ``W / (uᵀ W v)`` (u, v constant). Under bf16
  autocast the bf16 ``W / σ`` of every layer is written by one k5c launch
  (``mt_sn_scale_cast``) into a single flat buffer. A layer called
  again within the same network forward (weight sharing) falls back to its
  own power iteration — again the reference's behaviour.
"""
import os

import torch
from torch.nn.utils.spectral_norm import (SpectralNorm as _TorchSN,
                                          SpectralNormLoadStateDictPreHook,
                                          SpectralNormStateDictHook)
import torch.nn.functional as F

from imaginaire_amd.ops import _ext

# IMAGINAIRE_AMD_SN_FLIP=0: each conv flips its own weight for the data gradient
_SN_FLIP = os.environ.get('IMAGINAIRE_AMD_SN_FLIP', '1') == '1'
# IMAGINAIRE_AMD_SN_SHADOW=0: the power iteration and the W / sigma cast read the fp32 weights
# (default: a bf16 copy of each weight that the optimizer step writes in its own pass)
_SN_SHADOW = os.environ.get('IMAGINAIRE_AMD_SN_SHADOW', '1') == '1'
# IMAGINAIRE_AMD_SN_FUSED=0: every SN conv gets a materialised bf16(W / sigma) (the k5c cast)
# and the separate <G, W> / apply backward passes. Default (with shadows): a plain SN conv that
# runs on k10 / k11 takes its bf16 shadow directly, 1 / sigma rides in the conv epilogues
# (forward and data gradient) and the SN backward in the weight gradient's split-K sum
# (ops/conv.py _MfmaConv2d with an SNWeight): no W / sigma copy, no bf16 G round trip, no per-layer SN
# backward launches.
_SN_FUSED = os.environ.get('IMAGINAIRE_AMD_SN_FUSED', '1') == '1'


class _SNScale(torch.autograd.Function):
    """W / σ with σ = uᵀ W v (u, v constants): dW = G/σ − (⟨G, W⟩/σ²) u vᵀ."""

    @staticmethod
    def forward(ctx, weight, u, v, sigma):
        ctx.save_for_backward(weight, u, v, sigma)
        ctx.wparam = weight if isinstance(weight, torch.nn.Parameter) else None
        return weight / sigma

    @staticmethod
    def backward(ctx, grad):
        weight, u, v, sigma = ctx.saved_tensors
        if _ext.use_native(weight) and weight.dtype == torch.float32 and \
                grad.dtype in (torch.float32, torch.bfloat16):
            # <G, W> reads the bf16 shadow of W when the forward had one (half the bytes); dW
            # goes straight into the parameter's DDP bucket slice when one is armed
            from imaginaire_amd.ops.conv import _take_grad_dest
            dest = _take_grad_dest(getattr(ctx, 'wparam', None), tuple(weight.shape))
            return _ext.ext().sn_scale_backward(grad, weight, u, v, sigma,
                                                getattr(ctx, 'shadow', None), dest), \
                None, None, None
        g = grad.float()
        dot = (g * weight).sum()
        outer = torch.outer(u, v).view(weight.shape)
        dw = g / sigma - (dot / (sigma * sigma)) * outer
        return dw.to(weight.dtype), None, None, None


class _SNScaleCast(torch.autograd.Function):
    """As :class:`_SNScale`, but the forward value — ``bf16(W / σ)`` — was already
    produced for every layer at once by the k5c kernel (``mt_sn_scale_cast``),
    so autocast's per-layer divide + cast disappear from the forward."""

    @staticmethod
    def forward(ctx, weight, u, v, sigma, w16, shadow=None):
        ctx.save_for_backward(weight, u, v, sigma)
        ctx.shadow = shadow  # bf16(W) (the optimizer keeps it in sync), or None
        ctx.wparam = weight if isinstance(weight, torch.nn.Parameter) else None
        return w16

    @staticmethod
    def backward(ctx, grad):
        return _SNScale.backward(ctx, grad) + (None, None)


def w_shape(w):
    return tuple(w.shape)


def materialize_scaled(weight, sigma, shadow):
    """bf16(W / sigma) of ONE layer from its shadow (the fused group left it unmaterialised
    and a consumer needs the tensor: a linear layer, the tap-split head, an eager MIOpen conv)."""
    with torch.no_grad():
        return _ext.ext().mt_sn_scale_cast([weight], sigma.reshape(1), [shadow], 1)[0]


def _autocast_bf16(dev):
    return torch.is_autocast_enabled(dev) and torch.get_autocast_dtype(dev) == torch.bfloat16


class SpectralNorm(_TorchSN):
    def weight_ref(self, module):
        """The pending batched iteration's result as an ``ops.conv.SNWeight`` (unmaterialised
        W / sigma) for a plain conv whose group left it to the fused conv path; else None."""
        batched = getattr(self, '_batched', None)
        if batched is None or batched[3] is not None or batched[4] is None or \
                type(module) is not torch.nn.Conv2d or module.groups != 1 or \
                not _autocast_bf16(batched[4].device.type):
            return None
        self._batched = None
        from imaginaire_amd.ops.conv import SNWeight
        u, v, sigma, _, shadow = batched
        return SNWeight(getattr(module, self.name + '_orig'), shadow, u, v, sigma, self, module)

    def compute_weight(self, module, do_power_iteration):
        batched = getattr(self, '_batched', None)
        if batched is not None:
            self._batched = None  # consumed: a second call this forward iterates itself
            weight = getattr(module, self.name + '_orig')
            u, v, sigma, w16, shadow = batched
            if w16 is None and shadow is not None and _autocast_bf16(weight.device.type):
                w16 = materialize_scaled(weight, sigma, shadow)
            if w16 is not None and _autocast_bf16(weight.device.type):
                return _SNScaleCast.apply(weight, u, v, sigma, w16, shadow)
            return _SNScale.apply(weight, u, v, sigma)
        dev = getattr(module, self.name + '_orig').device.type
        with torch.autocast(device_type=dev, enabled=False):
            return super().compute_weight(module, do_power_iteration)

    @classmethod
    def apply(cls, module, name, n_power_iterations, dim, eps):
        for hook in module._forward_pre_hooks.values():
            if isinstance(hook, _TorchSN) and hook.name == name:
                raise RuntimeError('Cannot register two spectral_norm hooks on the same '
                                   'parameter {}'.format(name))
        fn = cls(name, n_power_iterations, dim, eps)
        weight = module._parameters[name]
        with torch.no_grad():
            weight_mat = fn.reshape_weight_to_matrix(weight)
            h, w = weight_mat.size()
            u = F.normalize(weight.new_empty(h).normal_(0, 1), dim=0, eps=fn.eps)
            v = F.normalize(weight.new_empty(w).normal_(0, 1), dim=0, eps=fn.eps)
        delattr(module, fn.name)
        module.register_parameter(fn.name + '_orig', weight)
        setattr(module, fn.name, weight.data)
        module.register_buffer(fn.name + '_u', u)
        module.register_buffer(fn.name + '_v', v)
        module.register_forward_pre_hook(fn)
        module._register_state_dict_hook(SpectralNormStateDictHook(fn))
        module._register_load_state_dict_pre_hook(SpectralNormLoadStateDictPreHook(fn))
        return fn


def spectral_norm(module, name='weight', n_power_iterations=1, eps=1e-12, dim=None):
    """Drop-in for ``torch.nn.utils.spectral_norm`` using :class:`SpectralNorm`."""
    if dim is None:
        dim = 1 if isinstance(module, (torch.nn.ConvTranspose1d, torch.nn.ConvTranspose2d,
                                       torch.nn.ConvTranspose3d)) else 0
    SpectralNorm.apply(module, name, n_power_iterations, dim, eps)
    return module


class _SNGroup:
    """Forward pre-hook of a network: one batched power iteration for all of
    its (dim-0, single-iteration) SN layers.

    ``sub=True``: the hook of a sub-module of a grouped network (an encoder / decoder / block
    with >= 2 SN layers). It iterates its layers only when every one of them has already
    consumed the network-level iteration — i.e. on a SECOND call of the sub-module within one
    network forward (MUNIT / UNIT re-encode translated images; reference torch semantics: one
    power iteration per layer call) — instead of each layer falling back to its own per-layer
    iteration (~10 small PyTorch launches forward and ~6 backward per layer per call)."""

    def __init__(self, net, sub=False):
        self.sub = sub
        self.entries = self._collect(net)
        self._snap = None  # (u, v) before this network forward's first iteration

    def finish(self, net, inputs, output):
        """Forward hook of the network: a layer the forward did NOT call gets its u / v back
        (the reference iterates a layer only when it runs — e.g. vid2vid's previous-frame
        encoder, idle on the first frame), and no stale σ is left pending for a later call."""
        snap, self._snap = self._snap, None
        if snap is None:
            return
        idle = [i for i, (_, h) in enumerate(self.entries) if getattr(h, '_batched', None)
                is not None]
        if not idle:
            return
        su, sv = snap
        dst, src = [], []
        ou = ov = 0
        offs = []
        for m, h in self.entries:
            u, v = getattr(m, h.name + '_u'), getattr(m, h.name + '_v')
            offs.append((ou, ov, u, v))
            ou += u.numel()
            ov += v.numel()
        for i in idle:
            o_u, o_v, u, v = offs[i]
            dst += [u, v]
            src += [su[o_u:o_u + u.numel()], sv[o_v:o_v + v.numel()]]
            self.entries[i][1]._batched = None
        with torch.no_grad():
            torch._foreach_copy_(dst, src)

    @staticmethod
    def _collect(net):
        entries = []
        for m in net.modules():
            for hook in m._forward_pre_hooks.values():
                if isinstance(hook, SpectralNorm) and hook.dim == 0 and \
                        hook.n_power_iterations == 1:
                    entries.append((m, hook))
        return entries

    def __call__(self, net, inputs):
        ends = (self.entries[0], self.entries[-1]) if self.entries else ()
        if not all(hasattr(m, h.name + '_orig') for m, h in ends):
            self.entries = self._collect(net)  # SN removed/added since (e.g. EMA copy)
        if not self.entries:
            return
        if self.sub and any(getattr(h, '_batched', None) is not None for _, h in self.entries):
            return  # first call within this forward: the network-level iteration is pending
        w0 = getattr(self.entries[0][0], self.entries[0][1].name + '_orig')
        if not _ext.use_native(w0):
            return
        ws, us, vs = [], [], []
        for m, h in self.entries:
            ws.append(getattr(m, h.name + '_orig'))
            us.append(getattr(m, h.name + '_u'))
            vs.append(getattr(m, h.name + '_v'))
        if any(w.dtype != torch.float32 for w in ws):
            return
        X = _ext.ext()
        eps = float(self.entries[0][1].eps)
        bf16 = _autocast_bf16(w0.device.type)
        with torch.no_grad():
            if net.training and not self.sub and self._snap is None:
                self._snap = (torch.cat(us), torch.cat(vs))
            shadows = self._shadows(ws) if (bf16 and net.training and _SN_SHADOW) else None
            fused = False
            if shadows is not None:
                # the optimizer's step writes bf16(W) with the update: the GEMV passes and the
                # W / sigma cast read half the bytes. Stale shadows (first step, a loaded or
                # restored state) are refreshed first, so the result depends on W alone —
                # an eager step and a graph replay from the same state agree bitwise.
                self._sync_stale(ws)
                sigma = X.mt_sn_power(ws, us, vs, True, eps, shadows)
                if _SN_FUSED:
                    # only the layers that must hand a tensor on (the SPADE γ|β pairs, one conv
                    # over their concatenated weights) get bf16(W / sigma), back to back in one
                    # launch; the others stay unmaterialised for the fused conv path
                    fused = True
                    pre = self._pre_materialize()
                    w16 = [None] * len(ws)
                    if pre:
                        sub = X.mt_sn_scale_cast([ws[i] for i in pre],
                                                 sigma.index_select(0, self._pre_index(sigma)),
                                                 [shadows[i] for i in pre], 1)
                        for i, t in zip(pre, sub):
                            w16[i] = t
                else:
                    w16 = X.mt_sn_scale_cast(ws, sigma, shadows, 1)
            else:
                sigma = X.mt_sn_power(ws, us, vs, bool(net.training), eps)
                w16 = X.mt_sn_scale_cast(ws, sigma) if bf16 else [None] * len(ws)
            # snapshots of u, v for the backward (the next forward updates them in place)
            u_all = torch.cat(us)
            v_all = torch.cat(vs)
        if torch.is_grad_enabled() and net.training and _SN_FLIP:
            if fused:
                # the fused convs' data gradients run on the flipped SHADOW (1 / sigma in the
                # epilogue); the γ|β pairs flip their concatenated weight in the backward
                self._flip_for_dgrad([shadows[i] if w16[i] is None else None
                                      for i in range(len(ws))])
            elif w16[0] is not None:
                self._flip_for_dgrad(w16)
        ou = ov = 0
        for i, (m, h) in enumerate(self.entries):
            nu, nv = us[i].numel(), vs[i].numel()
            h._batched = (u_all[ou:ou + nu], v_all[ov:ov + nv], sigma[i], w16[i],
                          shadows[i] if shadows is not None else None)
            ou += nu
            ov += nv

    def _pre_materialize(self):
        """Entries whose module asks for a materialised bf16(W / sigma) (``_iamd_sn_
        materialize``: the SPADE γ / β convs), in entry order; cached per group."""
        pre = getattr(self, '_pre', None)
        if pre is None or len(pre[1]) != len(self.entries):
            # (and every non-Conv2d SN layer — linear / 1-D / 3-D / transposed: no fused path)
            idx = [i for i, (m, _) in enumerate(self.entries)
                   if getattr(m, '_iamd_sn_materialize', False) or type(m) is not torch.nn.Conv2d
                   or m.groups != 1]
            pre = self._pre = (idx, list(self.entries))
            self._pre_t = None
        return pre[0]

    def _pre_index(self, like):
        t = getattr(self, '_pre_t', None)
        if t is None or t.device != like.device:
            t = self._pre_t = torch.tensor(self._pre_materialize(), dtype=torch.long,
                                           device=like.device)
        return t

    def _shadows(self, ws):
        """bf16 copies of the group's weights, one per parameter and shared by every group that
        holds it (optimizers/fused_adam.py registry), each laid out like its weight; the missing
        ones are allocated together, outside graph capture. None when unavailable."""
        from imaginaire_amd.optimizers import fused_adam as FA
        out = [FA.shadow_of(w) for w in ws]
        missing = [i for i, t in enumerate(out)
                   if t is None or t.shape != w_shape(ws[i]) or t.stride() != ws[i].stride()]
        if missing:
            if torch.cuda.is_current_stream_capturing():
                return None
            offs, tot = [], 0
            for i in missing:
                offs.append(tot)
                tot += (ws[i].numel() + 7) // 8 * 8  # 16-byte aligned views
            flat = torch.empty(tot, dtype=torch.bfloat16, device=ws[0].device)
            for i, o in zip(missing, offs):
                out[i] = flat.as_strided(ws[i].shape, ws[i].stride(), o)
                FA.register_shadow(ws[i], out[i])
        return out

    @staticmethod
    def _sync_stale(ws):
        from imaginaire_amd.optimizers import fused_adam as FA
        FA.sync_shadows([w for w in ws if not FA.shadow_synced(w)])

    def _flip_for_dgrad(self, w16):
        """The flipped, transposed bf16 copies of every stride-1 conv weight of the group, for
        the backward's data gradients, in ONE launch right after the W / sigma launch
        (instead of one flip per conv in the backward: ~220 small launches per SPADE step)."""
        from imaginaire_amd.ops import conv as nhwc_conv
        sel = [i for i, (m, _) in enumerate(self.entries)
               if w16[i] is not None and
               type(m) is torch.nn.Conv2d and tuple(m.stride) == (1, 1) and
               tuple(m.dilation) == (1, 1) and m.groups == 1 and w16[i].dim() == 4 and
               w16[i].shape[0] % 64 == 0 and w16[i].shape[1] % 64 == 0 and
               w16[i].is_contiguous(memory_format=torch.channels_last)]
        if not sel:
            return
        ws = [w16[i] for i in sel]
        with torch.no_grad():
            flipped = _ext.ext().mt_conv_weight_flip_t(ws)
        self._flip_keys = nhwc_conv.register_dgrad_weights(ws, flipped,
                                                           getattr(self, '_flip_keys', ()))


def install_batched_spectral_norm(net):
    """Register the batched SN pre-hook on ``net`` (and the re-call hooks of its sub-modules
    holding >= 2 SN layers); returns the number of layers covered."""
    group = _SNGroup(net)
    if group.entries:
        net.register_forward_pre_hook(group)
        net.register_forward_hook(group.finish)
        net._iamd_sn_group = group
        for m in net.modules():
            if m is net or any(isinstance(h, _SNGroup) for h in m._forward_pre_hooks.values()):
                continue
            sub = _SNGroup(m, sub=True)
            if len(sub.entries) >= 2:
                m.register_forward_pre_hook(sub)
    return len(group.entries)


def refresh_batched_spectral_norm(net):
    """Run the batched power iteration of ``net`` again inside one forward — for a network
    that calls its layers twice in one forward with the reference refreshing σ in between (the
    SPADE discriminator's real then fake pass, reference discriminators/spade.py:91-117).
    Without it each layer's second call falls back to its own per-layer power iteration
    (~7 small kernels + an fp32 W/σ and a cast per layer)."""
    group = getattr(net, '_iamd_sn_group', None)
    if group is not None:
        group(net, ())


@torch.no_grad()
def extra_sn_power_iteration(net):
    """One more spectral-norm power iteration for every SN layer of ``net`` before its next
    layer calls — so that a forward that calls each layer ONCE leaves u / v where a forward
    that calls each layer TWICE (the reference SPADE discriminator's real then fake pass)
    leaves them. With the batched group installed it is one more k5b pass (the layers then
    consume the refreshed σ without iterating again); otherwise each layer's own iteration runs
    once here and once more in its next call."""
    group = getattr(net, '_iamd_sn_group', None)
    if group is not None and group.entries and net.training:
        w0 = getattr(group.entries[0][0], group.entries[0][1].name + '_orig')
        if _ext.use_native(w0):
            group(net, ())
            return
    if not net.training:
        return
    for m in net.modules():
        for hook in list(m._forward_pre_hooks.values()):
            if isinstance(hook, _TorchSN) and hasattr(m, hook.name + '_orig'):
                hook._batched = None
                _TorchSN.compute_weight(hook, m, do_power_iteration=True)
