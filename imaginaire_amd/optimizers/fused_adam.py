"""Multi-tensor fused Adam / AdamW (k4, ``csrc/multi_tensor.hip``).

Replaces apex ``FusedAdam`` (reference utils/trainer.py:16, 271-281): one HIP
launch updates every parameter of a param group (fp32 master weights, fp32 or
bf16 gradients). Gradients are consumed as they are (no unscale pass: bf16
autocast needs no loss scaler). On CPU the update runs through
``torch._foreach_*`` with identical math.

State layout follows apex ``FusedAdam``: the step count lives in the param GROUP
(``group['step']``, one bias correction per group, advanced once per ``step()``
call that updates anything) and each parameter keeps only ``exp_avg`` /
``exp_avg_sq`` — so reference (apex) optimizer checkpoints load and resume
unchanged. States written by torch ``Adam`` (per-parameter ``'step'``) are
accepted too: the group step is taken from them when the group has none.
"""
import math
import weakref

import torch
from torch.optim import Optimizer

from imaginaire_amd.ops import _ext

# A parameter may carry a bf16 copy that the native step keeps in sync with it (the
# spectral-norm group's shadow weights, layers/spectral_norm.py), written in the same pass as the
# update. Stored as attributes of the parameter itself (tensors hash by identity but compare
# elementwise, so they make poor weak-dictionary keys).


_SHADOWED = {}  # id(param) -> weakref(param): every parameter that has a shadow


def register_shadow(param, shadow):
    """Have every native step of the optimizer owning ``param`` also write ``bf16(param)`` into
    ``shadow`` (same shape and strides); ``None`` unregisters."""
    param._iamd_shadow = shadow
    param._iamd_shadow_sync = None
    if shadow is None:
        _SHADOWED.pop(id(param), None)
    else:
        _SHADOWED[id(param)] = weakref.ref(param)


@torch.no_grad()
def sync_shadows(params):
    """shadow <- bf16(param) for each of ``params`` (one multi-tensor copy) and mark them synced."""
    if not params:
        return
    torch._foreach_copy_([shadow_of(p) for p in params], list(params))
    for p in params:
        p._iamd_shadow_sync = p._version


@torch.no_grad()
def resync_shadows():
    """Rewrite the shadow of every parameter changed since its shadow was last synced (a loaded
    checkpoint, a restored snapshot, any in-place write outside the native step). Eager forwards
    notice such writes themselves (:func:`shadow_synced`); a replayed graph cannot — its
    spectral-norm kernels read the shadows unconditionally — so graph replays call this first
    (utils/cuda_graph.py). A few microseconds of host work when nothing changed."""
    stale = []
    for key, ref in list(_SHADOWED.items()):
        p = ref()
        if p is None:
            del _SHADOWED[key]
            continue
        v = getattr(p, '_iamd_shadow_sync', None)
        if shadow_of(p) is None or v is None or v == p._version:
            continue  # never synced (its first forward writes it) or still in sync
        stale.append(p)
    sync_shadows(stale)
    return len(stale)


def shadow_of(param):
    return getattr(param, '_iamd_shadow', None)


def mark_shadow_synced(param):
    """``shadow_of(param)`` was just written from ``param``."""
    param._iamd_shadow_sync = param._version


def shadow_synced(param):
    """The shadow holds bf16(param): written from it and the parameter untouched since, or
    changed only by native optimizer steps (which rewrite the shadow in the same pass and do not
    bump the version counter; every other in-place write does)."""
    v = getattr(param, '_iamd_shadow_sync', None)
    return v is not None and v == param._version and shadow_of(param) is not None


class FusedAdam(Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0,
                 adam_w_mode=False, amsgrad=False):
        if amsgrad:
            raise NotImplementedError('amsgrad is not supported by FusedAdam')
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay,
                        adam_w_mode=adam_w_mode)
        super().__init__(params, defaults)

    def zero_grad(self, set_to_none=True):
        super().zero_grad(set_to_none=set_to_none)

    # -- capturable (hipGraph) support ------------------------------------------------
    # On the native path every group carries a device tensor [lr, step, lr/bc1, 1/sqrt(bc2)]
    # that the k4 launch advances itself (one 1-thread kernel ahead of the update), so the
    # same step can be captured into a hipGraph and replayed: the bias corrections move on
    # with every replay. group['step'] stays the host mirror (checkpoint format).
    def _hyper(self, group, device, step_before):
        h = group.get('_hyper')
        if h is None or h.device != device:
            h = torch.tensor([float(group['lr']), float(step_before), 0.0, 0.0],
                             dtype=torch.float32, device=device)
            group['_hyper'] = h
            group['_hyper_lr'] = float(group['lr'])
        return h

    def sync_hyper(self):
        """Push a changed learning rate (LR scheduler) into the device hyper-parameters.
        Call outside any capture — e.g. before replaying a captured step."""
        for group in self.param_groups:
            h = group.get('_hyper')
            lr = float(group['lr'])
            if h is not None and group.get('_hyper_lr') != lr:
                h[0:1].fill_(lr)
                group['_hyper_lr'] = lr

    def advance_host_step(self, n=1):
        """Host mirror of ``n`` replayed steps (the device counter advanced in the graph)."""
        for group in self.param_groups:
            if '_hyper' in group:
                group['step'] += n

    def state_dict(self):
        sd = super().state_dict()
        for g in sd['param_groups']:
            g.pop('_hyper', None)
            g.pop('_hyper_lr', None)
        return sd

    def load_state_dict(self, state_dict):
        hypers = [g.get('_hyper') for g in self.param_groups]
        super().load_state_dict(state_dict)
        for g, h in zip(self.param_groups, hypers):
            # refresh the device counters IN PLACE: a captured step keeps its pointer
            if h is not None:
                h.copy_(torch.tensor([float(g['lr']), float(g.get('step', 0)), 0.0, 0.0]))
                g['_hyper'] = h
                g['_hyper_lr'] = float(g['lr'])
            else:
                g.pop('_hyper', None)
                g.pop('_hyper_lr', None)

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        for group in self.param_groups:
            params, grads, m, v = [], [], [], []
            for p in group['params']:
                if p.grad is None:
                    continue
                if p.grad.is_sparse:
                    raise RuntimeError('FusedAdam does not support sparse gradients')
                state = self.state[p]
                if 'exp_avg' not in state:
                    state['exp_avg'] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    state['exp_avg_sq'] = torch.zeros_like(p, memory_format=torch.preserve_format)
                params.append(p)
                grads.append(p.grad)
                m.append(state['exp_avg'])
                v.append(state['exp_avg_sq'])
            if not params:
                continue
            if 'step' not in group:
                # torch-Adam-style state (per-parameter step): adopt the largest
                prev = [self.state[p].get('step', 0) for p in group['params']
                        if p in self.state]
                group['step'] = int(max([float(s) for s in prev], default=0))
            group['step'] += 1
            step = group['step']
            beta1, beta2 = group['betas']
            lr, eps, wd = group['lr'], group['eps'], group['weight_decay']
            adamw = group['adam_w_mode']
            if isinstance(lr, torch.Tensor):
                lr = float(lr)
            native = _ext.use_native(params[0]) and all(
                p.dtype == torch.float32 and _ext.is_dense(p) for p in params)
            if native:
                # device counter created at the pre-increment step: the launch advances it
                hyper = self._hyper(group, params[0].device, step - 1)
                if not torch.cuda.is_current_stream_capturing() and \
                        group.get('_hyper_lr') != float(lr):
                    hyper[0:1].fill_(float(lr))
                    group['_hyper_lr'] = float(lr)
                gdt = grads[0].dtype
                if gdt not in (torch.float32, torch.bfloat16):
                    gdt = torch.float32
                # grads must walk memory in the same order as their params
                # (channels-last conv weights): re-lay out only mismatching ones
                gl = [g if (g.dtype == gdt and g.stride() == p.stride())
                      else torch.empty_like(p, dtype=gdt).copy_(g)
                      for g, p in zip(grads, params)]
                shadows = []
                sh = [shadow_of(p) for p in params]
                if any(t is not None for t in sh):
                    none = params[0].new_empty(0, dtype=torch.bfloat16)
                    shadows = [t if t is not None else none for t in sh]
                _ext.ext().mt_adam(params, gl, m, v, shadows, lr, beta1, beta2, eps, int(step),
                                   wd, bool(adamw), 1.0, hyper)
            else:
                _reference_adam(params, grads, m, v, lr, beta1, beta2, eps, step, wd, adamw)
        return loss


def _reference_adam(params, grads, m, v, lr, beta1, beta2, eps, step, wd, adamw):
    grads = [g.float() for g in grads]
    if wd != 0 and not adamw:
        grads = torch._foreach_add(grads, params, alpha=wd)
    torch._foreach_mul_(m, beta1)
    torch._foreach_add_(m, grads, alpha=1 - beta1)
    torch._foreach_mul_(v, beta2)
    torch._foreach_addcmul_(v, grads, grads, value=1 - beta2)
    bc1 = 1 - beta1 ** step
    bc2 = 1 - beta2 ** step
    denom = torch._foreach_sqrt(v)
    torch._foreach_div_(denom, math.sqrt(bc2))
    torch._foreach_add_(denom, eps)
    if wd != 0 and adamw:
        torch._foreach_mul_(params, 1 - lr * wd)
    torch._foreach_addcdiv_(params, m, denom, value=-lr / bc1)
