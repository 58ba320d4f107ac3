"""Exponential moving average of the generator (reference utils/model_average.py:13-197).

Same semantics: deep-copied averaged model, optional spectral-norm removal in
the copy (the SN-normalised weight ``W/σ`` is what gets averaged), ``beta = 0``
until ``start_iteration``, ``num_updates_tracked`` buffer, BN re-estimation
helpers. On MI355X the whole update is two multi-tensor HIP launches (k5):
``mt_sn_sigma`` computes every σ = uᵀWv at once, then ``mt_ema`` lerps every
tensor with the per-tensor 1/σ folded in — instead of the reference's Python
loop over the state dict (hundreds of small kernels per iteration).
"""
import copy

import torch
from torch import nn
from torch.nn.utils.spectral_norm import remove_spectral_norm

from imaginaire_amd.ops import _ext
from imaginaire_amd.utils.misc import requires_grad


def reset_batch_norm(m):
    if hasattr(m, 'reset_running_stats'):
        m.reset_running_stats()


def calibrate_batch_norm_momentum(m):
    if hasattr(m, 'reset_running_stats') and 'BatchNorm' in m._get_name():
        m.momentum = 1.0 / float(m.num_batches_tracked + 1)


def _drop_sn_load_hooks(m):
    """``remove_spectral_norm`` leaves SN's load-state-dict pre-hook behind on
    this PyTorch version, which then demands ``weight_orig`` keys; drop it."""
    from torch.nn.utils.spectral_norm import SpectralNormLoadStateDictPreHook
    for k, h in list(m._load_state_dict_pre_hooks.items()):
        inner = getattr(h, 'hook', h)
        if isinstance(inner, SpectralNormLoadStateDictPreHook):
            del m._load_state_dict_pre_hooks[k]


def _drop_sn_group_hooks(net):
    """The deep-copied EMA network has no SN layers left: drop the batched-SN
    pre-hooks it inherited from the source network (the network-level one and the
    re-call hooks of its sub-modules)."""
    from imaginaire_amd.layers.spectral_norm import _SNGroup
    for m in net.modules():
        for k, h in list(m._forward_pre_hooks.items()):
            if isinstance(h, _SNGroup):
                del m._forward_pre_hooks[k]


class ModelAverage(nn.Module):
    def __init__(self, module, beta=0.9999, start_iteration=1000, remove_sn=True):
        super().__init__()
        self.module = module
        self.averaged_model = copy.deepcopy(self.module)
        self.beta = beta
        self.remove_sn = remove_sn
        self.start_iteration = start_iteration
        # on the module's device: DDP broadcasts every buffer over RCCL at construction
        dev = next(module.parameters()).device if any(True for _ in module.parameters()) \
            else torch.device('cpu')
        self.register_buffer('num_updates_tracked',
                             torch.tensor(0, dtype=torch.long, device=dev))
        requires_grad(self.averaged_model, False)
        if self.remove_sn:
            self.copy_s2t()

            def fn_remove_sn(m):
                if hasattr(m, 'weight_orig'):
                    remove_spectral_norm(m)
                    _drop_sn_load_hooks(m)
            self.averaged_model.apply(fn_remove_sn)
            _drop_sn_group_hooks(self.averaged_model)
            self.dim = 0
        else:
            self.averaged_model.eval()
        self._plan = None
        self._host_updates = 0

    def forward(self, *inputs, **kwargs):
        return self.module(*inputs, **kwargs)

    def _build_plan(self):
        """Pair every target tensor with its source (and SN u, v if absorbed)."""
        src = self.module.state_dict(keep_vars=True)
        tgt = self.averaged_model.state_dict(keep_vars=True)
        sn_t, sn_w, sn_u, sn_v = [], [], [], []
        plain = {}  # dtype -> (targets, sources)
        ints_t, ints_s = [], []
        for key, t in tgt.items():
            if self.remove_sn and key.endswith('weight') and key + '_orig' in src:
                sn_t.append(t.data)
                sn_w.append(src[key + '_orig'].data)
                sn_u.append(src[key + '_u'].data)
                sn_v.append(src[key + '_v'].data)
            else:
                s = src[key]
                if not t.is_floating_point():
                    ints_t.append(t.data)
                    ints_s.append(s.data)
                    continue
                plain.setdefault(t.dtype, ([], []))
                plain[t.dtype][0].append(t.data)
                plain[t.dtype][1].append(s.data)
        self._plan = (sn_t, sn_w, sn_u, sn_v, plain)
        self._ints = (ints_t, ints_s)

    @torch.no_grad()
    def update_average(self):
        self.num_updates_tracked += 1
        self._host_updates += 1
        beta = 0. if self._host_updates <= self.start_iteration else self.beta
        if not self.remove_sn:
            is_training = self.training
            self.eval()
            params = dict(self.module.named_parameters())
            for name, p_tgt in self.averaged_model.named_parameters():
                p_tgt.copy_(beta * p_tgt + (1. - beta) * params[name])
            bufs = dict(self.module.named_buffers())
            for name, b_tgt in self.averaged_model.named_buffers():
                if b_tgt.is_floating_point():
                    b_tgt.copy_(beta * b_tgt + (1. - beta) * bufs[name])
                else:
                    b_tgt.copy_(bufs[name])
            if is_training:
                self.train()
            return
        if self._plan is None:
            self._build_plan()
        sn_t, sn_w, sn_u, sn_v, plain = self._plan
        native = len(sn_t) > 0 and _ext.use_native(sn_t[0]) or \
            (len(sn_t) == 0 and plain and _ext.use_native(next(iter(plain.values()))[0][0]))
        if native:
            ext = _ext.ext()
            # the warm-up switch (beta = 0 until start_iteration) is evaluated on the device
            # from num_updates_tracked, so a captured step replays it correctly
            cnt, start = self.num_updates_tracked, int(self.start_iteration)
            if sn_t:
                sigma = ext.mt_sn_sigma(sn_w, sn_u, sn_v)
                ext.mt_ema(sn_t, sn_w, self.beta, sigma, cnt, start)
            for dt, (ts, ss) in plain.items():
                ext.mt_ema(ts, ss, self.beta, None, cnt, start)
        else:
            for t, w, u, v in zip(sn_t, sn_w, sn_u, sn_v):
                t.copy_(t * beta + self.sn_compute_weight(w, u, v) * (1 - beta))
            for dt, (ts, ss) in plain.items():
                if beta == 0.:
                    torch._foreach_copy_(ts, ss)
                else:
                    torch._foreach_lerp_(ts, ss, 1 - beta)
        # integer buffers (num_batches_tracked) are copied verbatim
        if self._ints[0]:
            torch._foreach_copy_(self._ints[0], self._ints[1])

    def copy_t2s(self):
        # (state_dict tensors share their parameter's version counter: the in-place copy is
        # visible to version checks — e.g. the spectral-norm group's bf16 shadow weights)
        target_dict = self.module.state_dict()
        source_dict = self.averaged_model.state_dict()
        with torch.no_grad():
            for key in source_dict:
                target_dict[key].copy_(source_dict[key])

    def copy_s2t(self):
        source_dict = self.module.state_dict()
        target_dict = self.averaged_model.state_dict()
        with torch.no_grad():
            for key in source_dict:
                target_dict[key].copy_(source_dict[key])

    def __repr__(self):
        return self.module.__repr__()

    def sn_reshape_weight_to_matrix(self, weight):
        weight_mat = weight
        if self.dim != 0:
            weight_mat = weight_mat.permute(self.dim,
                                            *[d for d in range(weight_mat.dim()) if d != self.dim])
        return weight_mat.reshape(weight_mat.size(0), -1)

    def sn_compute_weight(self, weight, u, v):
        weight_mat = self.sn_reshape_weight_to_matrix(weight)
        sigma = torch.sum(u * torch.mv(weight_mat, v))
        return weight / sigma

    def _load_from_state_dict(self, state_dict, prefix, *args, **kwargs):
        super()._load_from_state_dict(state_dict, prefix, *args, **kwargs)
        key = prefix + 'num_updates_tracked'
        if key in state_dict:
            self._host_updates = int(state_dict[key])
        self._plan = None
