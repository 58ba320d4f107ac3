"""The fused spectral-norm conv path: under bf16 autocast a plain spectrally normalised Conv2d
(ops/conv.py ``_MfmaConv2d`` with an ``SNWeight``) runs k10 on its bf16 shadow weight with
1 / sigma in the epilogue, and k11's weight gradient folds the SN backward (dW = G / sigma - (<G, W> / sigma^2)
u v^T) into its split-K sum. Checked against the materialised path (bf16(W / sigma) per layer,
IMAGINAIRE_AMD_SN_FUSED=0 semantics) and against fp32 PyTorch spectral norm (reference
layers/weight_norm.py -> torch.nn.utils.spectral_norm), over stride-1 / stride-2 / 1x1 convs,
channel counts that are not multiples of 64, reflect padding, bias-free and leaky / relu
epilogues, and three optimizer steps.
"""
import pytest
import torch
from torch import nn

pytestmark = pytest.mark.gpu


def _make():
    from imaginaire_amd.layers import Conv2dBlock
    sn = dict(weight_norm_type='spectral')
    return nn.Sequential(
        Conv2dBlock(64, 128, 3, 1, 1, nonlinearity='leakyrelu', **sn),          # conv + act
        Conv2dBlock(128, 185, 4, 2, 1, nonlinearity='leakyrelu', **sn),         # strided, Cout 185
        Conv2dBlock(185, 128, 3, 1, 1, padding_mode='reflect', **sn),           # Cin 185, reflect
        Conv2dBlock(128, 96, 1, 1, 0, nonlinearity='relu', **sn),               # 1x1
        Conv2dBlock(96, 64, 4, 2, 1, bias=False, **sn))                         # strided, Cin 96


def _rel(a, b):
    a, b = a.detach().float().reshape(-1), b.detach().float().reshape(-1)
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


def _cos(a, b):
    a, b = a.float().reshape(-1), b.float().reshape(-1)
    return float(torch.dot(a, b) / (a.norm() * b.norm()).clamp_min(1e-30))


@pytest.mark.parametrize('dot_ratio', [8.0, 0.0, 1e9])
def test_sn_fused_conv_matches_materialised_and_fp32(monkeypatch, dot_ratio):
    """(``dot_ratio``: where <G, W> comes from — the default mix of the k11 epilogue and the
    data-gradient identity sigma <dx, x>, the epilogue everywhere, the identity everywhere)"""
    from imaginaire_amd.layers import spectral_norm as snm
    from imaginaire_amd.ops import conv as C
    from imaginaire_amd.optimizers import fused_adam as FA
    torch.manual_seed(31)
    cl = torch.channels_last
    net = _make().cuda().to(memory_format=cl)
    ref = _make().cuda().to(memory_format=cl)
    f32 = _make().cuda().to(memory_format=cl)
    ref.load_state_dict(net.state_dict())
    f32.load_state_dict(net.state_dict())
    assert snm.install_batched_spectral_norm(net) == 5
    assert snm.install_batched_spectral_norm(ref) == 5
    opt = FA.FusedAdam(net.parameters(), lr=1e-3)

    calls = []
    orig = C._MfmaConv2d

    class Counting(orig):
        @staticmethod
        def forward(ctx, *a):
            if len(a) > 8 and a[8] is not None:  # an SNWeight: the fused path
                calls.append(tuple(a[1].shape))
            return orig.forward(ctx, *a)
    monkeypatch.setattr(C, '_MfmaConv2d', Counting)
    monkeypatch.setattr(C, '_SN_DOT_RATIO', dot_ratio)

    old_fused, old_shadow = snm._SN_FUSED, snm._SN_SHADOW
    snm._SN_SHADOW = True
    try:
        for it in range(3):
            x = torch.randn(4, 64, 64, 128, device='cuda').contiguous(memory_format=cl)
            g = torch.randn(4, 64, 16, 32, device='cuda').contiguous(memory_format=cl)
            outs = {}
            for tag, m, fused in (('fused', net, True), ('mat', ref, False)):
                snm._SN_FUSED = fused
                xi = x.clone().requires_grad_(True)
                with torch.autocast('cuda', dtype=torch.bfloat16):
                    y = m(xi)
                y.backward(g.to(y.dtype))
                outs[tag] = (y.detach(), xi.grad,
                             [(p.grad.clone() if p.grad is not None else None)
                              for p in m.parameters()])
            # fp32 PyTorch spectral norm from the same weights and u / v buffers
            xi = x.clone().requires_grad_(True)
            y32 = f32(xi)
            y32.backward(g)
            outs['fp32'] = (y32.detach(), xi.grad, [p.grad.clone() for p in f32.parameters()])
            if it == 0:
                assert len(calls) == 5, calls        # every conv took the fused path
                # after a fused forward, module.weight is the unmaterialised reference (not a
                # stale tensor) and materialises to the W / sigma the materialised path used
                from imaginaire_amd.layers.weight_norm import _sn_hook
                fmods = [m for m in net.modules() if _sn_hook(m) is not None]
                rmods = [m for m in ref.modules() if _sn_hook(m) is not None]
                assert len(fmods) == len(rmods) == 5
                for fm, rm in zip(fmods, rmods):
                    assert isinstance(fm.weight, C.SNWeight), type(fm.weight)
                    wm = fm.weight.materialize()
                    assert wm.shape == rm.weight.shape
                    assert _rel(wm, rm.weight) <= 1e-2, _rel(wm, rm.weight)
            yf, yr, y3 = outs['fused'][0], outs['mat'][0], outs['fp32'][0]
            assert _rel(yf, y3) <= max(2e-2, 1.5 * _rel(yr, y3)), (it, _rel(yf, y3), _rel(yr, y3))
            assert _rel(yf, yr) <= 2e-2, (it, _rel(yf, yr))
            cf, cr = _cos(outs['fused'][1], outs['fp32'][1]), _cos(outs['mat'][1], outs['fp32'][1])
            assert cf >= min(0.999, cr - 2e-3), (it, cf, cr)
            names = [n for n, _ in net.named_parameters()]
            for n, a, b, c in zip(names, outs['fused'][2], outs['mat'][2], outs['fp32'][2]):
                assert a is not None and b is not None, n
                cf, cr = _cos(a, c), _cos(b, c)
                # as close to fp32 as the materialised bf16 path (both round to bf16 operands)
                assert cf >= min(0.999, cr - 2e-3), (it, n, cf, cr)
                assert _rel(a, c) <= max(3e-2, 1.5 * _rel(b, c)), (it, n, _rel(a, c), _rel(b, c))
            for (n, bf), br in zip(net.named_buffers(), ref.buffers()):
                assert torch.allclose(bf, br, atol=2e-3, rtol=2e-2), (it, n)
            opt.step()
            opt.zero_grad()
            ref.zero_grad()
            f32.zero_grad()
            with torch.no_grad():  # the other two follow the fused net's weights and u / v
                for p, rp, fp in zip(net.parameters(), ref.parameters(), f32.parameters()):
                    rp.copy_(p)
                    fp.copy_(p)
                for b, rb, fb in zip(net.buffers(), ref.buffers(), f32.buffers()):
                    rb.copy_(b)
                    fb.copy_(b)
    finally:
        snm._SN_FUSED, snm._SN_SHADOW = old_fused, old_shadow


def test_sn_group_leaves_idle_layers_alone():
    """The batched power iteration runs for every SN layer of the network, but a layer the
    forward does not call keeps its u / v (the reference iterates a layer only when it runs —
    vid2vid's previous-frame encoder is idle on the first frame); the called layers advance
    exactly one iteration, as torch's spectral_norm does."""
    from imaginaire_amd.layers import Conv2dBlock
    from imaginaire_amd.layers import spectral_norm as snm

    class Two(nn.Module):
        def __init__(self):
            super().__init__()
            self.a = Conv2dBlock(64, 64, 3, 1, 1, weight_norm_type='spectral')
            self.b = Conv2dBlock(64, 64, 3, 1, 1, weight_norm_type='spectral')

        def forward(self, x, use_b):
            x = self.a(x)
            return self.b(x) if use_b else x

    torch.manual_seed(5)
    net = Two().cuda().to(memory_format=torch.channels_last)
    ref = Two().cuda().to(memory_format=torch.channels_last)
    ref.load_state_dict(net.state_dict())
    assert snm.install_batched_spectral_norm(net) == 2
    x = torch.randn(2, 64, 16, 16, device='cuda').contiguous(memory_format=torch.channels_last)
    bufs = lambda m: {k: v.clone() for k, v in m.state_dict().items()  # noqa: E731
                      if k.endswith(('_u', '_v'))}
    for use_b in (False, True, False):
        before = bufs(net)
        with torch.autocast('cuda', dtype=torch.bfloat16):
            net(x, use_b).float().sum().backward()
        with torch.autocast('cuda', enabled=False):
            ref(x.float(), use_b)  # torch spectral_norm on the CPU-free fallback path
        after, want = bufs(net), bufs(ref)
        for k in after:
            idle = k.startswith('b.') and not use_b
            if idle:
                assert torch.equal(after[k], before[k]), (use_b, k)
            else:
                assert not torch.equal(after[k], before[k]), (use_b, k)
            # (the batched iteration's GEMVs read the bf16 shadow of W: ~1e-3 relative)
            torch.testing.assert_close(after[k], want[k], rtol=2e-2, atol=2e-3)
