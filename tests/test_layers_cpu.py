"""Layer library semantics on CPU (reference-equivalent math)."""
from types import SimpleNamespace as NS

import pytest
import torch
import torch.nn.functional as F

from imaginaire_amd.layers import (Conv2dBlock, LinearBlock, Res2dBlock, UpRes2dBlock,
                                   DownRes2dBlock, PartialConv2dBlock, HyperConv2dBlock,
                                   NonLocal2dBlock, MultiOutRes2dBlock, PartialRes2dBlock)
from imaginaire_amd.layers.activation_norm import (SpatiallyAdaptiveNorm, AdaptiveNorm,
                                                   BatchNorm2d, InstanceNorm2d, LayerNorm2d)
from imaginaire_amd.ops.norm import fused_norm_act


def test_batchnorm_matches_torch():
    torch.manual_seed(0)
    bn = BatchNorm2d(8)
    ref = torch.nn.BatchNorm2d(8)
    x = torch.randn(4, 8, 5, 6)
    y = bn(x)
    yr = ref(x)
    assert torch.allclose(y, yr, atol=1e-5)
    assert torch.allclose(bn.running_mean, ref.running_mean, atol=1e-6)
    assert torch.allclose(bn.running_var, ref.running_var, atol=1e-5)
    bn.eval(); ref.eval()
    assert torch.allclose(bn(x), ref(x), atol=1e-5)
    assert set(bn.state_dict().keys()) == set(ref.state_dict().keys())


def test_instancenorm_matches_torch():
    x = torch.randn(2, 4, 7, 7)
    inn = InstanceNorm2d(4, affine=True)
    ref = torch.nn.InstanceNorm2d(4, affine=True)
    assert torch.allclose(inn(x), ref(x), atol=1e-5)


def test_conv_block_orders_and_fusion():
    torch.manual_seed(0)
    blk = Conv2dBlock(3, 8, 3, padding=1, nonlinearity='leakyrelu', order='CNA',
                      activation_norm_type='instance')
    x = torch.randn(2, 3, 8, 8)
    y = blk(x)
    conv = blk.layers.conv
    yr = F.leaky_relu(F.instance_norm(F.conv2d(x, conv.weight, conv.bias, padding=1),
                                      weight=blk.layers.norm.weight,
                                      bias=blk.layers.norm.bias), 0.2)
    assert torch.allclose(y, yr, atol=1e-5)
    blk2 = Conv2dBlock(3, 8, 3, padding=1, nonlinearity='relu', weight_norm_type='spectral')
    y2 = blk2(x)
    assert (y2 >= 0).all()
    assert 'layers.conv.weight_orig' in blk2.state_dict()


def test_spade_norm_separate_projection_equivalence():
    torch.manual_seed(0)
    norm = SpatiallyAdaptiveNorm(6, 5, num_filters=4, kernel_size=3, separate_projection=True,
                                 activation_norm_type='instance',
                                 activation_norm_params=NS(affine=False))
    x = torch.randn(2, 6, 8, 8)
    seg = torch.randn(2, 5, 16, 16)
    y = norm(x, seg)
    lm = F.interpolate(seg, size=(8, 8), mode='nearest')
    h = norm.mlps[0](lm)
    g = norm.gammas[0](h)
    b = norm.betas[0](h)
    yr = F.instance_norm(x) * (1 + g) + b
    assert torch.allclose(y, yr, atol=1e-5)


def test_adaptive_norm():
    an = AdaptiveNorm(6, 10, activation_norm_type='instance')
    x = torch.randn(3, 6, 4, 4)
    z = torch.randn(3, 10)
    y = an(x, z)
    gamma, beta = an.fc(z).chunk(2, 1)
    yr = F.instance_norm(x) * (1 + gamma[:, :, None, None]) + beta[:, :, None, None]
    assert torch.allclose(y, yr, atol=1e-5)


def test_res_blocks_shapes_and_grads():
    x = torch.randn(2, 8, 8, 8)
    for blk in [Res2dBlock(8, 4), UpRes2dBlock(8, 4, order='NACNAC',
                                               activation_norm_type='instance'),
                DownRes2dBlock(8, 16)]:
        y = blk(x)
        y.sum().backward()
    assert UpRes2dBlock(8, 4)(x).shape == (2, 4, 16, 16)
    assert DownRes2dBlock(8, 16)(x).shape == (2, 16, 4, 4)
    y, a0, a1 = MultiOutRes2dBlock(8, 8)(x) if False else (None, None, None)


def test_partial_conv_matches_reference_math():
    torch.manual_seed(0)
    blk = PartialConv2dBlock(3, 4, 3, padding=1)
    x = torch.randn(1, 3, 6, 6)
    mask = (torch.rand(1, 1, 6, 6) > 0.4).float()
    y, m = blk(x, mask_in=mask)
    conv = blk.layers.conv
    raw = F.conv2d(x * mask, conv.weight, conv.bias, padding=1)
    upd = F.conv2d(mask, torch.ones(1, 1, 3, 3), padding=1)
    ratio = 9 / (upd + 1e-6)
    updc = upd.clamp(0, 1)
    ratio = ratio * updc
    yr = ((raw - conv.bias.view(1, -1, 1, 1)) * ratio + conv.bias.view(1, -1, 1, 1)) * updc
    assert torch.allclose(y, yr, atol=1e-5)
    assert torch.allclose(m, updc)
    out, mask_out = PartialRes2dBlock(3, 3)(x, mask_in=mask)
    assert out.shape == x.shape


def test_hyper_conv_grouped_equals_loop():
    torch.manual_seed(0)
    blk = HyperConv2dBlock(4, 6, 3, padding=1, is_hyper_conv=True)
    x = torch.randn(3, 4, 5, 5)
    w = torch.randn(3, 6, 4, 3, 3)
    b = torch.randn(3, 6)
    y = blk(x, conv_weights=(w, b))
    yr = torch.cat([F.conv2d(x[i:i + 1], w[i], b[i], padding=1) for i in range(3)])
    assert torch.allclose(y, yr, atol=1e-5)


def test_non_local_equals_reference_formula():
    torch.manual_seed(0)
    nl = NonLocal2dBlock(16)
    with torch.no_grad():
        nl.gamma.fill_(0.5)
    x = torch.randn(2, 16, 6, 8)
    y = nl(x)
    n, c, h, w = x.shape
    theta = nl.theta(x).view(n, -1, h * w).permute(0, 2, 1)
    phi = nl.max_pool(nl.phi(x)).view(n, -1, h * w // 4)
    att = torch.softmax(torch.bmm(theta, phi), -1)
    g = nl.max_pool(nl.g(x)).view(n, -1, h * w // 4)
    out = torch.bmm(g, att.permute(0, 2, 1)).view(n, c // 2, h, w)
    yr = 0.5 * nl.out_conv(out) + x
    assert torch.allclose(y, yr, atol=1e-5)


def test_layernorm2d():
    ln = LayerNorm2d(4)
    assert ln(torch.randn(2, 4, 3, 3)).shape == (2, 4, 3, 3)


def test_linear_block_and_weight_demod():
    lb = LinearBlock(5, 7, nonlinearity='leakyrelu', weight_norm_type='spectral')
    assert lb(torch.randn(3, 5)).shape == (3, 7)
    from imaginaire_amd.layers.conv import Conv2dBlock as C2
    blk = C2(4, 6, 3, padding=1, weight_norm_type='weight_demod',
             weight_norm_params=NS(cond_dims=8))
    y = blk(torch.randn(2, 4, 5, 5), torch.randn(2, 8))
    assert y.shape == (2, 6, 5, 5)


def test_fpse_pool_first_embedding_matches_reference_order():
    """conv1x1 -> avg_pool (reference discriminators/fpse.py:118-122) == avg_pool -> conv1x1."""
    import torch
    from imaginaire_amd.discriminators.fpse import FPSEDiscriminator
    torch.manual_seed(0)
    d = FPSEDiscriminator(3, 7, 8, 3, 'spectral', 'none')
    img = torch.randn(2, 3, 32, 64)
    seg = torch.randn(2, 7, 32, 64)
    d.eval()
    assert d._embedding_is_linear()
    fast = d(img, seg)
    d._embedding_is_linear = lambda: False
    ref = d(img, seg)
    for a, b in zip(fast, ref):
        assert torch.allclose(a, b, atol=1e-5, rtol=1e-4)


def test_shadow_weight_registry_resync():
    """optimizers/fused_adam.py shadow registry: a parameter written outside the optimizer (its
    version counter moves) has its bf16 shadow rewritten by resync_shadows() — what every graph
    replay runs first — and one never synced (its first forward writes it) is left alone."""
    from imaginaire_amd.optimizers import fused_adam as FA
    p = torch.nn.Parameter(torch.randn(4, 3, 3, 3))
    q = torch.nn.Parameter(torch.randn(5))
    sp, sq = torch.zeros(4, 3, 3, 3, dtype=torch.bfloat16), torch.zeros(5, dtype=torch.bfloat16)
    FA.register_shadow(p, sp)
    FA.register_shadow(q, sq)
    FA.sync_shadows([p])
    assert FA.shadow_synced(p) and not FA.shadow_synced(q)
    assert torch.equal(sp, p.detach().to(torch.bfloat16))
    with torch.no_grad():
        p.add_(1.0)  # outside the optimizer
    assert not FA.shadow_synced(p)
    assert FA.resync_shadows() == 1
    assert FA.shadow_synced(p) and torch.equal(sp, p.detach().to(torch.bfloat16))
    assert torch.equal(sq, torch.zeros(5, dtype=torch.bfloat16))  # never synced: untouched
    FA.register_shadow(p, None)
    FA.register_shadow(q, None)
    assert FA.resync_shadows() == 0
