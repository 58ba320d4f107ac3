"""Perceptual loss pyramid semantics on CPU (reference losses/perceptual.py:108-140)."""
import torch
import torch.nn.functional as F

from imaginaire_amd.losses.perceptual import PerceptualLoss
from imaginaire_amd.utils.misc import apply_imagenet_normalization


def _per_layer_reference(loss_mod, inp, target, num_scales):
    """The reference formula written out: every scale sees a half-size pair."""
    inp = apply_imagenet_normalization(inp)[:, :3]
    target = apply_imagenet_normalization(target)[:, :3]
    total = 0.
    for scale in range(num_scales):
        fi = loss_mod.model(inp)
        with torch.no_grad():
            ft = loss_mod.model(target)
        for layer, w in zip(loss_mod.layers, loss_mod.weights):
            total = total + w * F.l1_loss(fi[layer], ft[layer].detach())
        if scale != num_scales - 1:
            inp = F.interpolate(inp, mode='bilinear', scale_factor=0.5, align_corners=False,
                                recompute_scale_factor=True)
            target = F.interpolate(target, mode='bilinear', scale_factor=0.5,
                                   align_corners=False, recompute_scale_factor=True)
    return total


def test_multiscale_l1_downsamples_every_scale():
    torch.manual_seed(0)
    layers = ['relu_1_1', 'relu_2_1', 'relu_3_1']
    weights = [0.25, 0.5, 1.0]
    ms = PerceptualLoss(None, 'vgg19', layers, weights, criterion='l1', num_scales=3)
    one = PerceptualLoss(None, 'vgg19', layers, weights, criterion='l1', num_scales=1)
    one.model.load_state_dict(ms.model.state_dict())
    x = torch.rand(2, 3, 32, 48) * 2 - 1
    y = torch.rand(2, 3, 32, 48) * 2 - 1
    got = ms(x, y)
    ref = _per_layer_reference(ms, x, y, 3)
    assert torch.allclose(got, ref, rtol=1e-5, atol=1e-6), (float(got), float(ref))
    # a pyramid is not three copies of the full-resolution term
    assert not torch.allclose(got, 3 * one(x, y), rtol=1e-3)


def test_multiscale_l2_matches_reference_order():
    torch.manual_seed(1)
    layers = ['relu_1_1', 'relu_2_1']
    m = PerceptualLoss(None, 'vgg19', layers, [1.0, 0.5], criterion='l2', num_scales=2)
    x = torch.rand(1, 3, 16, 16) * 2 - 1
    y = torch.rand(1, 3, 16, 16) * 2 - 1
    got = m(x, y)
    xi = apply_imagenet_normalization(x)[:, :3]
    yi = apply_imagenet_normalization(y)[:, :3]
    ref = 0.
    for s in range(2):
        fi, ft = m.model(xi), m.model(yi)
        ref = ref + F.mse_loss(fi['relu_1_1'], ft['relu_1_1']) + 0.5 * F.mse_loss(
            fi['relu_2_1'], ft['relu_2_1'])
        if s == 0:
            xi = F.interpolate(xi, scale_factor=0.5, mode='bilinear', align_corners=False,
                               recompute_scale_factor=True)
            yi = F.interpolate(yi, scale_factor=0.5, mode='bilinear', align_corners=False,
                               recompute_scale_factor=True)
    assert torch.allclose(got, ref, rtol=1e-5, atol=1e-6)
