"""CPU checks of the FlowNet2 op references (k6/k7/k8 oracles) and the FlowNet2 graph."""
import torch

from imaginaire_amd.ops.flownet_ops import (channelnorm_reference, correlation_out_size,
                                            correlation_reference, resample2d_reference)


def _naive_corr(a, b, pad, ks, md, s1, s2):
    n, c, h, w = a.shape
    ap = torch.nn.functional.pad(a, [pad] * 4)
    bp = torch.nn.functional.pad(b, [pad] * 4)
    kr = (ks - 1) // 2
    rad = md // s2
    d = 2 * rad + 1
    oh = correlation_out_size(h, pad, ks, md, s1)
    ow = correlation_out_size(w, pad, ks, md, s1)
    out = torch.zeros(n, d * d, oh, ow)
    for oy in range(oh):
        for ox in range(ow):
            y1, x1 = oy * s1 + md, ox * s1 + md
            for tj in range(-rad, rad + 1):
                for ti in range(-rad, rad + 1):
                    acc = torch.zeros(n)
                    for j in range(-kr, kr + 1):
                        for i in range(-kr, kr + 1):
                            acc += (ap[:, :, y1 + j, x1 + i] *
                                    bp[:, :, y1 + j + tj * s2, x1 + i + ti * s2]).sum(1)
                    out[:, (tj + rad) * d + ti + rad, oy, ox] = acc / (ks * ks * c)
    return out


def test_correlation_reference_matches_naive():
    torch.manual_seed(0)
    a, b = torch.randn(2, 3, 6, 7), torch.randn(2, 3, 6, 7)
    for params in [(2, 1, 2, 1, 1), (3, 3, 2, 2, 2), (4, 1, 4, 1, 2)]:
        assert torch.allclose(correlation_reference(a, b, *params), _naive_corr(a, b, *params),
                              atol=1e-5)


def test_resample2d_zero_flow_identity_and_channelnorm():
    x = torch.randn(1, 3, 5, 6)
    assert torch.allclose(resample2d_reference(x, torch.zeros(1, 2, 5, 6)), x)
    shifted = resample2d_reference(x, torch.ones(1, 2, 5, 6))
    assert torch.allclose(shifted[:, :, :-1, :-1], x[:, :, 1:, 1:])
    assert torch.allclose(channelnorm_reference(x), x.norm(dim=1, keepdim=True), atol=1e-6)
