"""Few-shot vid2vid attention / reference pooling formulations on CPU: the fused attention
(``AttentionModule.fused``: one scaled-dot-product attention with frame-indicator value
channels) equals the reference formulation (``AttentionModule.forward``: energy matrix,
softmax over K*HW, bmm, column sums), values and gradients; ``softmax_pool`` equals softmax +
bmm (reference generators/fs_vid2vid.py:780-788, 944-951)."""
import types

import torch


def _atn_module(k, c=16):
    from imaginaire_amd.generators.fs_vid2vid import AttentionModule
    from imaginaire_amd.layers import Conv2dBlock
    atn_cfg = types.SimpleNamespace(num_downsamples=1)
    data_cfg = types.SimpleNamespace(initial_few_shot_K=k, num_input_channels=3)

    def block(cin, cout, stride=1):
        return Conv2dBlock(cin, cout, 3, stride, 1, nonlinearity='leakyrelu')
    return AttentionModule(atn_cfg, data_cfg, block, [8, c])


def test_fused_attention_matches_reference_k2():
    torch.manual_seed(0)
    k, b, c, h, w = 2, 2, 16, 4, 6
    m = _atn_module(k, c)
    label = torch.randn(b, 3, 2 * h, 2 * w)
    ref_label = torch.randn(b * k, 3, 2 * h, 2 * w)
    x = torch.randn(b * k, c, h, w, requires_grad=True)
    xl = torch.randn(b * k, c, h, w, requires_grad=True)
    out, atn, vis = m(x, label, ref_label)
    out_l, _, _ = m(xl, None, None, atn)
    atn_full = atn.reshape(b, k, h * w, h * w).sum(2).reshape(b, k, h, w)
    (outs, vis_f) = m.fused([x, xl], label, ref_label)
    assert torch.allclose(outs[0], out, atol=1e-5)
    assert torch.allclose(outs[1], out_l, atol=1e-5)
    assert torch.allclose(vis_f, atn_full, atol=1e-5)
    assert torch.allclose(vis_f.sum(1), torch.ones(b, h, w), atol=1e-5)
    g0, g1 = torch.randn_like(out), torch.randn_like(out_l)
    gx_ref = torch.autograd.grad((out * g0).sum() + (out_l * g1).sum(),
                                 [x, xl] + list(m.parameters()), allow_unused=True)
    gx_f = torch.autograd.grad((outs[0] * g0).sum() + (outs[1] * g1).sum(),
                               [x, xl] + list(m.parameters()), allow_unused=True)
    for a, r in zip(gx_f, gx_ref):
        if r is None:
            assert a is None or float(a.abs().max()) == 0.0
            continue
        assert torch.allclose(a, r, atol=1e-4, rtol=1e-3)


def test_softmax_pool_matches_reference():
    from imaginaire_amd.ops.few_shot import softmax_pool
    torch.manual_seed(1)
    conv = torch.randn(2, 32, 5, 7, requires_grad=True)
    lab = torch.randn(2, 48, 5, 7, requires_grad=True)
    p = softmax_pool(conv, lab)
    ref = torch.bmm(conv.reshape(2, 32, 35), torch.softmax(lab, 1).reshape(2, 48, 35).transpose(1, 2))
    assert p.shape == (2, 32, 48) and torch.allclose(p, ref, atol=1e-6)


def test_fused_attention_op_cpu_path_matches_reference():
    """ops/attention.py off the GPU (PyTorch SDPA) equals the explicit formulation, values and
    gradients; the padding helpers map head dims onto the k16 kernel's sizes."""
    from imaginaire_amd.ops import attention as A
    assert [A._pad_head(d) for d in (1, 32, 33, 64, 100, 128, 129)] == [32, 32, 64, 64, 128, 128,
                                                                      None]
    assert [A._pad_value(d) for d in (2, 32, 130, 200, 224, 256, 258, 289)] == [
        32, 32, 160, 256, 256, 256, 288, None]
    assert A._value_chunks(258) == [(0, 258)] and A._value_chunks(600) == [(0, 256), (256, 256),
                                                                          (512, 88)]
    torch.manual_seed(0)
    q, k, v = (torch.randn(2, 64, 20, dtype=torch.float64), torch.randn(2, 128, 20,
                                                                        dtype=torch.float64),
               torch.randn(2, 128, 12, dtype=torch.float64))
    qa, ka, va = (t.clone().requires_grad_(True) for t in (q, k, v))
    qb, kb, vb = (t.clone().requires_grad_(True) for t in (q, k, v))
    assert not A.native_ok(qa, ka, va)
    o = A.fused_attention(qa, ka, va, 0.5)
    r = A.attention_reference(qb, kb, vb, 0.5)
    torch.testing.assert_close(o, r)
    g = torch.randn_like(r)
    o.backward(g)
    r.backward(g)
    for a, b in ((qa, qb), (ka, kb), (va, vb)):
        torch.testing.assert_close(a.grad, b.grad)
