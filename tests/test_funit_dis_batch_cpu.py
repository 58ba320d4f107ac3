"""FUNIT discriminator pass batching (discriminators/funit.py; reference
discriminators/funit.py:13-50 runs one ResDiscriminator pass per image set, each refreshing the
spectral-norm u / v once): the batched passes must match the reference passes' outputs up to the
one-iteration σ shift, and leave u / v exactly where the reference leaves them."""
import copy
import os

import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))


def _dis():
    from imaginaire_amd.config import Config
    from imaginaire_amd.discriminators.funit import Discriminator
    cfg = Config(os.path.join(HERE, '..', 'configs', 'unit_test', 'funit.yaml'))
    cfg.dis.num_filters = 8
    cfg.dis.max_num_filters = 32
    cfg.dis.num_layers = 3
    torch.manual_seed(0)
    d = Discriminator(cfg.dis, cfg.data)
    with torch.no_grad():  # converge the power iteration (u / v as after a few training steps)
        x = torch.rand(2, 3, 32, 32) * 2 - 1
        for _ in range(40):
            d.model(x, torch.tensor([0, 1]))
    return d, cfg


def _inputs(n=2, h=32, w=32, grad=False):
    g = torch.Generator().manual_seed(1)
    img = lambda: (torch.rand(n, 3, h, w, generator=g) * 2 - 1)  # noqa: E731
    data = {'images_style': img(), 'labels_content': torch.tensor([0, 1]),
            'labels_style': torch.tensor([1, 0])}
    out = {'images_trans': img().requires_grad_(grad), 'images_recon': img().requires_grad_(grad)}
    return data, out


def _sn_state(net):
    return {k: v.clone() for k, v in net.state_dict().items()
            if k.endswith(('weight_u', 'weight_v'))}


def _reference(d, data, out, recon):
    """The reference's pass order: translation, style, reconstruction."""
    m = d.model
    r = {}
    r['fake_out_trans'], r['fake_features_trans'] = m(out['images_trans'], data['labels_style'])
    r['real_out_style'], r['real_features_style'] = m(data['images_style'], data['labels_style'])
    if recon:
        r['fake_out_recon'], r['fake_features_recon'] = m(out['images_recon'],
                                                          data['labels_content'])
    return r


@pytest.mark.parametrize('recon,grad', [(False, True), (True, True), (True, False)])
def test_batched_passes_match_reference(recon, grad):
    d, _ = _dis()
    assert d.batched
    ref = copy.deepcopy(d)
    u0 = _sn_state(d)
    data, out = _inputs(grad=grad)
    got = d(data, out, recon=recon)
    want = _reference(ref, data, out, recon)
    assert set(got) == set(want)
    for k in want:
        torch.testing.assert_close(got[k], want[k], rtol=1e-3, atol=1e-3)
    one, two = _sn_state(d), _sn_state(ref)
    assert one.keys() == two.keys() and len(one) > 0
    for k in one:  # same number of power iterations as the reference's passes
        torch.testing.assert_close(one[k], two[k], rtol=1e-5, atol=1e-6)
    assert any(not torch.equal(one[k], u0[k]) for k in one)
    if grad:  # gradients reach every fake set through the concatenated pass
        loss = got['fake_out_trans'].sum() + (got['fake_out_recon'].sum() if recon else 0)
        loss.backward()
        assert out['images_trans'].grad is not None
        if recon:
            assert out['images_recon'].grad is not None


def test_unbatched_is_reference_order():
    d, _ = _dis()
    d.batched = False
    ref = copy.deepcopy(d)
    data, out = _inputs()
    with torch.no_grad():
        got = d(data, out)
        want = _reference(ref, data, out, True)
    for k in want:
        torch.testing.assert_close(got[k], want[k], rtol=0, atol=0)
