"""MUNIT discriminator pass batching (discriminators/munit.py; reference
discriminators/munit.py:56-99 runs each domain's discriminator once per image set, each pass
refreshing the spectral-norm u / v once)."""
import copy
import os

import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))


def _dis():
    from imaginaire_amd.config import Config
    from imaginaire_amd.discriminators.munit import Discriminator
    cfg = Config(os.path.join(HERE, '..', 'configs', 'unit_test', 'munit.yaml'))
    cfg.dis.num_filters = 8
    cfg.dis.max_num_filters = 32
    cfg.dis.num_layers = 3
    torch.manual_seed(0)
    d = Discriminator(cfg.dis, cfg.data)
    with torch.no_grad():  # converge the power iteration (u / v as after a few training steps)
        x = torch.rand(2, 3, 32, 32) * 2 - 1
        for _ in range(40):
            d.discriminator_a(x)
            d.discriminator_b(x)
    return d


def _inputs(grad):
    g = torch.Generator().manual_seed(1)
    img = lambda: torch.rand(2, 3, 32, 32, generator=g) * 2 - 1  # noqa: E731
    data = {'images_a': img(), 'images_b': img()}
    out = {k: img().requires_grad_(grad) for k in ('images_ab', 'images_ba', 'images_aa',
                                                     'images_bb')}
    return data, out


def _sn_state(net):
    return {k: v.clone() for k, v in net.state_dict().items()
            if k.endswith(('weight_u', 'weight_v'))}


def _flat(x):
    if torch.is_tensor(x):
        return [x]
    out = []
    for e in x:
        out += _flat(e)
    return out


@pytest.mark.parametrize('real,gan_recon', [(True, False), (True, True), (False, True)])
def test_batched_passes_match_reference(real, gan_recon):
    d = _dis()
    assert d.batched
    ref = copy.deepcopy(d)
    ref.batched = False
    u0 = _sn_state(d)
    data, out = _inputs(grad=True)
    got = d(data, out, real=real, gan_recon=gan_recon)
    want = ref(data, out, real=real, gan_recon=gan_recon)
    assert set(got) == set(want)
    for k in want:
        a, b = _flat(got[k]), _flat(want[k])
        assert len(a) == len(b) > 0
        for x, y in zip(a, b):
            torch.testing.assert_close(x, y, rtol=1e-3, atol=1e-3)
    one, two = _sn_state(d), _sn_state(ref)
    assert one.keys() == two.keys() and len(one) > 0
    for k in one:
        torch.testing.assert_close(one[k], two[k], rtol=1e-5, atol=1e-6)
    assert any(not torch.equal(one[k], u0[k]) for k in one)
    sum(t.float().sum() for t in _flat(got['out_ba'])).backward()
    assert out['images_ba'].grad is not None
