"""The WGAN-GP penalty (losses/gp.py) differentiates D's input gradient, so its D forward
must be twice differentiable. The HIP kernels' autograd Functions are first-order only;
trainers/munit.py therefore runs the penalty's D forward under ``_ext.eager_scope()``.
This checks that the penalty's gradient w.r.t. every D weight on the GPU matches the same
computation on the CPU (pure PyTorch), i.e. nothing is silently dropped."""
import copy
import os

import pytest
import torch

from imaginaire_amd.config import Config
from imaginaire_amd.losses.gp import GradientPenaltyLoss
from imaginaire_amd.ops import _ext
from imaginaire_amd.utils.trainer import get_model_optimizer_and_scheduler

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _gp_grads(net_D, xa, xb):
    gp = GradientPenaltyLoss()
    xa = xa.clone().requires_grad_(True)
    xb = xb.clone().requires_grad_(True)
    with _ext.eager_scope():
        out = net_D({}, dict(images_ab=xb, images_ba=xa), real=False)
    loss = gp(xa, out['out_ba']) + gp(xb, out['out_ab'])
    params = [p for p in net_D.parameters() if p.requires_grad]
    grads = torch.autograd.grad(loss, params, allow_unused=True)
    return loss.detach(), dict(zip([n for n, p in net_D.named_parameters() if p.requires_grad],
                                   grads))


def test_eager_scope_nests():
    assert not _ext.force_eager() or os.environ.get('IMAGINAIRE_AMD_EAGER') == '1'
    with _ext.eager_scope():
        with _ext.eager_scope():
            assert _ext.force_eager()
        assert _ext.force_eager()
    with _ext.eager_scope(enabled=False):
        assert _ext.force_eager() == (os.environ.get('IMAGINAIRE_AMD_EAGER') == '1')


@pytest.mark.gpu
def test_munit_gradient_penalty_reaches_d_weights():
    torch.manual_seed(0)
    cfg = Config(os.path.join(ROOT, 'configs', 'unit_test', 'munit.yaml'))
    net_G, net_D = get_model_optimizer_and_scheduler(cfg, seed=0)[:2]
    net_D = getattr(net_D, 'module', net_D)
    d_cpu = copy.deepcopy(net_D).cpu().float()
    d_gpu = copy.deepcopy(net_D).cuda()
    c = cfg.data.num_channels if hasattr(cfg.data, 'num_channels') else 3
    xa = torch.randn(2, 3, 64, 64)
    xb = torch.randn(2, 3, 64, 64)
    loss_c, g_c = _gp_grads(d_cpu, xa, xb)
    loss_g, g_g = _gp_grads(d_gpu, xa.cuda(), xb.cuda())
    torch.testing.assert_close(loss_g.cpu(), loss_c, rtol=2e-3, atol=1e-4)
    nonzero = 0
    for name, gc in g_c.items():
        gg = g_g[name]
        assert (gc is None) == (gg is None), name
        if gc is None:
            continue
        nonzero += int(gc.abs().max() > 0)
        scale = gc.abs().max().clamp_min(1e-6)
        err = (gg.cpu() - gc).abs().max() / scale
        assert err < 2e-2, (name, float(err))
    assert nonzero > 0
