"""Batch-concatenated discriminator passes on the HIP path (discriminators/funit.py; the reference
discriminators/funit.py:13-50 runs one ResDiscriminator pass per image set). The batched pass
normalises every set by the σ of the last power iteration, the reference passes each by its own,
so outputs and D gradients differ by one iteration's σ shift: this measures that deviation on the
GPU path (bf16 autocast, k10 / k11 convs, the batched spectral-norm group) for one D update and
one G update from the same state, and bounds it — within bf16 noise once the power iteration has
converged, as it has after a few training steps. (tests/test_funit_dis_batch_cpu.py checks the
same on the CPU fallback in fp32.)"""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _dis(batched):
    from imaginaire_amd.config import Config
    from imaginaire_amd.discriminators.funit import Discriminator
    from imaginaire_amd.layers.spectral_norm import install_batched_spectral_norm
    cfg = Config(os.path.join(ROOT, 'configs', 'unit_test', 'funit.yaml'))
    torch.manual_seed(0)
    d = Discriminator(cfg.dis, cfg.data).cuda().to(memory_format=torch.channels_last)
    assert install_batched_spectral_norm(d) > 0
    d.batched = batched
    with torch.no_grad(), torch.autocast('cuda', dtype=torch.bfloat16):
        x = (torch.rand(2, 3, 64, 64, device='cuda') * 2 - 1).contiguous(
            memory_format=torch.channels_last)
        for _ in range(40):  # converge u / v (as after a few training steps)
            d.model(x, torch.tensor([0, 1], device='cuda'))
    return d


def _inputs(grad):
    g = torch.Generator(device='cuda').manual_seed(1)

    def img():
        return (torch.rand(2, 3, 64, 64, generator=g, device='cuda') * 2 - 1).contiguous(
            memory_format=torch.channels_last)
    data = {'images_style': img(), 'labels_content': torch.tensor([0, 1], device='cuda'),
            'labels_style': torch.tensor([1, 0], device='cuda')}
    out = {'images_trans': img().requires_grad_(grad), 'images_recon': img().requires_grad_(grad)}
    return data, out


def _rel(a, b):
    a, b = a.float().reshape(-1), b.float().reshape(-1)
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


def _cos(a, b):
    a, b = a.float().reshape(-1), b.float().reshape(-1)
    return float(torch.dot(a, b) / (a.norm() * b.norm()).clamp_min(1e-30))


@pytest.mark.parametrize('update', ['D', 'G'])
def test_batched_d_passes_match_reference_passes_on_gpu(update):
    grad_fake = update == 'G'
    runs = {}
    for batched in (True, False):
        d = _dis(batched)
        data, out = _inputs(grad_fake)
        with torch.autocast('cuda', dtype=torch.bfloat16):
            o = d(data, out, recon=grad_fake)
            if update == 'D':  # hinge D loss on the translation (fake) and style (real) sets
                loss = torch.relu(1 + o['fake_out_trans'].float()).mean() + \
                    torch.relu(1 - o['real_out_style'].float()).mean()
            else:  # G: adversarial terms of both fakes + feature matching against the style set
                loss = -o['fake_out_trans'].float().mean() - o['fake_out_recon'].float().mean() + \
                    (o['fake_features_trans'].float() -
                     o['real_features_style'].float().detach()).abs().mean()
        loss.backward()
        grads = {n: p.grad.detach().float().clone() for n, p in d.named_parameters()
                 if p.grad is not None}
        ins = {k: v.grad.detach().float().clone() for k, v in out.items() if v.grad is not None}
        sn = {k: v.detach().clone() for k, v in d.state_dict().items()
              if k.endswith(('weight_u', 'weight_v'))}
        runs[batched] = (float(loss), {k: v.detach() for k, v in o.items()}, grads, ins, sn)
    (lb, ob, gb, ib, sb), (lr, orf, gr, ir, sr) = runs[True], runs[False]
    print('%s update: loss batched %.6f reference %.6f' % (update, lb, lr))
    assert abs(lb - lr) <= 1e-2 * max(1.0, abs(lr)), (lb, lr)
    assert ob.keys() == orf.keys()
    for k in orf:
        r = _rel(ob[k], orf[k])
        print('  %-22s rel %.2e' % (k, r))
        assert r <= 2e-2, (k, r)
    assert gb.keys() == gr.keys() and len(gr) > 0
    worst = min((_cos(gb[n], gr[n]), n) for n in gr if float(gr[n].norm()) > 0)
    print('  worst D-gradient cosine %.5f (%s)' % worst)
    for n in gr:
        if float(gr[n].norm()) == 0:
            continue
        assert _cos(gb[n], gr[n]) >= 0.995, (n, _cos(gb[n], gr[n]))
        assert _rel(gb[n], gr[n]) <= 5e-2, (n, _rel(gb[n], gr[n]))
    for k in ir:  # the G update's gradients reaching each fake set through the concatenated pass
        assert k in ib and _cos(ib[k], ir[k]) >= 0.995, k
    for k in sr:  # u / v advance by the same number of power iterations on both paths
        torch.testing.assert_close(sb[k], sr[k], rtol=1e-3, atol=1e-4)
