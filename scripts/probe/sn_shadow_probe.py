"""SN shadow path vs fp32 path on odd shapes: sigma, cast outputs, and the small-net gradients of
test_sn_scale_cast_under_bf16_autocast with and without shadows.

    python scripts/probe/sn_shadow_probe.py
"""
import os
import sys

import torch
from torch import nn

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from imaginaire_amd.ops import _ext  # noqa: E402
from imaginaire_amd.layers import spectral_norm as snm  # noqa: E402

X = _ext.ext()
torch.manual_seed(6)
cl = torch.channels_last
ws = [torch.randn(16, 6, 3, 3, device='cuda').contiguous(memory_format=cl),
      torch.randn(8, 16, 5, 5, device='cuda').contiguous(memory_format=cl),
      torch.randn(10, 288, device='cuda'), torch.randn(7, 13, device='cuda')]
sh = [w.to(torch.bfloat16) for w in ws]
for w, s in zip(ws, sh):
    assert s.stride() == w.stride()
mk = lambda: ([torch.nn.functional.normalize(torch.randn(w.shape[0], device='cuda'), dim=0)  # noqa
               for w in ws], [torch.zeros(w[0].numel(), device='cuda') for w in ws])
torch.manual_seed(1)
us, vs = mk()
us2 = [u.clone() for u in us]
vs2 = [v.clone() for v in vs]
s32 = X.mt_sn_power(ws, us, vs, True, 1e-12)
sbf = X.mt_sn_power([s.float() for s in sh], us2, vs2, True, 1e-12)
us3 = [u.clone() for u in us]
torch.manual_seed(1)
us3, vs3 = mk()
ssh = X.mt_sn_power(ws, us3, vs3, True, 1e-12, sh)
print('sigma fp32 W      ', s32.tolist())
print('sigma fp32(bf16 W)', sbf.tolist())
print('sigma shadow      ', ssh.tolist())
print('u err shadow vs fp32(bf16 W)', [float((a - b).abs().max()) for a, b in zip(us3, us2)])
c1 = X.mt_sn_scale_cast(ws, ssh, sh, 1)
for w, s, o, sg in zip(ws, sh, c1, ssh):
    ref = (s.float() / sg).bfloat16()
    print('cast mode1 shape', tuple(w.shape), 'max err vs bf16(bf16W/s)',
          float((o.float() - ref.float()).abs().max()), 'vs bf16(W/s)',
          float((o.float() - (w / sg).bfloat16().float()).abs().max()))


def make(sn):
    return nn.Sequential(sn(nn.Conv2d(6, 16, 3, padding=1)), nn.LeakyReLU(0.2),
                         sn(nn.Conv2d(16, 8, 5, padding=2)), nn.Flatten(),
                         sn(nn.Linear(8 * 6 * 6, 10)))


_orig_snb = X.sn_scale_backward
grads = {}
for mode in ('fp32', 'shadow', 'shadow_nobwd'):
    shadow = mode != 'fp32'
    if mode == 'shadow_nobwd':  # the shadow forward, fp32 W in the backward's <G, W>
        X.sn_scale_backward = lambda g, w, u, v, s, shadow=None: _orig_snb(g, w, u, v, s)
    torch.manual_seed(6)
    ref = make(torch.nn.utils.spectral_norm).cuda()
    net = make(snm.spectral_norm).cuda()
    net.load_state_dict(ref.state_dict())
    net = net.to(memory_format=cl)
    snm.install_batched_spectral_norm(net)
    snm._SN_SHADOW = shadow
    x = torch.randn(4, 6, 6, 6, device='cuda')
    acts = {}
    for i in (0, 1, 2):
        net[i].register_full_backward_hook(
            lambda m, gi, go, i=i: acts.__setitem__(i, go[0].detach().float().clone()))
    with torch.autocast('cuda', dtype=torch.bfloat16):
        y_ref = ref(x)
        y = net(x.contiguous(memory_format=cl))
    g = torch.randn_like(y)
    y_ref.backward(g)
    y.backward(g)
    grads[mode] = ({n: p.grad.clone() for n, p in net.named_parameters()}, acts)
    print('mode', mode, 'y err', float((y.float() - y_ref.float()).abs().max()), flush=True)
    for (n, p), (_, pr) in zip(net.named_parameters(), ref.named_parameters()):
        print('   %-12s grad err %.3e  ref max %.3e' % (n, float((p.grad - pr.grad).abs().max()),
                                                      float(pr.grad.abs().max())), flush=True)
X.sn_scale_backward = _orig_snb
for mode in ('shadow', 'shadow_nobwd'):
    for n in grads['fp32'][0]:
        print('%s vs fp32: %-12s %.3e' % (mode, n, float(
            (grads[mode][0][n] - grads['fp32'][0][n]).abs().max())))
    for i in sorted(grads['fp32'][1]):
        a, b = grads[mode][1].get(i), grads['fp32'][1][i]
        print('%s vs fp32: dy of module %d  %s (max %.3e)' % (
            mode, i, 'missing' if a is None else '%.3e' % float((a - b).abs().max()),
            float(b.abs().max())))
