"""Debug: multi-condition SPADE gradient, fused 'none'-mode modulation vs eager vs fp32."""
import copy
import os
import sys
from types import SimpleNamespace

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import imaginaire_amd.layers.activation_norm as AN  # noqa: E402
from imaginaire_amd.ops import _ext  # noqa: E402
from imaginaire_amd.ops.norm import fused_norm_act  # noqa: E402

torch.manual_seed(0)
cl = torch.channels_last
# 1) the k1 'none' mode alone, bf16 x / gb vs fp32 torch
x = torch.randn(2, 64, 32, 48, device='cuda').contiguous(memory_format=cl)
gb = torch.randn(2, 128, 32, 48, device='cuda').contiguous(memory_format=cl) * 0.5
for slope in (1.0, 0.2):
    xh = x.to(torch.bfloat16).requires_grad_(True)
    gh = gb.to(torch.bfloat16).requires_grad_(True)
    y = fused_norm_act(xh, 'none', gb=gh, slope=slope)
    xr = x.clone().requires_grad_(True)
    gr = gb.clone().requires_grad_(True)
    g, b = gr.chunk(2, 1)
    yr = xr * (1 + g) + b
    yr = torch.nn.functional.leaky_relu(yr, slope) if slope != 1.0 else yr
    go = torch.randn_like(yr)
    y.float().backward(go)
    yr.backward(go)
    rel = lambda a, r: float((a.float() - r).abs().max() / r.abs().max())  # noqa: E731
    print('none-mode slope %.1f: y %.4f dx %.4f dgb %.4f' % (
        slope, rel(y, yr), rel(xh.grad, xr.grad), rel(gh.grad, gr.grad)), flush=True)

# 2) the module: fused path, old eager path, fp32 reference
m = AN.SpatiallyAdaptiveNorm(64, [12, 3], num_filters=32, kernel_size=3,
                             activation_norm_type='instance',
                             activation_norm_params=SimpleNamespace(affine=False)).cuda()
m = m.to(memory_format=cl)
c1 = torch.randn(2, 12, 32, 48, device='cuda')
c2 = torch.randn(2, 3, 32, 48, device='cuda')
go = torch.randn(2, 64, 32, 48, device='cuda')


def run(mod, eager, bf16):
    xx = (x.to(torch.bfloat16) if bf16 else x.clone()).requires_grad_(True)
    with _ext.eager_scope(eager), torch.autocast('cuda', dtype=torch.bfloat16, enabled=bf16):
        y = mod(xx, c1, c2, act_slope=0.2)
    y.float().backward(go)
    return y.float().detach(), xx.grad.float()


ref_y, ref_dx = run(copy.deepcopy(m), True, False)
fy, fdx = run(copy.deepcopy(m), False, True)
orig = AN._modulate_more


def eager_more(out, gbs, act_slope):
    for gbx in gbs:
        g, b = gbx.chunk(2, dim=1)
        out = out * (1 + g) + b
    return torch.nn.functional.leaky_relu(out, act_slope) if act_slope != 1.0 else out


AN._modulate_more = eager_more
ey, edx = run(copy.deepcopy(m), False, True)
AN._modulate_more = orig
ey32, edx32 = run(copy.deepcopy(m), True, True)
r = lambda a, b: float((a - b).abs().max() / b.abs().max())  # noqa: E731
print('module fused-k1 vs fp32: y %.4f dx %.4f' % (r(fy, ref_y), r(fdx, ref_dx)))
print('module eager-bf16 (old path) vs fp32: y %.4f dx %.4f' % (r(ey, ref_y), r(edx, ref_dx)))
print('module plain-torch bf16 autocast vs fp32: y %.4f dx %.4f' % (r(ey32, ref_y),
                                                                   r(edx32, ref_dx)))
