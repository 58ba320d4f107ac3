"""Debug the k14 average-pool backward against F.avg_pool2d on a non-square map."""
import sys
sys.path.insert(0, '/root/repo')
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402
from imaginaire_amd.ops.pool import avg_pool2d  # noqa: E402
from imaginaire_amd.ops import _ext  # noqa: E402

for (k, s, p, inc) in [(3, 2, 1, True)]:
    torch.manual_seed(8)
    x = torch.randn(2, 24, 19, 26, device='cuda').contiguous(
        memory_format=torch.channels_last).requires_grad_(True)
    y = avg_pool2d(x, k, s, p, count_include_pad=inc)
    xr = x.detach().clone().requires_grad_(True)
    yr = F.avg_pool2d(xr, k, s, p, count_include_pad=inc)
    g = torch.randn_like(yr)
    print('g strides', g.stride(), g.is_contiguous(memory_format=torch.channels_last))
    y.backward(g)
    yr.backward(g)
    d = (x.grad - xr.grad).abs()
    print('max diff', float(d.max()), 'argmax', torch.nonzero(d == d.max())[:3].tolist())
    dx2 = _ext.ext().avg_pool_nhwc_bwd(g.contiguous(memory_format=torch.channels_last), 19, 26,
                                       k, k, s, s, p, p, inc)
    print('direct kernel diff', float((dx2 - xr.grad).abs().max()))
    print(x.grad[0, 0, :3, :6])
    print(xr.grad[0, 0, :3, :6])
    xc = x.detach().cpu().contiguous().requires_grad_(True)
    F.avg_pool2d(xc, k, s, p, count_include_pad=inc).backward(g.cpu().contiguous())
    xn = x.detach().contiguous().requires_grad_(True)  # NCHW on the GPU
    F.avg_pool2d(xn, k, s, p, count_include_pad=inc).backward(g.contiguous())
    print('k14 vs CPU', float((x.grad.cpu() - xc.grad).abs().max()),
          '| torch NHWC GPU vs CPU', float((xr.grad.cpu() - xc.grad).abs().max()),
          '| torch NCHW GPU vs CPU', float((xn.grad.cpu() - xc.grad).abs().max()))
