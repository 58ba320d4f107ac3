"""Audit PyTorch-ROCm's channels-last (NHWC) kernels against the CPU: forward and backward of
every spatial op the model families may run on NHWC activations. Prints max |GPU - CPU| per
op; anything above ~1e-4 (fp32) is a wrong kernel to route around."""
import torch
import torch.nn.functional as F

OPS = {
    'avg_pool2d k2s2': lambda x: F.avg_pool2d(x, 2, 2),
    'avg_pool2d k3s2p1': lambda x: F.avg_pool2d(x, 3, 2, 1),
    'avg_pool2d k3s2p1 no-pad-count': lambda x: F.avg_pool2d(x, 3, 2, 1, count_include_pad=False),
    'avg_pool2d k3s1p1': lambda x: F.avg_pool2d(x, 3, 1, 1),
    'max_pool2d k2': lambda x: F.max_pool2d(x, 2),
    'max_pool2d k3s2p1': lambda x: F.max_pool2d(x, 3, 2, 1),
    'adaptive_avg_pool2d 1': lambda x: F.adaptive_avg_pool2d(x, 1),
    'adaptive_avg_pool2d 5x7': lambda x: F.adaptive_avg_pool2d(x, (5, 7)),
    'adaptive_max_pool2d 4': lambda x: F.adaptive_max_pool2d(x, 4),
    'upsample nearest x2': lambda x: F.interpolate(x, scale_factor=2, mode='nearest'),
    'upsample bilinear x2': lambda x: F.interpolate(x, scale_factor=2, mode='bilinear',
                                                    align_corners=False),
    'bilinear down ac': lambda x: F.interpolate(x, scale_factor=0.5, mode='bilinear',
                                                align_corners=True),
    'bicubic x2': lambda x: F.interpolate(x, scale_factor=2, mode='bicubic', align_corners=False),
    'reflection_pad2d': lambda x: F.pad(x, (2, 2, 2, 2), mode='reflect'),
    'replication_pad2d': lambda x: F.pad(x, (2, 2, 2, 2), mode='replicate'),
    'instance_norm': lambda x: F.instance_norm(x),
    'group_norm': lambda x: F.group_norm(x, 4),
    'pixel_shuffle': lambda x: F.pixel_shuffle(x, 2),
    'grid_sample border': lambda x: F.grid_sample(
        x, torch.linspace(-1.1, 1.1, x.shape[2] * x.shape[3] * 2, device=x.device).view(
            1, x.shape[2], x.shape[3], 2).expand(x.shape[0], -1, -1, -1).contiguous(),
        mode='bilinear', padding_mode='border', align_corners=True),
}


def main():
    torch.manual_seed(0)
    base = torch.randn(2, 16, 19, 26)
    for name, fn in OPS.items():
        xc = base.clone().requires_grad_(True)
        yc = fn(xc)
        g = torch.randn_like(yc)
        yc.backward(g)
        xg = base.cuda().contiguous(memory_format=torch.channels_last).requires_grad_(True)
        yg = fn(xg)
        yg.backward(g.cuda().contiguous(memory_format=torch.channels_last)
                    if g.dim() == 4 else g.cuda())
        ef = float((yg.detach().cpu() - yc.detach()).abs().max())
        eb = float((xg.grad.cpu() - xc.grad).abs().max())
        flag = '   <-- WRONG' if max(ef, eb) > 1e-3 else ''
        print('%-32s fwd %.2e  bwd %.2e%s' % (name, ef, eb, flag))


if __name__ == '__main__':
    main()
