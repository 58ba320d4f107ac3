"""Per-stage finiteness of the random-init Inception-v3 features on the GPU (FID debug)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402
from imaginaire_amd.evaluation.common import get_inception  # noqa: E402
from imaginaire_amd.utils.misc import apply_imagenet_normalization  # noqa: E402

net = get_inception(torch.device('cuda', 0))
x = torch.rand(4, 3, 256, 512, device='cuda') * 2 - 1
for ac in (False, True):
    with torch.no_grad(), torch.autocast('cuda', dtype=torch.bfloat16, enabled=ac):
        h = apply_imagenet_normalization(x.float().clamp(-1, 1))
        h = F.interpolate(h, size=(299, 299), mode='bilinear', align_corners=True)
        h = h.contiguous(memory_format=torch.channels_last)
        print('autocast', ac, 'input', h.dtype, bool(torch.isfinite(h).all()), flush=True)
        for name in ('Conv2d_1a_3x3', 'Conv2d_2a_3x3', 'Conv2d_2b_3x3', 'maxpool1',
                     'Conv2d_3b_1x1', 'Conv2d_4a_3x3', 'maxpool2', 'Mixed_5b', 'Mixed_5c',
                     'Mixed_5d', 'Mixed_6a', 'Mixed_6b', 'Mixed_6c', 'Mixed_6d', 'Mixed_6e',
                     'Mixed_7a', 'Mixed_7b', 'Mixed_7c'):
            h = getattr(net, name)(h)
            print('  %-14s %-16s %s finite=%s max=%.3g' % (name, str(h.dtype), tuple(h.shape),
                  bool(torch.isfinite(h).all()), float(h.float().abs().max())), flush=True)
