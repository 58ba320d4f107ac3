"""FlowNet2 decoder transposed convs (4x4 / stride 2 / pad 1) at the vid2vid recipe's
512x1024 flow resolution: MIOpen (F.conv_transpose2d) vs the k10 phase-convolution path
(ops.conv.conv_transpose2d), plus one whole FlowNet2 forward with the path off / on."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from imaginaire_amd.ops import conv as C  # noqa: E402

cl = torch.channels_last


def t(fn, n=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / n


torch.manual_seed(0)
B = int(os.environ.get('B', 2))
# (Cin_t, Cout_t, H, W) of FlowNetC/S/SD/Fusion decoders at a 512x1024 input
shapes = [(1024, 512, 8, 16), (1026, 256, 16, 32), (770, 128, 32, 64), (386, 64, 64, 128),
          (1024, 512, 8, 16), (130, 64, 64, 128), (194, 32, 128, 256), (128, 32, 128, 256),
          (162, 16, 256, 512)]
with torch.no_grad():
    for cin, cout, h, w in shapes:
        x = torch.randn(B, cin, h, w, device='cuda').to(torch.bfloat16).contiguous(memory_format=cl)
        wt = (torch.randn(cin, cout, 4, 4, device='cuda') / (cin * 4) ** 0.5).to(torch.bfloat16)
        wt = wt.contiguous(memory_format=cl)
        ref = F.conv_transpose2d(x.float(), wt.float(), None, 2, 1)
        el = C.deconv_eligible(x, wt, (2, 2), (1, 1), (0, 0), 1, (1, 1))
        wt = torch.nn.Parameter(wt, requires_grad=False)  # cached phase weights, as FlowNet2's
        saved = C._DECONV_MIN_PIX
        C._DECONV_MIN_PIX, C._DECONV_FORCE = 0, 'k10s'
        y = C.conv_transpose2d(x, wt, None, 2, 1)
        err = float((y.float() - ref).abs().max() / ref.abs().max())
        t_k10 = t(lambda: C.conv_transpose2d(x, wt, None, 2, 1))
        C._DECONV_MIN_PIX, C._DECONV_FORCE = saved, None
        t_mi = t(lambda: F.conv_transpose2d(x, wt, None, 2, 1))
        fl = 2.0 * B * h * w * cin * cout * 16 / 1e12
        print('deconv %4d->%4d %3dx%3d  miopen %.3f ms (%4.0f TF/s)  k10s %.3f ms (%4.0f TF/s)  '
              'x%.2f  rel_err %.4f  eligible(default)=%s' % (
                  cin, cout, h, w, t_mi, fl / t_mi * 1e3, t_k10, fl / t_k10 * 1e3, t_mi / t_k10,
                  err, el), flush=True)

    from imaginaire_amd.third_party.flow_net.flow_net import FlowNet
    net = FlowNet(pretrained=False, fp16=True).cuda()
    im1 = torch.rand(B, 3, 512, 1024, device='cuda') * 2 - 1
    im2 = torch.rand(B, 3, 512, 1024, device='cuda') * 2 - 1
    for force in ('miopen', None):
        C._DECONV_FORCE = force
        ms = t(lambda: net(im1, im2), n=5)
        f, _ = net(im1, im2)
        print('FlowNet2 %dx3x512x1024 forward, transposed convs %s: %.2f ms  |flow| %.4f' % (
            B, 'on MIOpen' if force else 'tuned per shape (MIOpen / k10 phase)', ms,
            float(f.abs().mean())), flush=True)
    print('choices:', {'%s %s' % (k[0], k[1]): v for k, v in C._DECONV_CHOICE.items()})
