"""FlowNetC correlation on MI355X: forward diagonal multi-wave MFMA (diag, default) vs one-wave
MFMA (k6m) vs LDS-tiled VALU (k6); backward register-blocked tiled (reg, default) vs tiled
(corr_bwd_k1) vs per-element gather (corr_bwd), at the FlowNetC shapes (pad 20, max
displacement 20, stride2 2, kernel 1, 256-channel conv3 features at 1/8 of 512x1024 and of
256x512), interleaved rounds in one process, each checked against the fp32 PyTorch reference.

    python scripts/probe/corr_bwd_probe.py

Reference kernels: /root/reference/imaginaire/third_party/correlation/src/
correlation_cuda_kernel.cu:73-334 (forward / backward of the reference's CUDA extension).
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from imaginaire_amd.ops import _ext  # noqa: E402
from imaginaire_amd.ops.flownet_ops import correlation_reference  # noqa: E402

ext = _ext.ext()
CL = torch.channels_last
PAD, KS, MD, S1, S2 = 20, 1, 20, 1, 2


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


FWD = (('k6', '0', '0'), ('k6m', '1', '0'), ('diag', '1', '1'))
BWD = (('gather', '0'), ('tiled', '1'), ('reg', '2'))


def flops(N, C, H, W):
    D = 2 * (MD // S2) + 1
    return 2.0 * N * H * W * D * D * C  # one multiply-add per (pixel, displacement, channel)


for N, C, H, W in ((2, 256, 64, 128), (4, 256, 64, 128), (4, 256, 32, 64)):
    torch.manual_seed(0)
    a = torch.randn(N, C, H, W, device='cuda').to(torch.bfloat16).contiguous(memory_format=CL)
    b = torch.randn(N, C, H, W, device='cuda').to(torch.bfloat16).contiguous(memory_format=CL)
    # forward
    fw = {}
    for tag, env, dg in FWD:
        os.environ['IMAGINAIRE_AMD_CORR_MFMA'] = env
        os.environ['IMAGINAIRE_AMD_CORR_DIAG'] = dg
        y = ext.correlation_forward(a, b, PAD, KS, MD, S1, S2)
        fw[tag] = (y.float(), [])
    ref = correlation_reference(a.float(), b.float(), PAD, KS, MD, S1, S2)
    go = torch.randn_like(ref).contiguous(memory_format=CL)
    # backward reference via autograd on the fp32 reference
    a32 = a.float().requires_grad_(True)
    b32 = b.float().requires_grad_(True)
    correlation_reference(a32, b32, PAD, KS, MD, S1, S2).backward(go)
    bw = {}
    for tag, env in BWD:
        os.environ['IMAGINAIRE_AMD_CORR_BWD_TILED'] = env
        g1, g2 = ext.correlation_backward(a, b, go, PAD, KS, MD, S1, S2)
        err = max(float((g1 - a32.grad).norm() / a32.grad.norm()),
                  float((g2 - b32.grad).norm() / b32.grad.norm()))
        bw[tag] = (err, [])
    for _ in range(5):  # interleaved rounds
        for tag, env, dg in FWD:
            os.environ['IMAGINAIRE_AMD_CORR_MFMA'] = env
            os.environ['IMAGINAIRE_AMD_CORR_DIAG'] = dg
            fw[tag][1].append(timed(lambda: ext.correlation_forward(a, b, PAD, KS, MD, S1, S2)))
        for tag, env in BWD:
            os.environ['IMAGINAIRE_AMD_CORR_BWD_TILED'] = env
            bw[tag][1].append(timed(
                lambda: ext.correlation_backward(a, b, go, PAD, KS, MD, S1, S2), reps=3))
    fl = flops(N, C, H, W)
    fe = {k: float((v[0] - ref).norm() / ref.norm()) for k, v in fw.items()}
    t = {k: min(v[1]) for k, v in fw.items()}
    print('N=%d C=%d %dx%d fwd: k6 %.3f ms | k6m %.3f ms %.1f TF/s | diag %.3f ms %.1f TF/s '
          '(x%.2f vs k6) rel err %.1e/%.1e/%.1e' % (
              N, C, H, W, t['k6'], t['k6m'], fl / t['k6m'] / 1e9, t['diag'], fl / t['diag'] / 1e9,
              t['k6'] / t['diag'], fe['k6'], fe['k6m'], fe['diag']), flush=True)
    u = {k: min(v[1]) for k, v in bw.items()}
    print('N=%d C=%d %dx%d bwd: gather %.3f ms | tiled %.3f ms (x%.2f) | reg %.3f ms (x%.2f) '
          'rel err %.1e/%.1e/%.1e' % (
              N, C, H, W, u['gather'], u['tiled'], u['gather'] / u['tiled'], u['reg'],
              u['gather'] / u['reg'], bw['gather'][0], bw['tiled'][0], bw['reg'][0]), flush=True)
