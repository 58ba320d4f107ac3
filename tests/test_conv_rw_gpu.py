"""The row-window k10 tile (csrc/conv_rw.hip) against fp32 PyTorch convolutions.

Shapes cover every mode of the tile: stride 1 / 2 (the de-interleaved stride-2 window), filter
widths 1 / 3 / 4 / 5 / 7, BN = 64 / 128, Cin = 32 (two filter taps per 64-deep k-chunk, odd KW
with a zero half tap) and Cin multiples of 64, output widths that do not tile the 256 / 128
pixel block (masked virtual pixels: 5, 47, 100, 260), split-K, the residual / 1 / sigma
epilogue and the LDS-poison determinism check. Reference: the convolutions of
/root/reference/imaginaire/layers/conv.py:59-91 (cuDNN there)."""
import os

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

CL = torch.channels_last

# B, Cin, Cout, H, W, KH, KW, stride, pad
RW_CASES = [
    (2, 64, 64, 32, 64, 3, 3, 1, 1),       # BN 64, stride 1
    (2, 64, 128, 33, 47, 4, 4, 2, 1),      # 4x4 s2 (PatchGAN), odd sizes: Wo 24
    (2, 64, 128, 31, 33, 3, 3, 2, 1),      # 3x3 s2
    (1, 128, 128, 16, 100, 7, 7, 1, 3),    # 7x7, Wo 100 of a 128-pixel segment
    (2, 64, 64, 20, 30, 1, 1, 1, 0),       # 1x1
    (2, 128, 64, 17, 9, 1, 1, 2, 0),       # 1x1 s2
    (1, 64, 128, 13, 260, 3, 3, 1, 1),     # Wo 260: two 256-pixel segments per row
    (2, 192, 128, 16, 32, 4, 4, 2, 1),     # three channel blocks per filter row
    (1, 64, 64, 9, 9, 3, 3, 2, 1),         # Wo 5: 16-pixel segments
    (2, 256, 256, 8, 8, 3, 3, 1, 1),       # 8x8 map (split-K)
    (1, 64, 128, 12, 40, 5, 3, 1, 2),      # KH != KW
    (1, 64, 64, 20, 40, 7, 7, 2, 3),       # 7x7 s2
    (1, 64, 64, 19, 37, 5, 5, 2, 2),       # 5x5 s2
    (1, 32, 64, 24, 40, 3, 3, 1, 1),       # Cin 32: virtual taps (0, 1), (2, zero)
    (1, 32, 128, 20, 36, 4, 4, 2, 1),      # Cin 32, 4x4 s2
    (1, 32, 64, 16, 30, 7, 7, 1, 3),       # Cin 32, 7x7
    (1, 32, 64, 16, 16, 1, 1, 1, 0),       # Cin 32, 1x1 (one half-zero tap)
    (1, 32, 64, 15, 21, 5, 5, 2, 2),       # Cin 32, 5x5 s2
    (2, 32, 64, 64, 128, 3, 3, 1, 1),      # Cin 32 at a 128-wide row
    (1, 512, 128, 12, 32, 4, 4, 2, 1),     # 4x4 s2 over eight channel blocks (K 8192)
    (2, 64, 64, 16, 64, 7, 7, 1, 3),       # 7x7 stem-like, 64-pixel rows
    (2, 64, 128, 20, 64, 3, 3, 1, 2),      # Wo 66 (reflect-pad dgrad): 22-pixel segments
    (2, 128, 64, 16, 16, 3, 3, 1, 2),      # Wo 18: a non-power-of-two segment, BN 64
    (1, 64, 128, 9, 128, 5, 5, 1, 3),      # Wo 130
]


def _inputs(case, seed=5):
    B, cin, cout, H, W, kh, kw, s, p = case
    torch.manual_seed(seed)
    x = torch.randn(B, cin, H, W, device='cuda').to(torch.bfloat16).contiguous(memory_format=CL)
    # asymmetric weights: catches row / column swaps in the fragment maps
    w = (torch.randn(cout, cin, kh, kw, device='cuda') / (cin * kh * kw) ** 0.5 +
         torch.arange(cout, device='cuda').view(-1, 1, 1, 1) * 1e-3)
    w = w.to(torch.bfloat16).contiguous(memory_format=CL)
    b = torch.randn(cout, device='cuda') * 0.1
    return x, w, b


def _run(X, x, w, b, s, p, slope=0.2, res=None, asc=None, ver='6', splitk=None):
    os.environ['IMAGINAIRE_AMD_CONV_V'] = ver
    if splitk:
        os.environ['IMAGINAIRE_AMD_CONV_SPLITK'] = splitk
    try:
        y = X.conv2d_mfma(x, w, b, s, s, p, p, 1, 1, slope, 1, -1, res, asc)
        var = X.conv_last_variant()
    finally:
        os.environ.pop('IMAGINAIRE_AMD_CONV_V')
        os.environ.pop('IMAGINAIRE_AMD_CONV_SPLITK', None)
    return y, var


@pytest.mark.parametrize('case', RW_CASES)
def test_rw_forward_matches_fp32(case):
    from imaginaire_amd.ops import _ext
    X = _ext.ext()
    B, cin, cout, H, W, kh, kw, s, p = case
    x, w, b = _inputs(case)
    y, var = _run(X, x, w, b, s, p)
    assert var == 6, 'the row-window tile did not take %s (variant %d)' % (case, var)
    ref = F.leaky_relu(F.conv2d(x.float(), w.float(), b, s, p), 0.2)
    assert y.shape == ref.shape
    err = (y.float() - ref).abs().max().item()
    assert err <= 1e-2 * max(1.0, ref.abs().max().item()), err


@pytest.mark.parametrize('case', [RW_CASES[1], RW_CASES[3], RW_CASES[13], RW_CASES[14],
                                  RW_CASES[21]])
@pytest.mark.parametrize('splitk', ['2', '3'])
def test_rw_splitk_matches(case, splitk):
    from imaginaire_amd.ops import _ext
    X = _ext.ext()
    x, w, b = _inputs(case, seed=6)
    s, p = case[7], case[8]
    y1, _ = _run(X, x, w, b, s, p)
    y2, var = _run(X, x, w, b, s, p, splitk=splitk)
    assert var == 6
    ref = F.leaky_relu(F.conv2d(x.float(), w.float(), b, s, p), 0.2)
    for y in (y1, y2):
        err = (y.float() - ref).abs().max().item()
        assert err <= 1e-2 * max(1.0, ref.abs().max().item()), err


@pytest.mark.parametrize('case', [RW_CASES[0], RW_CASES[1], RW_CASES[14]])
def test_rw_residual_and_sigma_epilogue(case):
    """y = act(conv(x, W) / sigma + b) + res, the residual added after the activation."""
    from imaginaire_amd.ops import _ext
    X = _ext.ext()
    x, w, b = _inputs(case, seed=7)
    s, p = case[7], case[8]
    ref = F.conv2d(x.float(), w.float(), None, s, p)
    res = torch.randn(ref.shape, device='cuda').to(torch.bfloat16).contiguous(memory_format=CL)
    sig = torch.tensor([1.7], device='cuda')
    y, var = _run(X, x, w, b, s, p, res=res, asc=sig)
    assert var == 6
    ref = F.leaky_relu(ref / 1.7 + b.view(1, -1, 1, 1), 0.2) + res.float()
    err = (y.float() - ref).abs().max().item()
    assert err <= 1.5e-2 * max(1.0, ref.abs().max().item()), err


@pytest.mark.parametrize('case', [RW_CASES[0], RW_CASES[1], RW_CASES[3], RW_CASES[14],
                                  RW_CASES[9], RW_CASES[21], RW_CASES[22]])
def test_rw_never_reads_unwritten_lds(case):
    """Bitwise the same output after the LDS of every CU was filled with NaN bits."""
    from imaginaire_amd.ops import _ext
    X = _ext.ext()
    x, w, b = _inputs(case, seed=8)
    s, p = case[7], case[8]
    y0, _ = _run(X, x, w, b, s, p)
    X.lds_poison()
    y1, var = _run(X, x, w, b, s, p)
    torch.cuda.synchronize()
    assert var == 6
    assert torch.isfinite(y1.float()).all()
    assert torch.equal(y0, y1)


def test_rw_taken_by_default_for_long_filters():
    """Without a forced variant, long-filter shapes v4 / v5 do not take (7x7, 4x4 over three
    channel blocks) and Cin = 32 run on the row-window tile."""
    from imaginaire_amd.ops import _ext
    X = _ext.ext()
    for case in (RW_CASES[20], RW_CASES[19], RW_CASES[13]):
        x, w, b = _inputs(case)
        _, var = _run(X, x, w, b, case[7], case[8], ver='0')
        assert var == 6, (case, var)


def test_default_routing_of_narrow_and_odd_width_convs():
    """Default routing (round 6): a stride-1 Cout = 64 conv with a long filter row (3x3 over 128
    channels, K = 1152) takes the narrow two-blocks-per-CU row-window variant; the odd-width data
    gradient of a reflect-padded 3x3 conv (66 wide) stays on v1 (non-power-of-two segments ran at
    0.92x there) — and both match fp32."""
    from imaginaire_amd.ops import _ext
    X = _ext.ext()
    for case, want in (((2, 128, 64, 32, 64, 3, 3, 1, 1), 6),
                       ((2, 256, 128, 16, 64, 3, 3, 1, 2), 1)):
        x, w, b = _inputs(case, seed=10)
        y, var = _run(X, x, w, b, case[7], case[8], ver='0')
        assert var == want, (case, var)
        ref = F.leaky_relu(F.conv2d(x.float(), w.float(), b, case[7], case[8]), 0.2)
        err = (y.float() - ref).abs().max().item()
        assert err <= 1e-2 * max(1.0, ref.abs().max().item()), (case, err)


def test_cin32_never_takes_the_64_channel_tiles():
    """A Cin = 32 conv of a shape v4 / v5 take at Cin >= 64 (3x3 stride 1, Cout % 128 == 0,
    64-pixel rows) routes to the row-window tile: the v4 / v5 k loops step 64-channel chunks."""
    from imaginaire_amd.ops import _ext
    X = _ext.ext()
    case = (2, 32, 128, 16, 64, 3, 3, 1, 1)
    x, w, b = _inputs(case, seed=9)
    y, var = _run(X, x, w, b, 1, 1, ver='0')
    assert var == 6, var
    ref = F.leaky_relu(F.conv2d(x.float(), w.float(), b, 1, 1), 0.2)
    err = (y.float() - ref).abs().max().item()
    assert err <= 1e-2 * max(1.0, ref.abs().max().item()), err


# ---- tap-packed thin-input convolutions (csrc/im2col.hip + 1x1 k10 / k11) -----------------
# B, Cin, Cout, H, W, k, stride, pad, x layout
PACK_CASES = [
    (2, 3, 64, 38, 42, 7, 1, 3, 'nchw'),     # RGB stem (7x7, K 147 -> 192)
    (2, 3, 32, 40, 48, 4, 2, 1, 'nchw'),     # PatchGAN first layer on an image
    (1, 6, 64, 33, 35, 7, 2, 3, 'cl'),       # FlowNet-style two-image input, stride 2
    (2, 1, 64, 20, 24, 3, 1, 1, 'cl'),       # one-channel mask
    (1, 6, 128, 24, 24, 5, 1, 2, 'nchw'),    # K 150 -> 192 (Cin 8 / 16 stay on k10: the
                                             # packing must remove >= 8x of the padded k loop)
]


@pytest.mark.parametrize('case', PACK_CASES)
@pytest.mark.parametrize('slope,bias', [(1.0, False), (0.2, True)])
def test_tappack_conv_fwd_bwd(case, slope, bias):
    from imaginaire_amd.ops import conv as C
    C._TAPPACK_MIN_PIX = 0
    B, cin, cout, H, W, k, s, p, layout = case
    torch.manual_seed(9)
    x = torch.randn(B, cin, H, W, device='cuda')
    if layout == 'cl':
        x = x.contiguous(memory_format=CL)
    x.requires_grad_(True)
    w = (torch.randn(cout, cin, k, k, device='cuda') / (cin * k * k) ** 0.5 +
         torch.arange(cout, device='cuda').view(-1, 1, 1, 1) * 1e-3).requires_grad_(True)
    b = (torch.randn(cout, device='cuda') * 0.1).requires_grad_(True) if bias else None
    with torch.autocast('cuda', dtype=torch.bfloat16):
        assert C.tappack_eligible(x, w, (s, s), (p, p), (1, 1), 1)
        y = C.conv2d_act(x, w, b, s, p, 1, slope)
    # reference on the bf16-rounded operands in fp32
    xr = x.detach().to(torch.bfloat16).float().requires_grad_(True)
    wr = w.detach().to(torch.bfloat16).float().requires_grad_(True)
    br = b.detach().clone().requires_grad_(True) if bias else None
    yr = F.conv2d(xr, wr, br, s, p)
    if slope != 1.0:
        yr = torch.where(y.detach().float() > 0, yr, yr * slope)
    assert y.shape == yr.shape
    err = (y.float() - yr).abs().max().item()
    assert err <= 1e-2 * max(1.0, yr.abs().max().item()), err
    go = torch.randn_like(yr)
    y.backward(go.to(y.dtype))
    yr.backward(go)
    assert x.grad.dtype == x.dtype and x.grad.shape == x.shape
    for got, ref, name in ((x.grad, xr.grad, 'dx'), (w.grad, wr.grad, 'dw')) + \
            (((b.grad, br.grad, 'db'),) if bias else ()):
        e = (got.float() - ref).abs().max().item()
        assert e <= 2e-2 * max(1.0, ref.abs().max().item()), (name, e, ref.abs().max().item())


@pytest.mark.parametrize('case', [
    # B, Cin, Cout, H, W, k, pad
    (2, 64, 3, 30, 34, 7, 3),    # MUNIT / pix2pixHD RGB head
    (1, 128, 1, 20, 28, 3, 1),   # one-channel mask head
    (2, 64, 8, 16, 40, 5, 2),
    (1, 96, 3, 18, 22, 7, 0),    # unpadded head on a reflect-padded input
])
def test_thin_output_conv_grads(case):
    """Heads with Cout <= 16: the data and weight gradients from one tap-packed dy operand."""
    from imaginaire_amd.ops import conv as C
    C._MFMA_MIN_BLOCKS = 0
    C._MFMA_MIN_DGRAD_BLOCKS = 0
    B, cin, cout, H, W, k, p = case
    torch.manual_seed(11)
    x = torch.randn(B, cin, H, W, device='cuda').to(torch.bfloat16).contiguous(
        memory_format=CL).requires_grad_(True)
    w = (torch.randn(cout, cin, k, k, device='cuda') / (cin * k * k) ** 0.5).to(
        torch.bfloat16).contiguous(memory_format=CL).requires_grad_(True)
    b = (torch.randn(cout, device='cuda') * 0.1).requires_grad_(True)
    y = C.conv2d_act(x, w, b, 1, p, 1, 1.0)
    xr = x.detach().float().requires_grad_(True)
    wr = w.detach().float().requires_grad_(True)
    br = b.detach().clone().requires_grad_(True)
    yr = F.conv2d(xr, wr, br, 1, p)
    assert y.shape == yr.shape
    assert (y.float() - yr).abs().max().item() <= 1e-2 * max(1.0, yr.abs().max().item())
    go = torch.randn_like(yr)
    y.backward(go.to(y.dtype))
    yr.backward(go)
    for got, ref, name in ((x.grad, xr.grad, 'dx'), (w.grad, wr.grad, 'dw'),
                           (b.grad, br.grad, 'db')):
        e = (got.float() - ref).abs().max().item()
        assert e <= 2e-2 * max(1.0, ref.abs().max().item()), (name, e, ref.abs().max().item())
