"""Model-level parity on the GPU: one full training iteration (D update then G update) of a
BASELINE family run on the HIP kernels under bf16 autocast vs the same iteration run on the
plain PyTorch reference ops in fp32 (``IMAGINAIRE_AMD_EAGER=1``, amp O0), from identical
weights, inputs and RNG state. The loss dicts and the per-network gradient norms must agree
within bf16 tolerance, and every gradient tensor must agree with PyTorch's
own ops under the same bf16 autocast as closely as two PyTorch-bf16 runs agree with each other
(:func:`_same_precision_gate`); a negative control flips one k11 weight gradient and requires
the gate to fail.

Reference semantics: trainers/spade.py:128-187, trainers/munit.py, trainers/vid2vid.py."""
import math
import os

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _to_dev(x, dev):
    if torch.is_tensor(x):
        return x.to(dev)
    if isinstance(x, dict):
        return {k: _to_dev(v, dev) for k, v in x.items()}
    if isinstance(x, list):
        return [_to_dev(v, dev) for v in x]
    return x


def _fresh(x):
    if torch.is_tensor(x):
        return x.clone()
    if isinstance(x, dict):
        return {k: _fresh(v) for k, v in x.items()}
    if isinstance(x, list):
        return [_fresh(v) for v in x]
    return x


def _grads(net):
    """Every parameter's gradient as a CPU fp32 copy (unit-test configs: a few MB)."""
    return {name: p.grad.detach().float().cpu().clone() for name, p in net.named_parameters()
            if p.grad is not None}


def _grad_norms(net, exclude=()):
    sq = 0.0
    n = 0
    for name, p in net.named_parameters():
        if p.grad is not None and not any(e in name for e in exclude):
            sq += float(p.grad.float().pow(2).sum())
            n += 1
    return math.sqrt(sq), n


def _iteration(config, amp, eager, tmp, seq_len=None, overrides=(), grad_exclude=(), cudnn=None,
               perturb=0.0):
    from torch.utils.data import default_collate
    from imaginaire_amd.config import Config
    from imaginaire_amd.datasets.synthetic import Dataset
    from imaginaire_amd.utils.trainer import get_model_optimizer_and_scheduler, get_trainer
    old = os.environ.get('IMAGINAIRE_AMD_EAGER')
    os.environ['IMAGINAIRE_AMD_EAGER'] = '1' if eager else '0'
    # the fp32 reference runs PyTorch's own (im2col + rocBLAS) convolutions, not MIOpen: one
    # of MIOpen's fp32 backward solvers faulted (illegal memory access) on the pix2pixHD
    # reference iteration of one box (gpurun_out r4t, round 4)
    old_cudnn = torch.backends.cudnn.enabled
    # (``cudnn``: force MIOpen on / off — a second bf16 PyTorch run with other conv algorithms,
    # i.e. other roundings, measures how far bf16 alone moves each gradient)
    torch.backends.cudnn.enabled = (not eager) if cudnn is None else cudnn
    try:
        cfg = Config(os.path.join(ROOT, 'configs', 'unit_test', config))
        cfg.logdir = str(tmp)
        cfg.speed_benchmark = False
        cfg.trainer.amp = amp
        # lr 0: the G update sees the D both runs started from. Adam's first step moves every
        # weight by ~lr whatever the gradient's magnitude, so the sign flips of near-zero bf16
        # vs fp32 gradients would otherwise decorrelate the two D's before the G update.
        cfg.gen_opt.lr = 0.0
        cfg.dis_opt.lr = 0.0
        for key, val in overrides:
            node = cfg
            for k in key.split('.')[:-1]:
                node = getattr(node, k)
            setattr(node, key.split('.')[-1], val)
        video = hasattr(cfg.data, 'num_frames_G')
        if video and seq_len:
            cfg.data.train.initial_sequence_length = seq_len
            cfg.data.train.max_sequence_length = seq_len
        torch.manual_seed(0)
        ds = Dataset(cfg)

        class _Loader(list):
            dataset = ds

        nets = get_model_optimizer_and_scheduler(cfg, seed=0)
        if perturb:
            # every weight scaled by (1 + perturb * N(0, 1)): a rounding-sized change of the
            # starting point, to measure how far the model itself carries bf16-level noise
            g = torch.Generator(device='cpu').manual_seed(123)
            with torch.no_grad():
                for net in nets[:2]:
                    for prm in net.parameters():
                        prm.mul_(1 + perturb * torch.randn(prm.shape, generator=g).to(prm.device))
        tr = get_trainer(cfg, *nets, train_data_loader=_Loader(), val_data_loader=None)
        if video and seq_len:
            if hasattr(tr, 'init_temporal_network'):
                tr.init_temporal_network()
            ds.set_sequence_length(seq_len)
            tr.sequence_length = seq_len
        bs = cfg.data.train.batch_size
        torch.manual_seed(0)
        batch = _to_dev(default_collate([ds[j % max(1, len(ds))] for j in range(bs)]),
                        torch.device('cuda', 0))
        torch.manual_seed(1)
        data = tr.start_of_iteration(_fresh(batch), 0)
        torch.manual_seed(2)
        tr.dis_update(data)
        d_norm = _grad_norms(tr.net_D)
        d_grads = _grads(tr.net_D)
        torch.manual_seed(3)
        tr.gen_update(data)
        if video:  # (the video trainers step D per frame inside gen_update: its last frame's)
            d_norm = _grad_norms(tr.net_D)
            d_grads = _grads(tr.net_D)
        g_norm = _grad_norms(tr.net_G, grad_exclude)
        g_grads = _grads(tr.net_G)
        torch.cuda.synchronize()
        dl = {k: float(v) for k, v in tr.dis_losses.items() if torch.is_tensor(v)}
        gl = {k: float(v) for k, v in tr.gen_losses.items() if torch.is_tensor(v)}
        _LAST_GRADS[0] = (d_grads, g_grads)
        return dl, gl, d_norm, g_norm
    finally:
        torch.backends.cudnn.enabled = old_cudnn
        if old is None:
            os.environ.pop('IMAGINAIRE_AMD_EAGER', None)
        else:
            os.environ['IMAGINAIRE_AMD_EAGER'] = old


_LAST_GRADS = [None]


def _close(a, b, rtol, atol):
    # losses are O(1); a near-zero term (the hinge G loss -mean(D(fake)) of an untrained D)
    # is compared on the absolute scale
    return abs(a - b) <= atol + rtol * abs(b)


def _cos(a, b):
    a = a.reshape(-1)
    b = b.reshape(-1)
    return float(torch.dot(a, b) / (a.norm() * b.norm()).clamp_min(1e-30))


def _same_precision_gate(hip, e16, e16b, ref, floor_frac, tag, exclude=()):
    """Per-parameter-tensor gate of the HIP-bf16 gradients. A tensor passes if

    (a) it tracks PyTorch's own ops under the same bf16 autocast within bf16 noise: the two
        PyTorch-bf16 runs (im2col + rocBLAS convolutions; MIOpen's, from weights perturbed at
        bf16 rounding level) differ only by rounding-sized noise, so their MUTUAL cosine
        measures how far that noise moves the tensor, and
        1 - max(cos(hip, e16), cos(hip, e16b)) <= 3 (1 - cos(e16, e16b)) + 0.01; or
    (b) it tracks the fp32 reference at least as well as the better PyTorch-bf16 run does:
        cos(hip, fp32) >= max(cos(e16, fp32), cos(e16b, fp32)) - 0.01 — the HIP path keeping more
        of an op in fp32 than autocast does (k16's fp32 softmax, the fp32 flow warp) moves a
        gradient AWAY from PyTorch-bf16 towards the truth.

    A sign-flipped or otherwise wrong gradient fails both wherever the PyTorch-bf16 runs agree
    with each other (cos > 0.34) and with fp32 (the negative control below flips one k11 output
    and requires a failure). Tensors under ``floor_frac`` of the largest PyTorch-bf16 gradient
    norm are skipped (noise level), and so are the ``exclude`` tensors, which must only be
    finite (the K = 2 weight generator: see test_fs_vid2vid_iteration_hip_bf16_matches_eager_fp32)."""
    norms = {n: float(g.norm()) for n, g in e16.items()}
    top = max(norms.values()) if norms else 0.0
    bad, rows = [], []
    for n, g in e16.items():
        if norms[n] < floor_frac * top or n not in hip or n not in e16b or n not in ref:
            continue
        if any(e in n for e in exclude):
            if not bool(torch.isfinite(hip[n]).all()):
                bad.append('%s grad %s not finite' % (tag, n))
            continue
        c_mut = _cos(g, e16b[n])
        c_hip = max(_cos(hip[n], g), _cos(hip[n], e16b[n]))
        c_hf = _cos(hip[n], ref[n])
        c_ef = max(_cos(g, ref[n]), _cos(e16b[n], ref[n]))
        ok_a = (1 - c_hip) <= 3 * (1 - c_mut) + 0.01
        ok_b = c_hf >= c_ef - 0.01
        rows.append((c_hip, c_mut, c_hf, c_ef, n))
        if not (ok_a or ok_b):
            bad.append('%s grad %s cos(hip, torch-bf16) %.4f vs torch-bf16 mutual %.4f; '
                       'cos(hip, fp32) %.4f vs torch-bf16 %.4f' % (tag, n, c_hip, c_mut, c_hf,
                                                                    c_ef))
    rows.sort()
    print('%s grads: %d tensors gated; worst %s' % (
        tag, len(rows), ['%.4f (mutual %.4f; vs fp32 hip %.4f torch %.4f) %s' % r
                         for r in rows[:4]]))
    return bad


_REF_CACHE = {}


def _references(tmp_path, config, **kw):
    """fp32 eager run and the two PyTorch-bf16 runs of one config (cached per process: the
    negative control reuses them)."""
    key = (config, repr(sorted(kw.items())))
    if key not in _REF_CACHE:
        ref = _iteration(config, 'O0', True, tmp_path / 'ref', **kw)
        ref_grads = _LAST_GRADS[0]
        _iteration(config, 'O1', True, tmp_path / 'eager16', **kw)
        e16_grads = _LAST_GRADS[0]
        # the second PyTorch-bf16 run differs from the first in its conv algorithms (MIOpen) AND
        # starts from weights perturbed at bf16 rounding level (2^-9 relative): the two runs
        # then differ by bf16-sized noise in every op, not only in the convolutions, so their
        # mutual cosine is how far this model carries rounding noise to each gradient (the
        # unit-test video configs at random init amplify it: cos(torch-bf16, fp32) ~0.7 there)
        _iteration(config, 'O1', True, tmp_path / 'eager16b', cudnn=True, perturb=2.0 ** -9,
                   **kw)
        e16b_grads = _LAST_GRADS[0]
        _REF_CACHE[key] = (ref, ref_grads, e16_grads, e16b_grads)
    return _REF_CACHE[key]


def _compare(tmp_path, config, rtol=0.05, atol=1e-2, floor_frac=1e-3, flip=0, **kw):
    """Losses and gradient norms against the fp32 eager iteration, and every gradient tensor
    against the PyTorch-bf16 runs (:func:`_same_precision_gate`). Returns the list of failures
    (the positive tests assert it is empty). ``flip`` = k negates the k-th k11 weight gradient of
    the HIP run (negative control)."""
    from imaginaire_amd.ops import conv as conv_ops
    conv_ops._TEST_FLIP_WGRAD[:] = [flip, 0]
    try:
        hip = _iteration(config, 'O1', False, tmp_path / 'hip', **kw)
    finally:
        conv_ops._TEST_FLIP_WGRAD[:] = [0, 0]
    hip_grads = _LAST_GRADS[0]
    ref, ref_grads, e16_grads, e16b_grads = _references(tmp_path, config, **kw)
    (dl, gl, dn, gn), (rdl, rgl, rdn, rgn) = hip, ref
    print('%s: hip %s | fp32 eager %s' % (config, hip, ref))
    assert dl.keys() == rdl.keys() and gl.keys() == rgl.keys()
    bad = []
    for name, a, b in [('D.' + k, dl[k], rdl[k]) for k in dl] + \
            [('G.' + k, gl[k], rgl[k]) for k in gl]:
        assert math.isfinite(a), name
        if not _close(a, b, rtol, atol):
            bad.append('%s hip %.5g vs fp32 %.5g' % (name, a, b))
    assert dn[1] == rdn[1] and gn[1] == rgn[1], 'different sets of parameters got gradients'
    for name, a, b in (('|grad D|', dn[0], rdn[0]), ('|grad G|', gn[0], rgn[0])):
        if not _close(a, b, 2 * rtol, 1e-6):
            bad.append('%s hip %.5g vs fp32 %.5g' % (name, a, b))
    for tag, i in (('D', 0), ('G', 1)):
        bad += _same_precision_gate(hip_grads[i], e16_grads[i], e16b_grads[i], ref_grads[i],
                                    floor_frac, '%s %s' % (config, tag),
                                    kw.get('grad_exclude', ()))
    return bad


def test_spade_iteration_hip_bf16_matches_eager_fp32(tmp_path):
    bad = _compare(tmp_path, 'spade.yaml', overrides=[('gen.style_enc.freeze_random', True)])
    assert not bad, '; '.join(bad[:20])


def test_parity_gate_negative_control(tmp_path):
    # the gate must be able to fail: the first k11 weight gradient of the HIP iteration (D's
    # output conv, first in its backward) is negated; the same-precision gate has to name it
    bad = _compare(tmp_path, 'spade.yaml', overrides=[('gen.style_enc.freeze_random', True)],
                   flip=1)
    assert any('grad' in b and 'cos(hip' in b for b in bad), \
        'a sign-flipped weight gradient passed the parity gate: %s' % bad


def test_munit_iteration_hip_bf16_matches_eager_fp32(tmp_path):
    bad = _compare(tmp_path, 'munit.yaml')
    assert not bad, '; '.join(bad[:20])


def test_vid2vid_iteration_hip_bf16_matches_eager_fp32(tmp_path):
    # sequence length 2: the flow network, previous-frame warping (k9) and the temporal
    # discriminator are active
    bad = _compare(tmp_path, 'vid2vid_street.yaml', seq_len=2)
    assert not bad, '; '.join(bad[:20])


def test_pix2pixhd_iteration_hip_bf16_matches_eager_fp32(tmp_path):
    # 512-wide images with instance maps: the atomic-free instance-wise feature pooling
    # (ops/segment.py), reflect padding kernels and the multi-scale PatchGAN
    bad = _compare(tmp_path, 'pix2pixHD.yaml',
                   overrides=[('data.train.augmentations.resize_h_w', '256, 512')])
    assert not bad, '; '.join(bad[:20])


@pytest.mark.parametrize('k', [1, 2])
def test_fs_vid2vid_iteration_hip_bf16_matches_eager_fp32(tmp_path, k):
    # K = 1: the label-weighted reference pooling (k15 channel softmax + per-sample k11 GEMM);
    # K = 2: plus the fused few-shot attention; hyper (per-sample) SPADE convs, FlowNet2 flow
    # loss and the warped-reference path at sequence length 2
    # K = 2 leaves the weight generator (reference encoder, attention, hyper-weight MLPs) out of
    # the gradient norm: the attention softmax is unscaled (energies up to ~50 on this config),
    # so bf16 rounding of the energy moves the key / query towers' gradients by 0.3-20x and the
    # attended value features' gradients by ~16% relative — in the reference formulation (bmm +
    # softmax + bmm under autocast) exactly as much as on the fused path
    # (scripts/probe/fs_attn_probe.py, profiles/fs_attention_bf16_probe_mi355x.txt). The losses
    # and the rest of the generator are still compared; K = 1 covers the weight generator.
    # (round 5: the per-tensor direction check covered the weight generator too; round 6's
    # same-precision gate leaves it out at K = 2 for the same reason — the two PyTorch-bf16 runs
    # share one bf16 energy rounding, so their mutual cosine is high, while the fused kernel's
    # fp32 energies land elsewhere in that chaotic map: cos(hip, fp32) 0.83 vs torch-bf16 0.90
    # on ref_label_first, gpurun_out r6sn)
    bad = _compare(tmp_path, 'fs_vid2vid_face.yaml', seq_len=2,
                   overrides=[('data.initial_few_shot_K', k)],
                   grad_exclude=('weight_generator.',) if k > 1 else ())
    assert not bad, '; '.join(bad[:20])
