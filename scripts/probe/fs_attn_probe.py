"""Few-shot attention on the real fs_vid2vid inputs: the fused scaled-dot-product path vs the
reference formulation (energy bmm, softmax over K*HW, bmm) in bf16, both against the fp32
reference — outputs, per-frame attention mass, and the gradients of the value features and of
the key / query tower weights.

    python scripts/probe/fs_attn_probe.py [config] [K]
"""
import os
import sys

import torch

HERE = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, 'tests'))
import test_model_parity_gpu as T  # noqa: E402
from imaginaire_amd.generators import fs_vid2vid as FS  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else 'fs_vid2vid_face.yaml'
K = int(sys.argv[2]) if len(sys.argv) > 2 else 2
calls = []
orig = FS.AttentionModule.fused


def fused(self, features, label, ref_label):
    calls.append((self, [f.detach().clone() for f in features], label.detach().clone(),
                  ref_label.detach().clone()))
    return orig(self, features, label, ref_label)


FS.AttentionModule.fused = fused
T._iteration(cfg, 'O1', False, '/tmp/fsap', seq_len=2, overrides=[('data.initial_few_shot_K', K)])
FS.AttentionModule.fused = orig
print('captured %d attention calls' % len(calls))


def run(mod, feats, label, ref_label, mode, g):
    """mode: fp32 | bf16 | fused -> (outs, vis, grads of features + tower weights)"""
    params = [p for n, p in mod.named_parameters() if p.requires_grad]
    fs = [f.float().clone().requires_grad_(True) for f in feats]
    label, ref_label = label.float(), ref_label.float()
    for p in params:
        p.grad = None
    if mode == 'fused':
        with torch.autocast('cuda', dtype=torch.bfloat16):
            outs, vis = mod.fused(fs, label, ref_label)
    else:
        with torch.autocast('cuda', dtype=torch.bfloat16, enabled=(mode == 'bf16')):
            out, atn, _ = mod.forward(fs[0], label, ref_label)
            outs = [out]
            for f in fs[1:]:
                outs.append(mod.forward(f, None, None, atn)[0])
            b, k = out.shape[0], K
            hw = out.shape[2] * out.shape[3]
            vis = atn.reshape(b, k, hw, hw).sum(2).reshape(b, k, *out.shape[2:])
    loss = sum((o.float() * gi).sum() for o, gi in zip(outs, g))
    grads = torch.autograd.grad(loss, fs + params, allow_unused=True)
    return [o.float().detach() for o in outs], vis.float().detach(), grads, \
        [n for n, p in mod.named_parameters() if p.requires_grad]


def rel(a, b):
    if a is None or b is None:
        return float('nan')
    return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-30))


for ci, (mod, feats, label, ref_label) in enumerate(calls[:2]):
    mod.eval()  # the same sigma for every mode (no power iteration)
    print('call %d: features %s label %s ref_label %s' % (
        ci, [tuple(f.shape) for f in feats], tuple(label.shape), tuple(ref_label.shape)))
    torch.manual_seed(5)
    with torch.no_grad():
        key = mod.attention_encode(ref_label.float(), 'atn_key').float()
        qry = mod.attention_encode(label.float(), 'atn_query').float()
        b = qry.shape[0]
        e = torch.bmm(key.reshape(b, K, key.shape[1], -1).permute(0, 1, 3, 2).reshape(
            b, -1, key.shape[1]), qry.reshape(b, qry.shape[1], -1))
        p = torch.softmax(e, 1)
    print('  energy std %.3g max %.3g | softmax max mean %.3f' % (
        float(e.std()), float(e.abs().max()), float(p.max(1).values.mean())))
    ref_outs, _, _, _ = run(mod, feats, label, ref_label, 'fp32',
                            [torch.zeros(1, device='cuda')] * len(feats))
    g = [torch.randn_like(o) for o in ref_outs]
    R = run(mod, feats, label, ref_label, 'fp32', g)
    for mode in ('bf16', 'fused'):
        o, vis, grads, names = run(mod, feats, label, ref_label, mode, g)
        print('  %-5s out rel %s vis rel %.3g' % (
            mode, ' '.join('%.3g' % rel(a, b) for a, b in zip(o, R[0])), rel(vis, R[1])))
        nf = len(feats)
        print('        dfeat rel %s' % ' '.join('%.3g' % rel(a, b) for a, b in
                                                 zip(grads[:nf], R[2][:nf])))
        for n, a, b in zip(names, grads[nf:], R[2][nf:]):
            if 'weight' in n:
                print('        %-40s rel %.3g |fp32| %.3g' % (n, rel(a, b),
                                                             float(b.norm()) if b is not None
                                                             else float('nan')))
