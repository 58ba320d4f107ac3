"""Per-parameter gradient direction of one training iteration, three ways: HIP kernels under
bf16 autocast, PyTorch reference ops under bf16 autocast, and PyTorch reference ops in fp32 —
so a low cosine between HIP-bf16 and fp32 can be told apart from the model's own bf16
sensitivity (eager-bf16 vs fp32 equally low) and from a kernel defect (eager-bf16 close, HIP far).

    python scripts/probe/parity_cos_probe.py spade.yaml [vid2vid_street.yaml:2 fs_vid2vid_face.yaml:2:K2 ...]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests'))
import test_model_parity_gpu as P  # noqa: E402

import tempfile  # noqa: E402


def run(spec):
    parts = spec.split(':')
    config = parts[0]
    seq = int(parts[1]) if len(parts) > 1 and parts[1] else None
    kw = {'seq_len': seq}
    ov = []
    for extra in parts[2:]:
        if extra.startswith('K'):
            ov.append(('data.initial_few_shot_K', int(extra[1:])))
    if config == 'spade.yaml':
        ov.append(('gen.style_enc.freeze_random', True))
    if config == 'pix2pixHD.yaml':
        ov.append(('data.train.augmentations.resize_h_w', '256, 512'))
    kw['overrides'] = ov
    tmp = tempfile.mkdtemp()
    out = {}
    for tag, amp, eager in (('hip-bf16', 'O1', False), ('eager-bf16', 'O1', True),
                            ('fp32', 'O0', True)):
        P._iteration(config, amp, eager, os.path.join(tmp, tag), **kw)
        out[tag] = P._LAST_GRADS[0]
    for a in ('hip-bf16', 'eager-bf16'):
        for i, net in enumerate(('D', 'G')):
            rows, skipped = P._cosine_report(out[a][i], out['fp32'][i], 1e-3)
            if not rows:
                continue
            print('%-24s %-10s vs fp32 %s: %d tensors, worst %s' % (
                spec, a, net, len(rows), ['%.3f %s' % (c, n[-60:]) for c, n, _ in rows[:5]]),
                flush=True)
    for i, net in enumerate(('D', 'G')):
        rows, _ = P._cosine_report(out['hip-bf16'][i], out['eager-bf16'][i], 1e-3)
        if rows:
            print('%-24s hip-bf16 vs eager-bf16 %s: worst %s' % (
                spec, net, ['%.3f %s' % (c, n[-60:]) for c, n, _ in rows[:5]]), flush=True)


if __name__ == '__main__':
    for spec in sys.argv[1:]:
        run(spec)
