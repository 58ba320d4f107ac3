"""Per-parameter gradient norms of one training iteration, HIP bf16 vs eager fp32, for a unit
config (tests/test_model_parity_gpu.py helper): prints the parameters whose gradient norms
differ most.

    python scripts/probe/parity_grads_probe.py fs_vid2vid_face.yaml 2 [k]
"""
import os
import sys

import torch

HERE = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, 'tests'))
import test_model_parity_gpu as T  # noqa: E402


def grads(config, amp, eager, seq_len, overrides):
    norms = {}
    orig = T._grad_norms

    def capture(net, *args):
        for n, p in net.named_parameters():
            if p.grad is not None:
                norms[n] = float(p.grad.float().norm())
        return orig(net, *args)
    T._grad_norms = capture
    try:
        T._iteration(config, amp, eager, '/tmp/pgp_%d' % int(eager), seq_len=seq_len,
                     overrides=overrides)
    finally:
        T._grad_norms = orig
    return norms


cfg = sys.argv[1]
seq = int(sys.argv[2]) if len(sys.argv) > 2 else None
ov = [('data.initial_few_shot_K', int(sys.argv[3]))] if len(sys.argv) > 3 else []
h = grads(cfg, 'O1', False, seq, ov)
r = grads(cfg, 'O0', True, seq, ov)
rows = sorted(((abs(h[k] - r.get(k, 0.0)), k, h[k], r.get(k, 0.0)) for k in h), reverse=True)
for d, k, a, b in rows[:30]:
    print('%10.4g  hip %10.4g  fp32 %10.4g  %s' % (d, a, b, k))
