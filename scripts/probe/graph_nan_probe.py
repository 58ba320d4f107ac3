"""Bisect non-finite parameter updates of a hipGraph-replayed training iteration: capture the
family's step (unit-test config), replay once, list the G parameters whose update or gradient
is not finite. Run under different kernel switches (IMAGINAIRE_AMD_WGRAD_V2=0,
IMAGINAIRE_AMD_CONV_V4=0, ...) to find the kernel that reads memory it never wrote.

    python scripts/probe/graph_nan_probe.py pix2pixHD
"""
import os
import sys

import torch

HERE = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, 'tests'))
from test_graph_families_gpu import _build, _fresh  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else 'pix2pixHD'
seq = int(sys.argv[2]) if len(sys.argv) > 2 else None
from imaginaire_amd.utils.cuda_graph import make_trainer_step  # noqa: E402
torch.cuda.set_device(0)
torch.use_deterministic_algorithms(True, warn_only=True)
if os.environ.get('IAMD_PROBE_DET') == '1':  # MIOpen: deterministic (non-atomic) solvers
    torch.backends.cudnn.deterministic = True
cfg, tr, batches = _build(name, seq)
step, graphed = make_trainer_step(tr, warmup=2, enabled=True)
for i in range(3):
    torch.manual_seed(3)
    step(tr.start_of_iteration(_fresh(batches[i % 2]), i))
torch.cuda.synchronize()
names = [n for n, _ in tr.net_G.named_parameters()]
params = list(tr.net_G.parameters())
p0 = [p.detach().clone() for p in params]
for it in range(3):
    d = tr.start_of_iteration(_fresh(batches[1]), 3 + it)
    graphed(d)
    torch.cuda.synchronize()
    bad = [(n, p.shape) for n, p, q in zip(names, params, p0) if not torch.isfinite(p).all()]
    badg = [n for n, p in zip(names, params) if p.grad is not None and not torch.isfinite(p.grad).all()]
    print('replay %d: non-finite params %d %s | non-finite grads %d' % (
        it, len(bad), bad[:4], len(badg)), flush=True)
    for n in badg:
        print('    bad grad', n.replace('module.module.', ''))
    from imaginaire_amd.ops import conv as _C
    rep = _C.ps_check_report()
    nb = [r for r in rep if not r[1]]
    print('    per-sample checks: %d, non-finite %d: %s' % (len(rep), len(nb), nb[:12]))
    if bad:
        break
