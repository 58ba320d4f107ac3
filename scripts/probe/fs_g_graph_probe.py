"""fs_vid2vid generator alone in a hipGraph: one forward of net_G on a unit-config batch and a
random-projection loss, backward, captured and replayed several times; report the parameters
whose gradients are non-finite or differ from an eager run of the same computation.
Switches: IAMD_PROBE_PART=label_embedding|weight_generator (capture only that sub-module on
recorded inputs).

    python scripts/probe/fs_g_graph_probe.py
"""
import os
import sys

import torch

HERE = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, 'tests'))
from test_graph_families_gpu import _build  # noqa: E402

torch.cuda.set_device(0)
torch.use_deterministic_algorithms(True, warn_only=True)
cfg, tr, batches = _build('fs_vid2vid_face', 2)
G = tr.net_G.module.module if hasattr(tr.net_G.module, 'module') else tr.net_G.module
part = os.environ.get('IAMD_PROBE_PART', 'weight_generator.label_embedding')
mod = G
if part != 'G':
    for a in part.split('.'):
        mod = getattr(mod, a)
wg = G.weight_generator
rec = {}
orig_fwd = mod.forward


def recording(*a, **k):
    rec.setdefault('args', (a, k))
    return orig_fwd(*a, **k)


mod.forward = recording
from imaginaire_amd.utils.cuda_graph import make_trainer_step  # noqa: E402
step, _ = make_trainer_step(tr, enabled=False)
step(tr.start_of_iteration(batches[0], 0))
torch.cuda.synchronize()
mod.forward = orig_fwd
args, kwargs = rec['args']


def detach_all(x):
    if torch.is_tensor(x):
        return x.detach().clone().requires_grad_(x.requires_grad and x.is_floating_point())
    if isinstance(x, (list, tuple)):
        return type(x)(detach_all(v) for v in x)
    if isinstance(x, dict):
        return {k: detach_all(v) for k, v in x.items()}
    return x


args, kwargs = detach_all(args), detach_all(kwargs)
leaves = []


def collect(x):
    if torch.is_tensor(x):
        if x.requires_grad:
            leaves.append(x)
    elif isinstance(x, (list, tuple)):
        for v in x:
            collect(v)
    elif isinstance(x, dict):
        for v in x.values():
            collect(v)


collect(args)
collect(kwargs)
params = [p for p in mod.parameters() if p.requires_grad]
names = [n for n, p in mod.named_parameters() if p.requires_grad]
print('part %s: %d params, %d differentiable inputs' % (part, len(params), len(leaves)))
torch.manual_seed(7)
projs = {}


def flat_outputs(o):
    out = []
    if torch.is_tensor(o):
        out.append(o)
    elif isinstance(o, (list, tuple)):
        for v in o:
            out += flat_outputs(v)
    return out


def body():
    with torch.autocast('cuda', dtype=torch.bfloat16):
        outs = flat_outputs(mod(*args, **kwargs))
    loss = 0
    for i, o in enumerate(outs):
        if not o.is_floating_point() or not o.requires_grad:
            continue
        if i not in projs:
            projs[i] = torch.randn(o.shape, device=o.device)
        loss = loss + (o.float() * projs[i]).sum()
    loss.backward()


def zero():
    for t in params + leaves:
        t.grad = None


def grads():
    return [None if t.grad is None else t.grad.detach().float().clone() for t in params + leaves]


from imaginaire_amd.utils.cuda_graph import graph_routing  # noqa: E402
st = torch.cuda.Stream()
st.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(st), graph_routing():
    for _ in range(2):
        zero()
        body()
torch.cuda.current_stream().wait_stream(st)
torch.cuda.synchronize()
zero()
with graph_routing():
    body()
torch.cuda.synchronize()
ref = grads()
for t in params + leaves:  # static grads for the graph
    t.grad = torch.zeros_like(t)
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g, stream=st), graph_routing():
    body()
torch.cuda.synchronize()
allnames = names + ['input%d' % i for i in range(len(leaves))]
for rep in range(4):
    for t in params + leaves:
        t.grad.zero_()
    g.replay()
    torch.cuda.synchronize()
    got = grads()
    bad = [n for n, a in zip(allnames, got) if a is not None and not torch.isfinite(a).all()]
    diff = [(float((a - b).abs().max()) / max(1e-12, float(b.abs().max())), n)
            for n, a, b in zip(allnames, got, ref) if a is not None and b is not None]
    diff.sort(reverse=True)
    print('replay %d: non-finite %d %s | worst rel diff %s' % (rep, len(bad), bad[:4], diff[:3]),
          flush=True)
