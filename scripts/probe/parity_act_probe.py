"""Where does a HIP-bf16 training iteration leave PyTorch-bf16? Records every leaf module's
forward output and output gradient (module forward / full backward hooks on net_G and net_D) in
one iteration of tests/test_model_parity_gpu.py run three ways — HIP kernels under bf16
autocast, PyTorch ops under bf16 autocast with im2col convs, and the same with MIOpen convs —
and prints, in execution order, the modules whose HIP tensors are further from PyTorch-bf16
than the two PyTorch-bf16 runs are from each other (the first forward row is where the
forward diverges; the first backward row, read from the loss end, where the backward does).

    python scripts/probe/parity_act_probe.py vid2vid_street.yaml [seq_len] [max_rows]
"""
import os
import sys
import tempfile

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests'))
import test_model_parity_gpu as P  # noqa: E402
import imaginaire_amd.utils.trainer as T  # noqa: E402


ALL = os.environ.get('ACT_ALL', '1') == '1'  # composite modules too (post-order)


def _cos(a, b):
    a, b = a.reshape(-1).double(), b.reshape(-1).double()
    return float(torch.dot(a, b) / (a.norm() * b.norm()).clamp_min(1e-30))


def record(config, amp, eager, tmp, seq_len, cudnn=None):
    rec = []  # (kind, name, call, tensor) in execution order
    calls = {}
    orig = T.get_trainer

    def first(t):
        if torch.is_tensor(t):
            return t
        if isinstance(t, (tuple, list)):
            for v in t:
                r = first(v)
                if r is not None:
                    return r
        if isinstance(t, dict):
            for v in t.values():
                r = first(v)
                if r is not None:
                    return r
        return None

    def hooked(cfg, net_G, net_D, *a, **kw):
        tr = orig(cfg, net_G, net_D, *a, **kw)
        for tag, net in (('G', tr.net_G), ('D', tr.net_D)):
            for name, m in net.named_modules():
                if not name or (not ALL and len(list(m.children()))):
                    continue
                key = tag + ':' + name.replace('module.', '')

                def fwd(mod, inp, out, key=key):
                    t = first(out)
                    if t is None or not t.is_floating_point():
                        return
                    c = calls.get(('f', key), 0)
                    calls[('f', key)] = c + 1
                    rec.append(('fwd', key, c, t.detach().float().cpu()))
                    if t.requires_grad:
                        # a tensor hook (not a module backward hook: no output wrapping, so the
                        # models' in-place activations stay legal)
                        def bwd(g, key=key, c=c):
                            if g is not None:
                                rec.append(('bwd', key, c, g.detach().float().cpu()))
                        t.register_hook(bwd)
                m.register_forward_hook(fwd)
        return tr
    T.get_trainer = hooked
    try:
        P._iteration(config, amp, eager, tmp, seq_len=seq_len, cudnn=cudnn)
    finally:
        T.get_trainer = orig
    return rec


def main():
    config = sys.argv[1]
    seq = int(sys.argv[2]) if len(sys.argv) > 2 else None
    rows = int(sys.argv[3]) if len(sys.argv) > 3 else 40
    tmp = tempfile.mkdtemp()
    hip = record(config, 'O1', False, os.path.join(tmp, 'h'), seq)
    e16 = record(config, 'O1', True, os.path.join(tmp, 'e'), seq)
    e16b = record(config, 'O1', True, os.path.join(tmp, 'b'), seq, cudnn=True)
    idx = {(k, n, c): t for k, n, c, t in e16}
    idxb = {(k, n, c): t for k, n, c, t in e16b}
    out = []
    for order, (k, n, c, t) in enumerate(hip):
        a, b = idx.get((k, n, c)), idxb.get((k, n, c))
        if a is None or b is None or a.shape != t.shape or b.shape != t.shape:
            continue
        if float(a.norm()) == 0:
            continue
        ch = max(_cos(t, a), _cos(t, b))
        cm = _cos(a, b)
        out.append((order, k, n, c, ch, cm, float(t.norm()), float(a.norm())))
    print('%d hip records, %d compared' % (len(hip), len(out)))
    dump = os.environ.get('ACT_DUMP')  # 'a:b': every compared row with execution index in [a, b)
    if dump:
        a, b = (int(v) for v in dump.split(':'))
        for r in out:
            if a <= r[0] < b:
                print('  =%5d %s %-70s call %d  cos(hip, torch) %.6f  mutual %.6f  |hip| %.5g '
                      '|torch| %.5g' % r)
    bad = [r for r in out if (1 - r[4]) > 3 * (1 - r[5]) + 1e-3]
    print('rows where HIP is further from torch-bf16 than 3x the torch-bf16 mutual distance '
          '(execution order):')
    for r in bad[:rows]:
        print('  #%5d %s %-70s call %d  cos(hip, torch) %.5f  mutual %.5f  |hip| %.4g |torch| %.4g'
              % r)
    print('last backward rows (loss end first):')
    bw = [r for r in bad if r[1] == 'bwd']
    for r in bw[:rows]:
        print('  #%5d %s %-70s call %d  cos(hip, torch) %.5f  mutual %.5f  |hip| %.4g |torch| %.4g'
              % r)


if __name__ == '__main__':
    main()
