"""Attribute the ATen glue of one SPADE training step to Python call sites (GPU).

    python scripts/probe/op_sites.py [--config ...] [--ops copy_,cat,...]

A TorchDispatchMode records every listed aten op of one steady-state step (forward and
the autograd engine's backward thread) with its output bytes and the innermost repository
frames of the Python stack; the table is sorted by bytes moved.
"""
import argparse
import collections
import os
import sys
import threading
import traceback

HERE = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, HERE)

import torch  # noqa: E402
from torch.utils._python_dispatch import TorchDispatchMode  # noqa: E402


DEFAULT_OPS = ('copy_,_to_copy,cat,fill_,add_,add,mul,div,flip,upsample_nearest2d,'
               'upsample_bilinear2d,avg_pool2d,clone,sub,mul_,zero_,constant_pad_nd,contiguous,'
               'reflection_pad2d,index,grid_sampler_2d,sum,mean')


def main():
    p = argparse.ArgumentParser()
    p.add_argument('--config', default=os.path.join(HERE, 'configs', 'bench',
                                                    'spade_256x512_synthetic.yaml'))
    p.add_argument('--ops', default=DEFAULT_OPS)
    p.add_argument('--top', type=int, default=60)
    args = p.parse_args()
    from imaginaire_amd.config import Config
    from imaginaire_amd.utils.trainer import get_model_optimizer_and_scheduler, get_trainer
    from imaginaire_amd.datasets.synthetic import DeviceBatchSource
    torch.cuda.set_device(0)
    cfg = Config(args.config)
    cfg.logdir = '/tmp/iamd_opsites'
    nets = get_model_optimizer_and_scheduler(cfg, seed=0)
    tr = get_trainer(cfg, *nets, train_data_loader=[], val_data_loader=None)
    src = DeviceBatchSource(cfg, cfg.data.train.batch_size, torch.device('cuda', 0), pool=4)

    def step(i):
        d = tr.start_of_iteration(src.next(), i)
        tr.dis_update(d)
        tr.gen_update(d)

    for i in range(2):
        step(i)
    torch.cuda.synchronize()
    record_sites(lambda: step(2), args.ops, args.top)


def record_sites(step_fn, ops=DEFAULT_OPS, top=60, out=sys.stdout):
    """Run ``step_fn`` once under a dispatch-mode recorder of the listed aten ops; print the
    call sites sorted by output bytes (forward and the autograd engine's backward thread)."""
    wanted = set(ops.split(','))
    stats = collections.defaultdict(lambda: [0, 0])
    lock = threading.Lock()

    def site():
        fr = [f for f in traceback.extract_stack()
              if HERE in f.filename and 'op_sites' not in f.filename]
        return ' <- '.join('%s:%d' % (os.path.relpath(f.filename, HERE), f.lineno)
                           for f in reversed(fr[-3:])) or '<backward/engine>'

    class Mode(TorchDispatchMode):
        def __torch_dispatch__(self, func, types, args=(), kwargs=None):
            out_ = func(*args, **(kwargs or {}))
            name = func.__name__.split('.')[0]
            # '@fp32': every op (any name) whose output is a large fp32 tensor (>= 2M elements):
            # finds the forward producers of fp32 activations in a bf16 step
            if ('@fp32' in wanted and torch.is_tensor(out_) and out_.dtype == torch.float32 and
                    out_.numel() >= (1 << 21)) or name in wanted:
                t = out_ if torch.is_tensor(out_) else (args[0] if args and torch.is_tensor(
                    args[0]) else None)
                nbytes = t.numel() * t.element_size() if t is not None else 0
                shape = tuple(t.shape) if t is not None else ()
                dt = str(t.dtype).replace('torch.', '') if t is not None else ''
                with lock:
                    s = stats[(name, shape, dt, site())]
                    s[0] += 1
                    s[1] += nbytes
            return out_

    # the backward engine runs on its own thread: enable the mode there too
    torch.autograd.graph.set_warn_on_accumulate_grad_stream_mismatch(False)
    with Mode():
        step_fn()
    torch.cuda.synchronize()
    rows = sorted(stats.items(), key=lambda kv: -kv[1][1])
    tot = sum(v[1] for _, v in rows)
    print('recorded %d op calls, %.2f GB output' % (sum(v[0] for _, v in rows), tot / 1e9),
          file=out)
    for (name, shape, dt, st), (n, b) in rows[:top]:
        print('%8.1f MB %4d  %-20s %-9s %-26s %s' % (b / 1e6, n, name, dt, str(shape)[:26], st),
              file=out)
    # launch-count view: small ops cost a kernel each whatever their bytes
    by_site = collections.defaultdict(lambda: [0, 0])
    for (name, shape, dt, st), (n, b) in rows:
        s = by_site[(name, dt, st)]
        s[0] += n
        s[1] += b
    print('\nby call count (op, dtype, site; all shapes):', file=out)
    for (name, dt, st), (n, b) in sorted(by_site.items(), key=lambda kv: -kv[1][0])[:top]:
        print('%5d %9.1f MB  %-20s %-9s %s' % (n, b / 1e6, name, dt, st), file=out)


if __name__ == '__main__':
    main()
