"""Count the ``pad_channels_cast`` launches (ops/conv.py ``_pad_channels``) of one eager SPADE
training step by Python call site and operand shape (GPU). Used to compare routing variants,
e.g. ``IMAGINAIRE_AMD_SN_FUSED=0`` vs ``1``.

    python scripts/probe/pad_sites_probe.py [--config ...]
"""
import argparse
import collections
import os
import sys
import traceback

HERE = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, HERE)

import torch  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument('--config', default=os.path.join(HERE, 'configs', 'bench',
                                                    'spade_256x512_synthetic.yaml'))
    args = p.parse_args()
    from imaginaire_amd.config import Config
    from imaginaire_amd.utils.trainer import get_model_optimizer_and_scheduler, get_trainer
    from imaginaire_amd.datasets.synthetic import DeviceBatchSource
    torch.cuda.set_device(0)
    cfg = Config(args.config)
    cfg.logdir = '/tmp/iamd_padsites'
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
    record_ext_sites(lambda: step(2), ('pad_channels_cast',))


def record_ext_sites(step_fn, names, out=sys.stdout, depth=3):
    """Run ``step_fn`` once with the listed extension functions wrapped: count their calls by
    (function, Python call site, first operand's shape) and print the table to ``out``."""
    from imaginaire_amd.ops import _ext
    stats = collections.Counter()
    ext = _ext.ext()

    class Shim(object):
        def __getattr__(self, name):
            fn = getattr(ext, name)
            if name not in names:
                return fn

            def wrapped(*a, **k):
                fr = [f for f in traceback.extract_stack()[:-1] if HERE in f.filename]
                site = ' <- '.join('%s:%d' % (os.path.relpath(f.filename, HERE), f.lineno)
                                   for f in fr[-depth:][::-1])
                shape = tuple(a[0].shape) if a and torch.is_tensor(a[0]) else ()
                stats[(name, site, shape)] += 1
                return fn(*a, **k)
            return wrapped
    shim = Shim()
    old = _ext.ext
    _ext.ext = lambda: shim
    try:
        step_fn()
        torch.cuda.synchronize()
    finally:
        _ext.ext = old
    print('extension calls (%s): %d' % (','.join(names), sum(stats.values())), file=out)
    for (name, site, shape), n in stats.most_common():
        print('%5d  %-18s %-26s %s' % (n, name, shape, site), file=out)


if __name__ == '__main__':
    main()
