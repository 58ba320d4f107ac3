"""Who calls the channel pad / cast pass (``pad_channels_cast``, the ``pad_cast_kernel`` rows of
the recipe kernel tables)? Wraps the extension entry point, runs scripts/bench_families.py
in-process with the given arguments (eager: no --graph, so every call goes through Python), and
prints the calls per iteration grouped by (input shape, dtype, padded channels, call site).

    python scripts/probe/pad_cast_sites.py --config configs/unit_test/fs_vid2vid_face.yaml ...
"""
import collections
import os
import sys
import traceback

HERE = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, 'scripts'))

import imaginaire_amd._C as C  # noqa: E402

_orig = C.pad_channels_cast
_calls = collections.Counter()
_bytes = collections.Counter()


def _site():
    frames = [f for f in traceback.extract_stack()[:-2] if 'imaginaire_amd' in f.filename]
    return ' <- '.join('%s:%d' % (os.path.relpath(f.filename, HERE), f.lineno)
                       for f in frames[::-1][:3])


def _wrapped(x, cp, dtype):
    key = (tuple(x.shape), str(x.dtype).replace('torch.', ''), int(cp),
           'cl' if x.is_contiguous(memory_format=__import__('torch').channels_last) else 'nchw',
           _site())
    _calls[key] += 1
    _bytes[key] += x.numel() * x.element_size()
    return _orig(x, cp, dtype)


C.pad_channels_cast = _wrapped

import bench_families  # noqa: E402

iters = None
for i, a in enumerate(sys.argv):
    if a == '--steps':
        iters = int(sys.argv[i + 1])
    if a == '--warmup':
        iters = (iters or 0) + int(sys.argv[i + 1])
sys.argv = ['bench_families.py'] + sys.argv[1:]
try:
    bench_families.main()
except SystemExit:
    pass
n = max(1, iters or 1)
tot = sum(_calls.values())
print('pad_channels_cast: %d calls over %d iterations (%.1f per iteration)' % (tot, n, tot / n))
for key, c in sorted(_calls.items(), key=lambda kv: -_bytes[kv[0]]):
    shape, dt, cp, lay, site = key
    print('%7.1f/it %8.1f MB/it  %-22s %-8s -> %4d ch %-4s  %s'
          % (c / n, _bytes[key] / n / 1e6, shape, dt, cp, lay, site))
