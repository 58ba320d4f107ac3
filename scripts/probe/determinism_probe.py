"""Run the SPADE unit iteration of tests/test_determinism_gpu.py N times and print losses."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests'))
import torch  # noqa: E402

from test_determinism_gpu import _one_iteration  # noqa: E402


def main():
    from imaginaire_amd.config import Config
    from imaginaire_amd.datasets.synthetic import DeviceBatchSource
    torch.use_deterministic_algorithms(True, warn_only=True)
    cfg = Config(os.path.join(ROOT, 'configs', 'unit_test', 'spade.yaml'))
    src = DeviceBatchSource(cfg, 2, torch.device('cuda', 0), pool=1, seed=3)
    data = src.next()
    runs = []
    for r in range(int(sys.argv[1]) if len(sys.argv) > 1 else 3):
        losses, state = _one_iteration(data)
        runs.append((losses, state))
        print('run', r, {k: round(float(v), 6) for k, v in sorted(losses.items())})
    s0 = runs[0][1]
    for r in range(1, len(runs)):
        diff = [k for k in s0 if not torch.equal(s0[k], runs[r][1][k])]
        print('run', r, 'vs 0: %d tensors differ' % len(diff), diff[:8])


if __name__ == '__main__':
    main()
