"""bench.py's own multi-rank launcher (``--gpus N`` without torchrun), on CPU / gloo.

The driver runs ``python bench.py --gpus N`` and, for N > 1, also the torchrun form; both
must report ``n_gpus == N`` and ``parallelism == dpN``."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(extra, env=None):
    cmd = [sys.executable, 'bench.py', '--device', 'cpu', '--config',
           'configs/unit_test/spade.yaml', '--batch', '1', '--steps', '1', '--warmup', '1'] + extra
    e = dict(os.environ, OMP_NUM_THREADS='2')
    e.pop('WORLD_SIZE', None)
    if env:
        e.update(env)
    return subprocess.run(cmd, cwd=ROOT, env=e, capture_output=True, text=True, timeout=600)


def test_bench_launches_two_ranks_itself():
    r = _run(['--gpus', '2'])
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith('{')]
    assert len(lines) == 1, r.stdout  # rank 0 only
    out = json.loads(lines[0])
    assert out['n_gpus'] == 2
    assert out['config']['parallelism'] == 'dp2'
    assert out['config']['global_batch'] == 2
    assert out['steps'] == 1 and out['warmup'] == 1
    assert out['value'] > 0
    assert out['losses_finite'] is True and out['replicas_in_sync'] is True


def test_bench_refuses_mismatched_world():
    r = _run(['--gpus', '4'], env={'WORLD_SIZE': '1', 'RANK': '0', 'LOCAL_RANK': '0'})
    assert r.returncode != 0
    assert 'refusing' in r.stderr


def test_bench_families_launches_two_ranks_video():
    """the video BASELINE configs have a multi-GPU entry point —
    ``scripts/bench_families.py --gpus N`` (own child launcher, as bench.py). Two gloo ranks on
    the vid2vid street unit config: one JSON row from rank 0, whole-job frames/s, finite losses
    and bitwise identical replicas after the timed steps."""
    cmd = [sys.executable, 'scripts/bench_families.py', '--cpu', '--gpus', '2', '--backend',
           'gloo', '--config', 'configs/unit_test/vid2vid_street.yaml', '--seq-len', '2',
           '--steps', '1', '--warmup', '1']
    e = dict(os.environ, OMP_NUM_THREADS='2')
    e.pop('WORLD_SIZE', None)
    r = subprocess.run(cmd, cwd=ROOT, env=e, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith('{')]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out['n_gpus'] == 2 and out['parallelism'] == 'dp2'
    assert out['frames_per_sample'] == 2
    assert out['losses_finite'] is True and out['replicas_in_sync'] is True
    assert abs(out['frames_per_s'] - 2 * out['batch'] * 2 * 1e3 / out['ms_per_iteration']) < \
        1e-2 * out['frames_per_s']
