"""Failure detection / recovery (imaginaire_amd/utils/health.py): hang watchdog, fault
injection, straggler report, crash + auto-resume through train.py."""
import os
import socket
import subprocess
import sys

import pytest
import yaml

from imaginaire_amd.utils.health import CRASH_EXIT_CODE, FaultInjector, StragglerMonitor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _env(**kw):
    env = dict(os.environ, OMP_NUM_THREADS='2', PYTHONPATH=ROOT)
    env.pop('IMAGINAIRE_AMD_FAULT', None)
    env.update(kw)
    return env


def test_fault_spec_parsing():
    f = FaultInjector('hang@5:1, nan@3', rank=1)
    assert f.faults == [('hang', 5, 1), ('nan', 3, None)]
    assert f._due(5) == ['hang'] and f._due(3) == ['nan'] and f._due(4) == []
    assert FaultInjector('hang@5:1', rank=0)._due(5) == []
    assert not FaultInjector('', rank=0)
    with pytest.raises(ValueError):
        FaultInjector('explode@1', rank=0)


def test_nan_injection_poisons_inputs():
    import torch
    data = {'images': torch.zeros(2, 3, 4, 4), 'label': torch.ones(2, 5, 4, 4), 'key': 'x'}
    FaultInjector('nan@7', rank=0).apply(7, data)
    assert torch.isnan(data['images']).all() and torch.isnan(data['label']).all()


def test_straggler_monitor_single_process():
    m = StragglerMonitor()
    for _ in range(3):
        m.tick()
    slow, t, med, ratio = m.report()
    assert slow == 0 and ratio == 1.0 and t >= 0


def test_watchdog_dumps_stacks_and_exits(tmp_path):
    """A loop that stops beating: the native faulthandler thread writes the report and
    ends the process even though the main thread is blocked."""
    code = ('import time\n'
            'from imaginaire_amd.utils.health import Watchdog\n'
            'w = Watchdog(1.0, %r, first_timeout=1.0)\n'
            'w.beat(7)\n'
            'def stuck_in_collective():\n'
            '    time.sleep(60)\n'
            'stuck_in_collective()\n' % str(tmp_path))
    r = subprocess.run([sys.executable, '-c', code], env=_env(), capture_output=True,
                       text=True, timeout=60)
    assert r.returncode != 0
    rep = open(os.path.join(str(tmp_path), 'hang_rank0.txt')).read()
    assert 'no progress within 1 s after iteration 7' in rep
    assert 'stuck_in_collective' in rep


def test_watchdog_clean_exit_leaves_no_report(tmp_path):
    from imaginaire_amd.utils.health import Watchdog
    with Watchdog(30, str(tmp_path)) as w:
        w.beat(1)
        w.beat(2)
    assert not os.path.exists(os.path.join(str(tmp_path), 'hang_rank0.txt'))


def test_watchdog_grace_covers_slow_phase(tmp_path):
    """A phase longer than the steady-state bound (snapshot save / FID) under grace does
    not fire; a plain iteration that stalls afterwards still does."""
    code = ('import time\n'
            'from imaginaire_amd.utils.health import Watchdog\n'
            'w = Watchdog(1.0, %r, first_timeout=8.0)\n'
            'w.beat(1)\n'
            'w.beat(2)\n'
            'with w.grace(2, "write_metrics"):\n'
            '    time.sleep(2.5)\n'
            'print("survived", flush=True)\n'
            'def stalled_iteration():\n'
            '    time.sleep(60)\n'
            'stalled_iteration()\n' % str(tmp_path))
    r = subprocess.run([sys.executable, '-c', code], env=_env(), capture_output=True,
                       text=True, timeout=60)
    assert 'survived' in r.stdout
    assert r.returncode != 0
    rep = open(os.path.join(str(tmp_path), 'hang_rank0.txt')).read()
    assert 'after write_metrics' in rep and 'stalled_iteration' in rep


def test_train_py_slow_end_of_iteration_under_watchdog(tmp_path):
    """train.py with a 1 s watchdog and an end_of_iteration (checkpoint + metrics) that
    takes 2.5 s: the run finishes instead of being killed mid-eval."""
    cfg = _cfg(tmp_path, max_iter=3, snapshot_save_iter=2, logging_iter=1)
    logdir = os.path.join(str(tmp_path), 'log')
    code = ('import sys, time\n'
            'sys.argv = ["train.py", "--config", %r, "--logdir", %r, "--single_gpu",\n'
            '            "--watchdog-timeout", "1", "--watchdog-grace", "600"]\n'
            'from imaginaire_amd.trainers.base import BaseTrainer\n'
            '_orig = BaseTrainer.end_of_iteration\n'
            'def slow(self, *a, **k):\n'
            '    time.sleep(2.5)\n'
            '    return _orig(self, *a, **k)\n'
            'BaseTrainer.end_of_iteration = slow\n'
            'import train\n'
            'train.main()\n' % (cfg, logdir))
    r = subprocess.run([sys.executable, '-c', code], cwd=ROOT, env=_env(),
                       capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stderr[-3000:]
    assert 'Done with training' in r.stdout


def _cfg(tmp_path, **over):
    with open(os.path.join(ROOT, 'configs', 'unit_test', 'spade.yaml')) as f:
        cfg = yaml.safe_load(f)
    cfg.update(over)
    p = os.path.join(str(tmp_path), 'cfg.yaml')
    with open(p, 'w') as f:
        yaml.safe_dump(cfg, f)
    return p


def test_crash_then_auto_resume(tmp_path):
    """crash@3 after the iteration-2 checkpoint: the restarted job resumes at 2 and
    finishes (recovery = restart + latest_checkpoint.txt, reference trainers/base.py:225)."""
    cfg = _cfg(tmp_path, max_iter=4, snapshot_save_iter=2, logging_iter=1)
    logdir = os.path.join(str(tmp_path), 'log')
    cmd = [sys.executable, 'train.py', '--config', cfg, '--logdir', logdir, '--single_gpu']
    r = subprocess.run(cmd, cwd=ROOT, env=_env(IMAGINAIRE_AMD_FAULT='crash@2'),
                       capture_output=True, text=True, timeout=900)
    assert r.returncode == CRASH_EXIT_CODE, r.stderr[-3000:]
    assert '[fault-inject] rank 0: crash at iteration 2' in r.stderr
    with open(os.path.join(logdir, 'latest_checkpoint.txt')) as f:
        assert 'iteration_000000002' in f.read()
    assert not [f for f in os.listdir(logdir) if f.endswith('.tmp')]
    r = subprocess.run(cmd, cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stderr[-3000:]
    assert 'Load from:' in r.stdout and 'Done with training' in r.stdout
    with open(os.path.join(logdir, 'latest_checkpoint.txt')) as f:
        assert 'iteration_000000004' in f.read()


def test_two_rank_hang_is_detected(tmp_path):
    """Rank 1 hangs at iteration 2; rank 0 blocks in its next collective. Both watchdogs
    fire, the job ends non-zero instead of hanging, and rank 1's report names the stall."""
    cfg = _cfg(tmp_path, max_iter=6)
    logdir = os.path.join(str(tmp_path), 'log')
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node', '2',
           '--master-addr', '127.0.0.1', '--master-port', str(_free_port()), 'train.py',
           '--config', cfg, '--backend', 'gloo', '--logdir', logdir,
           '--watchdog-timeout', '45', '--watchdog-grace', '60']
    r = subprocess.run(cmd, cwd=ROOT, env=_env(IMAGINAIRE_AMD_FAULT='hang@2:1'),
                       capture_output=True, text=True, timeout=900)
    assert r.returncode != 0
    rep1 = open(os.path.join(logdir, 'hang_rank1.txt')).read()
    # the header names the last completed iteration (2) and the phase that followed it
    header = rep1.splitlines()[0]
    assert header.startswith('rank 1: no progress') and ' 2 (beat' in header, rep1
    assert 'health.py' in rep1, rep1
    assert os.path.exists(os.path.join(logdir, 'hang_rank0.txt'))
