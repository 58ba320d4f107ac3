"""Convolution-library flags (reference utils/cudnn.py:10-22).

On ROCm ``torch.backends.cudnn`` drives MIOpen. ``benchmark=True`` makes
MIOpen run an *exhaustive* kernel search per conv problem, which for a SPADE
step (~100 conv problems x fwd/bwd-data/bwd-weight) costs many minutes on a
fresh machine. We therefore honour ``cfg.cudnn.benchmark`` only when
``IMAGINAIRE_AMD_MIOPEN_TUNE=1``; otherwise MIOpen uses its heuristic /
find-db path, which also picks up the tuned records shipped in
``tuning/miopen`` (see ``setup_miopen_db``).
"""
import os

import torch
import torch.backends.cudnn as cudnn

from imaginaire_amd.utils.distributed import master_only_print as print

_REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
MIOPEN_DB_DIR = os.path.join(_REPO, 'tuning', 'miopen')


def setup_miopen_db():
    """Point MIOpen's user find/perf db at the in-repo tuning records.

    Must run before the first convolution (env is read at MIOpen handle
    creation). A user-provided ``MIOPEN_USER_DB_PATH`` wins.
    """
    if 'MIOPEN_USER_DB_PATH' not in os.environ and os.path.isdir(MIOPEN_DB_DIR):
        os.environ['MIOPEN_USER_DB_PATH'] = MIOPEN_DB_DIR


def miopen_tune_requested():
    return os.environ.get('IMAGINAIRE_AMD_MIOPEN_TUNE', '0') == '1'


def init_cudnn(deterministic, benchmark):
    setup_miopen_db()
    if torch.version.hip is not None and benchmark and not miopen_tune_requested():
        benchmark = False
    cudnn.deterministic = deterministic
    cudnn.benchmark = benchmark
    print('cudnn/MIOpen benchmark: {}'.format(benchmark))
    print('cudnn/MIOpen deterministic: {}'.format(deterministic))
