"""Phase ranges for ROCm tracing (SURVEY §5 "Tracing / profiling").

``IMAGINAIRE_AMD_TRACE=1`` emits roctx ranges (``torch.cuda.nvtx`` maps to
roctx on ROCm builds) around each trainer phase — ``gen/forward``,
``gen/backward``, ``gen/step``, ``gen/ema``, ``dis/*`` — so
``rocprofv3 --marker-trace --kernel-trace`` attributes kernels to phases.
Disabled (zero overhead beyond one env lookup at import) otherwise.
"""
import contextlib
import os

import torch

_ENABLED = os.environ.get('IMAGINAIRE_AMD_TRACE', '0') == '1'


def enabled():
    return _ENABLED


@contextlib.contextmanager
def phase(name):
    if not _ENABLED or not torch.cuda.is_available():
        yield
        return
    try:
        torch.cuda.nvtx.range_push(name)
        pushed = True
    except Exception:  # noqa: BLE001 (roctx not available in this build)
        pushed = False
    try:
        yield
    finally:
        if pushed:
            torch.cuda.nvtx.range_pop()
