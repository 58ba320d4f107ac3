"""imaginaire_amd: MI355X-native image / video GAN synthesis (the Imaginaire feature set).

HIP runtime setting applied at import (before any HIP call of a process that imports the
package first, as train.py / inference.py / bench.py do):

* ``DEBUG_CLR_GRAPH_PACKET_CAPTURE=0``: the ROCm runtime's graph "packet capture" mode (AQL
  packets of every kernel node pre-built at instantiation) made the replays of the few-shot
  vid2vid recipe's captured iteration — a graph of tens of thousands of nodes — read operands
  its predecessor nodes had not finished writing: the same tensor checked twice in a row inside
  one replay was non-finite, then finite (scripts/gpu/r5_fsnan4.sh with ``--op-probe``), and
  the recipe trained to NaN within 2-5 replays while the eager step from the same state stayed
  finite (``--ab-eager``). With packet capture off, 16 replays of the K = 1 and K = 2 recipes
  are finite, the in-graph checks all pass, and the SPADE step replays at the same speed
  (54.3 vs 54.5 images/s). An explicit value in the environment wins.

The runtime reads the variable once, when HIP starts. A process that started HIP before this
import (``torch.cuda`` used first) keeps the runtime default whatever ``os.environ`` says
afterwards: :data:`PACKET_CAPTURE_STATE` records what is actually in force, and
``utils/cuda_graph.py`` refuses to capture (running eagerly, with the reason printed) unless it
is ``'off'``.
"""
import os
import sys


def _hip_started():
    """True if this process has already initialised the HIP runtime through torch."""
    t = sys.modules.get('torch')
    if t is None:
        return False
    try:
        return bool(t.cuda.is_initialized())
    except Exception:  # noqa: BLE001 - a partially imported torch: nothing started yet
        return False


_PRESET = os.environ.get('DEBUG_CLR_GRAPH_PACKET_CAPTURE')
_HIP_STARTED_AT_IMPORT = _hip_started()
os.environ.setdefault('DEBUG_CLR_GRAPH_PACKET_CAPTURE', '0')
# 'off'       — the runtime starts (or started) with packet capture off;
# 'on'        — the variable was set to a non-zero value before this import;
# 'unknown'   — HIP was running before this import and the variable was unset then: the
#               runtime default (packet capture on) is in force.
if _PRESET is not None:
    PACKET_CAPTURE_STATE = 'off' if _PRESET == '0' else 'on'
elif _HIP_STARTED_AT_IMPORT:
    PACKET_CAPTURE_STATE = 'unknown'
else:
    PACKET_CAPTURE_STATE = 'off'
