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
"""
import os

os.environ.setdefault('DEBUG_CLR_GRAPH_PACKET_CAPTURE', '0')
