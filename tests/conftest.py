import os
import sys

# before anything in this process starts HIP (collection below calls torch.cuda.is_available):
# the runtime reads this once at start-up, and imaginaire_amd refuses graph capture when HIP
# started with packet capture on (profiles/r6/README_graph_root_cause.txt)
os.environ.setdefault('DEBUG_CLR_GRAPH_PACKET_CAPTURE', '0')

import pytest  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: test needs an MI355X (HIP) GPU')
    config.addinivalue_line('markers', 'slow: long-running test')


def pytest_collection_modifyitems(config, items):
    import torch
    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason='no GPU available')
    for item in items:
        if 'gpu' in item.keywords:
            item.add_marker(skip)
