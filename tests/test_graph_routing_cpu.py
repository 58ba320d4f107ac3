"""Host-side logic of the graphed-step helpers (utils/cuda_graph.py), no GPU needed:
graph_routing nests and restores, the static-batch copy ignores entries the captured step added
to its static batch, and batch signatures separate structures."""
import os

import torch


def test_graph_routing_nests_and_restores():
    from imaginaire_amd.ops import conv
    from imaginaire_amd.utils.cuda_graph import graph_routing
    assert conv._GRAPH_ROUTING[0] == 0
    with graph_routing():
        assert conv._GRAPH_ROUTING[0] == 1
        with graph_routing():
            assert conv._GRAPH_ROUTING[0] == 2
        assert conv._GRAPH_ROUTING[0] == 1
    assert conv._GRAPH_ROUTING[0] == 0
    try:
        with graph_routing():
            raise RuntimeError('x')
    except RuntimeError:
        pass
    assert conv._GRAPH_ROUTING[0] == 0


def test_static_copy_ignores_graph_added_keys():
    from imaginaire_amd.utils.cuda_graph import _static_copy
    dst = {'images': torch.zeros(2, 3), 'z': torch.zeros(2, 8), 'nested': [torch.zeros(1)]}
    src = {'images': torch.ones(2, 3), 'nested': [torch.full((1,), 2.0)]}
    _static_copy(dst, src)  # 'z' was added by the captured step: an output, not an input
    assert torch.equal(dst['images'], torch.ones(2, 3))
    assert torch.equal(dst['z'], torch.zeros(2, 8))
    assert float(dst['nested'][0]) == 2.0


def test_signature_separates_structures():
    from imaginaire_amd.utils.cuda_graph import _signature
    a = {'x': torch.zeros(2, 3), 'key': 'file_a'}
    b = {'x': torch.zeros(2, 3), 'key': 'file_b'}  # names never steer the computation
    c = {'x': torch.zeros(3, 3), 'key': 'file_a'}
    assert _signature(a) == _signature(b)
    assert _signature(a) != _signature(c)


def test_packet_capture_guard_refuses_unless_off(monkeypatch):
    """utils/cuda_graph.py refuses to capture when the runtime's packet-capture mode is (or may
    be) on: HIP started before the package import with the variable unset, or an explicit
    non-zero value (imaginaire_amd.PACKET_CAPTURE_STATE); the probe override captures anyway."""
    import imaginaire_amd
    from imaginaire_amd.utils import cuda_graph as G
    monkeypatch.delenv('IMAGINAIRE_AMD_GRAPH_ALLOW_PACKET_CAPTURE', raising=False)
    monkeypatch.setattr(imaginaire_amd, 'PACKET_CAPTURE_STATE', 'off')
    assert G.packet_capture_refusal() is None
    monkeypatch.setattr(imaginaire_amd, 'PACKET_CAPTURE_STATE', 'unknown')
    r = G.packet_capture_refusal()
    assert r is not None and 'before imaginaire_amd was imported' in r
    monkeypatch.setattr(imaginaire_amd, 'PACKET_CAPTURE_STATE', 'on')
    assert 'DEBUG_CLR_GRAPH_PACKET_CAPTURE' in G.packet_capture_refusal()
    monkeypatch.setenv('IMAGINAIRE_AMD_GRAPH_ALLOW_PACKET_CAPTURE', '1')
    assert G.packet_capture_refusal() is None


def test_packet_capture_state_detects_late_import():
    """A process that initialised HIP (torch.cuda) before importing the package is flagged
    'unknown' (run in a fresh interpreter with a stub torch whose cuda reports initialised)."""
    import subprocess
    import sys
    code = ('import sys, types, os\n'
            'os.environ.pop("DEBUG_CLR_GRAPH_PACKET_CAPTURE", None)\n'
            't = types.ModuleType("torch"); t.cuda = types.SimpleNamespace('
            'is_initialized=lambda: True)\n'
            'sys.modules["torch"] = t\n'
            'import imaginaire_amd\n'
            'print(imaginaire_amd.PACKET_CAPTURE_STATE)\n')
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = subprocess.run([sys.executable, '-c', code], cwd=root, capture_output=True, text=True,
                         timeout=60)
    assert out.stdout.strip().endswith('unknown'), (out.stdout, out.stderr[-1000:])
