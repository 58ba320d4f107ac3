"""Host-side logic of the graphed-step helpers (utils/cuda_graph.py), no GPU needed:
graph_routing nests and restores, the static-batch copy ignores entries the captured step added
to its static batch, and batch signatures separate structures."""
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
