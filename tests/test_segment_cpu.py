"""Instance-wise average pooling of the pix2pixHD feature encoder (ops/segment.py) vs the
reference's per-instance loop (reference generators/pix2pixHD.py:323-349)."""
import torch


def _reference(features, instance_map):
    out = torch.empty_like(features)
    for b in range(features.shape[0]):
        for v in instance_map[b].unique():
            m = instance_map[b, 0] == v
            for c in range(features.shape[1]):
                out[b, c][m] = features[b, c][m].mean()
    return out


def test_instance_mean_matches_reference_loop():
    from imaginaire_amd.ops.segment import instance_mean
    torch.manual_seed(0)
    f = torch.randn(3, 4, 12, 10)
    inst = (torch.randint(0, 6, (3, 1, 12, 10)) * 1000 + 26).float()
    inst[1] = 26.0  # one sample with a single instance
    torch.testing.assert_close(instance_mean(f, inst), _reference(f, inst), atol=1e-6, rtol=1e-5)
