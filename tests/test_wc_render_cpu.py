"""wc-vid2vid splat renderer vs numpy fancy-index semantics (reference
model_utils/wc_vid2vid/render.py:63-147: last write wins on duplicate targets)."""
import numpy as np
import torch

from imaginaire_amd.model_utils.wc_vid2vid.render import SplatRenderer, _last_rows


class _NumpyRenderer:
    """The reference algorithm in plain numpy (behavioural oracle)."""

    def __init__(self):
        self.colors = np.zeros((0, 3), np.uint8)
        self.seen_mask = np.zeros((0, 1), np.uint8)
        self.seen_time = np.zeros((0, 1), np.int64)
        self.call_idx = 0

    def _resize(self, n):
        if n > self.colors.shape[0]:
            pad = n - self.colors.shape[0]
            self.colors = np.concatenate([self.colors, np.zeros((pad, 3), np.uint8)])
            self.seen_mask = np.concatenate([self.seen_mask, np.zeros((pad, 1), np.uint8)])
            self.seen_time = np.concatenate([self.seen_time, np.zeros((pad, 1), np.int64)])

    def update(self, image, info):
        self.call_idx += 1
        i, j, p = info[:, 0], info[:, 1], info[:, 2]
        self._resize(p.max() + 1)
        self.colors[p] = self.seen_mask[p] * self.colors[p] + \
            (1 - self.seen_mask[p]) * image[i, j]
        self.seen_time[p] = self.seen_mask[p] * self.seen_time[p] + \
            (1 - self.seen_mask[p]) * self.call_idx
        self.seen_mask[p] = 1

    def render(self, info, w, h):
        out = np.zeros((h, w, 3), np.uint8)
        mask = np.zeros((h, w, 1), np.uint8)
        i, j, p = info[:, 0], info[:, 1], info[:, 2]
        self._resize(p.max() + 1)
        out[i, j] = self.colors[p]
        mask[i, j] = 255 * self.seen_mask[p]
        return out, mask


def test_last_rows():
    t = torch.tensor([3, 1, 3, 0, 1, 3])
    assert _last_rows(t, 4).tolist() == [False, False, False, True, True, True]


def test_renderer_matches_numpy_with_duplicates():
    rng = np.random.RandomState(0)
    h, w = 12, 16
    ours, ref = SplatRenderer(), _NumpyRenderer()
    for frame in range(4):
        image = rng.randint(0, 256, size=(h, w, 3)).astype(np.uint8)
        n = 150  # > h*w/2 rows over 40 point ids: many duplicate ids AND duplicate pixels
        info = np.stack([rng.randint(0, h, n), rng.randint(0, w, n),
                         rng.randint(0, 40 + 10 * frame, n)], 1)
        ours.update_point_cloud(image, info)
        ref.update(image, info)
        o, om = ours.render_image(info, w, h, return_mask=True)
        r, rm = ref.render(info, w, h)
        np.testing.assert_array_equal(o, r)
        np.testing.assert_array_equal(om, rm)
    n = ref.colors.shape[0]
    np.testing.assert_array_equal(ours.colors[:n].numpy(), ref.colors)
    np.testing.assert_array_equal(ours.seen_time[:n].numpy().astype(np.int64), ref.seen_time)
