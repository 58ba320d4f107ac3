"""Native Motion-JPEG mp4 demux/decode for the few-shot native-video dataset
(datasets/mp4.py; reference datasets/paired_few_shot_videos_native.py:117-150 decodes through
torchvision/PyAV, which this stack lacks). Round trips files written by the module's own muxer
(no reference fixture holds an mp4: parity with a third-party decoder is unpinned)."""
import numpy as np
import pytest

from imaginaire_amd.datasets import mp4
from imaginaire_amd.datasets.paired_few_shot_videos_native import read_video_frames


def _frames(t=5, h=48, w=64):
    rng = np.random.default_rng(0)
    base = np.linspace(0, 255, w, dtype=np.float32)[None, :, None]
    out = []
    for i in range(t):
        f = np.broadcast_to(base, (h, w, 3)).copy()
        f[:, :, 1] = (i * 40) % 256
        f[8:16, 8 + i:24 + i, 2] = 255
        out.append(np.clip(f + rng.normal(0, 2, f.shape), 0, 255).astype(np.uint8))
    return np.stack(out)


@pytest.mark.parametrize('per_chunk', [None, 2, 3])
def test_mjpeg_mp4_round_trip(per_chunk):
    frames = _frames()
    buf = mp4.write_mjpeg_mp4(frames, fps=25, samples_per_chunk=per_chunk)
    track = mp4.parse_video_track(buf)
    assert track['codec'] == b'jpeg' and (track['width'], track['height']) == (64, 48)
    assert len(track['samples']) == 5 and len(track['durations']) == 5
    out = read_video_frames(buf)
    assert out.shape == frames.shape and out.dtype == np.uint8
    assert np.abs(out.astype(np.int32) - frames).mean() < 4.0
    # frame order survives the chunk / run mapping
    for i in range(5):
        assert abs(int(out[i, :, :, 1].mean()) - (i * 40) % 256) < 6


def test_non_mjpeg_codec_names_the_codec():
    buf = bytearray(mp4.write_mjpeg_mp4(_frames(t=2)))
    i = buf.index(b'jpeg', buf.index(b'stsd'))
    buf[i:i + 4] = b'avc1'
    with pytest.raises(RuntimeError, match='avc1'):
        read_video_frames(bytes(buf))


def test_corrupt_files_raise_value_errors():
    buf = mp4.write_mjpeg_mp4(_frames(t=3))
    rng = np.random.default_rng(1)
    for cut in (10, len(buf) // 2, len(buf) - 7):
        with pytest.raises(ValueError):
            mp4.parse_video_track(buf[:cut])
    for _ in range(2000):  # flipped bytes: a clean ValueError or a (possibly wrong) parse
        b = bytearray(buf)
        for _ in range(4):
            b[int(rng.integers(0, len(b)))] = int(rng.integers(0, 256))
        try:
            mp4.parse_video_track(bytes(b))
        except ValueError:
            pass


def test_stsc_runs_must_advance():
    """A sample-to-chunk table whose runs do not start at increasing chunks is rejected
    up front (malformed clips must not cost O(runs x chunks) loader time)."""
    import struct
    import time
    buf = bytearray(mp4.write_mjpeg_mp4(_frames(t=5), samples_per_chunk=2))
    i = buf.index(b'stsc')
    n = struct.unpack_from('>I', buf, i + 8)[0]
    assert n >= 2
    # second run's first_chunk := first run's first_chunk
    struct.pack_into('>I', buf, i + 12 + 12, struct.unpack_from('>I', buf, i + 12)[0])
    t0 = time.perf_counter()
    with pytest.raises(ValueError, match='does not advance'):
        mp4.parse_video_track(bytes(buf))
    assert time.perf_counter() - t0 < 1.0
