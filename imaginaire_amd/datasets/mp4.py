"""Minimal ISO-BMFF (mp4 / mov) demuxer and Motion-JPEG muxer.

The reference's native few-shot video dataset decodes mp4 clips stored in LMDB through
torchvision / PyAV (reference datasets/paired_few_shot_videos_native.py:117-150); none of those
decoders ships with this stack. This module reads the container itself: it walks the box tree,
finds the video track, and maps every sample to its byte range (``stsz`` sizes, ``stco`` /
``co64`` chunk offsets, ``stsc`` chunk runs). Motion-JPEG tracks (``jpeg`` / ``mjpa`` /
``mjpb`` / ``MJPG`` sample entries — what ``ffmpeg -c:v mjpeg`` writes) are decoded frame by
frame with PIL; other codecs (H.264 / HEVC) need one of the optional decoders and raise an
error naming the codec. ``write_mjpeg_mp4`` produces such files (tests, dataset conversion).
"""
import io
import struct

import numpy as np
from PIL import Image

_CONTAINERS = {b'moov', b'trak', b'mdia', b'minf', b'stbl', b'dinf', b'edts', b'udta'}
MJPEG_CODECS = {b'jpeg', b'mjpa', b'mjpb', b'MJPG', b'AVDJ'}


def _boxes(buf, start, end):
    """Yield (type, payload_start, box_end) for the boxes in buf[start:end]."""
    pos = start
    while pos + 8 <= end:
        size, typ = struct.unpack_from('>I4s', buf, pos)
        hdr = 8
        if size == 1:
            if pos + 16 > end:
                raise ValueError('mp4: truncated 64-bit box header')
            size = struct.unpack_from('>Q', buf, pos + 8)[0]
            hdr = 16
        elif size == 0:
            size = end - pos
        if size < hdr or pos + size > end:
            raise ValueError('mp4: box %r at %d overruns its parent' % (typ, pos))
        yield typ, pos + hdr, pos + size
        pos += size


def _find(buf, start, end, path):
    """Payload ranges of every box reached by the type path (b'trak', b'mdia', ...)."""
    out = []
    for typ, a, b in _boxes(buf, start, end):
        if typ == path[0]:
            if len(path) == 1:
                out.append((a, b))
            elif typ in _CONTAINERS:
                out.extend(_find(buf, a, b, path[1:]))
    return out


def _u32s(buf, off, n):
    return struct.unpack_from('>%dI' % n, buf, off)


def parse_video_track(buf):
    """The first video track of an mp4 / mov: dict(codec, width, height, samples=[(off, size)],
    timescale, durations). Malformed files raise ValueError."""
    buf = memoryview(buf).tobytes() if not isinstance(buf, (bytes, bytearray)) else buf
    try:
        return _parse_video_track(buf)
    except (struct.error, IndexError) as e:
        raise ValueError('mp4: malformed sample tables (%s)' % e)


def _table(buf, box, head, entry):
    """(count, first entry offset) of a full-box table whose ``count`` u32 sits ``head`` bytes
    into the payload and whose entries are ``entry`` bytes, checked against the box end."""
    if box is None:
        raise ValueError('mp4: missing sample table box')
    a, b = box
    n = struct.unpack_from('>I', buf, a + head)[0]
    if a + head + 4 + n * entry > b:
        raise ValueError('mp4: table of %d entries overruns its box' % n)
    return n, a + head + 4


def _parse_video_track(buf):
    moovs = _find(buf, 0, len(buf), [b'moov'])
    if not moovs:
        raise ValueError('mp4: no moov box')
    for ta, tb in _find(buf, moovs[0][0], moovs[0][1], [b'trak']):
        hdlr = _find(buf, ta, tb, [b'mdia', b'hdlr'])
        if not hdlr or buf[hdlr[0][0] + 8:hdlr[0][0] + 12] != b'vide':
            continue
        mdhd = _find(buf, ta, tb, [b'mdia', b'mdhd'])
        stbl = _find(buf, ta, tb, [b'mdia', b'minf', b'stbl'])
        if not mdhd or not stbl:
            raise ValueError('mp4: video track without mdhd / stbl')
        ver = buf[mdhd[0][0]]
        timescale = struct.unpack_from('>I', buf, mdhd[0][0] + (20 if ver == 1 else 12))[0]
        a, b = stbl[0]

        def one(t):
            r = _find(buf, a, b, [t])
            return r[0] if r else None

        stsd = one(b'stsd')
        if stsd is None:
            raise ValueError('mp4: video track without stsd')
        # full box (4) + entry count (4), then the first sample entry: size, format, 6 reserved,
        # data ref index (2), 16 bytes pre-defined / reserved, width, height
        sd = stsd[0]
        if sd + 44 > stsd[1]:
            raise ValueError('mp4: short sample description')
        codec = bytes(buf[sd + 12:sd + 16])
        width, height = struct.unpack_from('>HH', buf, sd + 40)
        stsz = one(b'stsz')
        if stsz is None:
            raise ValueError('mp4: video track without stsz')
        fixed = struct.unpack_from('>I', buf, stsz[0] + 4)[0]
        if fixed:
            count = struct.unpack_from('>I', buf, stsz[0] + 8)[0]
            if count * fixed > len(buf):
                raise ValueError('mp4: %d samples of %d bytes exceed the file' % (count, fixed))
            sizes = [fixed] * count
        else:
            count, o = _table(buf, stsz, 8, 4)
            sizes = list(_u32s(buf, o, count))
        stco, co64 = one(b'stco'), one(b'co64')
        if stco is not None:
            n, o = _table(buf, stco, 4, 4)
            chunks = list(_u32s(buf, o, n))
        elif co64 is not None:
            n, o = _table(buf, co64, 4, 8)
            chunks = list(struct.unpack_from('>%dQ' % n, buf, o))
        else:
            raise ValueError('mp4: video track without chunk offsets')
        n, o = _table(buf, one(b'stsc'), 4, 12)
        runs = [_u32s(buf, o + 12 * i, 3) for i in range(n)]
        samples = []
        s = 0
        for i, (first, per_chunk, _) in enumerate(runs):
            if i + 1 < len(runs) and runs[i + 1][0] <= first:
                # chunk runs must start at strictly increasing chunk numbers; a malformed
                # table could otherwise cost O(runs x chunks) iterations
                raise ValueError('mp4: stsc run %d does not advance (first chunk %d -> %d)' % (
                    i, first, runs[i + 1][0]))
            last = runs[i + 1][0] - 1 if i + 1 < len(runs) else len(chunks)
            if first < 1 or last > len(chunks):
                raise ValueError('mp4: chunk run %d references missing chunks' % i)
            if per_chunk == 0:
                continue
            for c in range(first - 1, last):
                if s == count:
                    break
                off = chunks[c]
                for _ in range(min(per_chunk, count - s)):
                    samples.append((off, sizes[s]))
                    off += sizes[s]
                    s += 1
            if s == count:
                break
        if len(samples) != count:
            raise ValueError('mp4: sample table maps %d of %d samples' % (len(samples), count))
        for off, size in samples:
            if off + size > len(buf):
                raise ValueError('mp4: sample at %d+%d is past the end of the file' % (off, size))
        durations = []
        stts = one(b'stts')
        if stts is not None:
            n, o = _table(buf, stts, 4, 8)
            for i in range(n):
                cnt, delta = _u32s(buf, o + 8 * i, 2)
                durations.extend([delta] * min(cnt, count))
        return dict(codec=codec, width=width, height=height, samples=samples,
                    timescale=timescale, durations=durations[:count])
    raise ValueError('mp4: no video track')


def decode_mjpeg_mp4(buf):
    """Motion-JPEG mp4 / mov bytes -> uint8 [T, H, W, 3]."""
    track = parse_video_track(buf)
    if track['codec'] not in MJPEG_CODECS:
        raise RuntimeError('mp4: video codec %r needs torchvision.io, imageio or av '
                           '(only Motion-JPEG is decoded natively)' % track['codec'].decode(
                               'latin-1'))
    frames = []
    for off, size in track['samples']:
        with Image.open(io.BytesIO(buf[off:off + size])) as im:
            frames.append(np.asarray(im.convert('RGB')))
    return np.stack(frames)


def _box(typ, payload):
    return struct.pack('>I4s', 8 + len(payload), typ) + payload


def _full(typ, version, flags, payload):
    return _box(typ, struct.pack('>I', (version << 24) | flags) + payload)


_MATRIX = struct.pack('>9I', 0x10000, 0, 0, 0, 0x10000, 0, 0, 0, 0x40000000)


def write_mjpeg_mp4(frames, fps=30, quality=95, samples_per_chunk=None):
    """uint8 [T, H, W, 3] frames -> Motion-JPEG mp4 bytes (``jpeg`` sample entry; one chunk, or
    chunks of ``samples_per_chunk`` frames)."""
    frames = np.asarray(frames, dtype=np.uint8)
    t, h, w = frames.shape[:3]
    jpegs = []
    for f in frames:
        b = io.BytesIO()
        Image.fromarray(f).save(b, format='JPEG', quality=quality)
        jpegs.append(b.getvalue())
    timescale, delta = fps * 1000, 1000
    duration = t * delta
    ftyp = _box(b'ftyp', b'isom' + struct.pack('>I', 512) + b'isomiso2mp41')
    mdat_payload = b''.join(jpegs)
    mdat = _box(b'mdat', mdat_payload)
    data_off = len(ftyp) + 8
    mvhd = _full(b'mvhd', 0, 0, struct.pack('>IIIIIH10x', 0, 0, timescale, duration, 0x10000,
                                            0x100) + _MATRIX + b'\0' * 24 +
                 struct.pack('>I', 2))
    tkhd = _full(b'tkhd', 0, 3, struct.pack('>IIIII8xHHHH', 0, 0, 1, 0, duration, 0, 0, 0, 0) +
                 _MATRIX + struct.pack('>II', w << 16, h << 16))
    mdhd = _full(b'mdhd', 0, 0, struct.pack('>IIIIHH', 0, 0, timescale, duration, 0x55C4, 0))
    hdlr = _full(b'hdlr', 0, 0, struct.pack('>I4s12x', 0, b'vide') + b'VideoHandler\0')
    vmhd = _full(b'vmhd', 0, 1, struct.pack('>4H', 0, 0, 0, 0))
    dinf = _box(b'dinf', _full(b'dref', 0, 0, struct.pack('>I', 1) + _full(b'url ', 0, 1, b'')))
    name = b'Photo - JPEG'
    entry = _box(b'jpeg', b'\0' * 6 + struct.pack('>H', 1) + b'\0' * 16 +
                 struct.pack('>HHIIIH', w, h, 0x480000, 0x480000, 0, 1) +
                 bytes([len(name)]) + name + b'\0' * (31 - len(name)) +
                 struct.pack('>Hh', 24, -1))
    stsd = _full(b'stsd', 0, 0, struct.pack('>I', 1) + entry)
    stts = _full(b'stts', 0, 0, struct.pack('>III', 1, t, delta))
    per = min(t, samples_per_chunk or t)
    nfull, rem = divmod(t, per)
    runs = [(1, per)] + ([(nfull + 1, rem)] if rem else [])
    stsc = _full(b'stsc', 0, 0, struct.pack('>I', len(runs)) +
                 b''.join(struct.pack('>III', first, n, 1) for first, n in runs))
    chunk_starts, off = [], 0
    for i, j in enumerate(jpegs):
        if i % per == 0:
            chunk_starts.append(off)
        off += len(j)
    stsz = _full(b'stsz', 0, 0, struct.pack('>II', 0, t) +
                 struct.pack('>%dI' % t, *[len(j) for j in jpegs]))

    def moov_for(offset):
        stco = _full(b'stco', 0, 0, struct.pack('>I', len(chunk_starts)) +
                     b''.join(struct.pack('>I', offset + c) for c in chunk_starts))
        stbl = _box(b'stbl', stsd + stts + stsc + stsz + stco)
        minf = _box(b'minf', vmhd + dinf + stbl)
        mdia = _box(b'mdia', mdhd + hdlr + minf)
        return _box(b'moov', mvhd + _box(b'trak', tkhd + mdia))

    return ftyp + mdat + moov_for(data_off)
