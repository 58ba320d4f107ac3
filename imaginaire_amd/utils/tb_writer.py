"""Minimal TensorBoard event-file writer (no tensorboard/tensorflow dependency).

Writes ``events.out.tfevents.*`` records (TFRecord framing with masked
CRC32-C, hand-encoded ``Event``/``Summary`` protobufs) for scalars, so the
reference's TensorBoard scalar logging (utils/meters.py:54-104) keeps working
on images that ship without tensorboard. Images/hparams are written as scalar
placeholders + PNG files next to the event file.
"""
import os
import socket
import struct
import time

_CRC_TABLE = None


def _crc32c_table():
    global _CRC_TABLE
    if _CRC_TABLE is None:
        poly = 0x82F63B78
        table = []
        for i in range(256):
            c = i
            for _ in range(8):
                c = (c >> 1) ^ poly if c & 1 else c >> 1
            table.append(c)
        _CRC_TABLE = table
    return _CRC_TABLE


def crc32c(data):
    table = _crc32c_table()
    crc = 0xFFFFFFFF
    for b in data:
        crc = table[(crc ^ b) & 0xFF] ^ (crc >> 8)
    return crc ^ 0xFFFFFFFF


def _masked_crc(data):
    crc = crc32c(data)
    return (((crc >> 15) | (crc << 17)) + 0xA282EAD8) & 0xFFFFFFFF


def _varint(n):
    out = bytearray()
    while True:
        b = n & 0x7F
        n >>= 7
        if n:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _field(num, wire, payload):
    return _varint((num << 3) | wire) + payload


def _bytes_field(num, b):
    return _field(num, 2, _varint(len(b)) + b)


def _event(step, wall_time, summary=None, file_version=None):
    msg = _field(1, 1, struct.pack('<d', wall_time))
    msg += _field(2, 0, _varint(step & 0xFFFFFFFFFFFFFFFF))
    if file_version is not None:
        msg += _bytes_field(3, file_version.encode())
    if summary is not None:
        msg += _bytes_field(5, summary)
    return msg


def _scalar_summary(tag, value):
    val = _bytes_field(1, tag.encode()) + _field(2, 5, struct.pack('<f', float(value)))
    return _bytes_field(1, val)


class SummaryWriter(object):
    def __init__(self, log_dir):
        os.makedirs(log_dir, exist_ok=True)
        name = 'events.out.tfevents.%d.%s' % (int(time.time()), socket.gethostname())
        self.path = os.path.join(log_dir, name)
        self.log_dir = log_dir
        self._f = open(self.path, 'ab')
        self._write(_event(0, time.time(), file_version='brain.Event:2'))

    def _write(self, data):
        header = struct.pack('<Q', len(data))
        self._f.write(header + struct.pack('<I', _masked_crc(header)) + data +
                      struct.pack('<I', _masked_crc(data)))

    def add_scalar(self, tag, value, step):
        self._write(_event(int(step), time.time(), summary=_scalar_summary(tag, value)))
        self._f.flush()

    def add_histogram(self, tag, values, step):
        import numpy as np
        v = np.asarray(values.detach().cpu() if hasattr(values, 'detach') else values)
        self.add_scalar(tag + '/mean', float(v.mean()), step)
        self.add_scalar(tag + '/std', float(v.std()), step)

    def add_image(self, tag, img, step):
        from imaginaire_amd.utils.visualization.common import tensor2pilimage
        path = os.path.join(self.log_dir, 'images', '%s_%09d.png' % (tag, step))
        os.makedirs(os.path.dirname(path), exist_ok=True)
        tensor2pilimage(img, minus1to1_normalized=False).save(path)

    def flush(self):
        self._f.flush()

    def close(self):
        self._f.close()


def read_scalars(path):
    """Parse scalars back from an event file (used by tests)."""
    out = []
    with open(path, 'rb') as f:
        data = f.read()
    pos = 0
    while pos + 12 <= len(data):
        (n,) = struct.unpack('<Q', data[pos:pos + 8])
        rec = data[pos + 12:pos + 12 + n]
        pos += 12 + n + 4
        # extremely small protobuf walker for Event.summary.value.{tag, simple_value}
        i, step = 0, None
        while i < len(rec):
            key, i = _read_varint(rec, i)
            num, wire = key >> 3, key & 7
            if wire == 0:
                val, i = _read_varint(rec, i)
                if num == 2:
                    step = val
            elif wire == 1:
                i += 8
            elif wire == 5:
                i += 4
            elif wire == 2:
                ln, i = _read_varint(rec, i)
                payload = rec[i:i + ln]
                i += ln
                if num == 5:
                    out.extend((t, v, step) for t, v in _parse_summary(payload))
    return out


def _read_varint(b, i):
    shift = result = 0
    while True:
        byte = b[i]
        i += 1
        result |= (byte & 0x7F) << shift
        if not byte & 0x80:
            return result, i
        shift += 7


def _parse_summary(payload):
    res = []
    i = 0
    while i < len(payload):
        key, i = _read_varint(payload, i)
        ln, i = _read_varint(payload, i)
        val = payload[i:i + ln]
        i += ln
        j, tag, sv = 0, None, None
        while j < len(val):
            k, j = _read_varint(val, j)
            num, wire = k >> 3, k & 7
            if wire == 2:
                l2, j = _read_varint(val, j)
                if num == 1:
                    tag = val[j:j + l2].decode()
                j += l2
            elif wire == 5:
                if num == 2:
                    sv = struct.unpack('<f', val[j:j + 4])[0]
                j += 4
            elif wire == 0:
                _, j = _read_varint(val, j)
            elif wire == 1:
                j += 8
        res.append((tag, sv))
    return res
