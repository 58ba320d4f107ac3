"""Minimal TensorBoard event-file writer (no tensorboard/tensorflow dependency).

Writes ``events.out.tfevents.*`` records (TFRecord framing with masked
CRC32-C, hand-encoded ``Event``/``Summary`` protobufs) so the reference's
TensorBoard logging (utils/meters.py:54-159: scalars, histograms, the
"Visualizations" image grid and the hparams plugin's experiment / session
start / session end summaries) keeps working on images that ship without
tensorboard. Field numbers follow tensorflow's ``summary.proto`` /
``histogram.proto`` and tensorboard's ``plugins/hparams/{api,plugin_data}.proto``.
``read_events`` parses the records back (tests).
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


def _double(num, v):
    return _field(num, 1, struct.pack('<d', float(v)))


def _scalar_summary(tag, value):
    val = _bytes_field(1, tag.encode()) + _field(2, 5, struct.pack('<f', float(value)))
    return _bytes_field(1, val)


def _image_summary(tag, png, height, width, channels):
    # Summary.Image {height=1, width=2, colorspace=3, encoded_image_string=4}
    img = (_field(1, 0, _varint(height)) + _field(2, 0, _varint(width)) +
           _field(3, 0, _varint(channels)) + _bytes_field(4, png))
    return _bytes_field(1, _bytes_field(1, tag.encode()) + _bytes_field(4, img))


def _histogram_summary(tag, values, bins=64):
    import numpy as np
    v = np.asarray(values, dtype=np.float64).reshape(-1)
    v = v[np.isfinite(v)]
    if v.size == 0:
        v = np.zeros(1)
    counts, edges = np.histogram(v, bins=bins)
    # HistogramProto {min=1, max=2, num=3, sum=4, sum_squares=5, bucket_limit=6, bucket=7};
    # bucket i counts values in (bucket_limit[i-1], bucket_limit[i]]
    limits = struct.pack('<%dd' % bins, *edges[1:].tolist())
    buckets = struct.pack('<%dd' % bins, *counts.astype(np.float64).tolist())
    h = (_double(1, v.min()) + _double(2, v.max()) + _double(3, v.size) + _double(4, v.sum()) +
         _double(5, (v * v).sum()) + _bytes_field(6, limits) + _bytes_field(7, buckets))
    return _bytes_field(1, _bytes_field(1, tag.encode()) + _bytes_field(5, h))


def _pb_value(v):
    """google.protobuf.Value {number_value=2, string_value=3, bool_value=4}."""
    if isinstance(v, bool):
        return _field(4, 0, _varint(int(v)))
    if isinstance(v, (int, float)):
        return _double(2, v)
    return _bytes_field(3, str(v).encode())


def _hparams_summaries(hparam_dict, metric_dict):
    """The three summaries of tensorboard's hparams plugin (what
    ``torch.utils.tensorboard.summary.hparams`` returns; reference meters.py:67-104)."""
    infos = b''
    for k, v in hparam_dict.items():
        # HParamInfo {name=1, type=4}: DATA_TYPE_STRING=1, BOOL=2, FLOAT64=3
        dtype = 2 if isinstance(v, bool) else 3 if isinstance(v, (int, float)) else 1
        infos += _bytes_field(4, _bytes_field(1, k.encode()) + _field(4, 0, _varint(dtype)))
    for k in metric_dict:
        # MetricInfo {name=1: MetricName {tag=2}}
        infos += _bytes_field(5, _bytes_field(1, _bytes_field(2, k.encode())))
    experiment = infos
    ssi = b''
    for k, v in hparam_dict.items():
        ssi += _bytes_field(1, _bytes_field(1, k.encode()) + _bytes_field(2, _pb_value(v)))
    ssi += _double(5, time.time())
    sei = _field(1, 0, _varint(1)) + _double(2, time.time())  # STATUS_SUCCESS

    def wrap(tag, field, payload):
        plugin_content = _field(1, 0, _varint(0)) + _bytes_field(field, payload)
        meta = _bytes_field(1, _bytes_field(1, b'hparams') + _bytes_field(2, plugin_content))
        return _bytes_field(1, _bytes_field(1, tag.encode()) + _bytes_field(9, meta))

    return [wrap('_hparams_/experiment', 2, experiment),
            wrap('_hparams_/session_start_info', 3, ssi),
            wrap('_hparams_/session_end_info', 4, sei)]


def _encode_png(img):
    """[C,H,W] / [H,W,C] / [H,W] float (0..1) or uint8 image -> (png bytes, H, W, C)."""
    import io

    import numpy as np
    from PIL import Image
    a = img.detach().float().cpu().numpy() if hasattr(img, 'detach') else np.asarray(img)
    if a.ndim == 3 and a.shape[0] in (1, 3, 4) and a.shape[2] not in (1, 3, 4):
        a = a.transpose(1, 2, 0)
    if a.ndim == 2:
        a = a[:, :, None]
    if a.dtype != np.uint8:
        a = (np.clip(a, 0, 1) * 255 + 0.5).astype(np.uint8)
    h, w, c = a.shape
    buf = io.BytesIO()
    Image.fromarray(a[:, :, 0] if c == 1 else a).save(buf, format='PNG')
    return buf.getvalue(), h, w, c


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

    def add_histogram(self, tag, values, step, bins=64):
        if hasattr(values, 'detach'):
            values = values.detach().float().cpu().numpy()
        self._write(_event(int(step), time.time(), summary=_histogram_summary(tag, values, bins)))
        self._f.flush()

    def add_image(self, tag, img, step):
        """``img``: [C,H,W] in [0,1] (torch's ``dataformats='CHW'`` default) or uint8."""
        png, h, w, c = _encode_png(img)
        self._write(_event(int(step), time.time(), summary=_image_summary(tag, png, h, w, c)))
        self._f.flush()

    def add_hparams(self, hparam_dict, metric_dict):
        for summ in _hparams_summaries(hparam_dict, metric_dict):
            self._write(_event(0, time.time(), summary=summ))
        for k, v in metric_dict.items():
            self.add_scalar(k, v, 0)
        self._f.flush()

    def flush(self):
        self._f.flush()

    def close(self):
        self._f.close()


def _records(path):
    with open(path, 'rb') as f:
        data = f.read()
    pos = 0
    while pos + 12 <= len(data):
        (n,) = struct.unpack('<Q', data[pos:pos + 8])
        if struct.unpack('<I', data[pos + 8:pos + 12])[0] != _masked_crc(data[pos:pos + 8]):
            raise ValueError('corrupt record header at %d' % pos)
        rec = data[pos + 12:pos + 12 + n]
        if struct.unpack('<I', data[pos + 12 + n:pos + 16 + n])[0] != _masked_crc(rec):
            raise ValueError('corrupt record at %d' % pos)
        pos += 12 + n + 4
        yield rec


def _fields(buf):
    """Generic protobuf walk: yields (field number, wire type, value) — value is an int
    (varint), raw bytes (fixed64/fixed32) or the payload (length-delimited)."""
    i = 0
    while i < len(buf):
        key, i = _read_varint(buf, i)
        num, wire = key >> 3, key & 7
        if wire == 0:
            val, i = _read_varint(buf, i)
        elif wire == 1:
            val, i = buf[i:i + 8], i + 8
        elif wire == 5:
            val, i = buf[i:i + 4], i + 4
        elif wire == 2:
            ln, i = _read_varint(buf, i)
            val, i = buf[i:i + ln], i + ln
        else:
            raise ValueError('unsupported wire type %d' % wire)
        yield num, wire, val


def read_events(path):
    """All summary values of an event file as dicts {step, tag, kind, ...}: kind 'scalar'
    (value), 'image' (height, width, channels, png), 'histogram' (min, max, num, sum,
    buckets) or 'plugin' (plugin, content)."""
    out = []
    for rec in _records(path):
        step, summary = 0, None
        for num, wire, val in _fields(rec):
            if num == 2 and wire == 0:
                step = val
            elif num == 5 and wire == 2:
                summary = val
        if summary is None:
            continue
        for num, _, value in _fields(summary):
            if num != 1:
                continue
            ev = {'step': step}
            for vn, vw, vv in _fields(value):
                if vn == 1:
                    ev['tag'] = vv.decode()
                elif vn == 2 and vw == 5:
                    ev.update(kind='scalar', value=struct.unpack('<f', vv)[0])
                elif vn == 4:
                    img = {n: v for n, _, v in _fields(vv)}
                    ev.update(kind='image', height=img.get(1), width=img.get(2),
                              channels=img.get(3), png=img.get(4))
                elif vn == 5:
                    h = {}
                    for hn, _, hv in _fields(vv):
                        h[hn] = hv
                    bk = h.get(7, b'')
                    ev.update(kind='histogram', min=struct.unpack('<d', h[1])[0],
                              max=struct.unpack('<d', h[2])[0],
                              num=struct.unpack('<d', h[3])[0],
                              sum=struct.unpack('<d', h[4])[0],
                              buckets=list(struct.unpack('<%dd' % (len(bk) // 8), bk)))
                elif vn == 9:
                    pd = dict((n, v) for n, _, v in _fields(vv)).get(1, b'')
                    pdd = dict((n, v) for n, _, v in _fields(pd))
                    ev.update(kind='plugin', plugin=pdd.get(1, b'').decode(),
                              content=pdd.get(2, b''))
            out.append(ev)
    return out


def read_scalars(path):
    """(tag, value, step) of every scalar in an event file (used by tests)."""
    return [(e['tag'], e['value'], e['step']) for e in read_events(path)
            if e.get('kind') == 'scalar']


def _read_varint(b, i):
    shift = result = 0
    while True:
        byte = b[i]
        i += 1
        result |= (byte & 0x7F) << shift
        if not byte & 0x80:
            return result, i
        shift += 7
