"""Image / array decoding shared by the LMDB and folder handles
(reference datasets/lmdb.py:36-75, datasets/folder.py:29-82).

OpenCV is not part of this stack; PIL decodes the same formats: 8-bit
JPEG/PNG (RGB/RGBA/L) and 16-bit TIFF/PNG (returned as uint16, which
``BaseDataset.to_tensor`` scales by 1/65535 like the fork). Arrays come back
HxWxC (HxW for single-channel), RGB channel order.
"""
import io

import numpy as np
from PIL import Image

from imaginaire_amd.utils.data import IMG_EXTENSIONS


def decode_image(buf, ext):
    img = Image.open(io.BytesIO(buf))
    if 'tif' in ext.lower() or img.mode in ('I;16', 'I;16B', 'I;16L', 'I'):
        arr = np.array(img)
        if arr.dtype != np.uint16 and img.mode.startswith('I'):
            arr = arr.astype(np.uint16)
        return arr
    if ext.lower() in ('jpg', 'jpeg'):
        return np.array(img.convert('RGB'))
    if img.mode == 'P':
        return np.array(img)  # palette index maps (segmentation labels)
    if img.mode not in ('RGB', 'RGBA', 'L'):
        img = img.convert('RGB')
    return np.array(img)


def decode_numpy(buf):
    arr = np.load(io.BytesIO(buf), allow_pickle=False)
    if arr.ndim == 3 and arr.shape[2] >= 2:
        # fork convention (datasets/folder.py:78-79): the first two channels are stored (y, x)
        arr = arr.copy()
        arr[:, :, :2] = arr[:, :, 1::-1]
    return arr


def decode(buf, ext):
    if ext in IMG_EXTENSIONS:
        return decode_image(buf, ext)
    if ext is not None and 'npy' in ext:
        return decode_numpy(buf)
    return buf
