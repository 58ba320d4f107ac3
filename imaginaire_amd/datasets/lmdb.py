"""LMDB data-type handle (reference datasets/lmdb.py:17-79) on the native
mmap reader (csrc/lmdb_io.cpp): zero-copy page access, no locks, safe to
share across forked DataLoader workers."""
import json
import os

import torch.utils.data as data

from imaginaire_amd.datasets.decode import decode
from imaginaire_amd.utils.data import IMG_EXTENSIONS  # noqa: F401 (re-export)
from imaginaire_amd.utils.distributed import master_only_print as print


class LMDBDataset(data.Dataset):
    def __init__(self, root):
        from imaginaire_amd.ops import _ext
        self.root = os.path.expanduser(root)
        self.env = _ext.ext().LmdbReader(self.root)
        self.length = len(self.env)
        with open(os.path.join(self.root, '..', 'metadata.json')) as fin:
            self.extensions = json.load(fin)
        print('LMDB file at %s opened.' % root)

    def getitem_by_path(self, path, data_type):
        buf = self.env.get(path if isinstance(path, bytes) else path.encode())
        if buf is None:
            raise KeyError('%s not in %s' % (path, self.root))
        return decode(buf, self.extensions[data_type])

    def __len__(self):
        return self.length
