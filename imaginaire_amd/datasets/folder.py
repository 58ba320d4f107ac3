"""Folder data-type handle (reference datasets/folder.py:15-86): files at
``<root>/<sequence>/<filename>.<ext>``."""
import os

import torch.utils.data as data

from imaginaire_amd.datasets.decode import decode
from imaginaire_amd.utils.distributed import master_only_print as print


class FolderDataset(data.Dataset):
    def __init__(self, root, metadata):
        self.root = os.path.expanduser(root)
        self.extensions = metadata
        self.length = 0
        print('Folder at %s opened.' % root)

    def getitem_by_path(self, path, data_type):
        ext = self.extensions[data_type]
        path = path.decode() if isinstance(path, bytes) else path
        filepath = os.path.join(self.root, path + '.' + ext)
        assert os.path.exists(filepath), '%s does not exist' % filepath
        with open(filepath, 'rb') as f:
            return decode(f.read(), ext)

    def __len__(self):
        return self.length
