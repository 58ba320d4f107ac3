"""Shared helpers of the download scripts: Google-Drive fetch + safe tar extraction."""
import os
import sys
import tarfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from imaginaire_amd.utils.io import download_file_from_google_drive  # noqa: E402,F401


def safe_extract(archive, dest):
    """Extract ``archive`` under ``dest`` refusing absolute paths, ``..`` and links that
    escape ``dest`` (tarfile.extractall alone trusts the archive)."""
    dest = os.path.realpath(dest)
    with tarfile.open(archive) as tar:
        members = []
        for m in tar.getmembers():
            target = os.path.realpath(os.path.join(dest, m.name))
            if not (target == dest or target.startswith(dest + os.sep)):
                raise ValueError('unsafe path in archive: %s' % m.name)
            if m.issym() or m.islnk():
                link = os.path.realpath(os.path.join(os.path.dirname(target), m.linkname))
                if not link.startswith(dest + os.sep):
                    raise ValueError('unsafe link in archive: %s' % m.name)
            if m.isdev():
                raise ValueError('device node in archive: %s' % m.name)
            members.append(m)
        tar.extractall(dest, members=members)
