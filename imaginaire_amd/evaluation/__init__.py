from .fid import compute_fid, compute_fid_data  # noqa: F401
from .kid import compute_kid, compute_kid_data  # noqa: F401
from .prdc import compute_prdc  # noqa: F401

__all__ = ['compute_fid', 'compute_kid', 'compute_prdc', 'compute_fid_data', 'compute_kid_data']
