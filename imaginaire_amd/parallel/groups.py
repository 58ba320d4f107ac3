"""Process-group management.

SyncBatchNorm statistics exchanges are tiny (≤16 KB) and latency-bound; the
gradient all-reduces are hundreds of MB. On one communicator RCCL serialises
them on one stream, so a SyncBN all-reduce issued during the generator
backward would queue behind a 256 MB gradient bucket. SyncBN therefore gets
its own communicator (``get_syncbn_group``), i.e. its own HIP stream.
"""
import torch.distributed as dist

_SYNCBN_GROUP = None


def set_syncbn_group(group):
    global _SYNCBN_GROUP
    _SYNCBN_GROUP = group


def get_syncbn_group():
    """Dedicated group for SyncBN statistics (created lazily, collectively)."""
    global _SYNCBN_GROUP
    if _SYNCBN_GROUP is None and dist.is_available() and dist.is_initialized() and \
            dist.get_world_size() > 1:
        _SYNCBN_GROUP = dist.new_group(ranks=list(range(dist.get_world_size())))
    return _SYNCBN_GROUP


def assign_syncbn_group(module, group=None):
    """Point every SyncBatchNorm in ``module`` at the dedicated group."""
    from imaginaire_amd.layers.activation_norm import SyncBatchNorm
    group = group if group is not None else get_syncbn_group()
    for m in module.modules():
        if isinstance(m, SyncBatchNorm):
            m.process_group = group
