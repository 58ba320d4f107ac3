"""Parallelism for MI355X nodes: RCCL data parallel (ddp), process groups."""
from .ddp import DistributedDataParallel, WrappedModel  # noqa: F401
from .groups import get_syncbn_group, set_syncbn_group  # noqa: F401
