"""Process-group helpers (reference utils/distributed.py:11-93).

One process per GPU; the backend is ``nccl`` (which is RCCL on ROCm, riding
xGMI inside a node) on GPU and ``gloo`` on CPU-only hosts. Rank/world come from
the ``torchrun`` environment (``RANK``/``LOCAL_RANK``/``WORLD_SIZE``).
"""
import functools
import os

import torch
import torch.distributed as dist


def init_dist(local_rank=None, backend=None, **kwargs):
    """Initialise the default process group from ``env://``.

    ``backend=None`` picks ``nccl`` (RCCL) when a GPU is present and ``gloo``
    otherwise. Returns the local device index (or -1 on CPU).
    """
    if local_rank is None:
        local_rank = int(os.environ.get('LOCAL_RANK', 0))
    use_gpu = torch.cuda.is_available()
    if backend is None:
        backend = 'nccl' if use_gpu else 'gloo'
    if not dist.is_available():
        return local_rank
    if dist.is_initialized():
        return torch.cuda.current_device() if use_gpu else -1
    if use_gpu:
        torch.cuda.set_device(local_rank)
    os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
    os.environ.setdefault('MASTER_PORT', '29500')
    if backend == 'nccl' and use_gpu:
        kwargs.setdefault('device_id', torch.device('cuda', local_rank))
        # a collective that exceeds the timeout aborts the communicator and raises instead
        # of blocking every rank forever (utils/health.py)
        os.environ.setdefault('TORCH_NCCL_ASYNC_ERROR_HANDLING', '3')
    from imaginaire_amd.utils.health import dist_timeout
    kwargs.setdefault('timeout', dist_timeout())
    dist.init_process_group(backend=backend, init_method='env://', **kwargs)
    return local_rank if use_gpu else -1


def is_dist():
    return dist.is_available() and dist.is_initialized()


def get_rank():
    return dist.get_rank() if is_dist() else 0


def get_world_size():
    return dist.get_world_size() if is_dist() else 1


def master_only(func):
    """Run ``func`` only on rank 0 (reference utils/distributed.py:38-47)."""
    @functools.wraps(func)
    def wrapper(*args, **kwargs):
        if get_rank() == 0:
            return func(*args, **kwargs)
        return None
    return wrapper


def is_master():
    return get_rank() == 0


@master_only
def master_only_print(*args, **kwargs):
    print(*args, **kwargs)


def barrier():
    if is_dist():
        dist.barrier()


def dist_reduce_tensor(tensor):
    """Reduce to rank 0 and average there (reference utils/distributed.py:61-70)."""
    world_size = get_world_size()
    if world_size < 2:
        return tensor
    with torch.no_grad():
        dist.reduce(tensor, dst=0)
        if get_rank() == 0:
            tensor /= world_size
    return tensor


def dist_all_reduce_tensor(tensor):
    """All-reduce and average in place (reference utils/distributed.py:73-81)."""
    world_size = get_world_size()
    if world_size < 2:
        return tensor
    with torch.no_grad():
        dist.all_reduce(tensor)
        tensor.div_(world_size)
    return tensor


def dist_all_gather_tensor(tensor):
    """All-gather equally sized tensors (reference utils/distributed.py:84-93)."""
    world_size = get_world_size()
    if world_size < 2:
        return [tensor]
    tensor_list = [torch.ones_like(tensor) for _ in range(world_size)]
    with torch.no_grad():
        dist.all_gather(tensor_list, tensor)
    return tensor_list


def dist_all_gather_variable(tensor):
    """All-gather tensors whose first dimension differs across ranks."""
    world_size = get_world_size()
    if world_size < 2:
        return [tensor]
    n = torch.tensor([tensor.shape[0]], device=tensor.device, dtype=torch.long)
    sizes = [torch.zeros_like(n) for _ in range(world_size)]
    dist.all_gather(sizes, n)
    sizes = [int(s.item()) for s in sizes]
    max_n = max(sizes)
    pad = tensor.new_zeros((max_n - tensor.shape[0],) + tuple(tensor.shape[1:]))
    padded = torch.cat([tensor, pad], 0)
    out = [torch.zeros_like(padded) for _ in range(world_size)]
    dist.all_gather(out, padded)
    return [o[:s] for o, s in zip(out, sizes)]
