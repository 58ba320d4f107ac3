"""CPU-affinity for one-process-per-GPU jobs (reference utils/gpu_affinity.py:1-65).

The reference binds each rank to the CPU cores of its GPU's NUMA node via
NVML (and, in the fork, a Windows API). On MI355X nodes the GPU -> NUMA
mapping is read from sysfs (``/sys/class/drm/card*/device/numa_node`` via
the PCI bus id HIP reports), and the process is pinned with
``os.sched_setaffinity``. Everything degrades to a no-op where the
information is unavailable (containers, CPU-only hosts).
"""
import os

from imaginaire_amd.utils.distributed import master_only_print as print


def _cpus_of_numa_node(node):
    try:
        with open('/sys/devices/system/node/node%d/cpulist' % node) as f:
            spec = f.read().strip()
    except OSError:
        return None
    cpus = set()
    for part in spec.split(','):
        if '-' in part:
            a, b = part.split('-')
            cpus.update(range(int(a), int(b) + 1))
        elif part:
            cpus.add(int(part))
    return cpus or None


def _gpu_numa_node(gpu_id):
    try:
        import torch
        props = torch.cuda.get_device_properties(gpu_id)
        bus = getattr(props, 'pci_bus_id', None)
        dom = getattr(props, 'pci_domain_id', 0)
        dev = getattr(props, 'pci_device_id', 0)
        if bus is None:
            return None
        path = '/sys/bus/pci/devices/%04x:%02x:%02x.0/numa_node' % (dom, bus, dev)
        with open(path) as f:
            node = int(f.read().strip())
        return node if node >= 0 else None
    except Exception:  # noqa: BLE001 (no GPU / no sysfs)
        return None


def systemGetDriverVersion():  # noqa: N802 (reference name)
    """Kernel driver version (amdgpu module / KFD) as a string, '' if unknown."""
    for path in ('/sys/module/amdgpu/version', '/sys/class/kfd/kfd/topology/system_properties'):
        try:
            with open(path) as f:
                return f.read().strip().splitlines()[0]
        except (OSError, IndexError):
            continue
    return ''


def deviceGetCount():  # noqa: N802
    """Number of visible GPUs (without initialising the HIP runtime)."""
    import torch
    return torch.cuda.device_count()


class device(object):  # noqa: N801
    """Per-GPU handle exposing name and local CPU list (reference gpu_affinity.py:24-46)."""

    def __init__(self, device_idx):
        self.idx = device_idx

    def getName(self):  # noqa: N802
        import torch
        return torch.cuda.get_device_name(self.idx)

    def getCpuAffinity(self):  # noqa: N802
        node = _gpu_numa_node(self.idx)
        cpus = _cpus_of_numa_node(node) if node is not None else None
        if not cpus:
            cpus = os.sched_getaffinity(0) if hasattr(os, 'sched_getaffinity') else set()
        return sorted(cpus)


def set_affinity(gpu_id=None):
    """Pin this process to the CPUs local to ``gpu_id`` (default: $LOCAL_RANK); returns the
    CPU set used."""
    if gpu_id is None:
        gpu_id = int(os.getenv('LOCAL_RANK', 0))
    node = _gpu_numa_node(gpu_id)
    cpus = _cpus_of_numa_node(node) if node is not None else None
    if not cpus or not hasattr(os, 'sched_setaffinity'):
        return os.sched_getaffinity(0) if hasattr(os, 'sched_getaffinity') else None
    allowed = os.sched_getaffinity(0) & cpus
    if allowed:
        os.sched_setaffinity(0, allowed)
        print('GPU %d: pinned to NUMA node %d (%d CPUs)' % (gpu_id, node, len(allowed)))
    return os.sched_getaffinity(0)
