"""Loader for the gfx950 HIP extension ``imaginaire_amd._C``.

Policy: on a GPU tensor every op in ``imaginaire_amd.ops`` runs its HIP kernel.
If the extension is missing on a machine that has a GPU the op raises (no
silent eager fallback). CPU tensors use the PyTorch reference implementation
of the same math (this is what the CPU test-suite and the CPU plumbing config
exercise). Set ``IMAGINAIRE_AMD_EAGER=1`` to force the reference path on GPU
(used only by the self-baseline benchmark and numerics tests).
"""
import importlib
import contextlib
import os
import threading

import torch

_EXT = None
_ERR = None


def load():
    global _EXT, _ERR
    if _EXT is not None or _ERR is not None:
        return _EXT
    try:
        _EXT = importlib.import_module('imaginaire_amd._C')
    except ImportError as e:  # pragma: no cover - depends on build state
        _ERR = e
        _EXT = None
    if _EXT is not None:
        _check_provenance()
    return _EXT


def build_info():
    """The manifest ``_build`` wrote next to ``_C.so`` (arch, sources digest, compiler)."""
    import json
    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                        '_C.build.json')
    try:
        with open(path) as f:
            return json.load(f)
    except (OSError, ValueError):
        return None


def _check_provenance():
    """A _C.so built from different sources than the tree it sits in (stale build shipped to
    a GPU box) is an error: its kernels would not be the ones the Python side expects.
    ``IMAGINAIRE_AMD_ALLOW_STALE_EXT=1`` downgrades it to a warning."""
    info = build_info()
    if info is None:
        return
    from imaginaire_amd import _build
    try:
        digest = _build.sources_digest()
    except OSError:  # sources not shipped alongside the binary
        return
    if info.get('sources_sha1') != digest:
        msg = ('imaginaire_amd._C was built from sources %s but the tree holds %s: rebuild '
               'with `python -m imaginaire_amd._build`' % (
                   str(info.get('sources_sha1'))[:12], digest[:12]))
        if os.environ.get('IMAGINAIRE_AMD_ALLOW_STALE_EXT', '0') == '1':
            import warnings
            warnings.warn(msg)
        else:
            raise ImportError(msg)


def available():
    return load() is not None


_SCOPE = threading.local()


def force_eager():
    return os.environ.get('IMAGINAIRE_AMD_EAGER', '0') == '1' or \
        getattr(_SCOPE, 'depth', 0) > 0


@contextlib.contextmanager
def eager_scope(enabled=True):
    """Route every op dispatched inside the block to its plain PyTorch path.

    The HIP kernels' autograd Functions are first-order only (their backwards call raw
    kernels), so a forward whose gradient is itself differentiated -- the gradient
    penalty's ``autograd.grad(..., create_graph=True)`` -- must run on PyTorch ops, or the
    penalty's dependence on the weights is silently dropped."""
    if not enabled:
        yield
        return
    _SCOPE.depth = getattr(_SCOPE, 'depth', 0) + 1
    try:
        yield
    finally:
        _SCOPE.depth -= 1


def use_native(t):
    """True if tensor ``t`` should go through the HIP kernel."""
    if t is None or not t.is_cuda:
        return False
    if force_eager():
        return False
    ext = load()
    if ext is None:
        raise RuntimeError(
            'imaginaire_amd: the HIP extension _C is not built but a GPU tensor '
            'was given ({}). Run `python -m imaginaire_amd._build`.'.format(_ERR))
    return True


def ext():
    e = load()
    if e is None:
        raise RuntimeError('imaginaire_amd._C not available: {}'.format(_ERR))
    return e


def is_dense(t):
    """Python mirror of ``at::Tensor::is_non_overlapping_and_dense`` (not bound in torch):
    the elements exactly fill ``numel`` contiguous slots in some dimension order."""
    if t.is_contiguous() or (t.dim() == 4 and t.is_contiguous(memory_format=torch.channels_last)):
        return True
    dims = sorted((st, sz) for sz, st in zip(t.shape, t.stride()) if sz != 1)
    expect = 1
    for st, sz in dims:
        if st != expect:
            return False
        expect *= sz
    return True
