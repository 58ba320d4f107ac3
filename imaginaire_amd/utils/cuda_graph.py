"""hipGraph capture of a trainer's steady-state iteration (D update -> G update -> EMA).

The reference runs every iteration eagerly (trainers/base.py:594-666, apex AMP): ~1,450
kernel launches per SPADE step issued one by one from Python. On MI355X the whole
iteration is captured ONCE into a hipGraph (``torch.cuda.graph``) and replayed:

* inputs are copied into static device buffers before each replay;
* everything the step changes between iterations lives on the device: the Adam step
  counter / bias corrections / learning rate (FusedAdam's device hyper-parameters), the
  EMA warm-up switch (``num_updates_tracked``), BatchNorm running statistics, spectral-norm
  u/v vectors, the philox RNG offsets of the style-encoder noise;
* host-side mirrors (optimizer ``group['step']``, ``ModelAverage._host_updates``) are
  advanced after each replay, and a changed learning rate is pushed to the device
  (``FusedAdam.sync_hyper``) before it;
* device tables that the multi-tensor kernels build on first use are uploaded after the
  capture (``flush_deferred_uploads``), never as copy nodes inside the graph.

Multi-rank steps are captured too (the default since round 4), with their collectives: the
DDP bucket all-reduces and sync-BN exchanges run on the native RCCL communicator
(parallel/rccl.py: no torch Work objects for the watchdog to poll) and DDP uses its rank-local
unused-parameter mask (no host sync in ``finish()``), which holds for the trainers whose
``rank_uniform(cfg)`` is true: SPADE, pix2pixHD, MUNIT / UNIT, FUNIT, and the vid2vid family
unless its config adds the data-dependent hand / face discriminators
(trainers/vid2vid.py ``rank_uniform``); those keep the eager step at world > 1. Capture is
rank-local (nothing executes while
recording), so the ranks agree on its outcome afterwards: one all-reduce of a success flag and a
batch-signature hash; if any rank failed, every rank runs eagerly. Both paths run the same
kernels: the eager step also runs under :class:`graph_routing`. Batch structures must be
rank-uniform (every rank captures / replays the same graph at the same iteration), as a
``DistributedSampler`` with ``drop_last`` and the synthetic sources give.
"""
import os
import time

import torch

from imaginaire_amd.utils.distributed import get_world_size
from imaginaire_amd.utils.distributed import master_only_print as print


def graph_mode_default():
    """'1' (default: on for world size 1), '0' (off) or 'force' (also with world > 1)."""
    return os.environ.get('IMAGINAIRE_AMD_GRAPH', '1')


def graph_supported(trainer):
    mode = graph_mode_default()
    if mode == '0' or trainer.device.type != 'cuda':
        return False
    if getattr(trainer.cfg, 'speed_benchmark', False):
        return False  # per-phase host timers synchronise inside the step
    if getattr(trainer.cfg.trainer, 'skip_nonfinite_steps', False):
        return False  # host-side decision per step
    if get_world_size() > 1 and mode != 'force':
        return multirank_capturable(trainer)
    return True


def _capturable_wrapper(net):
    """A network wrapper whose collectives can be recorded: the single-process wrapper, or the
    bucketed DDP on the native RCCL communicator with the rank-local unused mask."""
    from imaginaire_amd.parallel.ddp import DistributedDataParallel
    if net is None:
        return True
    mod = getattr(net, 'module', None)
    if isinstance(net, torch.nn.parallel.DistributedDataParallel):
        return False
    if isinstance(net, DistributedDataParallel):
        return (not net._force) or (net.find_unused == 'local' and net._native is not None)
    if mod is not None and mod is not net and isinstance(mod, torch.nn.Module) and \
            isinstance(mod, (DistributedDataParallel, torch.nn.parallel.DistributedDataParallel)):
        return _capturable_wrapper(mod)
    return True


def multirank_capturable(trainer):
    """True when a world > 1 step of ``trainer`` can be captured: rank-uniform control flow and
    every network wrapper on the native communicator with the local unused mask."""
    if not getattr(trainer, 'rank_uniform_control_flow', False):
        return False
    return _capturable_wrapper(getattr(trainer, 'net_G', None)) and \
        _capturable_wrapper(getattr(trainer, 'net_D', None))


def _signature_hash(sig):
    import hashlib
    return int(hashlib.sha1(repr(sig).encode()).hexdigest()[:12], 16)


def agree_capture(ok, sig_hash, group=None):
    """Agree on a capture outcome across ranks: True only if every rank captured (``ok``) the
    same batch structure (``sig_hash``). One all-reduce of [min ok, min hash, -max hash]
    through the default group; world size 1: ``ok``."""
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return bool(ok)
    dev = torch.device('cpu') if dist.get_backend(group) == 'gloo' else \
        torch.device('cuda', torch.cuda.current_device())
    h = float(sig_hash % (1 << 40))  # exact in float64
    t = torch.tensor([1.0 if ok else 0.0, h, -h], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    t = t.cpu().tolist()
    return t[0] == 1.0 and t[1] == -t[2]


def _static_copy(dst, src):
    if torch.is_tensor(dst):
        dst.copy_(src, non_blocking=True)
    elif isinstance(dst, dict):
        # the captured step may have added entries to its static batch (e.g. the SPADE
        # trainer's style noise 'z'): those are outputs of the graph, not inputs
        for k in src:
            if k in dst:
                _static_copy(dst[k], src[k])
    elif isinstance(dst, (list, tuple)):
        for d, s in zip(dst, src):
            _static_copy(d, s)


def _clone(x):
    if torch.is_tensor(x):
        return x.clone()
    if isinstance(x, dict):
        return {k: _clone(v) for k, v in x.items()}
    if isinstance(x, list):
        return [_clone(v) for v in x]
    if isinstance(x, tuple):
        return tuple(_clone(v) for v in x)
    return x


def _same_structure(a, b):
    if torch.is_tensor(a):
        return torch.is_tensor(b) and a.shape == b.shape and a.dtype == b.dtype and \
            a.stride() == b.stride()
    if isinstance(a, dict):
        return isinstance(b, dict) and a.keys() == b.keys() and \
            all(_same_structure(a[k], b[k]) for k in a)
    if isinstance(a, (list, tuple)):
        return isinstance(b, (list, tuple)) and len(a) == len(b) and \
            all(_same_structure(x, y) for x, y in zip(a, b))
    return a == b


def _signature(x):
    """Hashable structure of a batch (tensor shapes / dtypes / strides, nested containers)."""
    if torch.is_tensor(x):
        return ('T', tuple(x.shape), str(x.dtype), tuple(x.stride()))
    if isinstance(x, dict):
        return ('D',) + tuple((k, _signature(v)) for k, v in sorted(x.items(), key=lambda kv: str(kv[0])))
    if isinstance(x, (list, tuple)):
        return ('L',) + tuple(_signature(v) for v in x)
    if isinstance(x, str):
        return ('S',)  # file keys / names: never steer the computation
    try:
        hash(x)
        return ('V', x)
    except TypeError:
        return ('V', repr(x))


def _resync_shadows():
    """bf16 shadow weights (optimizers/fused_adam.py) of parameters written outside the graph
    since the last replay — a restored snapshot, a loaded checkpoint — are refreshed before the
    replay reads them."""
    from imaginaire_amd.optimizers import fused_adam
    fused_adam.resync_shadows()


class graph_routing(object):
    """Kernel routing of a graphed step, for its warm-up, its capture and any eager run compared
    against its replay: every conv k10 / k11 can run takes them, whatever its grid size or
    channel-padding waste (ops/conv.py ``_capturing``). The small-problem MIOpen backward
    solvers accumulate with atomics into buffers zeroed outside the captured stream, so a replay
    adds onto the previous replay's values (and MIOpen's deterministic mode is no way out: it
    falls back to its naive direct kernels, ~11 s per MUNIT recipe iteration). Warm-up runs
    under it too, so the capture records the kernels the warm-up already ran."""

    def __enter__(self):
        from imaginaire_amd.ops import conv
        conv._GRAPH_ROUTING[0] += 1
        return self

    def __exit__(self, *exc):
        from imaginaire_amd.ops import conv
        conv._GRAPH_ROUTING[0] -= 1


_WARNED = [False]


def packet_capture_refusal():
    """None when graphs may be captured, else the reason they may not: the HIP runtime's graph
    packet-capture mode is (or may be) on in this process (imaginaire_amd/__init__.py
    ``PACKET_CAPTURE_STATE``). ``IMAGINAIRE_AMD_GRAPH_ALLOW_PACKET_CAPTURE=1`` captures anyway
    (probes that compare the two modes)."""
    import imaginaire_amd
    state = getattr(imaginaire_amd, 'PACKET_CAPTURE_STATE', 'off')
    if state == 'off' or os.environ.get('IMAGINAIRE_AMD_GRAPH_ALLOW_PACKET_CAPTURE') == '1':
        return None
    if state == 'unknown':
        return ('HIP was initialised before imaginaire_amd was imported, with '
                'DEBUG_CLR_GRAPH_PACKET_CAPTURE unset, so the runtime\'s packet-capture mode is '
                'on (replays of long graphs have read stale operands in that mode); import '
                'imaginaire_amd before using torch.cuda, or export '
                'DEBUG_CLR_GRAPH_PACKET_CAPTURE=0')
    return ('DEBUG_CLR_GRAPH_PACKET_CAPTURE=%s: packet-capture mode is on (replays of long '
            'graphs have read stale operands in that mode)' %
            os.environ.get('DEBUG_CLR_GRAPH_PACKET_CAPTURE'))


class GraphedStep(object):
    """Runs ``step_fn(data)`` eagerly for ``warmup`` iterations (on a side stream, as
    stream capture requires), then captures it and replays the graph from then on.

    One graph per batch structure (shapes / dtypes of the inputs): a new structure — the
    video trainers' growing sequence length, a ragged last batch — gets its own warm-up and
    capture, and its own memory pool: graphs replayed in any order (A, B, A) never rewrite
    each other's outputs (the trainers' loss dicts and images point into them). ``step_fn``
    must be the steady-state iteration for a given structure: no host synchronisation.
    ``pre_replay`` / ``post_replay`` are host hooks run around every replay.
    """

    MAX_GRAPHS = 8

    def __init__(self, step_fn, warmup=3, pre_replay=None, post_replay=None, name='step',
                 save_host=None, restore_host=None):
        self.step_fn = step_fn
        self.warmup = warmup
        self.pre_replay = pre_replay
        self.post_replay = post_replay
        # host-side counters the captured (not executed) iteration advanced: rolled back
        self.save_host = save_host
        self.restore_host = restore_host
        self.name = name
        self.entries = {}  # signature -> {'graph', 'static', 'n_eager'}
        self.failed = False
        self.capture_s = None
        self.stream = None
        self._last = None

    # the most recently used entry (tests and bench scripts read .graph / .static)
    @property
    def graph(self):
        return self._last['graph'] if self._last else None

    @property
    def static(self):
        return self._last['static'] if self._last else None

    @property
    def n_eager(self):
        return self._last['n_eager'] if self._last else 0

    def _side_stream(self):
        if self.stream is None:
            self.stream = torch.cuda.Stream()
            # parameters' AccumulateGrad nodes made by earlier default-stream iterations
            # meet the side stream here: a one-off stream sync during warm-up, not a
            # problem for the captured replay (no autograd engine runs there)
            _quiet = getattr(torch.autograd.graph,
                             'set_warn_on_accumulate_grad_stream_mismatch', None)
            if _quiet is not None:
                _quiet(False)
        return self.stream

    def __call__(self, data):
        if self.failed:
            return self.step_fn(data)
        sig = _signature(data)
        ent = self.entries.get(sig)
        if ent is None:
            if len(self.entries) >= self.MAX_GRAPHS:
                return self.step_fn(data)  # structure churn: stay eager for new ones
            ent = self.entries[sig] = {'graph': None, 'static': None, 'n_eager': 0,
                                       'sig': sig, 'pool': None}
        self._last = ent
        if ent['graph'] is not None:
            _static_copy(ent['static'], data)
            _resync_shadows()
            if self.pre_replay:
                self.pre_replay()
            ent['graph'].replay()
            if self.post_replay:
                self.post_replay()
            return None
        if ent['n_eager'] < self.warmup:
            # warm up on the stream the capture will use: autograd's AccumulateGrad nodes
            # remember the stream they were created on
            st = self._side_stream()
            st.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(st), graph_routing():
                self.step_fn(data)
            torch.cuda.current_stream().wait_stream(st)
            ent['n_eager'] += 1
            return None
        return self._capture_and_run(ent, data)

    def _capture_and_run(self, ent, data):
        from imaginaire_amd.ops import _ext
        refuse = packet_capture_refusal()
        if refuse is not None:
            if not _WARNED[0]:
                _WARNED[0] = True
                print('[graph] not capturing {}: {}; running eagerly'.format(self.name, refuse))
            self.failed = True
            ent['static'] = None
            return self.step_fn(data)
        torch.cuda.synchronize()
        t0 = time.time()
        # private copies: the batch source may hand out views of its own pool
        ent['static'] = _clone(data)
        saved = self.save_host() if self.save_host else None
        dot = os.environ.get('IMAGINAIRE_AMD_GRAPH_DOT')
        # (the DOT dump needs the captured hipGraph_t, which is freed at instantiation unless
        # the graph is kept)
        g = torch.cuda.CUDAGraph(keep_graph=True) if dot else torch.cuda.CUDAGraph()
        err = None
        try:
            st = self._side_stream()
            if ent['pool'] is None:
                ent['pool'] = torch.cuda.graph_pool_handle()
            # thread-local capture mode: the RCCL process group's watchdog thread keeps polling
            # its work events while a (seconds-long) step is being captured; under the default
            # global mode those calls from another thread are refused and abort the process
            if dot:  # hipGraphDebugDotPrint of the captured graph (scripts/probe/graph_dot.py)
                g.enable_debug_mode()
            with torch.cuda.graph(g, pool=ent['pool'], stream=st,
                                  capture_error_mode='thread_local'), graph_routing():
                self.step_fn(ent['static'])
            if dot:
                g.debug_dump(dot)
        except Exception as e:  # noqa: BLE001 - any capture failure: stay eager
            if os.environ.get('IMAGINAIRE_AMD_GRAPH_DEBUG'):
                raise
            err = e
        # every rank captured, or every rank runs eagerly (a rank replaying collectives its
        # peers issue eagerly would still match them, but one that failed mid-capture must not
        # leave the others replaying a graph it never recorded)
        if not agree_capture(err is None, _signature_hash(ent['sig'])) and err is None:
            err = RuntimeError('capture failed or differed on another rank')
        if err is not None:
            print('[graph] capture of {} failed ({}: {}); running eagerly'.format(
                self.name, type(err).__name__, str(err).splitlines()[0][:200]))
            self.failed = True
            g = None
            ent['static'] = None
            if self.restore_host:
                self.restore_host(saved)
            torch.cuda.synchronize()
            return self.step_fn(data)
        if self.restore_host:
            self.restore_host(saved)
        if _ext.available():
            _ext.ext().flush_deferred_uploads()
        torch.cuda.synchronize()
        ent['graph'] = g
        self.capture_s = time.time() - t0
        print('[graph] captured {} ({} graph(s)) in {:.1f} s'.format(
            self.name, sum(1 for e in self.entries.values() if e['graph'] is not None),
            self.capture_s))
        # the capture itself executed nothing: run this iteration as the first replay
        _resync_shadows()
        if self.pre_replay:
            self.pre_replay()
        g.replay()
        if self.post_replay:
            self.post_replay()
        return None


def make_trainer_step(trainer, warmup=None, enabled=True, force=False):
    """The steady-state iteration of an image trainer: ``dis_step`` D updates then
    ``gen_step`` G updates (reference train.py:72-84), as a GraphedStep when supported
    (``trainer.graph_capturable`` and :func:`graph_supported`). Returns (callable, graph or
    None)."""
    cfg = trainer.cfg
    if warmup is None:
        warmup = int(os.environ.get('IMAGINAIRE_AMD_GRAPH_WARMUP', '3'))

    from imaginaire_amd.ops.conv import tune_pending

    def step(data):
        # the eager step routes its convs as the captured one does (graph_routing): multi-rank
        # eager fallbacks and graph warm-ups run the same kernels as the replay
        with graph_routing():
            for _ in range(cfg.trainer.dis_step):
                trainer.dis_update(data)
            for _ in range(cfg.trainer.gen_step):
                trainer.gen_update(data)
        # per-shape kernel choices first seen in this iteration are timed and agreed across
        # ranks here, between iterations (every rank runs the same iterations), never inside a
        # backward; no-op once every shape is known and during graph capture
        tune_pending()

    # force: try any trainer (the capture falls back to eager on failure); used by
    # scripts/bench_families.py --graph to evaluate families not yet marked capturable
    if not (enabled and (force or getattr(trainer, 'graph_capturable', False)) and
            graph_supported(trainer)):
        return step, None

    opts = [o for o in (trainer.opt_G, trainer.opt_D) if o is not None]
    n_updates = {id(trainer.opt_D): cfg.trainer.dis_step, id(trainer.opt_G): cfg.trainer.gen_step}

    def pre():
        for o in opts:
            if hasattr(o, 'sync_hyper'):
                o.sync_hyper()

    def post():
        for o in opts:
            if hasattr(o, 'advance_host_step'):
                o.advance_host_step(n_updates.get(id(o), 1))
        if cfg.trainer.model_average:
            ma = trainer.net_G.module
            if hasattr(ma, '_host_updates'):
                ma._host_updates += cfg.trainer.gen_step

    def save_host():
        ma = trainer.net_G.module if cfg.trainer.model_average else None
        return ([[g.get('step') for g in o.param_groups] for o in opts],
                getattr(ma, '_host_updates', None))

    def restore_host(saved):
        steps, host_updates = saved
        for o, st in zip(opts, steps):
            for g, v in zip(o.param_groups, st):
                if v is not None:
                    g['step'] = v
        if host_updates is not None:
            trainer.net_G.module._host_updates = host_updates

    gs = GraphedStep(step, warmup=warmup, pre_replay=pre, post_replay=post,
                     name=type(trainer).__module__, save_host=save_host,
                     restore_host=restore_host)
    return gs, gs
