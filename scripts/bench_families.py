"""Training-step throughput of any model family on synthetic data (one GPU).

    python scripts/bench_families.py --config <reference-or-framework yaml> [--steps K]
        [--warmup W] [--batch B] [--seq-len T] [--pool P]

Runs the train.py iteration (``start_of_iteration`` -> ``dis_step`` x ``dis_update`` ->
``gen_step`` x ``gen_update``) of the family the config names, on batches of the config's
own shape produced by the synthetic dataset (``imaginaire_amd.datasets.synthetic``, random
init, no checkpoints) and kept resident on the GPU (a pool of P batches cycled), and prints
ONE JSON line: samples/s (images for image families, sequences x frames for video families)
and ms per iteration. The reference configs (configs/projects/... of the reference checkout)
load unchanged; only ``data.type`` is switched to the synthetic dataset.

Used for the BASELINE.json secondary configs (MUNIT 256x256, vid2vid 512x1024 seq 3, ...);
the flagship SPADE number comes from ``bench.py``.
"""
import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def main():
    p = argparse.ArgumentParser()
    p.add_argument('--config', required=True)
    p.add_argument('--steps', type=int, default=20)
    p.add_argument('--warmup', type=int, default=4)
    p.add_argument('--batch', type=int, default=None)
    p.add_argument('--seq-len', type=int, default=None,
                   help='video families: frames per training sequence')
    p.add_argument('--pool', type=int, default=2)
    p.add_argument('--cpu', action='store_true', help='plumbing check on the CPU')
    p.add_argument('--no-pipelined', dest='pipelined', action='store_false',
                   help='skip the second timed block (synchronised at its ends only)')
    p.add_argument('--op-sites', action='store_true',
                   help='after the timed steps, attribute the aten glue of one more iteration '
                        'to Python call sites (scripts/probe/op_sites.py) on stderr')
    p.add_argument('--ext-sites', default='',
                   help='after the timed steps, count the calls of these extension functions '
                        '(comma-separated, e.g. pad_channels_cast,conv_phase_scatter) of one more '
                        'eager iteration by Python call site, on stderr')
    p.add_argument('--graph', action='store_true',
                   help='replay the steady-state iteration from a captured hipGraph (any family)')
    p.add_argument('--conv-log', action='store_true',
                   help='after the timed steps, time every conv kernel call of one more '
                        'iteration and print time / TF/s per (kind, shape, kernel) to stderr')
    p.add_argument('--print-losses', action='store_true',
                   help='print every iteration\'s D and G losses to stderr (divergence hunts)')
    p.add_argument('--diag', action='store_true',
                   help='after every iteration: non-finite parameters / gradients per network and '
                        'spectral-norm bf16 shadows that differ from bf16(param), on stderr')
    p.add_argument('--poison', action='store_true',
                   help='fill every uninitialised allocation with NaN (deterministic mode\'s '
                        'fill_uninitialized_memory): a kernel reading memory nobody wrote shows')
    p.add_argument('--flag-probe', action='store_true',
                   help='with --graph: record isfinite() of every leaf module output / output '
                        'gradient into the captured graph and print the first non-finite ones '
                        'after each replay (locates a replay-only NaN)')
    p.add_argument('--static-batch', action='store_true',
                   help='prepare each pooled batch once and hand the same tensors to every '
                        'iteration (no host-side allocation between graph replays)')
    p.add_argument('--ab-eager', action='store_true',
                   help='with --graph: every timed iteration runs twice from one saved state — '
                        'graph replay, then the eager step — and prints where their losses and '
                        'gradients part; training continues from the eager result')
    p.add_argument('--op-probe', action='store_true',
                   help='like --flag-probe, plus the outputs (and in-place operands) of every HIP '
                        'extension call, labelled with the enclosing module')
    p.add_argument('--allow-nonfinite', action='store_true',
                   help='exit 0 even when a final loss is NaN/Inf (default: exit 3)')
    p.add_argument('--gpus', type=int, default=1,
                   help='ranks (one process per GPU, DDP over RCCL). Without a launcher (no '
                        'WORLD_SIZE) the script starts them itself through torch.distributed.run; '
                        'weak scaling: every rank trains its own batch of --batch samples')
    p.add_argument('--backend', default='nccl',
                   help='process-group backend for --gpus > 1 (nccl = RCCL; gloo for rehearsals)')
    p.add_argument('--share-gpu', action='store_true',
                   help='testing only: every rank uses cuda:0 (needs --backend gloo)')
    p.add_argument('--set', nargs='*', default=[], metavar='KEY=VALUE',
                   help='dotted config overrides, e.g. gen.num_filters=64 '
                        'data.train.augmentations.random_crop_h_w=256,256 (scale a unit-test '
                        'config up to a recipe without another YAML)')
    args = p.parse_args()
    world_env = os.environ.get('WORLD_SIZE')
    if world_env is None and args.gpus > 1:
        sys.exit(_launch_ranks(args, sys.argv[1:]))
    if world_env is not None and int(world_env) != args.gpus:
        sys.exit('bench_families.py: --gpus %d but WORLD_SIZE=%s' % (args.gpus, world_env))
    if args.share_gpu and args.gpus > 1 and args.backend == 'nccl':
        sys.exit('bench_families.py: --share-gpu needs --backend gloo')

    import torch
    import torch.distributed as dist
    from torch.utils.data import default_collate
    from imaginaire_amd.config import Config
    from imaginaire_amd.datasets.synthetic import Dataset
    from imaginaire_amd.utils.trainer import get_model_optimizer_and_scheduler, get_trainer

    real_stdout, sys.stdout = sys.stdout, sys.stderr
    if args.poison:
        torch.use_deterministic_algorithms(True, warn_only=True)
        torch.utils.deterministic.fill_uninitialized_memory = True
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local_rank = 0 if args.share_gpu else int(os.environ.get('LOCAL_RANK', '0'))
    device = torch.device('cpu') if args.cpu else torch.device('cuda', local_rank)
    if device.type == 'cuda':
        torch.cuda.set_device(local_rank)  # before the process group: rank r -> GPU r
    if world > 1:
        from imaginaire_amd.utils.distributed import init_dist
        init_dist(local_rank, backend=args.backend if device.type == 'cuda' else 'gloo')
    coll_dev = device if (world > 1 and args.backend == 'nccl' and device.type == 'cuda') \
        else torch.device('cpu')
    cfg = Config(args.config)
    cfg.logdir = '/tmp/imaginaire_amd_bench_families'
    for kv in args.set:
        key, val = kv.split('=', 1)
        node = cfg
        parts = key.split('.')
        for k in parts[:-1]:
            node = getattr(node, k)
        if val in ('True', 'False'):
            val = val == 'True'
        else:
            try:
                val = int(val)
            except ValueError:
                try:
                    val = float(val)
                except ValueError:
                    pass
        setattr(node, parts[-1], val)
    # the synthetic dataset is constructed directly below; cfg.data.type keeps naming the
    # reference dataset so the batch contract (few-shot keys, video axis) follows it
    if args.batch:
        cfg.data.train.batch_size = args.batch
    bs = cfg.data.train.batch_size
    video = hasattr(cfg.data, 'num_frames_G')
    if video and args.seq_len:
        cfg.data.train.initial_sequence_length = args.seq_len
        cfg.data.train.max_sequence_length = args.seq_len
    ds = Dataset(cfg)

    class _Loader(list):  # the trainers read train_data_loader.dataset (sequence schedule)
        dataset = ds

    net_G, net_D, opt_G, opt_D, sch_G, sch_D = get_model_optimizer_and_scheduler(cfg, seed=0)
    trainer = get_trainer(cfg, net_G, net_D, opt_G, opt_D, sch_G, sch_D,
                          train_data_loader=_Loader(), val_data_loader=None)
    if video and args.seq_len:
        # past the single-frame epochs: temporal network (flow, warping, temporal D) active
        if hasattr(trainer, 'init_temporal_network'):
            trainer.init_temporal_network()
        ds.set_sequence_length(args.seq_len)
        trainer.sequence_length = args.seq_len

    def to_dev(x):
        if torch.is_tensor(x):
            return x.to(device, non_blocking=True)
        if isinstance(x, dict):
            return {k: to_dev(v) for k, v in x.items()}
        if isinstance(x, list):
            return [to_dev(v) for v in x]
        return x

    # every rank trains its own samples (weak scaling)
    off = rank * bs * args.pool
    pool = [to_dev(default_collate([ds[(off + i * bs + j) % max(1, len(ds))] for j in range(bs)]))
            for i in range(args.pool)]

    def fresh(x):  # some pre-processing (DensePose label remap) edits the batch in place
        if torch.is_tensor(x):
            return x.clone()
        if isinstance(x, dict):
            return {k: fresh(v) for k, v in x.items()}
        if isinstance(x, list):
            return [fresh(v) for v in x]
        return x

    probe = _FlagProbe(trainer, ops=args.op_probe) if (args.flag_probe or args.op_probe) \
        else None
    graphed = None
    if args.graph:
        from imaginaire_amd.utils.cuda_graph import make_trainer_step
        cfg.speed_benchmark = False
        trainer.speed_benchmark = False
        train_step, graphed = make_trainer_step(trainer, warmup=max(1, args.warmup - 1),
                                                force=True)
    else:
        # the eager train.py step (incl. the between-iteration kernel-choice tuning)
        from imaginaire_amd.utils.cuda_graph import make_trainer_step
        train_step, graphed = make_trainer_step(trainer, enabled=False)

    prepared = {}

    def prepare(it):
        if args.static_batch:
            k = it % len(pool)
            if k not in prepared:
                prepared[k] = trainer.start_of_iteration(fresh(pool[k]), it)
            trainer.current_iteration = it
            return prepared[k]
        return trainer.start_of_iteration(fresh(pool[it % len(pool)]), it)

    def step(it):
        data = prepare(it)
        if probe is not None:
            probe.reset()
        train_step(data)
        if probe is not None:
            probe.report(it)
        return data

    step.prepare = prepare
    step.probe = probe

    def sync():
        if device.type == 'cuda':
            torch.cuda.synchronize()

    data = None
    for it in range(args.warmup):
        data = step(it)
        print('[bench_families] warmup %d done' % it, flush=True)
        if args.print_losses:
            print('[bench_families] it %d losses %s' % (it, json.dumps(_losses(trainer))),
                  flush=True)
        if args.diag:
            _diag(trainer, it)
    sync()
    if device.type == 'cuda':
        try:  # steady-state marker for scripts/gpu/summarize_kernels.py (after warm-up/autotune)
            from imaginaire_amd.ops import _ext
            _ext.ext().profile_marker(1)
        except Exception:  # noqa: BLE001 - the marker is a profiling aid only
            pass
    # per-iteration wall times (synchronised each iteration) -> median and spread; the mean over
    # the whole timed window is reported too (what a throughput number over K steps means)
    times = []
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for it in range(args.steps):
        t1 = time.perf_counter()
        if args.ab_eager and graphed is not None and graphed.graph is not None:
            data = _ab_step(trainer, graphed, step, args.warmup + it)
        else:
            data = step(args.warmup + it)
        sync()
        times.append(time.perf_counter() - t1)
        if args.print_losses:
            print('[bench_families] it %d losses %s' % (args.warmup + it,
                                                       json.dumps(_losses(trainer))), flush=True)
        if args.diag:
            _diag(trainer, args.warmup + it)
    if world > 1:
        dist.barrier()
    dt = (time.perf_counter() - t0) / args.steps
    if world > 1:  # the job is as fast as its slowest rank
        t = torch.tensor([dt], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    st = sorted(times)
    med = st[len(st) // 2] if len(st) % 2 else 0.5 * (st[len(st) // 2 - 1] + st[len(st) // 2])
    # the same number of iterations again, synchronised only at both ends (as train.py runs:
    # the host prepares iteration i + 1 while the GPU still runs iteration i); the loop above
    # makes the GPU wait for each iteration's host-side batch preparation and graph launch
    dt_pipe = None
    if args.pipelined and not args.ab_eager:
        if world > 1:
            dist.barrier()
        sync()
        t0 = time.perf_counter()
        for it in range(args.steps):
            data = step(args.warmup + args.steps + it)
        sync()
        if world > 1:
            dist.barrier()
        dt_pipe = (time.perf_counter() - t0) / args.steps
        if world > 1:
            t = torch.tensor([dt_pipe], dtype=torch.float64, device=coll_dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dt_pipe = float(t.item())
    if args.op_sites and device.type == 'cuda':
        sys.path.insert(0, os.path.join(HERE, 'probe'))
        from op_sites import record_sites
        record_sites(lambda: step(args.warmup + args.steps + 1), out=sys.stderr,
                     **({'ops': os.environ['OP_SITES_OPS']} if 'OP_SITES_OPS' in os.environ
                        else {}))
    if args.ext_sites and device.type == 'cuda':
        # one more eager iteration with the captured step's routing: extension calls by site
        sys.path.insert(0, os.path.join(HERE, 'probe'))
        from pad_sites_probe import record_ext_sites
        from imaginaire_amd.utils.cuda_graph import graph_routing
        with graph_routing():
            record_ext_sites(lambda: step(args.warmup + args.steps + 1),
                             tuple(args.ext_sites.split(',')), out=sys.stderr)
    if args.conv_log and device.type == 'cuda':
        from imaginaire_amd.ops import conv as conv_ops
        conv_ops.enable_conv_log(True)
        t1 = time.perf_counter()
        step(args.warmup + args.steps)
        sync()
        wall = (time.perf_counter() - t1) * 1e3
        rows = conv_ops.conv_log_summary()
        conv_ops.enable_conv_log(False)
        tot = sum(r[4] for r in rows)
        fl = sum(r[5] * r[4] * 1e9 for r in rows)
        print('conv kernels in one iteration: %.2f ms of %.1f ms wall, %.2f TFLOP, %.0f TF/s' % (
            tot, wall, fl / 1e12, fl / max(tot, 1e-9) / 1e9))
        for kind, path, desc, n, ms, tfs in rows[:60]:
            print('%8.3f ms %3d  %-6s %-8s %5.0f TF/s  %s' % (ms, n, kind, path, tfs, desc))
    frames = 1
    if video:
        img = data.get('images') if isinstance(data, dict) else None
        frames = img.shape[1] if torch.is_tensor(img) and img.dim() == 5 else \
            (args.seq_len or 1)
    losses = _losses(trainer)
    finite = all(v == v and abs(v) != float('inf')
                 for part in losses.values() for v in part.values())
    in_sync = None
    if world > 1:
        fl = torch.tensor([0.0 if finite else 1.0], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(fl, op=dist.ReduceOp.MAX)
        finite = float(fl.item()) == 0.0
        sys.path.insert(0, os.path.dirname(HERE))
        from bench import _replicas_in_sync
        in_sync = _replicas_in_sync(trainer, world, coll_dev)
    sys.stdout = real_stdout
    if rank == 0:
        _print_row(args, cfg, ds, bs, frames, dt, med, st, device, graphed, losses, finite,
                   world, in_sync, dt_pipe)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if not finite and not args.allow_nonfinite:
        print('[bench_families] NON-FINITE final losses: %s' % json.dumps(losses),
              file=sys.stderr, flush=True)
        sys.exit(3)
    if in_sync is False:
        print('[bench_families] replicas hold different parameters', file=sys.stderr, flush=True)
        sys.exit(4)


def _print_row(args, cfg, ds, bs, frames, dt, med, st, device, graphed, losses, finite, world,
               in_sync, dt_pipe=None):
    import torch
    h, w = ds.h, ds.w
    print(json.dumps({
        'config': os.path.relpath(args.config),
        'family': cfg.trainer.type.split('.')[-1],
        'resolution': '%dx%d' % (h, w), 'batch': bs, 'frames_per_sample': frames,
        'n_gpus': world, 'parallelism': 'dp%d' % world,
        'ms_per_iteration': round(dt * 1e3, 2),
        # whole-job throughput (every rank trains its own batch)
        'samples_per_s': round(world * bs / dt, 3),
        'frames_per_s': round(world * bs * frames / dt, 3),
        'timed_iterations': args.steps, 'warmup': args.warmup,
        'median_ms': round(med * 1e3, 2), 'min_ms': round(st[0] * 1e3, 2),
        'max_ms': round(st[-1] * 1e3, 2),
        # (sync only at the ends of the second timed block: see main)
        'ms_per_iteration_pipelined': round(dt_pipe * 1e3, 2) if dt_pipe else None,
        'frames_per_s_pipelined': round(world * bs * frames / dt_pipe, 3) if dt_pipe else None,
        'spread_pct': round(100.0 * (st[-1] - st[0]) / med, 2),
        'median_frames_per_s': round(world * bs * frames / med, 3),
        'routing': _routing(),
        'device': torch.cuda.get_device_name(device) if device.type == 'cuda' else 'cpu',
        'backend': args.backend if world > 1 else None,
        'replicas_in_sync': in_sync,
        'data': 'synthetic, random-init weights',
        'peak_mem_gb': round(torch.cuda.max_memory_allocated() / 2 ** 30, 2)
        if device.type == 'cuda' else None,
        'hipgraph': bool(graphed is not None and graphed.graph is not None),
        'losses': losses['gen'], 'dis_losses': losses['dis'],
        'losses_finite': finite}), flush=True)


def _launch_ranks(args, argv):
    """``--gpus N`` without a launcher: N ranks through a CHILD torch.distributed.run (nothing
    has touched the GPU yet; no exec from a process holding a HIP context)."""
    import socket
    import subprocess
    s = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1',
           '--nproc-per-node=%d' % args.gpus, '--master-addr=127.0.0.1',
           '--master-port=%d' % port, os.path.abspath(__file__)] + argv
    env = dict(os.environ)
    env.setdefault('HSA_ENABLE_IPC_MODE_LEGACY', '0')
    env.setdefault('OMP_NUM_THREADS', '4')
    print('[bench_families] launching %d ranks' % args.gpus, file=sys.stderr, flush=True)
    return subprocess.call(cmd, env=env)


class _FlagProbe(object):
    """isfinite() flags of every leaf module's outputs (forward) and output gradients (tensor
    hooks: no extra autograd nodes) recorded INSIDE the captured graph, read after each replay."""

    MAXF = 1 << 18

    def __init__(self, trainer, ops=False):
        import torch
        self.flags = torch.ones(self.MAXF, dtype=torch.bool, device='cuda')
        self.labels = []
        self.slot = 0
        self.stack = []
        for net, tag in ((trainer.net_G, 'G'), (trainer.net_D, 'D')):
            if net is None:
                continue
            for n, m in net.named_modules():
                m._probe_name = tag + '.' + n.replace('module.module.', '')
                if len(list(m.children())) == 0:
                    m.register_forward_hook(self._fwd)
                if ops:
                    m.register_forward_pre_hook(self._push)
                    m.register_forward_hook(self._pop)
        self.ops = ops
        # (a capture with tens of thousands of check nodes crashed graph instantiation: the
        # op probe stops after the first few thousand checks, i.e. within the first frame)
        self.limit = int(os.environ.get('IAMD_PROBE_LIMIT', '6000' if ops else str(self.MAXF)))
        if ops:
            self._install_op_hooks()

    def _push(self, mod, inp):
        self.stack.append(mod._probe_name)

    def _pop(self, mod, inp, out):
        if self.stack:
            self.stack.pop()

    def _where(self):
        return self.stack[-1] if self.stack else '-'

    def _install_op_hooks(self):
        import torch
        from imaginaire_amd.ops import _ext
        probe = self

        def rec_all(kind, out, pop=True):
            if torch.is_tensor(out):
                probe._record(kind, probe._where(), out, pop)
            elif isinstance(out, (list, tuple)):
                for o in out:
                    if torch.is_tensor(o):
                        probe._record(kind, probe._where(), o, pop)

        X = _ext.ext()
        arg_names = set(os.environ.get('IAMD_PROBE_ARGS', '').split(','))
        for name in dir(X):
            fn = getattr(X, name)
            if name.startswith('_') or not callable(fn) or name in (
                    'stream_capturing', 'flush_deferred_uploads', 'profile_marker'):
                continue

            def wrap(fn=fn, name=name):
                def w(*a, **k):
                    out = fn(*a, **k)
                    if torch.cuda.is_current_stream_capturing():
                        if name in arg_names:  # the operands too (IAMD_PROBE_ARGS=f1,f2)
                            for ai, t in enumerate(a):
                                if torch.is_tensor(t):
                                    probe._record('arg%d:%s' % (ai, name), probe._where(), t)
                        rec_all('ext:' + name, out)
                    return out
                return w
            setattr(X, name, wrap())

    def _record(self, kind, name, t, pop=True):
        import torch
        if not torch.cuda.is_current_stream_capturing() or not torch.is_tensor(t) or \
                not t.is_floating_point() or t.numel() == 0 or self.slot >= self.limit or \
                getattr(self, '_busy', False):
            return
        self._busy = True
        try:
            i = self.slot
            self.slot += 1
            self.labels.append((kind, name, tuple(t.shape)))
            self.flags[i:i + 1].copy_(torch.isfinite(t.detach()).all().reshape(1))
        finally:
            self._busy = False

    def _fwd(self, mod, inp, out):
        import torch
        for o in (out if isinstance(out, (tuple, list)) else [out]):
            self._record('fwd', mod._probe_name, o)
            if torch.cuda.is_current_stream_capturing() and torch.is_tensor(o) and \
                    o.requires_grad:
                nm = mod._probe_name
                o.register_hook(lambda g, nm=nm: self._record('dout', nm, g))

    def reset(self):
        self.flags.fill_(True)

    def report(self, it):
        if not self.slot:
            return
        f = self.flags[:self.slot].cpu()
        bad = [i for i in range(self.slot) if not bool(f[i])]
        print('[flag-probe] it %d: %d checks, %d non-finite' % (it, self.slot, len(bad)),
              flush=True)
        for i in bad[:12]:
            print('[flag-probe]    #%d %s %s %s' % ((i,) + self.labels[i]), flush=True)
        if bad and getattr(self, 'ops', False):
            # context around the first non-finite checks
            fl = f.tolist()
            for b in bad[:3]:
                for i in range(max(0, b - 6), min(self.slot, b + 5)):
                    print('[flag-probe]    %s #%d %s %s %s' % (
                        ('ok ' if fl[i] else 'BAD', i) + self.labels[i]), flush=True)


def _ab_state(tr):
    ts = list(tr.net_G.parameters()) + list(tr.net_G.buffers())
    ts += list(tr.net_D.parameters()) + list(tr.net_D.buffers())
    for o in (tr.opt_G, tr.opt_D):
        for st in o.state.values():
            ts += [v for v in st.values() if torch_is_tensor(v)]
        ts += [g['_hyper'] for g in o.param_groups if '_hyper' in g]
    return ts


def torch_is_tensor(v):
    import torch
    return torch.is_tensor(v)


def _ab_step(trainer, graphed, step, it, _refs={}):
    """One iteration run as the eager step and as a graph replay from the same saved state,
    continuing along the REPLAY trajectory; prints the loss differences and the parameters whose
    last-frame gradients differ most. The graph's own output tensors (loss dicts, parameter
    gradients) are grabbed once after a replay and re-installed after every eager run (an eager
    step rebinds them to fresh tensors)."""
    import torch
    from imaginaire_amd.utils.cuda_graph import graph_routing
    nets = (('G', trainer.net_G), ('D', trainer.net_D))
    if not _refs:
        _refs['gen'] = dict(trainer.gen_losses)
        _refs['dis'] = dict(trainer.dis_losses)
        _refs['grad'] = [(p, p.grad) for _, net in nets for p in net.parameters()]
    state = _ab_state(trainer)
    saved = [t.detach().clone() for t in state]

    def grads():
        out = {}
        for tag, net in nets:
            for n, p in net.named_parameters():
                if p.grad is not None:
                    out[tag + '.' + n.replace('module.', '')] = p.grad.detach().float().clone()
        return out

    data = step.prepare(it)
    with graph_routing():
        graphed.step_fn(data)
    torch.cuda.synchronize()
    le, ge = _losses(trainer), grads()
    with torch.no_grad():
        for t, c in zip(state, saved):
            t.copy_(c)
    trainer.gen_losses.clear()
    trainer.gen_losses.update(_refs['gen'])
    trainer.dis_losses.clear()
    trainer.dis_losses.update(_refs['dis'])
    for p, g in _refs['grad']:
        p.grad = g
    probe = getattr(step, 'probe', None)
    if probe is not None:
        probe.reset()
    graphed(data)
    torch.cuda.synchronize()
    if probe is not None:
        probe.report(it)
    lr, gr = _losses(trainer), grads()
    dl = {p + '/' + k: (lr[p][k], le[p][k]) for p in lr for k in lr[p]
          if k in le.get(p, {}) and lr[p][k] != le[p][k]}
    rows = []
    for n, b in ge.items():
        a = gr.get(n)
        if a is None:
            rows.append((float('inf'), n + ' (no replay grad)', float(b.norm())))
            continue
        d = float((a - b).norm())
        bn = float(b.norm())
        if not d == 0.0:
            rows.append((d / max(bn, 1e-30) if d == d else float('nan'), n, bn))
    nan_rows = [r for r in rows if r[0] != r[0]]
    rows = sorted((r for r in rows if r[0] == r[0]), key=lambda r: -r[0])
    print('[ab] it %d: losses replay vs eager %s | grads differing %d of %d, NaN %d' % (
        it, sorted(dl.items())[:8], len(rows) + len(nan_rows), len(ge), len(nan_rows)),
        flush=True)
    for r in nan_rows[:6] + rows[:8]:
        print('[ab]    rel %.3g  |eager| %.4g  %s' % (r[0], r[2], r[1][-90:]), flush=True)
    return data


def _diag(trainer, it):
    """Divergence hunt: non-finite parameters / gradients of every network and spectral-norm
    shadows (optimizers/fused_adam.py) that no longer equal bf16(param)."""
    import torch
    from imaginaire_amd.optimizers import fused_adam as FA
    out = []
    for tag in ('net_G', 'net_D'):
        net = getattr(trainer, tag, None)
        if net is None:
            continue
        bad_p, bad_g, bad_s, n_s = [], [], [], 0
        gn, pmax, top = 0.0, 0.0, ('', 0.0)
        for name, p in net.named_parameters():
            pmax = max(pmax, p.detach().abs().max().item())
            if p.grad is not None:
                g2 = p.grad.detach().float().norm().item()
                gn += g2 * g2
                if g2 > top[1]:
                    top = (name, g2)
            if not torch.isfinite(p).all():
                bad_p.append(name)
            if p.grad is not None and not torch.isfinite(p.grad).all():
                bad_g.append(name)
            sh = FA.shadow_of(p)
            if sh is not None:
                n_s += 1
                d = (sh.float() - p.detach().to(torch.bfloat16).float()).abs().max().item()
                if not d == 0.0:
                    bad_s.append('%s:%.3g' % (name, d))
        out.append('%s |g| %.3g (max %s %.3g) max|p| %.3g nonfinite params %d %s grads %d %s '
                   'shadows %d/%d off %s' % (
                       tag, gn ** 0.5, top[0][-48:], top[1], pmax, len(bad_p), bad_p[:2],
                       len(bad_g), bad_g[:2], len(bad_s), n_s, bad_s[:3]))
    print('[bench_families] it %d diag: %s' % (it, ' | '.join(out)), flush=True)


def _losses(trainer):
    """The last iteration's D and G losses as floats ({'gen': {...}, 'dis': {...}})."""
    import torch
    out = {}
    for part, src in (('gen', getattr(trainer, 'gen_losses', {})),
                      ('dis', getattr(trainer, 'dis_losses', {}))):
        out[part] = {k: round(float(v), 5) for k, v in src.items()
                     if torch.is_tensor(v) and v.numel() == 1}
    return out


def _routing():
    """Autotuned kernel choices of this process (k11 vs MIOpen wgrad, FlowNet2 deconv path) so
    run-to-run throughput differences can be attributed to routing."""
    try:
        from imaginaire_amd.ops import conv as conv_ops
        r = conv_ops.routing_table()
        return {k: {'n': len(v), 'counts': {c: list(v.values()).count(c) for c in set(v.values())}}
                for k, v in r.items()}
    except Exception:  # noqa: BLE001
        return None


if __name__ == '__main__':
    main()
