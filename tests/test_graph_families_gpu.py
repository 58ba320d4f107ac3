"""hipGraph-captured training iterations of the non-SPADE families vs the same iteration run
eagerly (GPU): MUNIT, pix2pixHD (capture-safe instance pooling), vid2vid and few-shot vid2vid
(the whole per-frame D / G update loop of a sequence as one graph).

The replayed iteration is compared with an eager iteration taken from the SAME saved state
(parameters, buffers, optimizer state) on the same batch, with the RNG reseeded identically
before each (graph-safe RNG: the replay draws from the generator's current seed/offset), so
the losses must agree to bf16 / atomic-order tolerance and the G update must point the same
way. Reference trainers: trainers/munit.py:210-241, trainers/vid2vid.py:238-288."""
import os

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _build(name, seq_len=None):
    from torch.utils.data import default_collate
    from imaginaire_amd.config import Config
    from imaginaire_amd.datasets.synthetic import Dataset
    from imaginaire_amd.utils.trainer import get_model_optimizer_and_scheduler, get_trainer
    torch.manual_seed(0)
    cfg = Config(os.path.join(ROOT, 'configs', 'unit_test', name + '.yaml'))
    cfg.speed_benchmark = False
    cfg.logdir = '/tmp/iamd_graph_fam_' + name
    video = hasattr(cfg.data, 'num_frames_G')
    if video and seq_len:
        cfg.data.train.initial_sequence_length = seq_len
        cfg.data.train.max_sequence_length = seq_len
    ds = Dataset(cfg)

    class _Loader(list):
        dataset = ds

    nets = get_model_optimizer_and_scheduler(cfg, seed=0)
    tr = get_trainer(cfg, *nets, train_data_loader=_Loader(), val_data_loader=None)
    if video and seq_len:
        if hasattr(tr, 'init_temporal_network'):
            tr.init_temporal_network()
        ds.set_sequence_length(seq_len)
        tr.sequence_length = seq_len
    bs = cfg.data.train.batch_size
    dev = torch.device('cuda', 0)

    def to_dev(x):
        if torch.is_tensor(x):
            return x.to(dev)
        if isinstance(x, dict):
            return {k: to_dev(v) for k, v in x.items()}
        if isinstance(x, list):
            return [to_dev(v) for v in x]
        return x
    batches = [to_dev(default_collate([ds[(i * bs + j) % max(1, len(ds))] for j in range(bs)]))
               for i in range(2)]
    return cfg, tr, batches


def _fresh(x):
    if torch.is_tensor(x):
        return x.clone()
    if isinstance(x, dict):
        return {k: _fresh(v) for k, v in x.items()}
    if isinstance(x, list):
        return [_fresh(v) for v in x]
    return x


def _state(tr):
    ts = list(tr.net_G.parameters()) + list(tr.net_G.buffers())
    ts += list(tr.net_D.parameters()) + list(tr.net_D.buffers())
    for o in (tr.opt_G, tr.opt_D):
        for st in o.state.values():
            ts += [v for v in st.values() if torch.is_tensor(v)]
        ts += [g['_hyper'] for g in o.param_groups if '_hyper' in g]
    return ts


def _losses(tr):
    out = {}
    for tag, d in (('D', tr.dis_losses), ('G', tr.gen_losses)):
        for k, v in d.items():
            if torch.is_tensor(v) and v.numel() == 1:
                out[tag + '/' + k] = float(v)
    return out


def _cases_worker(cases, q):
    """Capture + replay vs eager for every family, all in ONE process (see the test)."""
    import faulthandler
    import sys
    faulthandler.dump_traceback_later(170 * len(cases), exit=True, file=sys.__stderr__)
    for name, seq_len in cases:
        try:
            q.put((name, 'ok', _run_case(name, seq_len)))
        except BaseException as e:  # noqa: BLE001 - reported to the parent
            import traceback
            q.put((name, 'error', '%s: %s\n%s' % (type(e).__name__, e, traceback.format_exc())))


def _run_case(name, seq_len):
    from imaginaire_amd.utils.cuda_graph import graph_routing, make_trainer_step
    torch.cuda.set_device(0)
    # deterministic kernels on both paths: the flow-warp backward's image scatter (k9) uses
    # float atomics in the default mode, so vid2vid's replay and eager run would otherwise differ
    # in the last bits of the flow gradients and drift apart over the frames of a sequence
    torch.use_deterministic_algorithms(True, warn_only=True)
    cfg, tr, batches = _build(name, seq_len)
    capturable = bool(getattr(tr, 'graph_capturable', False))
    step, graphed = make_trainer_step(tr, warmup=2, enabled=True)
    if graphed is None:
        return {'capturable': capturable, 'graphed': False}
    for i in range(3):  # 2 eager warm-up iterations, then capture (+ first replay)
        torch.manual_seed(3)
        step(tr.start_of_iteration(_fresh(batches[i % 2]), i))
    torch.cuda.synchronize()
    captured = graphed.graph is not None and not graphed.failed
    state = _state(tr)
    saved = [t.detach().clone() for t in state]
    gparams = list(tr.net_G.parameters())
    p0 = [p.detach().clone() for p in gparams]
    d = tr.start_of_iteration(_fresh(batches[1]), 3)
    torch.manual_seed(11)
    graphed(d)
    torch.cuda.synchronize()
    lg = _losses(tr)
    dg = [p.detach() - q for p, q in zip(gparams, p0)]
    gg = [None if p.grad is None else p.grad.detach().float().clone() for p in gparams]
    with torch.no_grad():
        for t, c in zip(state, saved):
            t.copy_(c)
    torch.cuda.synchronize()
    d = tr.start_of_iteration(_fresh(batches[1]), 3)
    torch.manual_seed(11)
    with graph_routing():  # the kernels the capture recorded
        graphed.step_fn(d)
    torch.cuda.synchronize()
    le = _losses(tr)
    de = [p.detach() - q for p, q in zip(gparams, p0)]
    ge = [None if p.grad is None else p.grad.detach().float() for p in gparams]
    gnum = sum(float((x - y).pow(2).sum()) for x, y in zip(gg, ge) if x is not None)
    gden = sum(float(y.pow(2).sum()) for x, y in zip(gg, ge) if x is not None)
    names = [n for n, _ in tr.net_G.named_parameters()]
    bad = [n for n, x in zip(names, dg) if not torch.isfinite(x).all()]
    bad_eager = [n for n, x in zip(names, de) if not torch.isfinite(x).all()]
    num = sum(float((x - y).float().pow(2).sum()) for x, y in zip(dg, de))
    den = sum(float(y.float().pow(2).sum()) for y in de)
    return {'capturable': capturable, 'graphed': True, 'captured': captured, 'lg': lg,
            'le': le, 'bad': bad[:8], 'bad_eager': bad_eager[:8], 'num': num, 'den': den, 'gnum': gnum, 'gden': gden}


_CASES = [('munit', None), ('pix2pixHD', None), ('vid2vid_street', 3), ('fs_vid2vid_face', 2)]
_RESULTS = {}


def _results():
    """Run every family case once, sequentially in one spawned process that shares its
    allocator history across them (the setting in which round 3 saw fs-vid2vid's eager
    iteration drift from its replay: FlowNet2's 2 -> 2 flow upsamplers ran MIOpen backward-data
    solvers inside the graph, whose workspace zeroing the capture does not record; they now run
    k10 phase convolutions)."""
    if not _RESULTS:
        import multiprocessing as mp
        ctx = mp.get_context('spawn')
        q = ctx.Queue()
        proc = ctx.Process(target=_cases_worker, args=(_CASES, q))
        proc.start()
        try:
            for _ in _CASES:
                name, status, res = q.get(timeout=190)
                _RESULTS[name] = (status, res)
        finally:
            proc.join(30)
            if proc.is_alive():
                proc.kill()
    return _RESULTS


@pytest.mark.gpu
@pytest.mark.parametrize('name,seq_len', _CASES)
def test_family_graph_replay_matches_eager(name, seq_len):
    """The replayed iteration equals the eager one from the same state: losses to 1e-3 and the
    G gradients to 1e-2 relative L2 (both paths run the same kernels). The G UPDATE is
    compared more loosely: the first Adam steps move each weight by ~lr * sign(grad), so
    rounding-level differences of near-zero gradients flip whole-size update elements."""
    status, res = _results()[name]  # (run under torch.use_deterministic_algorithms)
    assert status == 'ok', res
    assert res['capturable'], name + ' is not marked capturable'
    assert res['graphed'] and res['captured'], 'step was not captured'
    lg, le = res['lg'], res['le']
    print(name, 'graph', lg, '\n', name, 'eager', le)
    assert not res['bad'], 'non-finite replayed G updates: %s (eager: %s; losses %s / %s)' % (
        res['bad'], res['bad_eager'], lg, le)
    assert lg.keys() == le.keys() and lg
    for k in le:
        assert lg[k] == lg[k], k  # finite
        assert abs(lg[k] - le[k]) <= 1e-3 * max(1.0, abs(le[k])), (k, lg[k], le[k])
    assert res['gden'] > 0 and res['gnum'] <= 1e-4 * res['gden'], (res['gnum'], res['gden'])
    assert res['den'] > 0 and res['num'] <= 1e-2 * res['den'], (res['num'], res['den'])
