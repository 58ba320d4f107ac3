"""Failure detection, fault injection and straggler monitoring for multi-GPU training.

The reference (SURVEY §5 "Failure detection") has only ``faulthandler.enable()``
(/root/reference/train.py:5), apex's overflow skip and restart-with-auto-resume
(/root/reference/imaginaire/trainers/base.py:225-233). At one process per MI355X
and 8 ranks per node the common failure is not a crash but a *hang*: one rank
stuck in an RCCL collective or a GPU wait while the others block on it. This
module adds:

* :class:`Watchdog` — a per-rank hang detector built on CPython's native
  ``faulthandler`` watchdog thread (a C thread that does not need the GIL, so it
  fires even when the main thread is blocked inside a HIP/RCCL call). The loop
  calls :meth:`Watchdog.beat` once per iteration; if no beat arrives within
  ``timeout`` seconds every Python thread's stack is written to
  ``<logdir>/hang_rank<R>.txt`` and the process exits (status 1, faulthandler's
  ``_exit``) so ``torch.distributed.run --max-restarts`` can restart the
  job, which then auto-resumes from ``latest_checkpoint.txt``.
* :class:`FaultInjector` — ``IMAGINAIRE_AMD_FAULT=<kind>@<iteration>[:<rank>]``
  (kinds ``hang``, ``crash``, ``nan``) drives the detection and recovery paths
  deliberately, for tests and drills.
* :class:`StragglerMonitor` — at logging boundaries, one all-gather of every
  rank's mean iteration time; rank 0 reports the slowest rank and its ratio to
  the median (a slow rank sets the whole job's step time under synchronous DP).
* :func:`dist_timeout` — the process-group timeout (collective hang bound) from
  ``IMAGINAIRE_AMD_DIST_TIMEOUT_S``.
"""
import datetime
import faulthandler
import math
import os
import sys
import time

import torch

CRASH_EXIT_CODE = 87


def dist_timeout(default_s=1800):
    """Timeout handed to ``init_process_group``: a collective that does not complete
    within it raises (gloo) or aborts the communicator (RCCL with async error handling)."""
    return datetime.timedelta(seconds=float(os.environ.get('IMAGINAIRE_AMD_DIST_TIMEOUT_S',
                                                           default_s)))


def _rank():
    try:
        import torch.distributed as dist
        if dist.is_available() and dist.is_initialized():
            return dist.get_rank()
    except Exception:  # noqa: BLE001
        pass
    return int(os.environ.get('RANK', 0))


class Watchdog(object):
    """Iteration-heartbeat hang detector.

    ``timeout`` <= 0 disables it. The first beat arms it (so model construction,
    MIOpen find and hipGraph capture in the first iterations are covered by the
    ``first_timeout`` grace period instead of the steady-state bound).
    """

    def __init__(self, timeout, logdir=None, first_timeout=None, exit_on_hang=True):
        self.timeout = float(timeout or 0)
        self.first_timeout = float(first_timeout if first_timeout is not None
                                   else max(self.timeout, 0) * 10)
        self.exit_on_hang = exit_on_hang
        self.rank = _rank()
        self.path = None
        self._file = None
        self.beats = 0
        if self.enabled:
            d = logdir or '.'
            os.makedirs(d, exist_ok=True)
            self.path = os.path.join(d, 'hang_rank%d.txt' % self.rank)

    @property
    def enabled(self):
        return self.timeout > 0

    def _open(self):
        if self._file is None:
            self._file = open(self.path, 'w')
        return self._file

    def beat(self, iteration=None, phase='iteration', grace=False):
        """Re-arm the deadline. Writes a one-line header naming the last completed
        iteration so the report says *where* the job stalled, then re-arms the native
        watchdog thread (the traceback goes right after the header).

        ``grace=True`` arms the long ``first_timeout`` bound instead: for phases that are
        legitimately slower than a steady-state iteration (checkpoint save, FID / metrics,
        end of epoch, data-loader start-up and first use of new shapes in the next
        iteration). The next plain beat restores the steady-state bound."""
        if not self.enabled:
            return
        deadline = self.first_timeout if grace else self._deadline()
        f = self._open()
        f.seek(0)
        f.truncate()
        f.write('rank %d: no progress within %.0f s after %s %s (beat %d, %s)\n' % (
            self.rank, deadline, phase, iteration, self.beats,
            time.strftime('%Y-%m-%d %H:%M:%S')))
        f.flush()
        faulthandler.dump_traceback_later(deadline, repeat=False, file=f,
                                          exit=self.exit_on_hang)
        self.beats += 1

    def grace(self, iteration=None, phase='phase'):
        """Context manager: the body runs under the long bound; leaving it re-arms the
        steady-state bound (the following iteration must then finish within ``timeout``)."""
        wd = self

        class _Grace(object):
            def __enter__(self):
                wd.beat(iteration, phase, grace=True)
                return wd

            def __exit__(self, *exc):
                if exc[0] is None:
                    wd.beat(iteration, 'after ' + phase)
                return False
        return _Grace()

    def _deadline(self):
        return self.first_timeout if self.beats == 0 else self.timeout

    def disarm(self):
        if self.enabled:
            faulthandler.cancel_dump_traceback_later()
        if self._file is not None:
            self._file.close()
            self._file = None
            # a clean shutdown leaves no hang report behind
            try:
                os.remove(self.path)
            except OSError:
                pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.disarm()
        return False


class FaultInjector(object):
    """``IMAGINAIRE_AMD_FAULT`` = comma-separated ``kind@iteration[:rank]`` entries.

    * ``hang``  — the rank sleeps forever at the start of that iteration (the peers block
      in their next collective; the watchdogs / process-group timeout must end the job);
    * ``crash`` — the rank exits at once with ``CRASH_EXIT_CODE`` (a lost process);
    * ``nan``   — the iteration's input images are poisoned with NaN (exercises
      ``trainer.skip_nonfinite_steps`` and the meters' non-finite reporting).
    Without a rank the fault fires on every rank.
    """

    KINDS = ('hang', 'crash', 'nan')

    def __init__(self, spec=None, rank=None):
        spec = os.environ.get('IMAGINAIRE_AMD_FAULT', '') if spec is None else spec
        self.rank = _rank() if rank is None else rank
        self.faults = []
        for item in filter(None, (s.strip() for s in spec.split(','))):
            kind, _, rest = item.partition('@')
            it, _, rk = rest.partition(':')
            if kind not in self.KINDS or not it:
                raise ValueError('IMAGINAIRE_AMD_FAULT: bad entry %r (want kind@iter[:rank], '
                                 'kind in %s)' % (item, self.KINDS))
            self.faults.append((kind, int(it), int(rk) if rk else None))

    def __bool__(self):
        return bool(self.faults)

    def _due(self, iteration):
        return [k for k, it, rk in self.faults
                if it == iteration and (rk is None or rk == self.rank)]

    def apply(self, iteration, data=None):
        """Call at the start of an iteration, before the step; returns ``data``."""
        for kind in self._due(iteration):
            sys.stderr.write('[fault-inject] rank %d: %s at iteration %d\n' % (
                self.rank, kind, iteration))
            sys.stderr.flush()
            if kind == 'crash':
                os._exit(CRASH_EXIT_CODE)
            if kind == 'hang':
                while True:
                    time.sleep(3600)
            if kind == 'nan' and isinstance(data, dict):
                for k in ('images', 'label'):
                    v = data.get(k)
                    if torch.is_tensor(v) and v.is_floating_point():
                        v.fill_(float('nan'))
        return data


class StragglerMonitor(object):
    """Per-rank iteration timing; :meth:`report` all-gathers the mean iteration time of
    every rank (one tiny collective, only at logging boundaries) and returns
    ``(slowest_rank, slowest_ms, median_ms, ratio)`` on every rank."""

    def __init__(self, warn_ratio=1.25):
        self.warn_ratio = warn_ratio
        self._t = None
        self._sum = 0.0
        self._n = 0
        self.last = None

    def tick(self):
        now = time.perf_counter()
        if self._t is not None:
            self._sum += now - self._t
            self._n += 1
        self._t = now

    def report(self, device=None):
        import torch.distributed as dist
        mean_ms = 1e3 * self._sum / max(self._n, 1)
        self._sum, self._n = 0.0, 0
        if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() < 2:
            self.last = (0, mean_ms, mean_ms, 1.0)
            return self.last
        if device is None:
            device = torch.device('cuda', torch.cuda.current_device()) \
                if dist.get_backend() == 'nccl' else torch.device('cpu')
        t = torch.tensor([mean_ms], dtype=torch.float64, device=device)
        out = torch.empty(dist.get_world_size(), dtype=torch.float64, device=device)
        dist.all_gather_into_tensor(out, t)
        times = out.cpu().tolist()
        order = sorted(times)
        median = order[len(order) // 2] if len(order) % 2 else \
            0.5 * (order[len(order) // 2 - 1] + order[len(order) // 2])
        slow = max(range(len(times)), key=lambda i: times[i])
        ratio = times[slow] / median if median > 0 else math.inf
        self.last = (slow, times[slow], median, ratio)
        if ratio > self.warn_ratio and _rank() == 0:
            print('[straggler] rank %d: %.1f ms/iter vs median %.1f ms (x%.2f)' % (
                slow, times[slow], median, ratio))
        return self.last
