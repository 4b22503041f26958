"""Fail-fast for synchronous data parallelism: a lost peer ends every rank promptly.

The reference gets this from TF: a worker whose gRPC peer disappears gets an error out
of ``sess.run`` and ``managed_session`` ends the process (worker.py:107-123, main.py:51-55,
SURVEY 5.3).  In sync DP the failure mode is different -- a rank whose peer died sits
inside a collective: gloo eventually times out (``--dist_timeout_secs``), but an RCCL or
xGMI all-reduce on the GPU waits on device memory the dead peer never writes, with the
host thread blocked in a stream wait.  :class:`PeerWatchdog` closes that gap:

* every rank bumps a heartbeat counter ``dtfx/hb/<rank>`` in the job's TCPStore (the
  rendezvous store torch.distributed already holds) every ``interval`` seconds from a
  daemon thread that never touches the GPU;
* it reads the peers' counters; a counter that has not moved for ``timeout`` seconds, or a
  store that stops answering (rank 0 hosts it), is a lost peer -- unless that peer first
  published ``dtfx/hb/<rank>/done`` (an orderly end: :meth:`stop`);
* on a lost peer it runs the registered abort hooks (``NativeComm.abort`` =
  ``ncclCommAbort``, which makes the RCCL kernels return), lets the device drain for at
  most ``drain_secs`` and ends the process with ``exit_code`` -- the launcher
  (``launch.launch_mirrored``) or torch.distributed.run then stops the remaining ranks.
"""
from __future__ import annotations

import contextlib
import os
import sys
import threading
import time

EXIT_PEER_LOST = 75


class PeerWatchdog:
    def __init__(self, store, rank, world_size, timeout=60.0, interval=1.0, drain_secs=10.0,
                 exit_code=EXIT_PEER_LOST, prefix="dtfx/hb", on_lost=None):
        self.store, self.rank, self.world = store, int(rank), int(world_size)
        self.timeout, self.interval = float(timeout), float(interval)
        self.drain_secs, self.exit_code = float(drain_secs), int(exit_code)
        self.prefix = prefix
        self.on_lost = on_lost  # tests: called instead of ending the process
        self._hooks = []
        self._stop = threading.Event()
        self._thread = None
        self.lost = None  # (peer or None, reason) once a loss was detected

    # -- public -----------------------------------------------------------------------------
    def add_abort_hook(self, fn):
        """``fn()`` runs (exceptions ignored) before the process ends on a lost peer."""
        self._hooks.append(fn)
        return self

    def start(self):
        if self.world < 2 or self.timeout <= 0:
            return self
        self.store.add(self._key(self.rank), 1)
        self._thread = threading.Thread(target=self._run, name="dtfx-peer-watchdog", daemon=True)
        self._thread.start()
        return self

    def stop(self, done=True):
        """Join the thread.  ``done`` (an orderly end): publish ``done`` so peers stop watching
        this rank.  Without it (this rank is failing) the heartbeat just stops and the peers
        declare this rank lost after ``timeout``."""
        if self._thread is None:
            return
        self._stop.set()
        self._thread.join(timeout=5 * self.interval + 5)
        self._thread = None
        if done:
            try:
                self.store.add(self._key(self.rank) + "/done", 1)
            except Exception:  # noqa: BLE001 -- the store host already left: nothing to tell
                pass

    # -- internals --------------------------------------------------------------------------
    def _key(self, r):
        return "%s/%d" % (self.prefix, r)

    def _run(self):
        seen = {p: (-1, time.monotonic()) for p in range(self.world) if p != self.rank}
        done = set()
        while not self._stop.wait(self.interval):
            try:
                self.store.add(self._key(self.rank), 1)
                now = time.monotonic()
                for p in list(seen):
                    if p in done:
                        continue
                    if self.store.add(self._key(p) + "/done", 0) > 0:
                        done.add(p)
                        continue
                    v = self.store.add(self._key(p), 0)
                    last, t = seen[p]
                    if v != last:
                        seen[p] = (v, now)
                    elif now - t > self.timeout:
                        return self._fail(p, "no heartbeat for %.1f s" % (now - t))
            except Exception as e:  # noqa: BLE001 -- the store (rank 0's) is gone
                if self._stop.is_set():
                    return
                return self._fail(None, "rendezvous store unreachable: %r" % (e,))

    def _fail(self, peer, reason):
        self.lost = (peer, reason)
        who = "rank %d" % peer if peer is not None else "the job"
        print("[watchdog] rank %d: lost %s (%s): aborting communicators and exiting with %d"
              % (self.rank, who, reason, self.exit_code), file=sys.stderr, flush=True)
        for fn in self._hooks:
            try:
                fn()
            except Exception as e:  # noqa: BLE001
                print("[watchdog] abort hook failed: %r" % (e,), file=sys.stderr, flush=True)
        if self.on_lost is not None:
            self.on_lost(peer, reason)
            return
        self._drain()
        os._exit(self.exit_code)

    def _drain(self):
        """Give in-flight kernels up to ``drain_secs`` to finish (the aborted RCCL kernels
        return at once; the xGMI kernels end at their own in-kernel timeout) so the process
        does not end with waves still resident."""
        try:
            import torch

            if not (torch.cuda.is_available() and torch.cuda.is_initialized()):
                return
        except Exception:  # noqa: BLE001
            return
        t = threading.Thread(target=torch.cuda.synchronize, daemon=True)
        t.start()
        t.join(self.drain_secs)


def start_for_job(comm=None, timeout=60.0, interval=1.0, key="dtfx/hb"):
    """The watchdog of this torch.distributed job (default store), with ``comm.abort`` as the
    abort hook when the communicator has one.  Returns None for a single process."""
    import torch.distributed as dist

    if not dist.is_initialized() or dist.get_world_size() < 2 or timeout <= 0:
        return None
    store = dist.distributed_c10d._get_default_store()
    wd = PeerWatchdog(store, dist.get_rank(), dist.get_world_size(), timeout=timeout,
                      interval=interval, prefix=key)
    abort = getattr(comm, "abort", None)
    if callable(abort):
        wd.add_abort_hook(abort)
    return wd.start()


_SCOPES = [0]


@contextlib.contextmanager
def watch_peers(comm=None, timeout=60.0, interval=1.0):
    """Watch the peers for the duration of a training loop.  A normal exit publishes
    ``done`` (a peer still finishing -- the chief's final checkpoint -- never counts this
    rank as lost); an exception only stops the heartbeat, so the peers, blocked in a
    collective this rank will never join, declare it lost and exit too."""
    _SCOPES[0] += 1  # a fresh key per scope: several training runs in one job
    wd = start_for_job(comm, timeout, interval, key="dtfx/hb/%d" % _SCOPES[0])
    try:
        yield wd
    except BaseException:
        if wd is not None:
            wd.stop(done=False)
        raise
    else:
        if wd is not None:
            wd.stop(done=True)


def init_process_group_with_timeout(backend="gloo", timeout_secs=None):
    """``dist.init_process_group`` with ``--dist_timeout_secs`` as the collective timeout (a
    gloo collective whose peer vanished raises after that long instead of torch's 30 min)."""
    import datetime

    import torch.distributed as dist

    kw = {}
    if timeout_secs:
        kw["timeout"] = datetime.timedelta(seconds=float(timeout_secs))
    dist.init_process_group(backend, **kw)


def maybe_inject_fault(rank, step):
    """Fault injection (tests only): ``DTFX_FAULT_KILL_AT_STEP=<rank>:<step>``
    SIGKILLs rank ``rank`` once its training loop has passed global step ``step`` -- a rank
    that dies without any chance to clean up, as on a node or driver failure."""
    spec = os.environ.get("DTFX_FAULT_KILL_AT_STEP")
    if not spec:
        return
    r, s = (int(v) for v in spec.split(":"))
    if int(rank) == r and int(step) >= s:
        import signal

        print("[fault-injection] rank %d: SIGKILL at step %d" % (rank, step), flush=True)
        os.kill(os.getpid(), signal.SIGKILL)
