"""Training-session lifecycle (``tf.train.Supervisor`` + ``managed_session``).

What the reference relies on (worker.py:107-123):

* chief (task 0): restore the latest checkpoint in ``logdir`` or run
  ``init_op``; then ``local_init_op``; write the graph (``graph.pbtxt`` in
  ``logdir`` + a ``graph_def`` event); start a checkpoint thread
  (``save_model_secs``) and a ``global_step/sec`` summary thread
  (``save_summaries_secs``);
* non-chief: poll ``ready_op`` (the list of uninitialized global variables)
  every ``recovery_wait_secs`` until empty, then ``local_init_op``;
* ``should_stop()`` / ``request_stop()`` via a coordinator; exiting the
  managed session stops and joins the service threads.

Everything is passed as callables so the same Supervisor drives the async
PS mode (variables on the parameter server) and the sync-DP mode (variables
replicated on the GPUs).

``checkpoint_on_main_thread=True`` (sync-DP trainers): the timer thread only
*requests* a checkpoint and the training loop performs it between steps via
:meth:`Supervisor.service`.  A trainer whose parameters live in ping-pong
device buffers with deferred updates (``train/fused_mlp.py``) must never be
read from another thread: flushing it there would mutate trainer state
concurrently with the loop and, with the xGMI exchange engines, start a peer
exchange that only the chief joins.
"""
from __future__ import annotations

import contextlib
import os
import threading
import time

from .saver import latest_checkpoint


class Coordinator:
    def __init__(self):
        self._stop = threading.Event()
        self._exc = None

    def request_stop(self, ex=None):
        if ex is not None and self._exc is None:
            self._exc = ex
        self._stop.set()

    def should_stop(self):
        return self._stop.is_set()

    def wait_for_stop(self, timeout=None):
        return self._stop.wait(timeout)

    def raise_requested_exception(self):
        if self._exc is not None:
            raise self._exc


class _LoopThread(threading.Thread):
    """TF's ``LooperThread`` with a timer: with ``run_at_start`` the first call happens when
    the thread starts ("next timer time starts as now"), which is why a TF chief writes
    ``model.ckpt-<start step>`` right after init/restore; later calls every ``period`` s."""

    def __init__(self, coord, period, fn, name, run_at_start=False):
        super().__init__(name=name, daemon=True)
        self.coord, self.period, self.fn = coord, float(period), fn
        self.run_at_start = bool(run_at_start)
        self._halt = threading.Event()

    def run(self):
        nxt = time.time() + (0.0 if self.run_at_start else self.period)
        while not self.coord.should_stop() and not self._halt.is_set():
            if self._halt.wait(max(nxt - time.time(), 0.0)):
                break
            nxt += self.period
            try:
                self.fn()
            except Exception as e:  # report, keep training (TF logs and continues)
                print("[supervisor] %s failed: %r" % (self.name, e), flush=True)

    def halt(self):
        self._halt.set()


class Supervisor:
    def __init__(self, is_chief=True, logdir=None, saver=None, summary_writer=None,
                 ready_op=None, global_step=None, save_model_secs=600, save_summaries_secs=120,
                 init_op=None, local_init_op=None, recovery_wait_secs=30, save_variables=None,
                 checkpoint_basename="model.ckpt", ready_timeout_secs=None, final_checkpoint=False,
                 checkpoint_on_main_thread=False, graph=None):
        self.is_chief = bool(is_chief)
        self.logdir = logdir
        self.saver = saver
        self.summary_writer = summary_writer
        self.ready_op = ready_op
        self.global_step = global_step
        self.save_model_secs = save_model_secs
        self.save_summaries_secs = save_summaries_secs
        self.init_op = init_op
        self.local_init_op = local_init_op
        self.recovery_wait_secs = recovery_wait_secs
        self.save_variables = save_variables
        self.save_path = os.path.join(logdir, checkpoint_basename) if logdir else None
        self.ready_timeout_secs = ready_timeout_secs
        self.final_checkpoint = final_checkpoint
        self.checkpoint_on_main_thread = bool(checkpoint_on_main_thread)
        self.graph = graph  # utils.graph.GraphDefBuilder: written by the chief at start
        self._ckpt_request = threading.Event()
        self.coord = Coordinator()
        self._threads = []
        self.restored_from = None

    # -- session bring-up ----------------------------------------------------
    def prepare_or_wait_for_session(self):
        if self.is_chief:
            ckpt = latest_checkpoint(self.logdir) if (self.logdir and self.saver) else None
            if ckpt:
                self.saver.restore(None, ckpt)
                self.restored_from = ckpt
            elif self.init_op is not None:
                self.init_op()
        else:
            self.wait_for_ready()
        if self.local_init_op is not None:
            self.local_init_op()
        if self.is_chief:
            self.start_standard_services()
        return self

    def wait_for_ready(self):
        if self.ready_op is None:
            return
        t0 = time.time()
        while True:
            not_ready = self.ready_op()
            if not not_ready:
                return
            if self.ready_timeout_secs is not None and time.time() - t0 > self.ready_timeout_secs:
                raise TimeoutError("variables never initialized by the chief: %s" % (not_ready,))
            if self.coord.wait_for_stop(self.recovery_wait_secs):
                raise RuntimeError("stop requested while waiting for the chief")

    # -- services (chief) -----------------------------------------------------
    def save_checkpoint(self):
        if self.saver is None or self.save_path is None:
            return None
        step = self.global_step() if callable(self.global_step) else self.global_step
        return self.saver.save(None, self.save_path, global_step=step,
                               variables=self.save_variables() if self.save_variables else None)

    def checkpoint_pending(self):
        """A main-thread checkpoint was requested and not yet written."""
        return self._ckpt_request.is_set()

    def service(self):
        """Run requested main-thread services (``checkpoint_on_main_thread``): call between
        training steps.  Returns the checkpoint path when one was written."""
        if self._ckpt_request.is_set():
            self._ckpt_request.clear()
            return self.save_checkpoint()
        return None

    def write_graph(self):
        """TF's Supervisor (chief): ``graph.pbtxt`` into ``logdir`` and the GraphDef through the
        summary writer (TensorBoard's Graphs tab)."""
        if self.graph is None:
            return
        if self.logdir:
            os.makedirs(self.logdir, exist_ok=True)
            with open(os.path.join(self.logdir, "graph.pbtxt"), "w") as f:
                f.write(self.graph.to_pbtxt())
        if self.summary_writer is not None and hasattr(self.summary_writer, "add_graph"):
            self.summary_writer.add_graph(self.graph)

    def start_standard_services(self):
        self.write_graph()
        if self.saver is not None and self.save_model_secs and self.save_path:
            fn = self._ckpt_request.set if self.checkpoint_on_main_thread else self.save_checkpoint
            self._threads.append(_LoopThread(self.coord, self.save_model_secs, fn,
                                             "SVTimerCheckpointThread", run_at_start=True))
        if self.summary_writer is not None and self.save_summaries_secs and self.global_step:
            state = {"t": time.time(), "s": self._step()}

            def step_rate():
                now, s = time.time(), self._step()
                rate = (s - state["s"]) / max(now - state["t"], 1e-9)
                state["t"], state["s"] = now, s
                self.summary_writer.add_summary({"global_step/sec": rate}, s)

            self._threads.append(_LoopThread(self.coord, self.save_summaries_secs, step_rate,
                                             "SVStepCounterThread"))
        for t in self._threads:
            t.start()

    def _step(self):
        g = self.global_step
        return int(g() if callable(g) else (g or 0))

    # -- coordination ---------------------------------------------------------
    def should_stop(self):
        return self.coord.should_stop()

    def request_stop(self, ex=None):
        self.coord.request_stop(ex)

    def stop(self, close_summary_writer=True):
        self.coord.request_stop()
        for t in self._threads:
            t.halt()
            t.join(timeout=60)
        self._threads = []
        if self.is_chief and self.final_checkpoint:
            self.save_checkpoint()
        if close_summary_writer and self.summary_writer is not None:
            self.summary_writer.close()

    @contextlib.contextmanager
    def managed_session(self, master=None, config=None, start_standard_services=True,
                        close_summary_writer=True):
        sess = self.prepare_or_wait_for_session()
        try:
            yield sess
        except Exception as e:
            self.request_stop(e)
            raise
        finally:
            self.stop(close_summary_writer)
