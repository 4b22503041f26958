"""Fused MNIST-MLP training engine: three HIP launches per step, hipGraph-replayed.

This is the MI355X-native replacement of the reference's per-step session
loop (worker.py:129-159).  Per step the reference makes three gRPC round
trips (pull 318 KB, push 318 KB + remote ApplyGradientDescent, AssignAdd),
a host->GPU feed of 317 KB and ~14 tiny TF kernels.  Here:

* the dataset is resident in HBM; each launch gets its batch's pointer, and
  one hipGraph is captured per epoch (``nbatches`` steps), so replaying it
  walks the dataset like ``next_batch`` with no host work per step;
* on one GPU the step is TWO launches (``pipeline=True``, default):
  ``mlp_fwdapply`` applies step t-1's update -- formed tile by tile from the
  factors the previous head left behind, never stored as a gradient -- and runs
  step t's forward; ``mlp_head`` finishes step t.  The last update stays pending
  until ``flush()`` (ping-pong parameter buffers, like the DP path below).
  ``pipeline=False``: the three-launch step ``mlp_fwd`` / ``mlp_head`` /
  ``mlp_wgrad`` with the SGD apply fused into ``mlp_wgrad``'s epilogue;
* in sync data-parallel mode the flat 318 KB gradient is all-reduced after
  ``mlp_wgrad`` by a pluggable ``allreduce(grad)`` callable (RCCL through
  ``torch.distributed`` or the native communicator) and applied, averaged
  through ``lr / world_size``, inside the next step's ``mlp_fwd``/``mlp_head``;
* or, with ``fused_comm`` (an ``XgmiComm`` with protocol "push"), the gradient
  exchange is fused into ``mlp_wgrad``'s epilogue (LL words pushed straight to
  the peers, gathered, summed in rank order and applied in the same launch):
  three launches per data-parallel step, no pending gradient;
* or, with ``factor_comm`` (also protocol "push") and ``x_all`` [world, n, 784]
  -- every rank's deterministic batch stream resident on every GPU, as every
  reference process loads the whole dataset (main.py:43-44) -- the ranks
  all-gather only the backprop factors dz1 (40 KB) inside ``mlp_head`` and
  each forms the global W1 gradient itself (sufficient-factor exchange);
* ``global_step`` is a device counter advanced by the kernels (AssignAdd of
  worker.py:32,141); loss/accuracy land in a device ring read back lazily.

Data-parallel update order: the all-reduced gradient of step t is applied at
the start of step t+1 (ping-pong parameter buffers make the apply race-free
across the launch's workgroups).  ``flush()`` applies the pending gradient,
so ``params`` after ``flush()`` is exactly the result of t full SGD steps.
"""
from __future__ import annotations

import os
import time

import torch

from ..ops import mlp_step, optim
from ..ops._ext import stream_handle


class FusedMLPTrainer:
    def __init__(self, params, x, labels, batch_size=100, learning_rate=0.001, allreduce=None,
                 world_size=1, stats_ring=4096, global_step=0, max_graph_steps=1024,
                 fused_comm=None, factor_comm=None, x_all=None, rank=0, pipeline=True):
        if not params.is_cuda:
            raise ValueError("FusedMLPTrainer runs on the GPU; use the generic path on CPU")
        if params.numel() != mlp_step.NPARAM:
            raise ValueError("params must be the flat 79,510-element MLP buffer")
        self.device = params.device
        self.B = int(batch_size)
        self.lr = float(learning_rate)
        self.world_size = int(world_size)
        self.allreduce = allreduce
        self.fused_comm = fused_comm
        if fused_comm is not None and (allreduce is not None or world_size < 2):
            raise ValueError("fused_comm replaces allreduce and needs world_size >= 2")
        self.factor_comm = factor_comm
        self.xstride = 0
        if factor_comm is not None:
            if fused_comm is not None or allreduce is not None or world_size < 2:
                raise ValueError("factor_comm replaces allreduce/fused_comm and needs world >= 2")
            if (x_all is None or x_all.dim() != 3 or x_all.shape[0] != world_size
                    or not x_all.is_contiguous() or x_all.dtype != torch.float32
                    or x_all.device != self.device):
                raise ValueError("factor_comm needs x_all: contiguous f32 [world, n, 784] on the GPU")
            x = x_all[int(rank)]  # a view: the other ranks' batches sit at +/- xstride
            self.xstride = x_all.stride(0)
            self.dz1A = torch.zeros(world_size * mlp_step.factor_plane(int(batch_size)),
                                    device=self.device, dtype=torch.float32)
        x = x.reshape(-1, mlp_step.D).to(self.device, torch.float32).contiguous()
        if factor_comm is not None and x.data_ptr() != x_all[int(rank)].data_ptr():
            raise ValueError("x_all slice must stay a view")
        labels = labels.reshape(-1).to(self.device, torch.int32).contiguous()
        self.nbatches = x.shape[0] // self.B
        if self.nbatches < 1:
            raise ValueError("dataset smaller than one batch")
        self.x, self.labels = x, labels
        self.bufs = [params.detach().clone().contiguous(), torch.empty_like(params)]
        self.cur = 0
        self.grad = torch.zeros_like(params)
        self.ws = mlp_step.StepWorkspace(self.B, self.device, stats_ring)
        self.ws.set_global_step(global_step)
        self.pos = int(global_step) % self.nbatches  # next batch (host mirror)
        self.pending = False
        # single GPU without a communicator, the fused engine or the factor engine (batch
        # <= 128): the two-launch pipelined step
        self.pipelined = bool(pipeline and allreduce is None and (
            (self.world_size == 1 and factor_comm is None and fused_comm is None)
            or fused_comm is not None
            or (factor_comm is not None and self.B <= 128)))
        self.max_graph_steps = int(max_graph_steps)
        self._graphs = {}
        self._pool = None
        self._ll = None   # granule buffer of the persistent engine (allocated on first use)
        self._ebase = 0   # epoch base of its next launch
        self._unchecked = False  # a persistent launch whose hand-offs were not verified yet
        self._host_args = None   # run_launched's cached launcher and buffer addresses

    # -- state --------------------------------------------------------------
    @property
    def direct(self):
        """SGD apply fused into the backward kernel (one GPU, or the fused xGMI exchange)."""
        return not self.pipelined and (
            self.fused_comm is not None or self.factor_comm is not None
            or (self.allreduce is None and self.world_size == 1))

    def _verified(self):
        """Raise before parameters or stats of a persistent launch whose in-kernel hand-off
        timed out are used (that launch writes zeros instead of valid parameters)."""
        if self._unchecked:
            self._unchecked = False
            self.check()

    @property
    def params(self):
        """Current parameters (excludes a pending, not yet applied gradient)."""
        self._verified()
        return self.bufs[self.cur]

    def flush(self):
        """Apply the pending update in place (DP: p -= lr/N * grad; pipelined: the last
        step's factors)."""
        self._verified()
        if self.pending:
            if self.pipelined and self.factor_comm is not None:
                xp, _ = self.batch((self.pos - 1) % self.nbatches)
                mlp_step.flush_factor(self.bufs[self.cur], xp, self.ws, self.lr / self.world_size,
                                      self.factor_comm, self.dz1A, self.xstride)
            elif self.pipelined and self.fused_comm is not None:
                xp, _ = self.batch((self.pos - 1) % self.nbatches)
                mlp_step.flush_xgmi(self.bufs[self.cur], self.bufs[self.cur ^ 1], xp, self.ws,
                                    self.lr / self.world_size, self.fused_comm)
                self.cur ^= 1
            elif self.pipelined:
                xp, _ = self.batch((self.pos - 1) % self.nbatches)
                mlp_step.flush_pipelined(self.bufs[self.cur], self.bufs[self.cur ^ 1], xp, self.ws,
                                         self.lr)
                self.cur ^= 1
            else:
                optim.sgd_(self.bufs[self.cur], self.grad, self.lr / self.world_size)
            self.pending = False
        return self.bufs[self.cur]

    def snapshot(self):
        """Parameters after every step run so far (a pending update included) as a NEW
        tensor, WITHOUT changing the trainer: no peer exchange starts and the replicas' update
        sequence is untouched, so one rank alone may call it (chief-only checkpoints and
        evals).  The all-reduce engine's pending gradient is already reduced: applied to a
        copy.  A pending update of the pipelined exchange engines needs every rank's
        exchange: raises (call flush() on every rank instead)."""
        self._verified()
        p = self.bufs[self.cur]
        if not self.pending:
            return p.clone()
        if not self.pipelined:
            out = p.clone()
            optim.sgd_(out, self.grad, self.lr / self.world_size)
            return out
        if self.world_size == 1:
            return self.flush().clone()
        raise RuntimeError("snapshot(): the pending update is a peer exchange; flush() on "
                           "every rank first")

    def load_params(self, p):
        self.bufs[self.cur].copy_(p)
        self.pending = False

    def global_step(self) -> int:
        # the pipelined step records step t (stats, global_step += 1) inside step t+1's
        # first launch (or flush())
        return self.ws.global_step() + (1 if (self.pipelined and self.pending) else 0)

    def batch(self, i):
        sl = slice(i * self.B, (i + 1) * self.B)
        return self.x[sl], self.labels[sl]

    # -- one step (eager) -----------------------------------------------------
    def _step_launches(self):
        xb, yb = self.batch(self.pos)
        self.pos = (self.pos + 1) % self.nbatches
        if self.factor_comm is not None and self.pipelined:
            xp, _ = self.batch((self.pos - 2) % self.nbatches)  # pos already advanced
            mlp_step.step_factor_pipelined(self.bufs[self.cur], self.bufs[self.cur ^ 1], xp, xb,
                                           yb, self.ws, self.lr / self.world_size, self.pending,
                                           self.factor_comm, self.dz1A, self.xstride)
            self.cur ^= 1
            self.pending = True
            return
        if self.factor_comm is not None:
            mlp_step.step_factor(self.bufs[self.cur], xb, yb, self.ws, self.lr / self.world_size,
                                 self.factor_comm, self.dz1A, self.xstride)
            return
        if self.fused_comm is not None and self.pipelined:
            xp, _ = self.batch((self.pos - 2) % self.nbatches)  # pos already advanced
            mlp_step.step_xgmi_pipelined(self.bufs[self.cur], self.bufs[self.cur ^ 1], xp, xb,
                                         yb, self.ws, self.lr / self.world_size, self.pending,
                                         self.fused_comm)
            self.cur ^= 1
            self.pending = True
            return
        if self.fused_comm is not None:
            mlp_step.step_xgmi(self.bufs[self.cur], xb, yb, self.ws, self.lr / self.world_size,
                               self.fused_comm)
            return
        if self.direct:
            mlp_step.step_direct(self.bufs[self.cur], xb, yb, self.ws, self.lr)
            return
        if self.pipelined:
            xp, _ = self.batch((self.pos - 2) % self.nbatches)  # pos already advanced
            mlp_step.step_pipelined(self.bufs[self.cur], self.bufs[self.cur ^ 1], xp, xb, yb,
                                    self.ws, self.lr, apply=self.pending)
            self.cur ^= 1
            self.pending = True
            return
        cur = self.bufs[self.cur]
        if self.pending:
            mlp_step.step_grad(cur, xb, yb, self.ws, self.grad, prev_grad=self.grad,
                               lr=self.lr / self.world_size, p_new=self.bufs[self.cur ^ 1])
            self.cur ^= 1
        else:
            mlp_step.step_grad(cur, xb, yb, self.ws, self.grad)
        if self.allreduce is not None:
            self.allreduce(self.grad)
        self.pending = True

    def step(self):
        self._step_launches()

    # -- hipGraph capture/replay ---------------------------------------------
    def _graph(self, n):
        """Graph of ``n`` steps starting at batch ``self.pos`` and parity ``self.cur``.

        Capture records without executing, so only the host mirrors (batch
        position, ping-pong parity, pending flag) move during capture; they are
        restored afterwards and advanced by the caller at replay.
        """
        key = (n, self.pos, self.cur)
        g = self._graphs.get(key)
        if g is None:
            pos, cur, pend = self.pos, self.cur, self.pending
            assert self.direct or pend
            s = torch.cuda.Stream(self.device)
            s.wait_stream(torch.cuda.current_stream(self.device))
            g = torch.cuda.CUDAGraph()
            with torch.cuda.stream(s):
                with torch.cuda.graph(g, pool=self._pool, stream=s):
                    for _ in range(n):
                        self._step_launches()
            torch.cuda.current_stream(self.device).wait_stream(s)
            self._pool = g.pool()
            self.pos, self.cur, self.pending = pos, cur, pend
            self._graphs[key] = g
        return g

    def _plan(self, steps):
        """Split ``steps`` into epoch-aligned graph chunks -> list of n."""
        out, pos = [], self.pos
        while steps > 0:
            n = min(steps, self.nbatches - pos, self.max_graph_steps)
            out.append(n)
            pos = (pos + n) % self.nbatches
            steps -= n
        return out

    @property
    def host_loop_ok(self):
        """The step can be issued by a C++ host loop: the plain single-GPU pipelined step
        (``mlp_run_pipelined``) or a pipelined exchange engine -- fused2 / fused2x / factor2
        (``XgmiComm`` ``mlp_run_engine``)."""
        if not self.pipelined or self.allreduce is not None:
            return False
        if self.world_size == 1:
            return self.fused_comm is None and self.factor_comm is None
        c = self.fused_comm if self.fused_comm is not None else self.factor_comm
        return c is not None and hasattr(getattr(c, "_h", None), "mlp_run_engine")

    def run_launched(self, steps, flush=False):
        """``steps`` pipelined single-GPU steps issued by ONE C++ call (kernel launches, no
        graph): no ~15 us graph-submission latency before the first kernel.  ``flush``: the
        last step's update is applied by the same call (one more launch, as ``flush()``).
        The buffer addresses are read once: a short timed region (bench.py --steps 20) pays
        the Python side of this call before its first kernel starts."""
        steps = int(steps)
        if not self.host_loop_ok:
            raise RuntimeError("run_launched: pipelined single-GPU step or exchange engine only")
        if steps <= 0:
            if flush:
                self.flush()
            return
        if self.world_size > 1:
            return self._run_launched_engine(steps, flush)
        a = self._host_args
        if a is None:
            from ..ops._ext import hip, ptr

            ws = self.ws
            if os.environ.get("DTFX_MLP_PLAN", "1") != "0":
                # the buffers bound once in a C++ plan: the call before the first kernel
                # converts 7 arguments instead of 17 (a short timed region starts on the host)
                plan = hip().MlpRunPlan(ptr(self.bufs[0]), ptr(self.bufs[1]), ptr(self.x),
                                        ptr(self.labels), self.nbatches, ptr(ws.buf),
                                        ptr(ws.ctr), ptr(ws.stats), ws.stats_ring, self.B)
                a = self._host_args = (plan.run, self.device.index, None)
            else:  # (A/B: the 17-argument entry point)
                a = self._host_args = (hip().mlp_run_pipelined, self.device.index,
                                       (ptr(self.bufs[0]), ptr(self.bufs[1]), ptr(self.x),
                                        ptr(self.labels), ptr(ws.buf), ptr(ws.ctr),
                                        ptr(ws.stats), ws.stats_ring))
        run, dix, full = a
        if full is None:
            run(self.cur, 1 if self.pending else 0, self.lr, self.pos, steps, 1 if flush else 0,
                stream_handle(dix))
        else:
            p0, p1, xp, lp, wb, wc, wst, ring = full
            run(p0, p1, self.cur, 1 if self.pending else 0, self.lr, xp, lp, self.nbatches,
                self.pos, steps, wb, wc, wst, ring, self.B, stream_handle(dix), 1 if flush else 0)
        self.pos = (self.pos + steps) % self.nbatches
        self.cur ^= (steps + (1 if flush else 0)) & 1
        self.pending = not flush

    def _run_launched_engine(self, steps, flush):
        """run_launched for the pipelined exchange engines: every rank issues the same steps
        from one C++ call (the in-kernel exchanges pair them up across ranks)."""
        from ..ops._ext import ptr

        factor = self.factor_comm is not None
        comm = self.factor_comm if factor else self.fused_comm
        kind = 2 if factor else (1 if getattr(comm, "two_shot", False) else 0)
        a = self._host_args
        if a is None:
            ws = self.ws
            a = self._host_args = (comm._h.mlp_run_engine, ptr(self.bufs[0]), ptr(self.bufs[1]),
                                   ptr(self.x), ptr(self.labels), ptr(ws.buf), ptr(ws.ctr),
                                   ptr(ws.stats), ws.stats_ring,
                                   ptr(self.dz1A) if factor else 0)
        fn, p0, p1, xp, lp, wb, wc, wst, ring, dz = a
        fn(kind, p0, p1, self.cur, 1 if self.pending else 0, self.lr / self.world_size, xp,
           int(self.xstride), lp, self.nbatches, self.pos, steps, wb, wc, wst, ring, self.B, dz,
           stream_handle(self.device.index), float(comm.timeout_s),
           1 if flush else 0)
        self.pos = (self.pos + steps) % self.nbatches
        self.cur ^= (steps + (1 if (flush and not factor) else 0)) & 1
        self.pending = not flush

    # -- persistent single-launch engine (csrc/kernels/mlp_persistent.hip) ----------------
    @property
    def persistent_ok(self):
        """The plain single-GPU step with batch <= 128 can run as ONE persistent launch."""
        return self.host_loop_ok and self.world_size == 1 and self.B <= 128

    def run_persistent(self, steps, timeout_s=2.0, trace=None):
        """``steps`` complete SGD steps (every update applied, nothing left pending) in ONE
        launch: 105 co-resident workgroups hand z1 partials / backprop factors / small
        parameters to each other as epoch-tagged 8-byte granules instead of ending a kernel.
        Same trajectory as the pipelined two-launch step (to f32 rounding).  ``timeout_s`` bounds every in-kernel
        wait; a timed-out run raises at the next ``check()``.  ``trace``: optional int64
        [blocks, trace_steps, 12] buffer of in-kernel s_memrealtime stamps (probe only)."""
        from ..ops._ext import hip, ptr, stream_handle

        steps = int(steps)
        if not self.persistent_ok:
            raise RuntimeError("run_persistent: single-GPU step with batch <= 128 only")
        if steps <= 0:
            return
        self.flush()  # a pending pipelined update is applied first (params exact)
        h = hip()
        if self._ll is None or self._ebase + steps + 2 >= 2 ** 32:
            self._ll = torch.zeros(int(h.mlp_persistent_ll_words()), dtype=torch.int64,
                                   device=self.device)
            self._ebase = 0
        ws = self.ws
        h.mlp_persistent(ptr(self.bufs[self.cur]), ptr(self.x), ptr(self.labels), self.nbatches,
                         self.pos, steps, self.lr, self._ebase, ptr(self._ll), ptr(ws.ctr),
                         ptr(ws.stats), ws.stats_ring, self.B, int(timeout_s * 1e8),
                         stream_handle(), 0 if trace is None else ptr(trace))
        self._ebase += steps + 1
        self.pos = (self.pos + steps) % self.nbatches
        self._unchecked = True

    def check(self):
        """Raise if an in-kernel wait of the persistent engine, or of the terminal head +
        apply launch of ``run_launched(.., flush=True)``, ever timed out."""
        if self._ll is not None and int(self._ll[-32].item()) != 0:
            raise RuntimeError("persistent MLP engine: an in-kernel hand-off timed out "
                               "(parameters are not valid)")
        ws = getattr(self, "ws", None)
        if ws is not None and ws.buf.is_cuda:
            sync = ws.buf[-4:].view(torch.int32)  # mlp::Bufs::sync (the workspace's last words)
            if int(sync[2].item()) != 0:
                sync.zero_()
                raise RuntimeError("fused MLP step: the terminal head + apply hand-off timed "
                                   "out (the last update was not applied)")
        self._unchecked = False  # verified

    def run(self, steps, use_graph=True, lead=0):
        """Run ``steps`` training steps (epoch-aligned hipGraph replays).  ``lead`` > 0 (single
        GPU): the first ``lead`` steps are launched directly from C++ so the GPU starts at
        once, and the graph replay of the rest is submitted while they run."""
        steps = int(steps)
        if not use_graph:
            for _ in range(steps):
                self._step_launches()
            return
        if lead > 0 and self.host_loop_ok:
            k = min(int(lead), steps)
            self.run_launched(k)
            steps -= k
        if steps > 0 and not self.direct and not self.pending:
            self._step_launches()  # the first DP step has nothing to apply
            steps -= 1
        for n in self._plan(steps):
            self._graph(n).replay()
            self.pos = (self.pos + n) % self.nbatches
            if not self.direct:
                self.cur ^= n & 1

    def prepare(self, steps, lead=0):
        """Capture (not run) every graph a following ``run(steps, lead=lead)`` replays."""
        steps = int(steps)
        if steps > 0 and not self.direct and not self.pending:
            raise RuntimeError("prepare() in DP mode needs one eager step first")
        pos, cur = self.pos, self.cur
        if lead > 0 and self.host_loop_ok:
            k = min(int(lead), steps)
            self.pos = (self.pos + k) % self.nbatches
            self.cur ^= k & 1
            steps -= k
        for n in self._plan(steps):
            self._graph(n)
            self.pos = (self.pos + n) % self.nbatches
            if not self.direct:
                self.cur ^= n & 1
        self.pos, self.cur = pos, cur

    # -- observability ------------------------------------------------------
    def stats(self, step=None):
        """(loss, accuracy) recorded by the kernel for ``step`` (default: last)."""
        self._verified()
        if self.pipelined and self.pending:
            self.flush()  # the last step's record is written by its apply
        s = (self.global_step() - 1) if step is None else int(step)
        v = self.ws.stats[s % self.ws.stats_ring].tolist()
        return float(v[0]), float(v[1])

    def stats_range(self, start, end):
        """Loss/accuracy for steps [start, end) as a CPU tensor [n, 2]."""
        self._verified()
        if self.pipelined and self.pending:
            self.flush()
        ring = self.ws.stats_ring
        if end - start > ring:
            start = end - ring
        idx = torch.arange(start, end) % ring
        return self.ws.stats[idx.to(self.device)].cpu()


def benchmark_steps(trainer, steps, warmup, barrier=None, use_graph=True):
    """Time exactly ``steps`` steps after ``warmup`` (synchronised both sides)."""
    trainer.run(warmup, use_graph)
    if use_graph:
        trainer.prepare(steps)
    if barrier:
        barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    trainer.run(steps, use_graph)
    torch.cuda.synchronize()
    if barrier:
        barrier()
    return time.perf_counter() - t0
