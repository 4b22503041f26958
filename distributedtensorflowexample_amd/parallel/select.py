"""Choice of the all-reduce backend for the latency-bound MLP gradient.

``pick_small_allreduce`` creates one xGMI communicator per protocol (LL pull,
LL push one-shot, LL push two-shot, flag), verifies each against RCCL on random
gradients (every rank must agree), times all of them and RCCL inside captured
hipGraphs (max over ranks) and returns the fastest -- RCCL whenever no xGMI
protocol is available, correct and faster.  Used by ``bench.py`` and
the mirrored MLP trainer for N > 1.
"""
from __future__ import annotations

import sys
import time

import torch
import torch.distributed as dist

from ..ops import mlp_step
from .xgmi import XgmiComm


def xgmi_protocols(world):
    """Candidate xGMI protocols for a world size.  The LL variants (epoch inside every data
    word) need world <= 8; the flag protocol (separate per-block flags, release-ordered)
    is the fallback beyond that only -- a 3-rank probe caught it serving stale slices
    before its flag store was release-ordered (tools/probes/fused_flake.py)."""
    return ["push2", "push", "ll"] if world <= 8 else ["flag"]


def pick_small_allreduce(rccl, mode, world, rank, dev, iters=200, n=None, xgmi_key="dtfx/xgmi/0",
                         protocols=None, timeout_s=2.0):
    """MLP gradient all-reduce backend.  Every candidate xGMI protocol (``xgmi_protocols``)
    that can be created on every rank and agrees with RCCL on ten random gradients is timed
    against RCCL inside captured hipGraphs (max over ranks, interleaved, best of three); mode
    "auto" returns the fastest of all, mode "xgmi" the fastest xGMI protocol.  Falls back to
    RCCL when no xGMI protocol qualifies.  Every rank takes the same decision (gloo control
    plane).  Returns (communicator, {name: us_per_call} or None)."""
    n = mlp_step.NPARAM if n is None else n

    def agree(ok):
        t = torch.tensor([1 if ok else 0], dtype=torch.int32)
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        return bool(t.item())

    cands = {}
    for proto in (protocols or xgmi_protocols(world)):
        xg, err = None, ""
        try:
            xg = XgmiComm(rank, world, n, device=dev, key="%s/%s" % (xgmi_key, proto),
                          protocol=proto, timeout_s=timeout_s)
        except Exception as e:  # no IPC / peer mapping on this node
            err = repr(e)
            print("[bench] rank %d: xgmi-%s: %s" % (rank, proto, err), file=sys.stderr)
        if not agree(xg is not None):
            if xg is not None:
                xg.destroy()
            if rank == 0:
                print("[bench] xgmi-%s unavailable (%s)" % (proto, err), file=sys.stderr)
            continue
        g = torch.Generator(device="cpu").manual_seed(1000 + rank)
        ok = True
        # Every rank issues the SAME sequence of collectives whatever happens locally: a rank
        # that left this loop early (a timed-out wait raising on it but not on a peer) would
        # leave its peers blocked in the next RCCL call.  Timeouts are read without raising
        # (failed()) and the verdict is agreed on after all ten rounds.
        for it in range(10):  # fresh random gradients: both backends must agree every time
            base = torch.randn(n, generator=g).to(dev) * (1 + it)
            ra, xa = base.clone(), base.clone()
            rccl.allreduce_sum_(ra)
            torch.cuda.synchronize()
            dist.barrier()
            try:
                xg.allreduce_sum_(xa)
                bad = xg.failed()
            except Exception as e:  # noqa: BLE001 - host-side launch error: same on every call
                bad, err = True, repr(e)
            ok &= not bad and bool(((ra - xa).abs().max() <= 1e-5 * ra.abs().max()).item())
        if agree(ok):
            cands["xgmi-" + proto] = xg
        else:
            if rank == 0:
                print("[bench] xgmi-%s failed verification (%s)" % (proto, err), file=sys.stderr)
            xg.destroy()
    if not cands:
        print("[bench] no xgmi protocol available: RCCL", file=sys.stderr)
        return rccl, None
    if mode != "xgmi":
        cands["rccl"] = rccl

    def graph_of(c, buf):
        s = torch.cuda.Stream(dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):
            c.allreduce_sum_(buf)
        torch.cuda.current_stream(dev).wait_stream(s)
        torch.cuda.synchronize()
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr):
            for _ in range(iters):
                c.allreduce_sum_(buf)
        gr.replay()  # warm replay (first-launch costs stay out of the timing)
        torch.cuda.synchronize()
        return gr

    def timed(gr):
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        gr.replay()
        torch.cuda.synchronize()
        dt = torch.tensor([(time.perf_counter() - t0) / iters * 1e6], dtype=torch.float64)
        dist.all_reduce(dt, op=dist.ReduceOp.MAX)
        return float(dt.item())

    names = sorted(cands)  # same order on every rank
    graphs = {k: graph_of(cands[k], torch.zeros(n, device=dev)) for k in names}
    probe = {k: float("inf") for k in names}
    for _ in range(3):  # interleaved, best of three each
        for k in names:
            probe[k] = min(probe[k], timed(graphs[k]))
    for k in names:  # a protocol that timed out on ANY rank is out, on every rank
        if k != "rccl" and not agree(not cands[k].failed()):
            probe[k] = float("inf")
    probe = {k: round(v, 2) for k, v in probe.items()}
    best = min(names, key=lambda k: (probe[k], k))  # times are max-reduced: identical everywhere
    if probe[best] == float("inf"):
        best = "rccl"
        cands["rccl"] = rccl
    for k in names:
        if k not in (best, "rccl"):
            cands[k].destroy()
    if rank == 0:
        print("[bench] small all-reduce probe (us/call, max over ranks): %s -> %s"
              % (probe, best), file=sys.stderr)
    return cands[best], probe


def pick_mlp_engine(params, x, y, batch_size, lr, ar_comm, world, rank, dev, mode="auto",
                    xgmi_key="dtfx/xgmi/fused", verify_steps=20, time_steps=400, x_all=None,
                    timeout_s=2.0):
    """Data-parallel engine of the fused MLP trainer, one of
      ``("allreduce", ar_comm)`` -- flat gradient, separate all-reduce launch, deferred apply;
      ``("fused", XgmiComm)``   -- gradient exchange inside the weight-gradient kernel;
      ``("fused2", XgmiComm)``  -- the same exchange in the two-launch pipelined step (step
                                   t-1's local gradient tiles exchanged and applied inside
                                   step t's forward launch);
      ``("fused2x", XgmiComm)`` -- fused2 with the W1 tiles exchanged two-shot (each element
                                   reduced by one owner rank and broadcast back: 2 (W-1)/W
                                   words per element per rank instead of W-1; world >= 3);
      ``("factor", XgmiComm)``  -- sufficient-factor exchange: the backprop factors dz1 are
                                   all-gathered inside the head kernel and every rank forms
                                   the global W1 gradient from them and every rank's batch
                                   (needs ``x_all`` [world, n, 784], ``x = x_all[rank]``);
      ``("factor2", XgmiComm)`` -- the same exchange in the two-launch pipelined step (the
                                   global update of step t-1 inside step t's forward launch).
    An xGMI engine must (on every rank) build, agree with the all-reduce engine after
    ``verify_steps`` identical SGD steps, keep the replicas bit-identical, and (mode "auto") be
    the fastest over ``time_steps`` graph-replayed steps (max over ranks); mode "fused" /
    "factor" forces that engine once verified.  Every rank takes the same decision.
    Returns (kind, comm, {engine: us_per_step} or None)."""
    from ..train.fused_mlp import FusedMLPTrainer

    def agree(ok):
        t = torch.tensor([1 if ok else 0], dtype=torch.int32)
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        return bool(t.item())

    if world < 2 or world > 8 or mode == "allreduce":
        return "allreduce", ar_comm, None
    kinds = {"auto": ["fused", "fused2", "fused2x", "factor", "factor2"], "fused": ["fused"],
             "fused2": ["fused2"], "fused2x": ["fused2x"], "factor": ["factor"],
             "factor2": ["factor2"]}[mode]
    if world < 3:  # two-shot moves no fewer words than one-shot at 2 ranks, for one more hop
        kinds = [k for k in kinds if k != "fused2x"]
    if x_all is None:
        kinds = [k for k in kinds if not k.startswith("factor")]
    if batch_size > 128:
        kinds = [k for k in kinds if k != "factor2"]
    comms = {}
    for kind in kinds:
        c, err = None, ""
        try:
            c = XgmiComm(rank, world, mlp_step.engine_slot_words(kind), device=dev,
                         key="%s/%s" % (xgmi_key, kind),
                         protocol="push", timeout_s=timeout_s)
        except Exception as e:
            err = repr(e)
            print("[bench] rank %d: %s xgmi engine: %s" % (rank, kind, err), file=sys.stderr)
        if c is not None and kind == "fused2x":
            c.two_shot = True
        if agree(c is not None):
            comms[kind] = c
        else:
            if c is not None:
                c.destroy()
            if rank == 0:
                print("[bench] %s xgmi engine unavailable (%s)" % (kind, err), file=sys.stderr)
    if not comms:
        return "allreduce", ar_comm, None

    def make(kind):
        if kind in ("fused", "fused2", "fused2x"):  # fused2 / fused2x: two-launch pipelined
            return FusedMLPTrainer(params, x, y, batch_size, lr, world_size=world,
                                   fused_comm=comms[kind], pipeline=kind != "fused")
        if kind in ("factor", "factor2"):  # factor2: the two-launch pipelined variant
            return FusedMLPTrainer(params, None, y, batch_size, lr, world_size=world,
                                   factor_comm=comms[kind], x_all=x_all, rank=rank,
                                   pipeline=kind == "factor2")
        return FusedMLPTrainer(params, x, y, batch_size, lr, allreduce=ar_comm.allreduce_sum_,
                               world_size=world)

    ta = make("allreduce")
    ta.run(verify_steps, use_graph=False)
    pa = ta.flush().clone()
    trainers = {"allreduce": ta}
    for kind in list(comms):
        # the control-plane collectives below run on every rank whatever happened locally
        # (an exception on one rank must not leave the others waiting in a broadcast)
        ok, err = True, ""
        chk = torch.full((1,), float("nan"), dtype=torch.float64)
        try:
            tk = make(kind)
            tk.run(verify_steps, use_graph=False)
            pk = tk.flush()
            if comms[kind].failed():  # a timed-out in-kernel wait (no raise: see above)
                ok, err = False, "xGMI exchange timed out waiting for a peer"
            tol = 1e-4 * (1.0 + float(pa.abs().max()))
            ok &= bool(((pk - pa).abs().max() <= tol).item())
            chk = pk.double().sum().reshape(1).cpu()  # replicas must stay bit-identical
        except Exception as e:
            ok, err = False, repr(e)
        ref = chk.clone()
        dist.broadcast(ref, 0)
        ok &= bool(torch.equal(chk, ref))
        if agree(ok):
            trainers[kind] = tk
        else:
            if rank == 0:
                print("[bench] %s xgmi engine failed verification (%s)" % (kind, err),
                      file=sys.stderr)
            comms.pop(kind).destroy()
    if not comms:
        return "allreduce", ar_comm, None
    if mode != "auto":
        kind = next(iter(comms))
        return kind, comms[kind], None

    def timed(tr):
        tr.run(50)  # warm (captures the graphs)
        tr.prepare(time_steps)
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        tr.run(time_steps)
        torch.cuda.synchronize()
        dt = torch.tensor([(time.perf_counter() - t0) / time_steps * 1e6], dtype=torch.float64)
        dist.all_reduce(dt, op=dist.ReduceOp.MAX)
        return float(dt.item())

    names = sorted(trainers)  # same order on every rank
    probe = {k: float("inf") for k in names}
    for _ in range(2):
        for k in names:
            probe[k] = min(probe[k], timed(trainers[k]))
    for k, c in comms.items():  # an engine that timed out on ANY rank is out, on every rank
        if not agree(not c.failed()):
            probe[k] = float("inf")
    probe = {k: round(v, 2) for k, v in probe.items()}
    best = min(names, key=lambda k: (probe[k], k))  # max-reduced: identical everywhere
    if rank == 0:
        print("[bench] MLP step engine probe (us/step, max over ranks): %s -> %s"
              % (probe, best), file=sys.stderr)
    del trainers
    for k in list(comms):
        if k != best:
            comms.pop(k).destroy()
    if best == "allreduce":
        return "allreduce", ar_comm, probe
    return best, comms[best], probe


class HybridComm:
    """RCCL communicator with the large f32 all-reduces routed to the xGMI bandwidth-mode
    two-shot (protocol "bw") where ``pick_large_allreduce`` measured it faster: tensors with
    ``lo <= numel <= bw.max_numel``, f32 and contiguous.  Everything else (other collectives,
    dtypes, sizes) goes to RCCL.  The route depends only on properties every rank shares
    (dtype, numel, ``lo``) -- never on a per-rank property such as the address -- so both
    communicators see the same call sequence on every rank; both are graph-capturable.  A
    routed tensor that is not 16-byte aligned goes through an aligned copy instead of
    silently switching one rank to RCCL (which would leave its peers waiting in the kernel).
    """

    def __init__(self, rccl, bw, lo):
        self.rccl, self.bw, self.lo = rccl, bw, int(lo)
        self.rank, self.world_size = rccl.rank, rccl.world_size
        self.device = getattr(rccl, "device", bw.device)

    def _use_bw(self, t):
        if not (t.is_cuda and t.dtype == torch.float32 and self.lo <= t.numel() <= self.bw.max_numel):
            return False
        if not t.is_contiguous():
            raise ValueError("HybridComm: a routed all-reduce tensor must be contiguous")
        return True

    def _bw_sum(self, t):
        if t.data_ptr() % 16 == 0:
            return self.bw.allreduce_sum_(t)
        tmp = t.clone()  # fresh allocations are 512-byte aligned
        self.bw.allreduce_sum_(tmp)
        return t.copy_(tmp)

    def allreduce_sum_(self, t):
        return self._bw_sum(t) if self._use_bw(t) else self.rccl.allreduce_sum_(t)

    def allreduce_avg_(self, t):
        if self._use_bw(t):
            self._bw_sum(t)
            return t.div_(self.world_size)
        return self.rccl.allreduce_avg_(t)

    def _shard_bw(self, full):
        """Route an in-place reduce-scatter / all-gather over ``full`` to the two-shot's halves
        (same size rule as the all-reduce; bf16 counted in f32 words)."""
        if not (full.is_cuda and full.is_contiguous()):
            return False
        if full.dtype == torch.float32:
            words = full.numel()
        elif full.dtype == torch.bfloat16 and full.numel() % 2 == 0:
            words = full.numel() // 2
        else:
            return False
        return (self.lo <= words <= self.bw.max_numel and words % (4 * self.world_size) == 0
                and full.data_ptr() % 16 == 0)

    def reduce_scatter(self, out, inp):
        if inp.dtype == torch.float32 and self._shard_bw(inp) and \
                out.data_ptr() == inp.data_ptr() + self.rank * out.numel() * 4:
            return self.bw.reduce_scatter(out, inp)
        return self.rccl.reduce_scatter(out, inp)

    def all_gather(self, out, inp):
        if self._shard_bw(out) and \
                inp.data_ptr() == out.data_ptr() + self.rank * inp.numel() * inp.element_size():
            return self.bw.all_gather(out, inp)
        return self.rccl.all_gather(out, inp)

    def check(self):
        self.bw.check()

    def failed(self):
        return self.bw.failed() or bool(getattr(self.rccl, "failed", lambda: False)())

    def abort(self):
        """Peer-watchdog hook: release the two-shot's peer waits (host abort word), then
        abort the RCCL communicator."""
        self.bw.abort()
        ab = getattr(self.rccl, "abort", None)
        if callable(ab):
            ab()

    def __getattr__(self, name):  # broadcast_, reduce_scatter, all_gather, barrier, ...
        return getattr(self.rccl, name)

    def destroy(self):
        self.bw.destroy()


def pick_large_allreduce(rccl, world, rank, dev, max_numel, sizes=None, iters=10,
                         xgmi_key="dtfx/xgmi/bw", timeout_s=2.0, bw_blocks=128,
                         train_timeout_s=None, peer_timeout_s=60.0):
    """Bucketed all-reduce backend for the large gradients (BERT / ResNet buckets): the xGMI
    bandwidth-mode two-shot is created on every rank (or not at all), verified against RCCL
    on random buckets, and timed against RCCL inside captured hipGraphs at each size in
    ``sizes`` (max over ranks, best of three).  Returns ``(HybridComm, probe)`` routing every
    bucket of at least the smallest size from which bw won at every larger probed size, or
    ``(rccl, probe)`` when it never wins.  The same decision on every rank.

    ``timeout_s`` bounds the in-kernel peer waits of the probe; the returned communicator
    waits up to ``train_timeout_s`` (a rank that is away for seconds -- the chief writing a
    checkpoint, first-step graph capture -- must not time its peers out: a timed-out
    two-shot leaves the bucket partly reduced, where RCCL would simply have blocked).
    Trainers still poll ``failed()`` collectively (``check_comm_collective``).

    ``bw_blocks`` (default 128 of the kernel's 256 workgroups): the two-shot runs BESIDE the
    backward on the comm stream, and fewer workgroups take fewer CUs from it -- the simulated
    world-8 step (tools/probes/dp_sim.py, profiles/r5/dp_sim/) ran BERT-base +7.4 % over the
    1-GPU step with 128 against +8.5 % with 256 (+8.0 % with 64), ResNet-50 +5.7 % against +6.5 %.

    Default ``train_timeout_s``: 120 s, independent of the peer watchdog's timeout, so a live
    but slow peer (a chief writing a checkpoint while its heartbeats still flow) does not time
    the two-shot out.  A peer that is really lost is the watchdog's job
    (``--peer_timeout_secs``): its abort hook (``HybridComm.abort`` -> ``XgmiComm.abort``) sets
    the communicator's host-visible abort word, which the kernel's peer waits poll about once
    per millisecond, and calls queued behind read it at entry -- so the two-shot leaves the GPU
    within the watchdog's drain window, before it ends the process.  ``peer_timeout_s`` is
    accepted for compatibility and not used."""
    if train_timeout_s is None:
        train_timeout_s = 120.0
    max_numel = int(max_numel)
    sizes = [s for s in (sizes or (1 << 18, 1 << 20, 1 << 22, 7 << 20, 1 << 24))
             if s <= max_numel] or [max_numel]

    def agree(ok):
        t = torch.tensor([1 if ok else 0], dtype=torch.int32)
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        return bool(t.item())

    bw, err = None, ""
    try:
        bw = XgmiComm(rank, world, max_numel, device=dev, key=xgmi_key, protocol="bw",
                      timeout_s=timeout_s, bw_blocks=bw_blocks)
    except Exception as e:  # no IPC / peer mapping on this node
        err = repr(e)
    if not agree(bw is not None):
        if bw is not None:
            bw.destroy()
        if rank == 0:
            print("[bench] xgmi-bw unavailable (%s): RCCL for every bucket" % err, file=sys.stderr)
        return rccl, None
    g = torch.Generator(device="cpu").manual_seed(2000 + rank)
    ok = True
    for n in (sizes[0] + 3, sizes[-1]):  # (a ragged size too) -- same collectives on every rank
        base = (torch.randn(n, generator=g) * (1 + rank)).to(dev)
        ra, xa = base.clone(), base.clone()
        rccl.allreduce_sum_(ra)
        torch.cuda.synchronize()
        dist.barrier()
        try:
            bw.allreduce_sum_(xa)
            bad = bw.failed()
        except Exception as e:  # noqa: BLE001
            bad, err = True, repr(e)
        ok &= not bad and bool(((ra - xa).abs().max() <= 1e-5 * ra.abs().max()).item())
        del base, ra, xa
    if not agree(ok):
        if rank == 0:
            print("[bench] xgmi-bw failed verification (%s): RCCL" % err, file=sys.stderr)
        bw.destroy()
        return rccl, None

    def timed(c, buf):
        s = torch.cuda.Stream(dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):
            c.allreduce_sum_(buf)
        torch.cuda.current_stream(dev).wait_stream(s)
        torch.cuda.synchronize()
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr):
            for _ in range(iters):
                c.allreduce_sum_(buf)
        gr.replay()
        torch.cuda.synchronize()
        best = float("inf")
        for _ in range(3):
            dist.barrier()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            gr.replay()
            torch.cuda.synchronize()
            dt = torch.tensor([(time.perf_counter() - t0) / iters * 1e6], dtype=torch.float64)
            dist.all_reduce(dt, op=dist.ReduceOp.MAX)
            best = min(best, float(dt.item()))
        return best

    probe = {}
    for n in sizes:
        buf = torch.zeros(n, device=dev)
        probe[n] = {"rccl": round(timed(rccl, buf), 1), "bw": round(timed(bw, buf), 1)}
        del buf
    if not agree(not bw.failed()):
        probe["bw_timed_out"] = True
        bw.destroy()
        return rccl, probe
    lo = None
    for n in reversed(sizes):  # smallest size from which bw wins at every larger size
        if probe[n]["bw"] < probe[n]["rccl"]:
            lo = n
        else:
            break
    if rank == 0:
        print("[bench] large all-reduce probe (us/call, max over ranks): %s -> %s"
              % (probe, "xgmi-bw from %d elements" % lo if lo else "rccl"), file=sys.stderr)
    if lo is None:
        bw.destroy()
        return rccl, probe
    bw.timeout_s = float(train_timeout_s)  # read at every launch / graph capture from here on
    return HybridComm(rccl, bw, lo), probe


def check_comm_collective(comm, where=""):
    """Raise on EVERY rank if the xGMI communicator of ANY rank latched a timed-out in-kernel
    wait (its buffer then holds a partial reduction and the replicas have diverged).  A
    collective over the gloo control plane, so every rank must call it at the same step."""
    failed = getattr(comm, "failed", None)
    bad = bool(failed()) if callable(failed) else False
    if dist.is_initialized() and dist.get_world_size() > 1:
        t = torch.tensor([1 if bad else 0], dtype=torch.int32)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        bad = bool(t.item())
    if bad:
        raise RuntimeError("xGMI all-reduce timed out waiting for a peer%s: replicas are no "
                           "longer identical" % ((" (" + where + ")") if where else ""))
