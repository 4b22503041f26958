"""xGMI peer-memory all-reduce communicators: LL one-/two-shot for small buckets and the
bandwidth-mode two-shot ("bw") for large ones; ``HybridComm`` routes by bucket size.

Wraps ``csrc/kernels/xgmi_allreduce.hip`` / ``xgmi_comm.cpp``: every rank
exports an uncached IPC slot, the handles are exchanged through the
torch.distributed TCP store, and each ``allreduce_sum_`` is ONE kernel that
publishes, flags and sums straight from peer memory over the direct xGMI
links (protocol: ``docs/COMM.md``).  Graph-capturable (epochs live on the
device).  Only f32, and only up to ``max_numel`` elements.  The LL protocols exist for the
latency-bound 318 KB gradient of the MNIST MLP; the "bw" protocol (f32 payload, per-block
release flags, all W-1 links at once) for large buckets, where it is selected against RCCL
per bucket size at startup (``select.pick_large_allreduce`` -> ``select.HybridComm``).
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from ..ops import hip


class XgmiComm:
    def __init__(self, rank, world_size, max_numel, device=None, store=None,
                 key="dtfx/xgmi/0", timeout_s=2.0, protocol=None, bw_blocks=None):
        self.rank, self.world_size = int(rank), int(world_size)
        self.device = torch.device("cuda", torch.cuda.current_device() if device is None
                                   else torch.device(device).index)
        self.timeout_s = float(timeout_s)
        self.max_numel = int(max_numel)
        # fused MLP engine: exchange the W1 gradient tiles two-shot (reduce-scatter +
        # all-gather inside the kernel) instead of one-shot (set by the engine selection)
        self.two_shot = False
        # "ll": 8-byte {value, epoch} words (no flag round trip; world <= 8); "flag": slots +
        # per-block epoch flags (any world <= 16)
        self.protocol = protocol or ("ll" if self.world_size <= 8 else "flag")
        if store is None:
            store = dist.distributed_c10d._get_default_store()
        # Every rank ALWAYS publishes its key -- an empty handle when its own allocation or
        # export failed -- so no peer blocks in store.get on a rank that gave up; every rank
        # then fails the same way (callers agree on availability through a collective).
        err, handle = None, b""
        try:
            self._h = hip().XgmiAllReduce(self.rank, self.world_size, self.device.index,
                                          self.max_numel, self.protocol)
            handle = self._h.handle()
        except Exception as e:  # noqa: BLE001 - re-raised below, after publishing
            err, self._h = e, None
        store.set("%s/%d" % (key, self.rank), handle)
        handles = [bytes(store.get("%s/%d" % (key, j))) for j in range(self.world_size)]
        if err is not None:
            raise RuntimeError("xgmi rank %d: %r" % (self.rank, err))
        missing = [j for j, h in enumerate(handles) if not h]
        if missing:
            self._h.close()
            raise RuntimeError("xgmi: ranks %s could not export their buffers" % missing)
        self._h.open(handles)
        if bw_blocks is not None:
            self._h.set_bw_blocks(int(bw_blocks))

    @classmethod
    def with_local_peers(cls, rank, world_size, max_numel, regions=None, device=None,
                         protocol="push", timeout_s=2.0, bw_blocks=None):
        """Test harness ("peer buffers that are local allocations"): a communicator
        for ``rank`` of a ``world_size``-rank job whose peer slot regions are plain allocations
        on this device -- ``regions`` (one int64 tensor per rank, ``region_words`` long) or new
        zeroed ones.  The kernels and the slot layout are those of a real communicator; one
        process can therefore run ANY rank's kernels of ANY world size, with the other ranks'
        words staged into the regions by the caller.  Returns (comm, regions)."""
        self = cls.__new__(cls)
        self.rank, self.world_size = int(rank), int(world_size)
        self.device = torch.device("cuda", torch.cuda.current_device() if device is None
                                   else torch.device(device).index)
        self.timeout_s = float(timeout_s)
        self.max_numel = int(max_numel)
        self.protocol = protocol
        self.two_shot = False
        self._h = hip().XgmiAllReduce(self.rank, self.world_size, self.device.index,
                                      self.max_numel, protocol, False)
        words = self._h.region_bytes() // 8
        if regions is None:
            regions = [torch.zeros(words, dtype=torch.int64, device=self.device)
                       for _ in range(self.world_size)]
        if len(regions) != self.world_size or any(
                r.dtype != torch.int64 or r.numel() < words or not r.is_cuda for r in regions):
            raise ValueError("need %d int64 device regions of >= %d words" % (world_size, words))
        self._h.open_local([r.data_ptr() for r in regions])
        if bw_blocks is not None:
            self._h.set_bw_blocks(int(bw_blocks))
        self.regions = regions
        return self, regions

    @property
    def slot_stride(self):
        """Elements per slot (S): the stride of the LL slot layout (``docs/COMM.md``)."""
        return self._h.slot_stride()

    def allreduce_sum_(self, t):
        if not (t.is_cuda and t.dtype == torch.float32 and t.is_contiguous()):
            raise ValueError("XgmiComm: contiguous f32 GPU tensors only")
        if t.numel() > self.max_numel:
            raise ValueError("XgmiComm: %d elements > max_numel %d" % (t.numel(), self.max_numel))
        self._h.all_reduce(t.data_ptr(), t.numel(), torch.cuda.current_stream().cuda_stream,
                           self.timeout_s)
        return t

    def _shard_view(self, out, inp, dtype_ok=(torch.float32,)):
        """(f32 word view of ``inp``, its word count) for an in-place shard op: ``out`` must be
        this rank's chunk of ``inp`` (``inp[rank * n : (rank + 1) * n]``, n = out.numel()).
        bf16 tensors travel as f32 words (all-gather only: the
        kernel moves them, it does not sum them)."""
        if inp.dtype not in dtype_ok or out.dtype != inp.dtype:
            raise ValueError("XgmiComm shard op: dtype %s not supported here" % inp.dtype)
        if not (inp.is_cuda and inp.is_contiguous() and out.is_contiguous()):
            raise ValueError("XgmiComm shard op: contiguous GPU tensors only")
        n = out.numel()
        if inp.numel() != n * self.world_size or \
                out.data_ptr() != inp.data_ptr() + self.rank * n * inp.element_size():
            raise ValueError("XgmiComm shard op: out must be this rank's chunk of inp (in place)")
        words = inp.view(torch.float32) if inp.dtype != torch.float32 else inp
        if words.numel() % (4 * self.world_size) or words.numel() > self.max_numel:
            raise ValueError("XgmiComm shard op: %d words (need a multiple of %d, <= %d)"
                             % (words.numel(), 4 * self.world_size, self.max_numel))
        return words

    def reduce_scatter(self, out, inp):
        """In-place reduce-scatter (protocol "bw"): ``out`` = this rank's chunk of ``inp``
        receives the sum over ranks of that chunk."""
        w = self._shard_view(out, inp)
        self._h.shard_op(1, w.data_ptr(), w.numel(), torch.cuda.current_stream().cuda_stream,
                         self.timeout_s)
        return out

    def all_gather(self, out, inp):
        """In-place all-gather (protocol "bw"): every rank's chunk ``inp`` of ``out`` lands in
        every rank's ``out``.  f32 or bf16 (moved as f32 words)."""
        w = self._shard_view(inp, out, (torch.float32, torch.bfloat16))
        self._h.shard_op(2, w.data_ptr(), w.numel(), torch.cuda.current_stream().cuda_stream,
                         self.timeout_s)
        return out

    def mlp_wgrad(self, p, lr, x, ws, stats=True):
        """MNIST-MLP weight-gradient launch with the gradient all-reduce fused into its
        epilogue (protocol "push"): ``p -= lr * sum over ranks of the gradient``; see
        ``ops.mlp_step.step_xgmi``."""
        from ..ops._ext import ptr

        self._h.mlp_wgrad(ptr(p), float(lr), ptr(x), ptr(ws.buf), ptr(ws.ctr),
                          ptr(ws.stats) if stats else 0, ws.stats_ring, ws.B,
                          torch.cuda.current_stream().cuda_stream, self.timeout_s)

    def mlp_head(self, p, labels, ws, dz1A, nslab=7):
        """Factor engine: MLP head launch that also all-gathers every rank's backprop factors
        dz1 into ``dz1A`` [world, BP, 112] (row-major; protocol "push"); see ``ops.mlp_step.step_factor``.
        ``nslab``: partial-z1 planes left by the forward (7: 3-launch, 28: pipelined)."""
        from ..ops._ext import ptr

        self._h.mlp_head(ptr(p), ptr(labels), ptr(ws.buf), ptr(dz1A), ws.B,
                         torch.cuda.current_stream().cuda_stream, self.timeout_s, int(nslab))

    def mlp_fwdapply_factor(self, p_old, p_new, lr, x_prev, x, xstride, dz1A, ws, apply,
                            stats=True):
        """Pipelined factor engine, first launch: step t-1's global W1 update from the
        gathered factors and every rank's previous batch (+ small-parameter exchange),
        fused with step t's forward; ``p_old`` -> ``p_new``."""
        from ..ops._ext import ptr

        self._h.mlp_fwdapply_factor(ptr(p_old), ptr(p_new), float(lr) if apply else 0.0,
                                    ptr(x_prev if apply else x), ptr(x), int(xstride), ptr(dz1A),
                                    ptr(ws.buf), ptr(ws.ctr), ptr(ws.stats) if stats else 0,
                                    ws.stats_ring, ws.B, 1 if apply else 0,
                                    torch.cuda.current_stream().cuda_stream, self.timeout_s)

    def mlp_fwdapply(self, p_old, p_new, lr, x_prev, x, ws, apply, stats=True, trace=None):
        """Pipelined fused engine, first launch: step t-1's local gradient tiles (from the
        factors its head left in ``ws`` and ``x_prev``) exchanged with the peers, summed in
        rank order and applied ``p_old`` -> ``p_new``, fused with step t's forward.
        ``trace``: int64 [blocks * 4, 8] in-kernel stamp buffer (probe builds, world 2/4/8)."""
        from ..ops._ext import ptr

        self._h.mlp_fwdapply(ptr(p_old), ptr(p_new), float(lr) if apply else 0.0,
                             ptr(x_prev if apply else x), ptr(x), ptr(ws.buf), ptr(ws.ctr),
                             ptr(ws.stats) if stats else 0, ws.stats_ring, ws.B,
                             1 if apply else 0, torch.cuda.current_stream().cuda_stream,
                             self.timeout_s, 1 if self.two_shot else 0,
                             0 if trace is None else ptr(trace))

    def mlp_wgrad_factor(self, p, lr, x, xstride, dz1A, ws, stats=True):
        """Factor engine: global dW1 from the gathered factors and every rank's batch
        (``x`` = this rank's batch, rank q's at ``x + (q - rank) * xstride`` elements),
        small-parameter gradients exchanged, SGD applied in place."""
        from ..ops._ext import ptr

        self._h.mlp_wgrad_factor(ptr(p), float(lr), ptr(x), int(xstride), ptr(dz1A), ptr(ws.buf),
                                 ptr(ws.ctr), ptr(ws.stats) if stats else 0, ws.stats_ring, ws.B,
                                 torch.cuda.current_stream().cuda_stream, self.timeout_s)

    def broadcast_(self, t, root=0):
        """Broadcast as a sum with zeros off the root (small control-path use)."""
        if self.rank != root:
            t.zero_()
        return self.allreduce_sum_(t)

    def allreduce_max_(self, t):
        """Element-wise max over ranks for control-path checks (``--check_replicas_every``):
        over the default torch.distributed group (the gloo control plane), not xGMI."""
        c = t.detach().cpu()
        dist.all_reduce(c, op=dist.ReduceOp.MAX)
        t.copy_(c)
        return t

    def failed(self):
        """True if any call timed out waiting for a peer (synchronizes the device)."""
        torch.cuda.synchronize(self.device)
        return bool(self._h.error())

    def check(self):
        """Raise if any all-reduce timed out waiting for a peer (synchronizes the device)."""
        torch.cuda.synchronize(self.device)
        if self._h.error():
            raise RuntimeError("xGMI all-reduce timed out waiting for a peer")

    def abort(self):
        """Peer-watchdog abort hook: every bandwidth-mode peer wait of this communicator
        (running or queued) gives up within ~1 ms and latches ``failed()``.  A host store to a
        pinned word -- no HIP call, no GIL held in C++ -- so it is safe from the watchdog
        thread while the stream is blocked in the kernel."""
        if self._h is not None:
            self._h.abort()

    def destroy(self):
        self._h.close()


class SimulatedPeersComm:
    """Rank 0 of a ``world_size``-rank data-parallel job on ONE GPU, for timing the DP shape of
    a training step: every all-reduce runs the real bandwidth-mode
    two-shot kernel (``xgmi_bw_kernel<W>``, protocol "bw") of rank 0 over simulated local
    peers -- its reduce-scatter stores into the W-1 "peer" receive slots, the owner sum over
    W contributions and the all-gather copies, all in this GPU's HBM, every peer flag
    pre-raised (``XgmiComm.with_local_peers``).  So a trainer driven with it runs its world > 1
    path exactly (comm stream, bucket hooks, no split-K fold, side-stream defaults, 1/W
    scaling) and its comm kernels compete with the backward for CUs and HBM as on a node --
    minus the link time, which this cannot show.  The simulated peers never write: their
    contributions and their reduced chunks read as zeros, so the result keeps only this rank's
    own chunk (chunk 0 of W, unscaled) and zeros elsewhere -- a timing harness, not a
    training one (``tests/test_xgmi_sim_gpu.py::test_simulated_peers_comm_shape``).

    Buckets above ``max_numel`` elements are reduced in ``max_numel`` pieces."""

    def __init__(self, world_size, max_numel, device=None, bw_blocks=None, timeout_s=5.0):
        self.rank, self.world_size = 0, int(world_size)
        self.comm, regs = XgmiComm.with_local_peers(0, self.world_size, int(max_numel),
                                                    device=device, protocol="bw",
                                                    timeout_s=timeout_s, bw_blocks=bw_blocks)
        self.device = self.comm.device
        self.max_numel = int(max_numel)
        W, S = self.world_size, self.comm.slot_stride
        CS = ((S + W - 1) // W + 3) // 4 * 4
        f0 = 2 * W * CS + 2 * S  # the flag array, past the data slots (xgmi_ll_bytes, XG_BW)
        for r in regs:  # every flag any call could wait for: already raised (epoch 0x7fffffff)
            r.view(torch.int32)[f0:f0 + 2 * W * 256] = 0x7FFFFFFF
        self.regions = regs

    def allreduce_sum_(self, t):
        flat = t.view(-1)
        for lo in range(0, flat.numel(), self.max_numel):
            self.comm.allreduce_sum_(flat[lo:lo + self.max_numel])
        return t

    def allreduce_avg_(self, t):
        return self.allreduce_sum_(t).div_(self.world_size)

    def _pieces(self, out, inp, esize_words):
        """Split an in-place shard op over pieces of at most ``max_numel`` words whose
        lengths are multiples of 4 x W words (timing harness: rank 0's chunk of each piece
        stands in for its chunk of the whole)."""
        flat = inp.view(-1)
        step = max(4 * self.world_size, self.max_numel // (4 * self.world_size) * 4 * self.world_size)
        step = int(step / esize_words)
        for lo in range(0, flat.numel(), step):
            piece = flat[lo:lo + step]
            n = piece.numel() // self.world_size
            yield piece[:n], piece

    def reduce_scatter(self, out, inp):
        for o, i in self._pieces(out, inp, 1.0):
            self.comm.reduce_scatter(o, i)
        return out

    def all_gather(self, out, inp):
        for i, o in self._pieces(inp, out, 0.5 if out.dtype == torch.bfloat16 else 1.0):
            self.comm.all_gather(o, i)
        return out

    def broadcast_(self, t, root=0):
        return t  # rank 0 is the root: its values are the broadcast values

    def barrier(self):
        torch.cuda.synchronize(self.device)

    def failed(self):
        return self.comm.failed()

    def check(self):
        self.comm.check()

    def destroy(self):
        self.comm.destroy()
