"""Data-parallel engine: bucketed gradient all-reduce on RCCL, overlapped with backward.

Re-implements what main_dist.py:140-144 gets from ``torch.nn.parallel.DistributedDataParallel``
(SURVEY §2.6 / §2.9 C3-C5), designed for one MI355X node:

* parameters, gradients and momentum live in flat arenas (:mod:`..engine.arena`) laid out in
  reverse registration order; buckets are contiguous slices of the gradient arena (no copy-in /
  copy-out, i.e. ``gradient_as_bucket_view=True``) of ~``bucket_cap_mb`` each, with the first
  bucket capped at 1 MiB like DDP so the all-reduce pipeline starts early in backward;
* gradient delivery (native kernels or AccumulateGrad) fires a ready hook per parameter; a bucket
  whose parameters are all ready is all-reduced (``ncclAvg`` = sum / world) on a dedicated
  high-priority HIP stream ordered after the producing kernels by an event, so communication of
  late layers overlaps the backward of early layers;
* a callback queued on the autograd engine closes the pass: buckets left unlaunched (parameters
  that got no gradient — EfficientNet-B0's unused ``layers.0.conv1`` / ``bn1``, efficientnet.py:
  61-67, 96) are reduced as zeros, which is what ``find_unused_parameters=True`` yields, and
  the compute stream waits for the communication stream before the optimizer runs;
* ``broadcast_buffers=True`` (DDP default): rank 0's BN running statistics reach every rank
  before any forward that follows a grad-enabled forward (C4) — one collective per dtype arena.
  DDP issues it at the start of that next forward, where it sits on the critical path; nothing
  touches the buffers between the end of a forward and the next one (backward never does), so
  with ``overlap_buffer_broadcast`` (default) it is issued right after the grad-enabled forward
  on the communication stream and runs under the backward (joined with the gradient buckets).
  Every forward then sees exactly the buffers DDP would give it; only the non-zero ranks' own
  copies between a step's forward and the next forward differ (they already hold rank 0's);
* the initial rank-0 parameters and buffers are broadcast at construction (C3).

Bucket size on xGMI (why the launchers default to 4 MiB, not DDP's 25). xGMI is point-to-point
(7 links per GPU, ~150 GB/s each way per link); an 8-rank ring all-reduce of S bytes moves
2(N-1)/N * S = 1.75 S through every GPU. At the 8-GPU shard (bs128 per rank) ResNet-18's backward
is ~1.2 ms and produces its 44.7 MB of fp32 gradients back to front: layer 4 (33.6 MB) in the first
~0.35 ms, layers 3-1 and the stem (11.1 MB) in the remaining ~0.85 ms. What the step cannot hide is
the all-reduce of the LAST bucket, which only starts after the stem's weight gradient:
  * 25 MiB buckets: the last bucket holds layers 1-3 (~11 MB) -> 1.75 * 11 MB / ~150 GB/s (one
    ring's per-link rate; more channels only help until the per-message latency dominates) ~ 130 us
    exposed per step (7 % of a 1.88 ms step);
  * 4 MiB buckets: the last bucket is ~4 MB -> ~47 us exposed, and the earlier buckets (each
    ~20-30 us of RCCL launch/latency) still finish under the backward (11 collectives in ~1 ms of
    backward leave the link idle >70 % of the time);
  * 1 MiB buckets: ~45 collectives per step; their fixed per-call cost (~20 us) adds up to most of
    the backward, so the pipeline no longer drains behind the last gradient.
Hence ``bucket_cap_mb`` defaults to DDP's 25 MiB in this class (API parity) and to 4 MiB in
bench.py / main_dist.py (``--bucket_mb``). The first bucket is capped at 1 MiB like DDP.

``grad_compress`` (opt-in, off by default = exact DDP semantics): "bf16" all-reduces every bucket
as bf16 (compressed into a persistent bf16 copy on the communication stream, decompressed into the
fp32 arena after the collective: half the link bytes, the sum rounded to bf16 — what torch's
``bf16_compress_hook`` does); "bf16_tail" compresses only the last bucket, the one whose all-reduce
is exposed after the backward (see above).

The communicator is the native :class:`RcclComm` on GPU ranks; a torch.distributed fallback
(gloo) runs the same logic in the CPU multi-process tests.
"""
from __future__ import annotations

import torch
import torch.distributed as dist
import torch.nn as nn

from ..engine import grads as G
from ..ops import functional as F
from ..engine.arena import BufferArena, ParamArena


class _TorchDistComm:
    """Communicator facade over torch.distributed (gloo / fallback)."""

    def all_reduce(self, t, op, stream):
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        if op == "avg":
            t.div_(dist.get_world_size())

    def broadcast(self, t, root, stream):
        dist.broadcast(t, src=root)


class Bucket:
    __slots__ = ("index", "start", "end", "params", "pending", "launched", "view", "low")

    def __init__(self, index, start, end, params, flat):
        self.index, self.start, self.end, self.params = index, start, end, params
        self.view = flat[start:end]
        self.pending = len(params)
        self.launched = False
        self.low = None       # persistent bf16 copy (grad_compress)


class DistributedDataParallel(nn.Module):
    def __init__(self, module: nn.Module, ctx, bucket_cap_mb: float = 25.0,
                 first_bucket_mb: float = 1.0, broadcast_buffers: bool = True,
                 find_unused_parameters: bool = True, arena: ParamArena | None = None,
                 force_collectives: bool = False, overlap_buffer_broadcast: bool = True,
                 grad_compress: str | None = None):
        super().__init__()
        if grad_compress not in (None, "none", "bf16", "bf16_tail"):
            raise ValueError(f"grad_compress must be None, 'bf16' or 'bf16_tail', not {grad_compress!r}")
        self.grad_compress = None if grad_compress == "none" else grad_compress
        self.module = module
        self.ctx = ctx
        self.world = ctx.world
        # issue every collective even on a 1-rank clique (GPU tests exercise the RCCL-in-hipGraph
        # path on a single-GPU box this way; a world-1 RCCL all-reduce is a device copy)
        self._collectives = self.world > 1 or force_collectives
        self.broadcast_buffers = broadcast_buffers
        self.overlap_buffer_broadcast = overlap_buffer_broadcast
        self.find_unused_parameters = find_unused_parameters
        params = [p for p in module.parameters() if p.requires_grad]
        self.arena = arena if arena is not None else ParamArena(params)
        self.buffers_arena = BufferArena(module) if any(True for _ in module.buffers()) else None
        self.is_cuda = self.arena.param_flat.is_cuda
        if self.is_cuda and ctx.comm is not None:
            self.comm = ctx.comm
            self.comm_stream = torch.cuda.Stream(device=self.arena.param_flat.device, priority=-1)
        else:
            self.comm = _TorchDistComm()
            self.comm_stream = None
        self._build_buckets(bucket_cap_mb, first_bucket_mb)
        self._require_forward_param_sync = True
        self._bcast_pending = False
        self._pass_active = False
        self.last_unused = []
        for p in self.arena.params:
            G.register_grad_ready_hook(p, self._on_grad_ready)
        self._sync_initial_state()

    # ------------------------------------------------------------------------- set-up
    def _build_buckets(self, cap_mb, first_mb):
        cap = int(cap_mb * 1024 * 1024 / 4)
        first = int(first_mb * 1024 * 1024 / 4)
        buckets, cur, start = [], [], None
        limit = first
        for p in self.arena.order:  # reverse registration order = backward order
            off, n = self.arena.slice_of(p)
            if cur and off + n - start > limit:  # close before overflowing (a lone big param
                buckets.append((start, end, cur))  # still gets its own bucket)
                cur, start, limit = [], None, cap
            if start is None:
                start = off
            cur.append(p)
            end = off + n
        if cur:
            buckets.append((start, end, cur))
        flat = self.arena.grad_flat
        self.buckets = []
        for i, (s, e, ps) in enumerate(buckets):
            if i == len(buckets) - 1:
                e = flat.numel()
            if i > 0:
                s = self.buckets[-1].end
            self.buckets.append(Bucket(i, s, e, ps, flat))
        if self.buckets:
            self.buckets[0].start = 0
            self.buckets[0].view = flat[0: self.buckets[0].end]
        self._bucket_of = {id(p): b for b in self.buckets for p in b.params}
        for b in self.buckets:
            if self.grad_compress == "bf16" or (self.grad_compress == "bf16_tail" and b is self.buckets[-1]):
                b.low = torch.empty(b.end - b.start, dtype=torch.bfloat16, device=flat.device)

    def bucket_sizes_mib(self):
        return [round((b.end - b.start) * 4 / 2 ** 20, 3) for b in self.buckets]

    def _stream_ctx(self):
        if self.comm_stream is None:
            return _Null()
        return torch.cuda.stream(self.comm_stream)

    def _sid(self):
        return self.comm_stream.cuda_stream if self.comm_stream is not None else 0

    def _fork(self):
        if self.comm_stream is not None:
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream())
            self.comm_stream.wait_event(ev)
            # weight gradients may still be in flight on the side stream (ops/functional.py)
            side = F.wgrad_stream(self.comm_stream.device)
            if side is not None:
                self.comm_stream.wait_stream(side)

    def _join(self):
        if self.comm_stream is not None:
            ev = torch.cuda.Event()
            ev.record(self.comm_stream)
            torch.cuda.current_stream().wait_event(ev)

    @torch.no_grad()
    def _sync_initial_state(self):
        if not self._collectives:
            return
        self._fork()
        with self._stream_ctx():
            self.comm.broadcast(self.arena.param_flat, 0, self._sid())
            if self.buffers_arena is not None:
                for t in self.buffers_arena.flat_tensors():
                    self.comm.broadcast(t, 0, self._sid())
        self._join()

    # ------------------------------------------------------------------------ forward
    def _broadcast_buffers(self, join: bool):
        with torch.no_grad():
            self._fork()
            with self._stream_ctx():
                for t in self.buffers_arena.flat_tensors():
                    self.comm.broadcast(t, 0, self._sid())
            if join:
                self._join()

    def forward(self, *args, **kwargs):
        if self._bcast_pending:          # previous grad-enabled forward had no backward
            self._join()
            self._bcast_pending = False
        sync = self.broadcast_buffers and self._collectives and self.buffers_arena is not None
        if sync and self._require_forward_param_sync:
            self._broadcast_buffers(join=True)
        out = self.module(*args, **kwargs)
        self._require_forward_param_sync = torch.is_grad_enabled()
        if sync and self._require_forward_param_sync and self.overlap_buffer_broadcast \
                and self.comm_stream is not None:
            # issued now on the communication stream (after this forward's kernels), overlapped
            # with the backward; the pass-closing join orders it before the optimizer / next step
            self._broadcast_buffers(join=False)
            self._require_forward_param_sync = False
            self._bcast_pending = True
        return out

    # ----------------------------------------------------------------------- backward
    def _start_pass(self):
        self._pass_active = True
        for b in self.buckets:
            b.pending = len(b.params)
            b.launched = False
        self._ready = set()
        torch.autograd.Variable._execution_engine.queue_callback(self._finish_pass)

    def _on_grad_ready(self, p):
        if not self._pass_active:
            self._start_pass()
        if id(p) in self._ready:
            return
        self._ready.add(id(p))
        b = self._bucket_of[id(p)]
        b.pending -= 1
        if b.pending == 0:
            self._launch(b)

    def _launch(self, b):
        if b.launched:
            return
        b.launched = True
        if not self._collectives:
            return
        # deferred weight-gradient slab reductions (ops/functional.py) complete this bucket's
        # gradients: one batched launch on the compute stream, before the fork orders the
        # collective after it
        F.flush_wgrads()
        self._fork()
        with self._stream_ctx():
            if b.low is not None:
                # compressed bucket: bf16 over the links, fp32 back into the arena (comm stream)
                b.low.copy_(b.view)
                self.comm.all_reduce(b.low, "avg", self._sid())
                b.view.copy_(b.low)
            else:
                self.comm.all_reduce(b.view, "avg", self._sid())

    def _finish_pass(self):
        unused = []
        for b in self.buckets:
            if not b.launched:
                if not self.find_unused_parameters:
                    raise RuntimeError(
                        "parameters did not receive gradients (set find_unused_parameters=True)")
                unused += [p for p in b.params if id(p) not in self._ready]
                self._launch(b)
        self.last_unused = unused
        self._join()
        self._bcast_pending = False
        self._pass_active = False

    def state_dict(self, *args, **kwargs):
        # the overlapped BN-buffer broadcast of a grad-enabled forward may still be writing the
        # buffers on the communication stream: order it before anyone reads them
        self.finish()
        return super().state_dict(*args, **kwargs)

    def finish(self):
        """Explicitly close a pass (no-op if the autograd callback already ran)."""
        if self._pass_active:
            self._finish_pass()
        elif self._bcast_pending:        # a grad-enabled forward without a backward
            self._join()
            self._bcast_pending = False


class _Null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False
