"""Training engine: the step, hipGraph capture, epoch loops and on-device metrics.

Reference loop (main.py:93-113, main_dist.py:166-202): per batch ``zero_grad -> net(x) -> CE ->
backward -> step`` and two ``.item()`` host syncs per step for the running loss/accuracy.

Here a step is: on-device batch gather+augment, forward, fused CE (which also accumulates loss
sum / correct / count in an fp64 device buffer), backward (native kernels write gradients into
the flat arena, RCCL buckets overlap), one SGD launch.  No host sync per step; the metrics buffer
is read once per log interval. With ``graph=True`` the whole step is captured once into a
hipGraph (``torch.cuda.CUDAGraph`` on ROCm = hipGraph) and replayed: the batch indices are
copied into a static buffer before each replay and the learning rate lives in a device scalar,
so one capture serves the whole run.
"""
from __future__ import annotations

import os
import time

import torch

from ..ops.functional import cross_entropy, unit_grad
from ..utils.profiling import trace_range


class NonFiniteLossError(FloatingPointError):
    """Raised by the trainer's loss guard (SURVEY §5 failure detection: NaN/inf loss guard)."""


class TrainStep:
    def __init__(self, net, optimizer, loader, batch_size, ddp=None, graph=False, metrics=None,
                 clear_grads_in_step=None):
        self.net = net
        self.opt = optimizer
        self.loader = loader
        self.B = batch_size
        inner = getattr(net, "module", net)
        if loader.device.type == "cuda" and os.environ.get("PCA_BATCHED_WPREP", "1") != "0":
            from ..ops.functional import enable_batched_weight_prep

            enable_batched_weight_prep(inner)
            # the optimizer step writes the bf16 operands (no prep pass at the next forward)
            if getattr(optimizer, "arena", None) is not None and hasattr(optimizer, "attach_weight_prep") \
                    and os.environ.get("PCA_FUSED_SGD_PREP", "1") != "0":
                optimizer.attach_weight_prep(inner.__dict__["_pca_wplan"])
        # the arena step clears the gradients it consumed, so the next step needs no zero_grad
        # fill (one launch and a full gradient-arena write per step). This changes what the
        # optimizer's step() does to .grad (it reads zero afterwards), so it is an explicit
        # opt-in of this TrainStep: ``clear_grads_in_step`` (default on, PCA_SGD_ZERO_GRAD=0 off),
        # and close() puts the optimizer's previous setting back.
        self._prev_zero_in_step = getattr(optimizer, "zero_grad_in_step", None)
        if clear_grads_in_step is None:
            clear_grads_in_step = os.environ.get("PCA_SGD_ZERO_GRAD", "1") != "0"
        if getattr(optimizer, "arena", None) is not None and hasattr(optimizer, "zero_grad_in_step") \
                and clear_grads_in_step:
            optimizer.zero_grad_in_step = True
        self._grads_clean = False
        self.ddp = ddp
        self.device = loader.device
        self.metrics = metrics if metrics is not None else torch.zeros(3, dtype=torch.float64, device=self.device)
        self.graph_requested = graph and self.device.type == "cuda"
        self.graph = None
        self.static_idx = torch.zeros(batch_size, dtype=torch.int64, device=self.device)
        self.last_loss = None
        self.graph_error = None
        self.selection_hash = None   # kernel selection after the first (tuning) step

    def close(self):
        """Give the optimizer back its own gradient semantics (step() leaves .grad as computed)."""
        if self._prev_zero_in_step is not None:
            self.opt.zero_grad_in_step = self._prev_zero_in_step
        self._grads_clean = False

    # one eager step on a given index batch
    def _body(self, idx):
        with trace_range("data"):
            x, y = self.loader.make_batch(idx)
        if not self._grads_clean:
            self.opt.zero_grad()
        self._grads_clean = False
        with trace_range("forward"):
            out = self.net(x)
            loss = cross_entropy(out, y, self.metrics)
        with trace_range("backward"):
            loss.backward(unit_grad(loss))
            if self.ddp is not None:
                self.ddp.finish()
        with trace_range("optimizer"):
            self.opt.step()
        self._grads_clean = bool(getattr(self.opt, "_zeroed_grads", False))
        if self.selection_hash is None and self.device.type == "cuda" and not getattr(self.opt, "capturing", False):
            self._sync_selection()
        return loss

    def _sync_selection(self):
        """After the first step (the one that autotuned every conv geometry): every rank adopts
        rank 0's kernel selection (engine/tuning.py), and its hash is recorded."""
        from .. import _native
        from .tuning import selection_hash, selection_rows, sync_selection

        lib = _native.lib()
        ctx = getattr(self.ddp, "ctx", None)
        if ctx is not None and ctx.world > 1:
            self.selection_hash = sync_selection(ctx, lib)
        else:
            self.selection_hash = selection_hash(selection_rows(lib))

    def _fresh_operands(self):
        """A captured step with the fused optimizer has no prep pass: when the masters changed
        outside it (restore, checkpoint load, user writes), refresh the operands before replay."""
        plan = getattr(self.opt, "_wplan", None)
        if plan is not None and plan.skip_when_fresh and plan.entries and not plan.is_fresh():
            with torch.no_grad():
                plan.run()

    def _state_tensors(self):
        """Every tensor a training step mutates: parameters, BN buffers, momenta, metrics."""
        inner = getattr(self.net, "module", self.net)
        seen, out = set(), []

        def add(t):
            if t is not None and id(t) not in seen:
                seen.add(id(t))
                out.append(t)

        arena = getattr(self.opt, "arena", None)
        if arena is not None:
            add(arena.param_flat)
            add(arena.mom_flat)
        else:
            for p in inner.parameters():
                add(p.data)
            for st in self.opt.state.values():
                add(st.get("momentum_buffer"))
        for b in inner.buffers():
            add(b)
        from ..ops.functional import bn_pilots, rng_states

        for r in rng_states(inner):      # dropout Philox step counters
            add(r)
        for k in bn_pilots(inner):       # BN-statistics shifts (previous batch means)
            add(k)
        add(self.metrics)
        return out

    def _capture(self):
        # The warm-up bodies below are real steps (SGD update, BN running stats, metrics). Snapshot
        # the state first and roll it back before capture, so the first captured replay is the
        # first step this batch takes (N graph steps == N eager steps). Any failure on the way
        # (a warm-up raising, capture unsupported) restores the snapshot and the optimizer's
        # first-step flag before the caller falls back to eager, so the eager step that follows
        # sees exactly the state it would have seen without the attempt.
        state = self._state_tensors()
        snap = [t.clone() for t in state]
        first = getattr(self.opt, "_arena_first", None)
        known = {id(t) for t in state}

        def restore():
            torch.cuda.synchronize()
            with torch.no_grad():
                for t, v in zip(state, snap):
                    t.copy_(v)
                for st in self.opt.state.values():   # momenta created by the warm-ups start at zero
                    b = st.get("momentum_buffer")
                    if b is not None and id(b) not in known and getattr(self.opt, "arena", None) is None:
                        b.zero_()
            if first is not None:
                self.opt._arena_first = first

        def born_in_warmup():
            # state created by the warm-ups themselves (the dropout Philox states and the BN
            # pilots appear on the first training forward): roll it back to its creation value
            # ({seed, step 0, tickets 0}; a zero shift)
            from ..ops.functional import bn_pilots, rng_states

            inner = getattr(self.net, "module", self.net)
            with torch.no_grad():
                for r in rng_states(inner):
                    if id(r) not in known:
                        r[1:].zero_()
                for k in bn_pilots(inner):
                    if id(k) not in known:
                        k.zero_()

        try:
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                for _ in range(3):
                    self._body(self.static_idx)
            torch.cuda.current_stream().wait_stream(s)
        except BaseException:
            torch.cuda.current_stream().wait_stream(s)
            restore()
            born_in_warmup()
            raise
        restore()
        born_in_warmup()
        self._fresh_operands()   # (the restore rewrote the masters: the capture sees current operands)
        # If this is the run's first step, the restored momenta are zero and the captured
        # steady-state rule buf = 0.9 * buf + d equals the first-step rule buf = d (dampening 0),
        # so the graph is exact from its first replay; keep recording the steady-state rule.
        if first and self.opt.param_groups[0].get("dampening", 0) != 0:
            raise RuntimeError("hipGraph capture of the first SGD step needs dampening == 0")
        if first:
            self.opt._arena_first = False   # record the steady-state rule (see above)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        self.opt.capturing = True
        try:
            with torch.cuda.graph(g):
                self.static_loss = self._body(self.static_idx)
        except BaseException:
            self.opt.capturing = False
            restore()                      # (also puts back the first-step flag)
            raise
        finally:
            self.opt.capturing = False
        # (the captured step recorded the steady-state rule and left _arena_first False: the replay
        # that follows is the first real step, exact on the restored zero momenta as noted above)
        del snap
        self.graph = g

    def __call__(self, idx: torch.Tensor):
        """Run one training step on the sample indices ``idx`` (device int64)."""
        full = idx.numel() == self.B
        if self.graph_requested and full:
            if self.graph is None and self.graph_error is None:
                try:
                    self.static_idx.copy_(idx)
                    self._capture()
                except Exception as e:  # capture unsupported -> stay eager
                    self.graph_error = e
                    self.graph = None
                    torch.cuda.synchronize()
            if self.graph is not None:
                self.static_idx.copy_(idx)
                self.opt.sync_lr()
                self._fresh_operands()
                self.graph.replay()
                self.last_loss = self.static_loss
                return self.last_loss
        self.last_loss = self._body(idx)
        return self.last_loss


def read_metrics(metrics: torch.Tensor, reset: bool = True):
    """(mean loss per step, correct, total) from the device accumulator (one host sync)."""
    m = metrics.tolist()
    if reset:
        metrics.zero_()
    return m


def build_bench_step(model_name, per_rank_batch, device, ctx, graph=True, baseline=False,
                     bucket_mb=25.0, n_images=50000, grad_compress=None):
    """Closure running one timed training step of the headline benchmark + metadata."""
    from ..data.loader import DeviceLoader
    from ..data.synthetic import synthetic_cifar10

    images, labels = synthetic_cifar10(n_images, seed=1234)
    if baseline:
        from .stock import build_stock_step

        return build_stock_step(model_name, per_rank_batch, device, ctx, images, labels)

    from .. import models
    from .arena import ParamArena
    from .optim import SGD

    torch.manual_seed(0)
    model = models.build_model(model_name).to(device)
    arena = ParamArena(model.parameters())
    opt = SGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=5e-4).attach_arena(arena)
    ddp = None
    net = model
    if ctx.world > 1:
        from ..parallel.ddp import DistributedDataParallel

        ddp = DistributedDataParallel(model, ctx, bucket_cap_mb=bucket_mb, arena=arena,
                                      grad_compress=grad_compress)
        net = ddp
    loader = DeviceLoader(images, labels, per_rank_batch, device, train=True, crop_pad=4, flip=True,
                          world=ctx.world, rank=ctx.rank, seed=0, drop_last=True)
    step = TrainStep(net, opt, loader, per_rank_batch, ddp=ddp, graph=graph)
    state = {"it": None, "epoch": 0}

    def next_idx():
        while True:
            if state["it"] is None:
                loader.set_epoch(state["epoch"])
                state["it"] = iter(loader.batch_indices())
            try:
                idx = next(state["it"])
                if idx.numel() == per_rank_batch:
                    return idx
            except StopIteration:
                state["it"] = None
                state["epoch"] += 1

    def run():
        step(next_idx())

    meta = {"buckets_mib": ddp.bucket_sizes_mib() if ddp else None}

    def info():
        from .tuning import table_rows_loaded

        return {"graph_captured": step.graph is not None,
                "graph_error": repr(step.graph_error) if step.graph_error else None,
                "kernel_selection": step.selection_hash,
                "tune_table_rows": table_rows_loaded()}

    run.info = info
    return run, meta


class EpochTimer:
    def __init__(self):
        self.t0 = time.perf_counter()

    def elapsed(self):
        return time.perf_counter() - self.t0


class Trainer:
    """Epoch driver shared by main.py and main_dist.py.

    train_epoch / test_epoch reproduce the reference loops (main.py:93-148, main_dist.py:166-252)
    including their console/log formats, with three changes: metrics accumulate on the device and
    are read every ``log_every`` steps (not two ``.item()`` syncs per step); the test set is sharded
    across ranks and its counts all-reduced (the reference evaluated the full set on every rank and
    checkpointed on rank 0's local accuracy); full batches replay a captured
    hipGraph of the whole step when ``graph`` is on.
    """

    def __init__(self, net, optimizer, train_loader, test_loader, ctx, ddp=None, graph=False,
                 log_every=20, progress=None, is_main=True, max_steps=None, nan_guard=True,
                 profiler=None):
        self.net = net
        self.opt = optimizer
        self.train_loader = train_loader
        self.test_loader = test_loader
        self.ctx = ctx
        self.ddp = ddp
        self.device = train_loader.device
        self.log_every = max(1, log_every)
        self.progress = progress
        self.is_main = is_main
        self.max_steps = max_steps
        self.step = TrainStep(net, optimizer, train_loader, train_loader.batch_size, ddp=ddp,
                              graph=graph)
        self.images_per_sec = None
        self.nan_guard = nan_guard
        self.profiler = profiler   # torch.profiler session stepped once per train step

    def _check_finite(self, loss_sum, b, epoch):
        # the metrics buffer is read at every log point anyway: the guard costs no extra sync
        if self.nan_guard and not (loss_sum == loss_sum and abs(loss_sum) != float("inf")):
            raise NonFiniteLossError(
                f"non-finite training loss at epoch {epoch}, step {b} (rank {self.ctx.rank}); "
                "lower the learning rate or resume from the last checkpoint")

    def _reduce(self, m):
        t = torch.tensor(m, dtype=torch.float64, device=self.device if self.device.type == "cuda" else "cpu")
        self.ctx.all_reduce_sum(t)
        return t.tolist()

    def train_epoch(self, epoch):
        self.net.train()
        loader = self.train_loader
        loader.set_epoch(epoch)
        metrics = self.step.metrics
        metrics.zero_()
        n = len(loader)
        if self.max_steps:
            n = min(n, self.max_steps)
        t0 = time.perf_counter()
        imgs = 0
        for b, idx in enumerate(loader.batch_indices()):
            if b >= n:
                break
            if loader.drop_last and idx.numel() < loader.batch_size:
                break
            with trace_range("train_step"):
                self.step(idx)
            if self.profiler is not None:
                self.profiler.step()
            imgs += idx.numel()
            if b % self.log_every == 0 or b == n - 1:
                loss_sum, correct, total = metrics.tolist()
                self._check_finite(loss_sum, b, epoch)
                if hasattr(self.ctx, "health_check"):
                    self.ctx.health_check()
                if self.progress is not None:
                    self.progress(b, n, "Loss: %.3f | Acc: %.3f%% (%d/%d)"
                                  % (loss_sum / (b + 1), 100.0 * correct / max(total, 1), correct, total))
        if self.device.type == "cuda":
            torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        loss_sum, correct, total = metrics.tolist()
        self._check_finite(loss_sum, n, epoch)
        steps = max(1, min(n, b + 1) if n else 1)
        self.images_per_sec = imgs * self.ctx.world / dt if dt > 0 else None
        return loss_sum / steps, 100.0 * correct / max(total, 1), int(correct), int(total)

    @torch.no_grad()
    def test_epoch(self, epoch):
        self.net.eval()
        loader = self.test_loader
        metrics = torch.zeros(3, dtype=torch.float64, device=self.device)
        n = len(loader)
        if self.max_steps:
            n = min(n, self.max_steps)
        for b, idx in enumerate(loader.batch_indices()):
            if b >= n:
                break
            with trace_range("eval_step"):
                x, y = loader.make_batch(idx)
                out = self.net(x)
                cross_entropy(out, y, metrics)
            if self.progress is not None and (b % self.log_every == 0 or b == n - 1):
                loss_sum, correct, total = metrics.tolist()
                self.progress(b, n, "Loss: %.3f | Acc: %.3f%% (%d/%d)"
                              % (loss_sum / (b + 1), 100.0 * correct / max(total, 1), correct, total))
        # ranks may hold one batch more or less (unpadded eval shards): reduce the batch count too
        loss_sum, correct, total, steps = self._reduce(metrics.tolist() + [float(min(n, b + 1) if n else 0)])
        steps = max(1.0, steps)
        return loss_sum / steps, 100.0 * correct / max(total, 1), int(correct), int(total)
