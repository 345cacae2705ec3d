"""SGD with momentum / weight decay as one multi-tensor gfx950 kernel launch.

Semantics are those of ``torch.optim.SGD`` used by the reference (main.py:87-88,
main_dist.py:160-161: lr 0.1, momentum 0.9, weight_decay 5e-4, dampening 0, nesterov off):

    d = g + wd * p ;  buf = d (first step) | momentum * buf + (1 - dampening) * d
    d = d + momentum * buf (nesterov) | buf ;  p -= lr * d

The state_dict layout (``state[p]['momentum_buffer']``, ``param_groups``) matches torch's, so
checkpoints interoperate. The learning rate lives in a device scalar per group, refreshed from
``group['lr']`` before each step, so the captured hipGraph of a training step keeps reading the
current schedule value on replay.
"""
from __future__ import annotations

import torch

from .. import _native
from . import grads

_CHUNK = 8192


class SGD(torch.optim.Optimizer):
    def __init__(self, params, lr=0.1, momentum=0.0, dampening=0.0, weight_decay=0.0, nesterov=False,
                 grad_scale=1.0):
        if lr < 0.0:
            raise ValueError(f"Invalid learning rate: {lr}")
        if nesterov and (momentum <= 0 or dampening != 0):
            raise ValueError("Nesterov momentum requires a momentum and zero dampening")
        defaults = dict(lr=lr, momentum=momentum, dampening=dampening, weight_decay=weight_decay,
                        nesterov=nesterov)
        super().__init__(params, defaults)
        self.grad_scale = grad_scale
        self._lr_dev = {}
        self._lr_host = {}
        self._tables = {}
        self.capturing = False
        # arena step only: clear each gradient after reading it (the trainer then skips the next
        # zero_grad fill); _zeroed_grads reports whether the last step did. While this is set,
        # step() leaves every arena .grad reading ZERO (gradient-norm logging or hooks must read
        # the gradients before step()); a TrainStep sets it for its lifetime and close() restores it.
        self.zero_grad_in_step = False
        self._zeroed_grads = False

    # -------------------------------------------------------------------------- helpers
    def sync_lr(self):
        """Copy every group's python lr into its device scalar (call outside graph capture)."""
        for i, g in enumerate(self.param_groups):
            self._set_lr(i, g)

    def _set_lr(self, i, group):
        # the device scalar is rewritten only when the schedule moved (one fill per epoch, not per
        # step: a captured step's replay otherwise pays a launch for an unchanged value)
        t = self._lr_dev.get(i)
        lr = float(group["lr"])
        if t is not None and self._lr_host.get(i) != lr:
            t.fill_(lr)
            self._lr_host[i] = lr

    def _lr_tensor(self, i, group, device):
        t = self._lr_dev.get(i)
        if t is None or t.device != device:
            t = torch.full((1,), float(group["lr"]), dtype=torch.float32, device=device)
            self._lr_dev[i] = t
            self._lr_host[i] = float(group["lr"])
        elif not self.capturing:
            self._set_lr(i, group)
        return t

    def _table(self, i, params, grads, bufs):
        key = (i, tuple(p.data_ptr() for p in params), tuple(g.data_ptr() for g in grads),
               tuple(b.data_ptr() for b in bufs))
        ent = self._tables.get(i)
        if ent is not None and ent[0] == key:
            return ent[1]
        dev = params[0].device
        chunks = []
        for t, p in enumerate(params):
            n = p.numel()
            for s in range(0, n, _CHUNK):
                chunks.append((t, s, min(n, s + _CHUNK)))
        chunks_t = torch.tensor(chunks, dtype=torch.int64).to(dev)
        pp = torch.tensor([p.data_ptr() for p in params], dtype=torch.int64).to(dev)
        gp = torch.tensor([g.data_ptr() for g in grads], dtype=torch.int64).to(dev)
        bp = torch.tensor([b.data_ptr() for b in bufs], dtype=torch.int64).to(dev)
        tab = (chunks_t, pp, gp, bp)
        self._tables[i] = (key, tab)
        return tab

    def attach_arena(self, arena):
        """Run the update as one launch over the arena's flat param/grad/momentum buffers.

        Only valid when every trainable parameter is in a single param group (the reference's
        configuration); per-parameter ``momentum_buffer`` state entries become arena views so the
        optimizer state_dict keeps torch's layout.
        """
        if len(self.param_groups) != 1:
            raise ValueError("arena SGD needs a single param group")
        ids = {id(p) for p in self.param_groups[0]["params"]}
        if ids != {id(p) for p in arena.params}:
            raise ValueError("arena and optimizer parameters differ")
        self.arena = arena
        mom = arena.ensure_momentum()
        self._arena_first = True
        for p in arena.params:
            old = self.state[p].get("momentum_buffer")
            v = arena.view(mom, p)
            if old is not None:
                v.copy_(old)
                self._arena_first = False
            self.state[p]["momentum_buffer"] = v
        return self

    def attach_weight_prep(self, plan):
        """Fuse the model's bf16 conv-operand refresh (ops.functional.WeightPrepPlan) into the
        arena step: one launch updates every master and writes the operands from the new values
        (the optimizer emits the bf16 shadows), so the forward's separate prep pass
        (a full re-read of the masters) disappears. Needs ``attach_arena`` first."""
        if getattr(self, "arena", None) is None:
            raise ValueError("attach_weight_prep needs attach_arena first")
        self._wplan = plan
        plan.skip_when_fresh = True
        plan.watch = (self.arena.param_flat,)
        return self

    def _fused_tables(self, plan):
        """(sgd chunks of the arena ranges outside the plan, desc, prep chunks, {grad, mom} table)
        or None when some plan weight is not an arena member."""
        tabs = plan.ensure_tables()
        if tabs is None:
            return None
        arena = self.arena
        key = (id(tabs[0]), id(tabs[1]), tabs[2], arena.param_flat.data_ptr(), arena.mom_flat.data_ptr())
        ent = getattr(self, "_fused", None)
        if ent is not None and ent[0] == key:
            return ent[1]
        ranges, gm = [], []
        for e in plan.entries:
            if id(e.w) not in arena.offsets:
                self._fused = (key, None)
                return None
            off, n = arena.offsets[id(e.w)]
            if grads.physical(e.w).data_ptr() != arena.param_flat.data_ptr() + 4 * off:
                self._fused = (key, None)
                return None
            ranges.append((off, off + n))
            gm.append([arena.grad_flat.data_ptr() + 4 * off, arena.mom_flat.data_ptr() + 4 * off])
        ranges.sort()
        free, pos = [], 0
        for a, b in ranges:
            if a > pos:
                free.append((pos, a))
            pos = max(pos, b)
        if pos < arena.numel:
            free.append((pos, arena.numel))
        chunks = [(0, s, min(b, s + _CHUNK)) for a, b in free for s in range(a, b, _CHUNK)]
        dev = arena.param_flat.device
        out = (torch.tensor(chunks, dtype=torch.int64).reshape(-1, 3).to(dev),
               torch.tensor([arena.param_flat.data_ptr()], dtype=torch.int64).to(dev),
               torch.tensor([arena.grad_flat.data_ptr()], dtype=torch.int64).to(dev),
               torch.tensor([arena.mom_flat.data_ptr()], dtype=torch.int64).to(dev),
               torch.tensor(gm, dtype=torch.int64).to(dev))
        self._fused = (key, out)
        return out

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        arena = getattr(self, "arena", None)
        if arena is not None:  # keep momentum buffers as views of the arena
            mom = arena.ensure_momentum()
            have = False
            for p in arena.params:
                v = arena.view(mom, p)
                b = self.state[p].get("momentum_buffer")
                if b is not None and b.data_ptr() != v.data_ptr():
                    v.copy_(b)
                    have = True
                elif b is None:
                    v.zero_()
                self.state[p]["momentum_buffer"] = v
            self._arena_first = not have
        self._tables = {}

    # ----------------------------------------------------------------------------- step
    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        arena = getattr(self, "arena", None)
        if arena is not None and arena.param_flat.is_cuda:
            group = self.param_groups[0]
            lr = self._lr_tensor(0, group, arena.param_flat.device)
            plan = getattr(self, "_wplan", None)
            fused = self._fused_tables(plan) if plan is not None and plan.entries else None
            if fused is not None:
                chunks, pp, gp, bp, gm = fused
                _native.lib().sgd_prep_step(chunks, pp, gp, bp, lr, group["momentum"],
                                            group["dampening"], group["weight_decay"],
                                            self.grad_scale, group["nesterov"], self._arena_first,
                                            plan.tables[0], plan.tables[1], gm,
                                            self.zero_grad_in_step)
                plan.mark_fresh()      # masters and operands updated together, versions untouched
            else:
                chunks, pp, gp, bp = self._table(0, [arena.param_flat], [arena.grad_flat], [arena.mom_flat])
                _native.lib().sgd_step(chunks, pp, gp, bp, None, lr, group["momentum"], group["dampening"],
                                       group["weight_decay"], self.grad_scale, group["nesterov"],
                                       self._arena_first, self.zero_grad_in_step)
                if plan is not None:
                    plan.invalidate()   # raw-pointer update: the operands are stale
            self._arena_first = False
            self._zeroed_grads = self.zero_grad_in_step
            return loss
        self._zeroed_grads = False
        for i, group in enumerate(self.param_groups):
            params = [p for p in group["params"] if p.grad is not None]
            if not params:
                continue
            if params[0].is_cuda:
                self._native_step(i, group, params)
            else:
                self._reference_step(group, params)
        return loss

    def _native_step(self, i, group, params):
        C = _native.lib()
        first = False
        bufs = []
        for p in params:
            st = self.state[p]
            b = st.get("momentum_buffer")
            if b is None:
                b = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["momentum_buffer"] = b
                first = True
            bufs.append(b)
        for p, g, b in zip(params, [p.grad for p in params], bufs):
            dense = p.is_contiguous() or (p.dim() == 4 and p.is_contiguous(memory_format=torch.channels_last))
            if not (dense and g.stride() == p.stride() and b.stride() == p.stride()
                    and p.dtype == torch.float32 and g.dtype == torch.float32):
                raise RuntimeError("SGD native path needs fp32 params/grads/buffers with equal strides")
        chunks, pp, gp, bp = self._table(i, params, [p.grad for p in params], bufs)
        lr = self._lr_tensor(i, group, params[0].device)
        C.sgd_step(chunks, pp, gp, bp, None, lr, group["momentum"], group["dampening"],
                   group["weight_decay"], self.grad_scale, group["nesterov"], first)

    def _reference_step(self, group, params):
        for p in params:
            d = p.grad * self.grad_scale if self.grad_scale != 1.0 else p.grad
            if group["weight_decay"] != 0:
                d = d.add(p, alpha=group["weight_decay"])
            if group["momentum"] != 0:
                st = self.state[p]
                b = st.get("momentum_buffer")
                if b is None:
                    b = torch.clone(d).detach()
                    st["momentum_buffer"] = b
                else:
                    b.mul_(group["momentum"]).add_(d, alpha=1 - group["dampening"])
                d = d.add(b, alpha=group["momentum"]) if group["nesterov"] else b
            p.add_(d, alpha=-group["lr"])

    def zero_grad(self, set_to_none: bool = False):
        """Zero gradients in place (keeps buffer addresses stable for graphs / RCCL buckets)."""
        arena = getattr(self, "arena", None)
        if arena is not None:
            arena.zero_grad()
            return
        for group in self.param_groups:
            for p in group["params"]:
                if p.grad is not None:
                    if set_to_none:
                        p.grad = None
                    else:
                        p.grad.zero_()
