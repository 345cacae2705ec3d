"""Autograd wiring of the native gfx950 kernels.

Tensor convention: activations are NCHW-shaped tensors whose memory is NHWC (torch
``channels_last``) bf16 on the GPU, so ``x.permute(0, 2, 3, 1)`` is the contiguous [N,H,W,C]
matrix the kernels consume and the model code keeps the reference's NCHW indexing
(``torch.cat(dim=1)``, ``x[:, :c]``, ``out.view(N, -1)``).  CPU tensors take the pure PyTorch
reference path with identical semantics (used by the CPU tests and the LeNet CPU config).

Every GPU op here calls the extension; nothing silently falls back to stock PyTorch kernels
except pure data movement (cat/slice/shuffle views) which has no arithmetic.
"""
from __future__ import annotations

import functools
import math
import os

import torch
import torch.nn.functional as F

from .. import _native
from ..engine import grads as G

ACT = {None: 0, "none": 0, "relu": 1, "swish": 2, "silu": 2, "sigmoid": 3}
COMPUTE_DTYPE = torch.bfloat16


def _C():
    return _native.lib()


_FORCE_REFERENCE = False


def set_reference_mode(on: bool) -> None:
    """Process-wide: GPU tensors take the stock-PyTorch path too (``--dtype fp32`` runs)."""
    global _FORCE_REFERENCE
    _FORCE_REFERENCE = bool(on)


def _ref(x: torch.Tensor) -> bool:
    """True when ``x`` takes the pure-PyTorch reference path (CPU, or reference mode forced)."""
    return _FORCE_REFERENCE or not x.is_cuda


class reference_kernels:
    """Context manager: run GPU tensors through stock PyTorch ops (the comparator / oracle)."""

    def __enter__(self):
        global _FORCE_REFERENCE
        self._prev = _FORCE_REFERENCE
        _FORCE_REFERENCE = True
        return self

    def __exit__(self, *a):
        global _FORCE_REFERENCE
        _FORCE_REFERENCE = self._prev
        return False


# ------------------------------------------------------------------------------- layout
def to_nhwc(x: torch.Tensor, pad_to: int | None = None) -> torch.Tensor:
    """Contiguous NHWC bf16 [N,H,W,C'] view/copy of an NCHW-shaped tensor (C' >= C if padded)."""
    N, C, H, W = x.shape
    if pad_to is not None and pad_to != C:
        # channel-padded storage produced by the loader / a previous pad: reuse it
        base = getattr(x, "_pca_padded", None)
        if base is not None and base.shape[-1] == pad_to:
            return base
        if x.dtype == torch.float32 and x.is_contiguous():
            return _C().nchw_to_nhwc(x, pad_to)
        v = to_nhwc(x)
        return F.pad(v, (0, pad_to - C))
    v = x.permute(0, 2, 3, 1)
    if v.dtype == COMPUTE_DTYPE and v.is_contiguous():
        return v
    if x.dtype == torch.float32 and x.is_contiguous():
        return _C().nchw_to_nhwc(x, C)
    out = torch.empty((N, H, W, C), dtype=COMPUTE_DTYPE, device=x.device)
    out.copy_(v)
    return out


def to_nchw(y: torch.Tensor) -> torch.Tensor:
    """NCHW-shaped channels_last view of an NHWC tensor (no copy)."""
    return y.permute(0, 3, 1, 2)


def padded_input(x_nhwc_padded: torch.Tensor, C: int) -> torch.Tensor:
    """Wrap a channel-padded NHWC buffer as an NCHW-shaped tensor with ``C`` visible channels.

    The returned tensor remembers its padded storage so the first conv can consume it without a
    copy (the GPU augmentation kernel writes 3 RGB channels into 8-channel pixels).
    """
    v = to_nchw(x_nhwc_padded)[:, :C]
    v._pca_padded = x_nhwc_padded
    return v


# ------------------------------------------------------------------------------- conv
def _round8(c: int) -> int:
    return (c + 7) // 8 * 8


# ------------------------------------------------------------- gradient hand-off slots
# An activation read by several ops (a residual block's input: conv1 and the skip path) gets its
# gradient summed by autograd with a separate elementwise add (3 tensor passes). A GradSlot on the
# activation lets the first MFMA conv that read it ("owner") fold the other contribution into its
# dgrad epilogue instead: a producer (the residual BN or another conv on the same input) whose
# backward runs first deposits its gradient and returns None; the owner's dgrad adds it while
# storing dX. Order-safe: a producer that runs after the owner returns its gradient normally.
_FUSE_GRAD = os.environ.get("PCA_FUSE_RESIDUAL_GRAD", "1") != "0"


class GradSlot:
    # s2c: the owner is a 3x3 / stride-2 / pad-1 conv, so a 1x1 / stride-2 sibling may hand over
    # its dX in compact form (even-even pixels only; the owner's parity dgrad adds it in place)
    __slots__ = ("grad", "closed", "s2c")

    def __init__(self):
        self.grad = None
        self.closed = False
        self.s2c = False

    def offer(self, g) -> bool:
        if self.closed or self.grad is not None or g is None:
            return False
        self.grad = g
        return True

    def take(self):
        g, self.grad = self.grad, None
        self.closed = True
        return g


class _DenseSlot(GradSlot):
    """GradSlot of a dense-block slab suffix; ``claimed`` once a BatchNorm whose backward will
    take it has read the suffix (only then may the append hand its gradient over)."""
    __slots__ = ("claimed",)

    def __init__(self):
        super().__init__()
        self.claimed = False


def _slot_for_conv(x):
    """(slot, is_owner) for an MFMA conv reading the user-level activation ``x``."""
    if not (_FUSE_GRAD and x.requires_grad and torch.is_grad_enabled()):
        return None, False
    s = getattr(x, "_pca_slot", None)
    if s is None:
        s = GradSlot()
        try:
            x._pca_slot = s
        except Exception:
            return None, False
        return s, True
    return s, False


class BiasRec:
    """Hand-off of a conv bias gradient to the BatchNorm that alone consumes the conv's output
    (googlenet.py / vgg.py ``Conv2d(bias=True) -> BatchNorm2d``, the fused Sequential marks the
    pair): the BN backward adds sum_m dY from the per-channel sums it already holds (its
    finalize, csrc/batchnorm.hip set_bn_dbias) and the conv backward skips its column-sum pass."""
    __slots__ = ("bias", "armed", "done")

    def __init__(self, bias):
        self.bias = bias
        self.armed = False    # the conv kernel path can hand its bias gradient over
        self.done = False     # the BN backward added it


def _slot_for_residual(x):
    if not (_FUSE_GRAD and x is not None and x.requires_grad):
        return None
    return getattr(x, "_pca_slot", None)


# ------------------------------------------------------------- concurrent weight gradients
# dW of a conv depends only on (x, dY); the rest of the backward chain depends on dX only. The
# weight-gradient kernels therefore run on a second HIP stream, concurrently with the dgrad /
# BatchNorm-backward chain of the layers below: at a per-GPU batch of 128 (the 8-GPU
# strong-scaling shard) no single backward kernel fills the 256 CUs, so two independent kernel
# streams recover the idle CUs. Ordering: the side stream waits for the main stream when a dW
# is issued; a callback at the end of the backward pass joins it back into the main stream
# (before the optimizer, and inside hipGraph capture); the data-parallel engine's bucket
# launches also wait on it (parallel/ddp.py).
# Measured on MI355X (ResNet-18, hipGraph step): the per-conv cross-stream dependencies cost more
# than the overlap recovers (bs128 2.28 -> 2.40 ms, bs1024 7.30 -> 7.50 ms), so the side stream
# is opt-in: PCA_WGRAD_STREAM=1. Round 4 re-measured it with the wgrad issued before its conv's
# dgrad (so the two can overlap): bs128 1.88 -> 1.96-1.99 ms, bs1024 6.59 -> 6.88-6.93 ms (same
# box) — each conv kernel holds its CUs' LDS / registers, so the branches do not co-reside; they
# only serialise behind the cross-stream edges.
_WGRAD_STREAM = os.environ.get("PCA_WGRAD_STREAM", "0") == "1"
_side = {}          # device index -> torch.cuda.Stream
_join_pending = {"on": False}


def wgrad_stream(device):
    """The side stream carrying weight-gradient kernels on ``device`` (None when disabled)."""
    if not _WGRAD_STREAM:
        return None
    idx = device.index if device.index is not None else torch.cuda.current_device()
    s = _side.get(idx)
    if s is None:
        s = torch.cuda.Stream(device=idx)
        _side[idx] = s
    return s


def _join_side_streams():
    _join_pending["on"] = False
    cur = torch.cuda.current_stream()
    for s in _side.values():
        if s.device == cur.device:
            cur.wait_stream(s)


def _schedule_join():
    if not _join_pending["on"]:
        _join_pending["on"] = True
        torch.autograd.Variable._execution_engine.queue_callback(_join_side_streams)


def join_wgrad_streams():
    """Make the current stream wait for all outstanding side-stream weight gradients."""
    if _side:
        _join_side_streams()


# Deferred weight-gradient reductions. A split-K wgrad that writes slab rows records its reduce
# instead of launching it (csrc/conv_halo.hip wgrad_flush_launch); every pending one then runs in
# ONE batched launch when the gradients are next needed: at the end of the backward pass (an
# autograd-engine callback queued by the first deferred wgrad), or earlier by a DDP bucket about
# to be all-reduced (parallel/ddp.py). Bitwise the per-conv reduce kernels' result (same order).
# ResNet-18 bs128: 12 reduce launches (117 us) -> 1.
# Measured SLOWER and therefore opt-in (PCA_WGRAD_DEFER=1), same box, 2 reps: ResNet-18 bs128
# 1.867 -> 1.886-1.890 ms, bs1024 6.479-6.483 -> 6.513-6.544 ms. The per-conv reduce reads its slab
# right after the wgrad wrote it (L2-resident); deferred, every slab is re-read from MALL / HBM at
# the end of the pass, which costs more than the ~11 launches it saves (ResNet-152 bs128: 779 us
# for the 3 batched launches).
_DEFER_MODE = os.environ.get("PCA_WGRAD_DEFER", "piggy")
_WGRAD_DEFER = _DEFER_MODE == "1"
# Default ("piggy"): the recorded reductions ride along in the NEXT fused BatchNorm-backward launch
# as extra workgroups (csrc/batchnorm.hip bn_bwd_apply_acc_rows_red_kernel) — right after their
# wgrad, beside the BN pass they are independent of, so the slabs are still cache-resident and no
# launch of their own is left; whatever no BN launch took is flushed as above. (Not bitwise the
# per-conv kernels: 4 split lanes per column instead of up to 16; still a fixed order.)
_WGRAD_PIGGY = _DEFER_MODE == "piggy"
_piggy_set = [None]
_defer_queued = {"on": False}


def flush_wgrads():
    """Launch every deferred weight-gradient reduction on the current stream (no-op if none)."""
    _defer_queued["on"] = False
    if _native._lib is not None:
        _C().wgrad_flush()


def _after_deferred_wgrad():
    if _defer_queued["on"]:
        return
    try:
        torch.autograd.Variable._execution_engine.queue_callback(flush_wgrads)
        _defer_queued["on"] = True
    except RuntimeError:      # not inside a backward pass: nobody would flush later
        flush_wgrads()


# ------------------------------------------------------------------ batched weight prep
# Each MFMA conv consumes a bf16 copy of its fp32 master weight (plus a transposed copy for
# dgrad). Converting them per conv costs one small launch per layer per step; a WeightPrepPlan
# attached to the model converts ALL of them in one multi-tensor launch from a forward
# pre-hook, into persistent buffers (stable addresses for hipGraph replay). The conversion runs
# every forward from the current masters, so it can never serve a stale weight.
_PLAN = {"cur": None}
_PREP_CHUNK = int(os.environ.get("PCA_PREP_CHUNK", "4096"))   # fp32 elements per convert block


class _PrepEntry:
    __slots__ = ("w", "groups", "wb", "wt", "dwbuf")

    def __init__(self, w, groups, wb, wt):
        self.w, self.groups, self.wb, self.wt = w, groups, wb, wt
        self.dwbuf = None     # zero-padded convs: persistent padded weight-gradient accumulator


class WeightPrepPlan:
    """The model's bf16 conv operands, refreshed from the fp32 masters in one launch.

    With a fused optimizer attached (``SGD.attach_weight_prep``) the optimizer step itself writes
    the operands from the updated masters (sgd_prep_kernel), and the forward pre-hook skips the
    refresh while the masters are unchanged since the operands were last written. "Unchanged" is
    tracked through the autograd version counters of every weight and of the parameter arena
    (in-place writes, checkpoint loads and snapshot restores all bump them); writers that bypass
    them (the native optimizer kernels) either refresh the operands themselves or ``invalidate``.
    """

    def __init__(self):
        self.entries = []
        self.by_id = {}
        self.tables = None
        self.owner = None
        self.skip_when_fresh = False   # set by a fused optimizer
        self.watch = ()                # extra tensors whose versions guard freshness (the arena)
        self.fresh_key = None

    def _key(self):
        return (tuple(e.w._version for e in self.entries), tuple(t._version for t in self.watch),
                self.tables[2] if self.tables is not None else None)

    def is_fresh(self):
        return self.fresh_key is not None and self.tables is not None and self.fresh_key == self._key()

    def mark_fresh(self):
        self.fresh_key = self._key() if self.tables is not None else None

    def invalidate(self):
        self.fresh_key = None

    def ensure_tables(self):
        if self.entries and (self.tables is None or self.tables[2] != tuple(G.physical(e.w).data_ptr() for e in self.entries)):
            self._build()
        return self.tables

    def lookup(self, w, groups):
        e = self.by_id.get(id(w))
        if e is not None and e.w is w and e.groups == groups and e.wb.device == w.device:
            return e
        if e is not None:   # stale (deep copy / device move): rebuild the plan
            self.entries, self.by_id, self.tables = [], {}, None
        return None

    def register(self, w, groups, w_phys):
        if isinstance(groups, tuple) and groups[0] in ("gpad", "gdense"):
            # per-group zero-padded operands (odd-width grouped / narrow convs): w_phys is the
            # padded fp32 weight [G*op][KH][KW][cp], converted now (first sight)
            wb, wt = _C().weight_prep(w_phys, groups[1], True)
        elif isinstance(groups, tuple):
            # ("pad", Cp): forward-only bf16 copy with channels zero-padded to Cp (stem convs)
            co, cg, kh, kw = w.shape
            wb = torch.empty((co, kh, kw, groups[1]), dtype=COMPUTE_DTYPE, device=w.device)
            wt = None
        elif groups == DW_PREP:
            # depthwise: fp32 tap-major copy [KH*KW][Co] (valid for this forward already)
            co = w.shape[0]
            wb = w.detach().reshape(co, -1).t().contiguous()
            wt = None
        else:
            wb, wt = _C().weight_prep(w_phys, groups, True)
        e = _PrepEntry(w, groups, wb, wt)
        self.entries.append(e)
        self.by_id[id(w)] = e
        self.tables = None
        self.fresh_key = None
        return e

    def _build(self):
        desc, chunks = [], []
        for t, e in enumerate(self.entries):
            wp = G.physical(e.w)
            Cout, KH, KW, Cg = wp.shape
            n = wp.numel()
            if isinstance(e.groups, tuple) and e.groups[0] == "gpad":
                _, g, cout_g, op, cg, cp = e.groups
                desc.append([wp.data_ptr(), e.wb.data_ptr(), e.wt.data_ptr(), g, op, KH * KW, cp,
                             (cout_g << 32) | cg])
                tiles = g * KH * KW * ((op + 63) // 64) * ((cp + 63) // 64)
                chunks += [[t, k, 0, 5] for k in range(tiles)]
                continue
            if isinstance(e.groups, tuple) and e.groups[0] == "gdense":
                _, g, cout_g, cg, S = e.groups
                cn = Cout // g
                desc.append([wp.data_ptr(), e.wb.data_ptr(), e.wt.data_ptr(), g, cn, KH * KW, S,
                             (cout_g << 32) | cg])
                tiles = g * KH * KW * ((cn + 63) // 64) * ((S + 63) // 64)
                chunks += [[t, k, 0, 6] for k in range(tiles)]
                continue
            if isinstance(e.groups, tuple):
                cp = e.groups[1]
                rows = Cout * KH * KW
                desc.append([wp.data_ptr(), e.wb.data_ptr(), 0, 1, Cout, KH * KW, Cg, cp])
                step = max(1, 2048 // cp)
                chunks += [[t, r0, min(rows, r0 + step), 3] for r0 in range(0, rows, step)]
                continue
            if e.groups == DW_PREP:
                # [Co][K] -> [K][Co] with K = KH*KW*Cg: a depthwise weight's taps (Cg = 1), or a
                # 1x1 weight's input channels (the squeeze-excite W2 transposed)
                desc.append([wp.data_ptr(), e.wb.data_ptr(), 0, 1, Cout, KH * KW * Cg, 1, n])
                chunks += [[t, c0, min(Cout, c0 + 64), 2] for c0 in range(0, Cout, 64)]
                continue
            desc.append([wp.data_ptr(), e.wb.data_ptr(), e.wt.data_ptr(), e.groups,
                         Cout // e.groups, KH * KW, Cg, n])
            cn, cr = Cout // e.groups, Cg
            tiles = e.groups * KH * KW * ((cn + 63) // 64) * ((cr + 63) // 64)
            # pass 4: each transpose tile also writes its elements' forward copy (one read of
            # the fp32 master for both bf16 operands)
            chunks += [[t, k, 0, 4] for k in range(tiles)]
        dev = self.entries[0].wb.device
        self.tables = (torch.tensor(desc, dtype=torch.int64).to(dev),
                       torch.tensor(chunks, dtype=torch.int64).to(dev),
                       tuple(G.physical(e.w).data_ptr() for e in self.entries))

    def run(self):
        if not self.entries:
            return
        self.ensure_tables()
        _C().weight_prep_multi(self.tables[0], self.tables[1])
        self.mark_fresh()


def _plan_pre_hook(module, args):
    plan = module.__dict__.get("_pca_wplan")
    # replicas made by torch DataParallel share __dict__ entries: only the owner runs the plan
    if plan is not None and plan.owner == id(module) and not _FORCE_REFERENCE and \
            next(iter(module.parameters())).is_cuda:
        if not (plan.skip_when_fresh and plan.is_fresh()):
            plan.run()
        _PLAN["cur"] = plan


def _plan_post_hook(module, args, out):
    _PLAN["cur"] = None


def enable_batched_weight_prep(model):
    """Attach a WeightPrepPlan to ``model`` (idempotent). Returns the model."""
    if "_pca_wplan" not in model.__dict__:
        plan = WeightPrepPlan()
        plan.owner = id(model)
        model.__dict__["_pca_wplan"] = plan
        model.register_forward_pre_hook(_plan_pre_hook)
        model.register_forward_hook(_plan_post_hook)
    return model


DW_PREP = -1      # WeightPrepPlan "groups" key of a depthwise weight's tap-major fp32 copy


def _dw_weight(weight):
    """Depthwise weight [Co,1,KH,KW] as the fp32 tap-major [KH*KW][Co] operand of the kernels:
    from the active plan (refreshed by its one batched launch per forward) when there is one."""
    plan = _PLAN["cur"]
    if plan is not None and weight.is_leaf and weight.dtype == torch.float32 and \
            weight.permute(0, 2, 3, 1).is_contiguous():
        e = plan.lookup(weight, DW_PREP)
        if e is None:
            e = plan.register(weight, DW_PREP, None)
        return e.wb
    Co = weight.shape[0]
    return weight.detach().reshape(Co, -1).t().contiguous()


def _prepped_weight(weight, groups, w_phys, need_dx):
    """(wb, wt) for an MFMA conv: from the active plan when there is one, else converted now."""
    plan = _PLAN["cur"]
    if plan is not None and weight.is_leaf and weight.dim() == 4 and \
            weight.permute(0, 2, 3, 1).is_contiguous():
        e = plan.lookup(weight, groups)
        if e is None:
            e = plan.register(weight, groups, w_phys)
        return e.wb, e.wt
    return _C().weight_prep(w_phys, groups, need_dx)


# ------------------------------------------------- BN-backward reduce in the dgrad epilogue
# The BatchNorm+ReLU backward needs per-channel sums of dz and dz*xhat over the whole batch before
# it can produce dy. When that BN's output feeds an MFMA conv, the conv's dgrad epilogue holds
# exactly dz's source (the gradient it stores) in registers: it also reads the BN input y and the
# 1-bit ReLU mask and emits the two sums as slab rows, so the BN backward skips its separate
# reduce pass (one full read of dout + y + mask) and launch. The sums are used only if the BN's
# incoming gradient IS that dgrad's output (same storage): any other gradient contribution makes
# autograd produce a new tensor and the BN falls back to its own reduce.
_FUSE_BN_BWD = os.environ.get("PCA_FUSE_BN_BWD", "1") != "0"
# the same for a dual BN (act(BN(y) + BN2(y2)), the projection-shortcut block tail): generic
# igemm / split-K stride-1 dgrads add the third sum dz * xhat2 (PCA_DUAL_BN_FUSE=0: separate pass)
_DUAL_BN_FUSE = os.environ.get("PCA_DUAL_BN_FUSE", "1") != "0"


def set_dual_bn_fuse(on: bool) -> None:
    global _DUAL_BN_FUSE
    _DUAL_BN_FUSE = bool(on)


def set_fuse_bn_backward(on: bool) -> None:
    """Enable/disable the BN-backward reduce fusion into the consumer conv's dgrad epilogue."""
    global _FUSE_BN_BWD
    _FUSE_BN_BWD = bool(on)


# A BatchNorm without activation (MobileNetV2 / EfficientNet-B0 block tails: the project conv's
# BN, reference mobilenetv2.py:37, efficientnet.py:103) hands its consumer dgrad an all-ones
# "ReLU mask": dz = dout * 1, so the same fused epilogue reduces its backward sums (PCA_FUSE_BN_NOACT=0
# keeps the separate reduce + finalize passes). One persistent buffer per size (stable addresses
# for hipGraph replay); the kernels read 1 bit per element of it.
_FUSE_BN_NOACT = os.environ.get("PCA_FUSE_BN_NOACT", "1") != "0"
_ONES_MASK = {}


# A BatchNorm reading a row-strided slab slice (DenseNet's suffix BNs) hands its backward reduce
# to the consumer conv's dgrad epilogue too (PCA_STRIDED_BN_FUSE=0: separate reduce + finalize)
_STRIDED_BN_FUSE = os.environ.get("PCA_STRIDED_BN_FUSE", "1") != "0"
# DenseNet slabs cache each channel's batch sums as it is produced (PCA_SLAB_STATS=0: every
# suffix BatchNorm runs its own statistics + finalize passes)
_SLAB_STATS = os.environ.get("PCA_SLAB_STATS", "1") != "0"


def _ones_mask(numel, device):
    key = (int(numel), device.index if device.index is not None else torch.cuda.current_device())
    m = _ONES_MASK.get(key)
    if m is None:
        m = _ONES_MASK[key] = torch.full(((int(numel) + 7) // 8,), 255, dtype=torch.uint8, device=device)
    return m


class _BNSrc:
    __slots__ = ("y", "mask", "aux", "part", "dx", "acc", "act", "y2", "aux2")

    def __init__(self, y, mask, aux, acc=None, act=1, y2=None, aux2=None):
        self.y, self.mask, self.aux = y, mask, aux
        self.y2, self.aux2 = y2, aux2   # dual BN (projection-shortcut tail): NS = 3 sums
        self.part = None
        self.dx = None
        self.acc = acc        # the BN's backward StatAcc (sharded-accumulator mode) or None
        self.act = act        # 1: ReLU (1-bit mask); 2: swish (z from y and aux scale | shift;
                              #    only the depthwise dgrad epilogue computes it)


# ------------------------------------------------- sharded BatchNorm-sum accumulators
# Training BatchNorm needs per-channel batch sums before it can normalize (forward: sum, sumsq of
# the conv output; backward: sum dz, sum dz*xhat). Their producers (conv / dgrad epilogues, the
# reduce kernels) add per-workgroup partials with fp32 atomics into a small accumulator of R shard
# rows (persistent, owned by the producing conv / the BN); the consuming BN kernel folds the R
# rows in its prologue. Each accumulator is re-zeroed by block 0 of the OTHER pass of the same BN
# (the forward kernel clears the BN's backward accumulator, the backward kernel the forward
# one(s)), so a training step needs no finalize launch (37 per ResNet-18 step), no memset and no
# cross-block ticket, and the buffers stay valid under hipGraph replay. A small state machine
# (clean -> filled -> used) falls back to a memset only when a pass is skipped (a forward without
# backward). Deterministic mode (ordered slab rows + finalize kernel) and PCA_BN_ACC=0 turn it off.
_BN_ACC = os.environ.get("PCA_BN_ACC", "1") != "0"
# BNs whose input comes with no conv statistics get their own statistics pass into an accumulator
# (off by default: measured slower, its reduction runs on few blocks to bound atomic contention)
_BN_OWN_STATS = os.environ.get("PCA_BN_OWN_STATS", "0") != "0"
_DETERMINISTIC = False


def set_deterministic_flag(on: bool) -> None:
    global _DETERMINISTIC
    _DETERMINISTIC = bool(on)


def acc_shards(C: int) -> int:
    """Shard rows of a C-channel accumulator: the consumer folds R*2*C <= 4096 floats per block
    (64 <= C <= 1024) while the producers' same-address atomics spread over R rows."""
    return max(2, min(32, 2048 // max(1, C)))


class StatAcc:
    """[R][NS][C] fp32 accumulator of sharded BN partial sums.

    ``state``: "clean" (all zero), "filled" (a producer added into it), "used" (a consumer folded
    it; it is cleared by the other pass of its BN, or by a memset before the next production)."""

    __slots__ = ("buf", "R", "NS", "C", "state", "shifted")

    def __init__(self, C, NS, device):
        self.C, self.NS, self.R = C, NS, acc_shards(C)
        # [R][NS][C] sums + one K row (the shift a forward-statistics producer subtracted)
        self.buf = torch.zeros(self.R * NS * C + C, dtype=torch.float32, device=device)
        self.state = "clean"
        self.shifted = False   # the last producer subtracted K (and wrote the K row)

    def slab(self, ns=2):
        """[R][ns][C] view (finalize fallback path)."""
        return self.buf[: self.R * ns * self.C].view(self.R, ns, self.C)

    def krow(self):
        """The K row of a shifted forward accumulator, or None."""
        if not self.shifted:
            return None
        o = self.R * 2 * self.C
        return self.buf[o: o + self.C]

    def ensure_clean(self):
        if self.state != "clean":
            self.buf.zero_()
            self.state = "clean"

    def begin(self):
        """Called before a producer adds in."""
        self.ensure_clean()
        self.state = "filled"
        self.shifted = False


class _SlabStats(StatAcc):
    """Channels [off, off + C) of a dense slab's statistics cache ([R][2][ld] centred sums + K row,
    ``DenseSlab.sbuf``): read in place by the fused finalize+apply kernel (acc_off / acc_ld)."""

    __slots__ = ("off", "ld")

    def __init__(self, buf, R, off, ld, C):
        self.buf, self.R, self.off, self.ld, self.C, self.NS = buf, R, off, ld, C, 2
        self.state = "filled"
        self.shifted = True


# ------------------------------------------------- shifted (robust) BatchNorm forward sums
# A conv that delivers its output's BN statistics subtracts a per-channel pilot mean K from every
# value before summing (csrc/common.h stat_shift): var = E[(x-K)^2] - E[x-K]^2 has no catastrophic
# cancellation once K is near the batch mean, which the previous batch's mean is. The pilot
# lives on the producing conv (persistent, so hipGraph replays see a stable address); the
# consuming BN links it on first sight and its finalize / fold writes each batch mean into it.
_BN_SHIFT = os.environ.get("PCA_BN_SHIFT", "1") != "0"   # 0: unshifted sums (A/B)


def conv_pilot(conv, device):
    """The pilot tensor of ``conv`` on ``device`` (None until a BN linked it)."""
    if not _BN_SHIFT:
        return None
    d = conv.__dict__.get("_pca_pilot")
    if d is None:
        return None
    return d.get(device.index if device.index is not None else torch.cuda.current_device())


def link_pilot(conv, C, device):
    """The consuming BN makes sure its producer has a pilot ([C] fp32, zero until the first batch
    mean lands in it) and returns it."""
    d = conv.__dict__.setdefault("_pca_pilot", {})
    key = device.index if device.index is not None else torch.cuda.current_device()
    t = d.get(key)
    if t is None or t.numel() != C:
        t = d[key] = torch.zeros(C, dtype=torch.float32, device=device)
    return t


def bn_pilots(model):
    """Every pilot tensor of ``model``'s convs (training-step state, like the BN buffers)."""
    out = []
    for m in model.modules():
        out += list(m.__dict__.get("_pca_pilot", {}).values())
    return out


def acc_enabled(C: int, device) -> bool:
    return (_BN_ACC and device.type == "cuda" and C % 8 == 0 and C <= 2048
            and not _FORCE_REFERENCE and not (_DETERMINISTIC or _C().deterministic()))


def stat_acc(owner, role: str, C: int, NS: int, device) -> StatAcc:
    """The persistent accumulator of ``owner`` (a module) for ``role`` on ``device``."""
    d = owner.__dict__.get("_pca_acc")
    if d is None:
        d = owner.__dict__["_pca_acc"] = {}
    key = (role, device.index if device.index is not None else torch.cuda.current_device())
    a = d.get(key)
    if a is None or a.C != C or a.NS < NS:
        a = d[key] = StatAcc(C, NS, device)
    return a


def _bn_fusable(C, act, has_res, dual, bn, bn2=None):
    """Can the fused finalize+apply row kernel serve this BN (training mode)?"""
    a = ACT[act]
    if not (C % 8 == 0 and C <= 2048 and (a in (0, 1) or (a == 2 and not has_res and not dual))
            and not (has_res and dual)):
        return False
    return bn.running_mean is not None and (bn2 is None or bn2.running_mean is not None)


_ACC_MAX = []


def _acc_max_elems():
    if not _ACC_MAX:
        _ACC_MAX.append(_C().bn_acc_max_elems())
    return _ACC_MAX[0]


def _own_stats(bn, role, y_nhwc, stats):
    if stats is not None:
        return stats
    a = stat_acc(bn, role, y_nhwc.shape[-1], 2, y_nhwc.device)
    a.begin()
    if _C().bn_stats_acc(y_nhwc, a.buf, a.R):
        return a
    a.state = "clean"             # too large for the accumulator form: nothing was added
    return None


def _dgrad_bn(C, src, dy, wt, H, W, stride, padding, groups, add):
    s2c = add is not None and getattr(add, "_pca_s2c", False)
    if src is None or src.act != 1 or src.mask is None or (src.y2 is not None and src.acc is None):
        return C.conv_dgrad(dy, wt, H, W, stride, padding, groups, add, s2c)
    acc = src.acc
    if acc is not None:
        acc.begin()
        dx, part = C.conv_dgrad_bn(dy, wt, H, W, stride, padding, groups, add, src.y, src.mask,
                                   src.aux, acc.buf, acc.R, src.y2, src.aux2, s2c)
    else:
        dx, part = C.conv_dgrad_bn(dy, wt, H, W, stride, padding, groups, add, src.y, src.mask,
                                   src.aux, addend_s2c=s2c)
    if part.numel():
        src.part, src.dx = part, dx   # the reference to dx keeps autograd from adding into it
    elif acc is not None:
        acc.state = "clean"           # the selected kernel could not fuse: nothing was added
    return dx


class _ConvMFMA(torch.autograd.Function):
    """Implicit-GEMM MFMA conv (fwd + BN-stat epilogue, dgrad, split-K wgrad)."""

    @staticmethod
    def forward(ctx, x, weight, bias, stride, padding, groups, want_stats, cin_pad, slot=None,
                owner=False, bnsrc=None, acc=None, pilot=None, padded=None, brec=None):
        # padded = (wb, wt, remap): operands of the per-group zero-padded form of ``weight``
        # (_conv_group_padded, from the plan); the weight gradient is gathered back by ``remap``
        C = _C()
        ctx.brec = brec
        if brec is not None:
            brec.armed = bias is not None and padded is None and not cin_pad
        ctx.padded = padded[2:] if padded is not None else None
        ctx.slot, ctx.owner = slot, owner
        ctx.bnsrc = bnsrc
        if slot is not None and owner:
            slot.s2c = (_S2C_ADDEND and stride == 2 and padding == 1 and groups == 1 and
                        weight.shape[2] == 3 and weight.shape[3] == 3 and
                        x.shape[1] % 2 == 0 and x.shape[2] % 2 == 0)
        w_phys = G.physical(weight)
        if not w_phys.is_contiguous():
            w_phys = w_phys.contiguous()
        need_dx = ctx.needs_input_grad[0]
        if cin_pad:
            wb = None
            plan = _PLAN["cur"]
            if plan is not None and not need_dx and groups == 1 and weight.is_leaf and \
                    weight.permute(0, 2, 3, 1).is_contiguous():
                # zero-padded copy made by the plan's one batched launch (no pad + convert here)
                key = ("pad", cin_pad)
                e = plan.lookup(weight, key) or plan.register(weight, key, None)
                wb, wt = e.wb, None
                if plan.tables is None:          # first sight of this weight: fill it now
                    wb.copy_(F.pad(w_phys, (0, cin_pad - w_phys.shape[-1])).to(COMPUTE_DTYPE))
            if wb is None:
                w_phys = F.pad(w_phys, (0, cin_pad - w_phys.shape[-1]))
                wb, wt = C.weight_prep(w_phys, groups, need_dx)
        elif padded is not None:
            wb, wt = padded[0], padded[1]
        else:
            wb, wt = _prepped_weight(weight, groups, w_phys, need_dx)
        if not want_stats:
            pilot = None
        if acc is not None and want_stats:
            acc.begin()
            y, _ = C.conv_fwd(x, wb, bias, stride, padding, groups, True, acc.buf, acc.R, pilot)
            acc.shifted = pilot is not None
            stats = None                  # delivered through the accumulator (conv2d returns it)
        else:
            y, stats = C.conv_fwd(x, wb, bias, stride, padding, groups, want_stats, None, 0, pilot)
            if pilot is not None and stats is not None and stats.numel():
                # the slab's sums are of x - pilot (finalize adds it back). A snapshot, not the live
                # pilot: a finalize writes the new batch mean into the pilot, and a second finalize
                # of these sums (one conv output read by two BNs, or the conv called twice before
                # its BN finalizes) must still add back the K its sums were taken against
                stats._pca_kin = pilot.clone()
        ctx.geom = (stride, padding, groups, cin_pad, x.shape[1], x.shape[2])
        ctx.save_for_backward(x, wt if need_dx else None)
        ctx.weight = weight
        ctx.bias = bias
        if stats is None or not want_stats:
            stats = torch.empty(0, device=x.device)
        ctx.mark_non_differentiable(stats)
        # no zero-filled gradient for the (non-differentiable) statistics output: autograd
        # would otherwise launch one fill kernel per conv per step
        ctx.set_materialize_grads(False)
        return y, stats

    @staticmethod
    def backward(ctx, dy, _dstats):
        if dy is None:
            return (None,) * 15
        C = _C()
        x, wt = ctx.saved_tensors
        stride, padding, groups, cin_pad, H, W = ctx.geom
        dy = dy.contiguous()
        weight, bias = ctx.weight, ctx.bias
        dx = None
        # with the side stream the weight gradient is issued first, so it runs beside this
        # conv's dgrad (both only need dy); otherwise dgrad then wgrad on the one stream
        side_first = wgrad_stream(x.device) is not None

        def do_dgrad():
            nonlocal dx
            if ctx.needs_input_grad[0]:
                slot = ctx.slot
                src = ctx.bnsrc
                ctx.bnsrc = None
                if slot is not None and ctx.owner:
                    add = slot.take()            # the other branch's dX, summed in the epilogue
                    dx = _dgrad_bn(C, src, dy, wt, H, W, stride, padding, groups, add)
                elif slot is None:
                    dx = _dgrad_bn(C, src, dy, wt, H, W, stride, padding, groups, None)
                elif (slot.s2c and slot.grad is None and stride == 2 and padding == 0 and
                      groups == 1 and wt.shape[1] == 1 and wt.shape[2] == 1 and
                      H == 2 * dy.shape[1] and W == 2 * dy.shape[2]):
                    # 1x1 stride-2 projection shortcut: its dX is nonzero only at the even-even
                    # pixels — computed compact as a plain 1x1 dgrad (a GEMM, no parity classes
                    # writing zeros) and added by the owner's parity dgrad in its class 0
                    dxc = C.conv_dgrad(dy, wt, dy.shape[1], dy.shape[2], 1, 0, 1)
                    dxc._pca_s2c = True
                    if slot.offer(dxc):
                        dx = None
                    else:
                        dx = C.conv_dgrad(dy, wt, H, W, stride, padding, groups)
                else:
                    # another consumer's gradient already waiting in the slot (GoogLeNet's
                    # Inception input feeds three 1x1 convs and a max-pool; a DLA level-2 tree
                    # input feeds two blocks with projection shortcuts): this dgrad adds it in
                    # its epilogue and hands the sum on, so the owner finally stores the total —
                    # no autograd add between the branches. A compact stride-2 pending gradient
                    # is added by a 3x3 / stride-2 dgrad's parity class 0 (or expanded by the
                    # binding when the selected kernel cannot).
                    pend = slot.grad
                    s2c = pend is not None and getattr(pend, "_pca_s2c", False)
                    want = ((dy.shape[0], H // 2, W // 2, wt.shape[0]) if s2c
                            else (dy.shape[0], H, W, wt.shape[0]))
                    if (pend is None or pend.dim() != 4 or tuple(pend.shape) != want
                            or not pend.is_contiguous() or pend.dtype != dy.dtype
                            or (s2c and (stride != 2 or H % 2 or W % 2))):
                        pend, s2c = None, False
                    else:
                        slot.grad = None
                    dx = C.conv_dgrad(dy, wt, H, W, stride, padding, groups, pend, s2c)
                    if slot.offer(dx):
                        dx = None                # delivered through the owner's epilogue

        if not side_first:
            do_dgrad()
        KH, KW = weight.shape[2], weight.shape[3]
        dw_ret = db_ret = None
        if weight.requires_grad and cin_pad and weight.is_leaf and KH == 3 and KW == 3:
            # stem conv: dedicated small-Cin wgrad adds straight into the fp32 gradient
            sbuf = G.grad_buffer(weight)
            if sbuf is not None and C.stem_wgrad(x, dy, stride, padding, sbuf):
                G.fire(weight)
                weight = None
        if weight is not None and weight.requires_grad and cin_pad and weight.is_leaf and groups == 1:
            # other channel-padded convs (stems the dedicated kernel does not cover: GoogLeNet's
            # 3 -> 192, ShuffleNetV2's 3 -> 24): the padded dW accumulates in a persistent buffer
            # whose real entries one native remap adds into the arena and zeroes (its padding
            # entries stay exact zeros: the padded input channels are zero) — no fill, no slice
            # + autograd add
            buf = G.grad_buffer(weight)
            Co, Ci = weight.shape[0], weight.shape[1]
            if buf is not None and tuple(buf.shape) == (Co, KH, KW, Ci):
                pbuf = weight.__dict__.get("_pca_pad_dw")
                if pbuf is None or pbuf.shape != (Co, KH, KW, cin_pad) or pbuf.device != x.device:
                    pbuf = torch.zeros((Co, KH, KW, cin_pad), dtype=torch.float32, device=x.device)
                    weight.__dict__["_pca_pad_dw"] = pbuf
                C.conv_wgrad(x, dy, KH, KW, stride, padding, groups, pbuf)
                _weight_pad_remap(1, Co, Co, Ci, cin_pad, KH * KW).apply(
                    pbuf, inverse=True, acc=buf, clear_src=True)
                G.fire(weight)
                weight = None
        if weight is not None and weight.requires_grad and ctx.padded is not None:
            # padded-form dW [G*op][KH][KW][cp], its real entries gathered into the arena
            remap, dwbuf = ctx.padded
            dw = C.conv_wgrad(x, dy, KH, KW, stride, padding, groups, dwbuf)
            clear = dwbuf is not None
            buf = G.grad_buffer(weight)
            phys = G.physical(weight).shape
            flat = remap.flat
            if flat:
                dw = dw.reshape(-1)
            if buf is not None and tuple(buf.shape) == tuple(phys):
                remap.apply(dw, inverse=True, acc=buf.view(-1) if flat else buf, clear_src=clear)
                G.fire(weight)
            else:
                G.accumulate(weight, remap.apply(dw, inverse=True, clear_src=clear).view(phys))
            weight = None
        if weight is not None and weight.requires_grad:
            buf = None if (cin_pad or not weight.is_leaf) else G.grad_buffer(weight)
            side = wgrad_stream(x.device) if buf is not None else None
            if side is not None:
                side.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(side):
                    C.conv_wgrad(x, dy, KH, KW, stride, padding, groups, buf)
                x.record_stream(side)
                dy.record_stream(side)
                _schedule_join()
                G.fire(weight)
            elif buf is not None:
                piggy = _WGRAD_PIGGY and not _WGRAD_DEFER
                if _piggy_set[0] != piggy:
                    C.wgrad_piggy(piggy)
                    _piggy_set[0] = piggy
                C.conv_wgrad(x, dy, KH, KW, stride, padding, groups, buf,
                             defer=_WGRAD_DEFER or piggy)
                if (_WGRAD_DEFER or piggy) and C.wgrad_deferred():
                    _after_deferred_wgrad()
                G.fire(weight)
            else:
                dw = C.conv_wgrad(x, dy, KH, KW, stride, padding, groups, None)
                if cin_pad:
                    dw = dw[..., : weight.shape[1]]
                if weight.is_leaf:
                    G.accumulate(weight, dw)
                else:
                    dw_ret = dw.permute(0, 3, 1, 2)
        if side_first:
            do_dgrad()
        if ctx.brec is not None and ctx.brec.done:
            bias = None                      # added by the consuming BN's backward finalize
        if bias is not None and bias.requires_grad:
            bbuf = G.grad_buffer(bias) if bias.is_leaf else None
            if bbuf is not None:
                C.bias_grad(dy, bbuf)        # summed straight into the gradient arena
                G.fire(bias)
            else:
                db = C.bias_grad(dy)
                if bias.is_leaf:
                    G.accumulate(bias, db)
                else:
                    db_ret = db
        return dx, dw_ret, db_ret, None, None, None, None, None, None, None, None, None, None, None, None


class _ConvDirect(torch.autograd.Function):
    """Generic direct conv for odd channel counts / tiny groups (LeNet, DPN, PNASNet-A...)."""

    @staticmethod
    def forward(ctx, x, weight, bias, stride, padding, groups):
        C = _C()
        w_phys = G.physical(weight).contiguous()
        y = C.direct_fwd(x, w_phys, bias, stride, padding, groups)
        ctx.save_for_backward(x, w_phys)
        ctx.geom = (stride, padding, groups)
        ctx.weight, ctx.bias = weight, bias
        return y

    @staticmethod
    def backward(ctx, dy):
        C = _C()
        x, w_phys = ctx.saved_tensors
        stride, padding, groups = ctx.geom
        dy = dy.contiguous()
        weight, bias = ctx.weight, ctx.bias
        dx = None
        if ctx.needs_input_grad[0]:
            dx = C.direct_dgrad(dy, w_phys, x.shape[1], x.shape[2], stride, padding, groups)
        with_bias = bias is not None and bias.requires_grad
        dw_ret = db_ret = None
        if weight.requires_grad or with_bias:
            flat = C.direct_wgrad(x, dy, weight.shape[2], weight.shape[3], stride, padding, groups, with_bias)
            nw = w_phys.numel()
            if weight.requires_grad:
                dw = flat[:nw].view_as(w_phys)
                if weight.is_leaf:
                    G.accumulate(weight, dw)
                else:
                    dw_ret = dw.permute(0, 3, 1, 2)
            if with_bias:
                if bias.is_leaf:
                    G.accumulate(bias, flat[nw:])
                else:
                    db_ret = flat[nw:]
        return dx, dw_ret, db_ret, None, None, None


class _ConvDepthwise(torch.autograd.Function):
    """Depthwise conv (groups == Cin, multiplier Cout/Cin), bandwidth-bound direct kernels.

    With ``acc`` (the consuming BatchNorm's StatAcc) the forward kernel adds that BN's batch
    statistics into it (``out[0]`` reports whether it did); with ``bnsrc`` (the producing
    BN(+ReLU/swish) record) the dgrad kernel adds that BN's backward sums into its accumulator —
    the two separate passes + finalize launches of each BN around a depthwise conv disappear
    (mobilenetv2.py:33-36, efficientnet.py:96-103)."""

    @staticmethod
    def forward(ctx, x, weight, stride, padding, acc=None, bnsrc=None, out=None, slot=None):
        C = _C()
        ctx.slot = slot
        Co, _, KH, KW = weight.shape
        wT = _dw_weight(weight)
        if acc is not None:
            acc.begin()
            y, ok = C.dw_fwd_stats(x, wT, KH, KW, stride, padding, acc.buf, acc.R)
            if not int(ok):
                acc.state = "clean"           # nothing was added
            elif out is not None:
                out.append(acc)
        else:
            y = C.dw_fwd(x, wT, KH, KW, stride, padding)
        ctx.save_for_backward(x, wT)
        ctx.geom = (stride, padding, KH, KW)
        ctx.weight = weight
        ctx.bnsrc = bnsrc
        return y

    @staticmethod
    def backward(ctx, dy):
        C = _C()
        x, wT = ctx.saved_tensors
        stride, padding, KH, KW = ctx.geom
        dy = dy.contiguous()
        dx = None
        src = ctx.bnsrc
        ctx.bnsrc = None
        if ctx.needs_input_grad[0]:
            H, W, Cx = x.shape[1], x.shape[2], x.shape[3]
            if (src is not None and src.acc is not None and src.y2 is None   # (no dual-BN sums)
                    and src.y.is_contiguous()):
                src.acc.begin()
                dx, ok = C.dw_dgrad_bn(dy, wT, H, W, Cx, KH, KW, stride, padding, src.y, src.mask,
                                       src.aux, src.act, src.acc.buf, src.acc.R)
                if int(ok):
                    src.part, src.dx = src.acc.buf, dx   # the BN backward finds its sums filled
                else:
                    src.acc.state = "clean"
            else:
                dx = C.dw_dgrad(dy, wT, H, W, Cx, KH, KW, stride, padding)
                if ctx.slot is not None and ctx.slot.offer(dx):
                    # (ShuffleNetV2 DownBlock, shufflenetv2.py:84-90: x feeds this depthwise conv
                    # and a 1x1 conv — the 1x1's dgrad epilogue adds this gradient)
                    dx = None
        w = ctx.weight
        dw_ret = None
        if w.requires_grad:
            buf = G.grad_buffer(w) if w.is_leaf else None
            if buf is not None and buf.is_contiguous():
                # channels_last [Co,1,KH,KW] == physical [Co][KH][KW]: the final reduce adds into
                # the arena view directly
                C.dw_wgrad(x, dy, KH, KW, stride, padding, buf.view(-1))
                G.fire(w)
            else:
                dw = C.dw_wgrad(x, dy, KH, KW, stride, padding)  # [Co, KH*KW]
                if w.is_leaf:
                    G.accumulate(w, dw.view(w.shape[0], KH, KW, 1))
                else:
                    dw_ret = dw.view(w.shape)
        return dx, dw_ret, None, None, None, None, None, None


# PCA_DW_BN_FUSE=1: depthwise k3 convs carry the BatchNorm sums of their neighbours in their
# epilogues (dwconv.hip dwk_epi_*: 2 launches fewer per BN). Off by default: measured same-box,
# the fused kernels (2-3 waves per SIMD against the plain kernels' 3) cost more than the
# bandwidth-bound passes + finalize they replace — MobileNetV2 bs1024 13.64 -> 14.52 ms,
# EfficientNet-B0 bs128 3.93 -> 3.99 ms.
_DW_BN_FUSE = os.environ.get("PCA_DW_BN_FUSE", "0") == "1"


def conv2d(x, weight, bias=None, stride=1, padding=0, groups=1, want_stats=False, acc=None,
           pilot=None, brec=None):
    """NCHW-shaped conv. On GPU returns (y, stats) where stats are BN partials (a slab tensor, or
    ``acc`` — a :class:`StatAcc` the epilogue added into — when one is given), or None. With
    ``pilot`` (the consuming BN's shift, :func:`link_pilot`) the MFMA paths sum x - pilot."""
    if isinstance(stride, (tuple, list)):
        assert stride[0] == stride[1]
        stride = stride[0]
    if isinstance(padding, (tuple, list)):
        assert padding[0] == padding[1]
        padding = padding[0]
    if _ref(x):
        # the reference path computes in the default (NCHW) format: PyTorch's CPU channels_last
        # kernels lose ~1e-3 relative accuracy in BN/conv backward chains (tests/test_models_cpu)
        if x.device.type == "cpu":
            weight = weight.contiguous()
            x = x.contiguous()
        return F.conv2d(x, weight, bias, stride, padding, 1, groups), None
    Cout, Cg, KH, KW = weight.shape
    Cin = x.shape[1]
    cout_g = Cout // groups
    if groups > 1 and groups == Cin and Cg == 1:
        got = []
        fuse = _DW_BN_FUSE and bias is None
        bnsrc = getattr(x, "_pca_bnsrc", None) if (x.requires_grad and fuse) else None
        y = _ConvDepthwise.apply(to_nhwc(x), weight, stride, padding,
                                 acc if (want_stats and fuse) else None, bnsrc, got,
                                 _slot_for_residual(x))
        if bias is not None:
            y = add_bias(y, bias)
        return to_nchw(y), (got[0] if got else None)
    if Cg % 8 == 0 and cout_g % 8 == 0:
        slot, owner = _slot_for_conv(x)
        bnsrc = getattr(x, "_pca_bnsrc", None) if x.requires_grad else None
        y, stats = _ConvMFMA.apply(to_nhwc(x), weight, bias, stride, padding, groups, want_stats, 0,
                                   slot, owner, bnsrc, acc if want_stats else None, pilot, None,
                                   brec)
        if want_stats and acc is not None:
            return to_nchw(y), acc
        return to_nchw(y), (stats if want_stats else None)
    if groups == 1 and cout_g % 8 == 0 and Cin < 8 * 2 and Cout >= 16:
        # stem conv on 3-channel images: pad channels to 8 and run on MFMA
        cp = _round8(Cin)
        # (BN partial sums into the accumulator as for every other MFMA conv: no finalize launch)
        y, stats = _ConvMFMA.apply(to_nhwc(x, pad_to=cp), weight, bias, stride, padding, groups, want_stats, cp,
                                   None, False, None, acc if want_stats else None, pilot)
        if want_stats and acc is not None:
            return to_nchw(y), acc
        return to_nchw(y), (stats if want_stats else None)
    S = _group_dense_width(Cin, Cout, Cg, cout_g, groups)
    if S:
        return _conv_group_dense(x, weight, bias, stride, padding, groups, S, want_stats, acc, pilot)
    if _GROUP_PAD:
        return _conv_group_padded(x, weight, bias, stride, padding, groups, want_stats)
    y = _ConvDirect.apply(to_nhwc(x), weight, bias, stride, padding, groups)
    return to_nchw(y), None


# Convs whose per-group widths are not multiples of 8 (ShuffleNet's 25/50/100-channel
# groups, shufflenet.py:26-33; DPN's groups=32 with 3..24 channels, dpn.py:15; ResNeXt29_32x4d's
# 4, resnext.py:19; LeNet 3->6->16, densenet_cifar's growth 12, PNASNet-A's 44) run on the MFMA
# implicit GEMM with every group zero-padded to a multiple of 8 channels on both sides: pad
# (input, weight) and slice (output,
# BN statistics) are plain differentiable tensor ops, so autograd carries the gradients back
# through them. Even where the padded group leaves most of a 64-wide MFMA tile empty (DPN's
# 3-channel groups) this beats the scalar direct kernels by 10-30x (tools/zoo_bench.py).
_GROUP_PAD = os.environ.get("PCA_GROUP_PAD", "1") != "0"
# zero-padded convs (groups == 1) hand their output to the consumer as a row-strided prefix view
_PAD_VIEW = os.environ.get("PCA_PAD_VIEW", "1") != "0"


# Narrow groups as block-diagonal super-groups: P = S / Cg neighbouring groups become one group of
# S input channels whose weight is block-diagonal (zeros between the original groups). The
# activations keep their layout (no pad / slice passes, and the conv keeps its fused BN
# statistics / gradient hand-offs), the weight is expanded by one native remap per step and its
# gradient's diagonal blocks are gathered back by the adjoint remap. It trades S / Cg x MFMA work
# for tiles the implicit GEMM runs efficiently: DPN's 3..24-channel groups (dpn.py:15) ran at
# ~15 TFLOP/s padded to 8 per group, plus two activation remap passes per conv each way.
# PCA_GROUP_DENSE: 1 (default) for widths that are not multiples of 8, "all" also for multiples
# of 8 below 64, 0 off.
_GROUP_DENSE = os.environ.get("PCA_GROUP_DENSE", "1")
# PCA_S2C_ADDEND=0: projection-shortcut dX written whole (zeros at 3 of 4 pixels) and added as a
# full addend, instead of the compact even-even form
_S2C_ADDEND = os.environ.get("PCA_S2C_ADDEND", "1") != "0"


def _group_dense_width(Cin, Cout, Cg, cout_g, groups):
    """Super-group input width S for a grouped conv (0: keep the plain / padded path): the
    smallest multiple of Cg that is >= 64, divides Cin and keeps both super-group widths
    multiples of 8 (else the largest such)."""
    if groups <= 1 or _GROUP_DENSE == "0" or (Cg % 8 == 0 and cout_g % 8 == 0 and
                                               (_GROUP_DENSE != "all" or Cg >= 64)):
        return 0
    best = 0
    for P in range(1, groups + 1):
        if groups % P:
            continue
        S, So = P * Cg, P * cout_g
        if S % 8 or So % 8:
            continue
        best = S
        if S >= 64:
            break
    return best


def _group_dense_remap(Cout, cout_g, Cg, S, K):
    """Weight [Cout][K][Cg] (flat) -> block-diagonal [Cout][K][S] (flat)."""
    def build():
        # (vectorised: DPN92's widest conv maps 663k weight slots)
        P = S // Cg
        r = torch.arange(Cout).view(Cout, 1, 1)
        k = torch.arange(K).view(1, K, 1)
        j = torch.arange(S).view(1, 1, S)
        lg = (r // cout_g) % P
        inside = (j >= lg * Cg) & (j < (lg + 1) * Cg)
        src = (r * K + k) * Cg + j - lg * Cg
        cmap = torch.where(inside, src, torch.full_like(src, -1)).reshape(-1).tolist()
        m = Remap(cmap, Cout * K * Cg)
        m.flat = True
        return m
    return Remap.get(("gdense", Cout, cout_g, Cg, S, K), build)


def _conv_group_dense(x, weight, bias, stride, padding, groups, S, want_stats, acc, pilot):
    Cout, Cg, KH, KW = weight.shape
    Cin = x.shape[1]
    remap = _group_dense_remap(Cout, Cout // groups, Cg, S, KH * KW)
    plan = _PLAN["cur"]
    padded = None
    if (plan is not None and weight.is_leaf and weight.dtype == torch.float32
            and weight.permute(0, 2, 3, 1).is_contiguous()):
        # block-diagonal bf16 operands written by the plan's batched launch / the fused
        # optimizer (weight_prep pass 6) from the master: no per-step expansion + convert
        key = ("gdense", Cin // S, Cout // groups, Cg, S)
        e = plan.lookup(weight, key)
        if e is None:
            e = plan.register(weight, key, remap.apply(G.physical(weight).detach().reshape(-1))
                              .view(Cout, KH, KW, S))
        padded = (e.wb, e.wt, remap, None)
        wp = weight
    else:
        wp = to_nchw(_remap_param(weight, remap, (Cout, KH, KW, S)))
    slot, owner = _slot_for_conv(x)
    bnsrc = getattr(x, "_pca_bnsrc", None) if x.requires_grad else None
    y, stats = _ConvMFMA.apply(to_nhwc(x), wp, bias, stride, padding, Cin // S, want_stats, 0,
                               slot, owner, bnsrc, acc if want_stats else None, pilot, padded)
    if want_stats and acc is not None:
        return to_nchw(y), acc
    return to_nchw(y), (stats if want_stats else None)


def _group_pad_remap(groups, n, npad):
    """[groups * npad] <- [groups * n]: each group's n channels followed by npad - n zeros."""
    def build():
        return Remap([(j // npad) * n + j % npad if j % npad < n else -1
                      for j in range(groups * npad)], groups * n)
    return Remap.get(("gpad", groups, n, npad), build)


def _group_unpad_remap(groups, n, npad):
    """[groups * n] <- [groups * npad] (the slice back to the logical channels)."""
    def build():
        return Remap([(j // n) * npad + j % n for j in range(groups * n)], groups * npad)
    return Remap.get(("gunpad", groups, n, npad), build)


def _weight_pad_remap(groups, cout_g, op, Cg, cp, K):
    """Conv weight [G*cout_g][K][Cg] -> [G*op][K][cp]: zero output rows and input channels."""
    def build():
        cmap = [c if c < Cg else -1 for c in range(cp)]
        rmap = [(r // op) * cout_g + r % op if r % op < cout_g else -1 for r in range(groups * op)]
        return Remap(cmap, Cg, rmap, groups * cout_g, K)
    return Remap.get(("wpad", groups, cout_g, op, Cg, cp, K), build)


def _conv_group_padded(x, weight, bias, stride, padding, groups, want_stats):
    """Odd-width grouped conv on the MFMA kernels: the per-group zero padding of the input,
    weight and bias and the slice of the output / BN statistics are native channel remaps
    (one launch each way, gradients of the weight and bias added into the arena)."""
    Cout, Cg, KH, KW = weight.shape
    cout_g = Cout // groups
    cp, op = _round8(Cg), _round8(cout_g)
    if groups == 1 and cp != Cg and getattr(x, "_pca_zpad", 0) == cp:
        # the producer left x as the prefix of a zero-padded buffer of this width: read in place
        xv = x.permute(0, 2, 3, 1)
        N, H, W, _ = xv.shape
        assert xv.stride() == (H * W * cp, W * cp, cp, 1), "zero-padded input layout"
        xn = _ZeroPadView.apply(xv, cp)
    else:
        xn = to_nhwc(x)
        N, H, W, _ = xn.shape
        if cp != Cg and groups == 1:
            # x feeds other consumers too (ShuffleNetV2 DownBlock: this 1x1 conv3 and the left
            # depthwise conv1, shufflenetv2.py:84-90): the unpad of this conv's dX adds their
            # gradient in the same pass (_PadInput)
            pslot, powner = _slot_for_conv(x)
            xn = _PadInput.apply(xn, _group_pad_remap(groups, Cg, cp), (N, H, W, groups * cp),
                                 pslot if powner else None)
        elif cp != Cg:
            xn = _RemapFn.apply(xn, _group_pad_remap(groups, Cg, cp), (N, H, W, groups * cp), None)
    # weight [Cout, Cg, KH, KW] -> [G*op, cp, KH, KW], channels_last (the MFMA B layout): with a
    # plan, the padded bf16 operands are written by its batched launch (or the fused optimizer
    # step) straight from the master — no per-step fp32 remap + convert
    padded = None
    if cp != Cg or op != cout_g:
        wr = _weight_pad_remap(groups, cout_g, op, Cg, cp, KH * KW)
        plan = _PLAN["cur"]
        if (plan is not None and weight.is_leaf and weight.dtype == torch.float32
                and weight.permute(0, 2, 3, 1).is_contiguous()):
            key = ("gpad", groups, cout_g, op, Cg, cp)
            e = plan.lookup(weight, key)
            if e is None:
                e = plan.register(weight, key, wr.apply(G.physical(weight).detach())
                                  .view(groups * op, KH, KW, cp))
            if e.dwbuf is None:
                # the padded dW accumulates here and the adjoint remap that gathers its real
                # entries zeroes them (its padding entries stay exact zeros: the padded input
                # channels and output-gradient channels are zero) — no fill launch per step
                e.dwbuf = torch.zeros((groups * op, KH, KW, cp), dtype=torch.float32,
                                      device=weight.device)
            padded = (e.wb, e.wt, wr, e.dwbuf)
            wp = weight
        else:
            wp = to_nchw(_remap_param(weight, wr, (groups * op, KH, KW, cp)))
    else:
        wp = weight
    bp = None
    if bias is not None:
        bp = bias if op == cout_g else _remap_param(bias, _group_pad_remap(groups, cout_g, op),
                                                    (groups * op,))
    # an unpadded input (only the output width is odd) is x itself: the conv takes part in x's
    # gradient slot like any MFMA conv (ShuffleNetV2 DownBlock conv3, shufflenetv2.py:84-90)
    slot, owner = _slot_for_conv(x) if (groups == 1 and cp == Cg) else (None, False)
    y, stats = _ConvMFMA.apply(xn, wp, bp, stride, padding, groups, want_stats, 0, slot, owner,
                               None, None, None, padded)
    if op != cout_g and groups == 1 and _PAD_VIEW:
        # the real channels are a prefix: consumers read them in place (BatchNorm: row-strided
        # vector kernels, its dY handed back already padded)
        slot = _PadSlot()
        yv = to_nchw(_UnpadView.apply(y, Cout, slot))
        yv._pca_padslot = slot
        if want_stats and stats is not None and stats.numel():
            stats = stats.view(stats.shape[0], 2, op)[:, :, :Cout]
        return yv, (stats if want_stats and stats is not None and stats.numel() else None)
    if op != cout_g:
        Ho, Wo = y.shape[1], y.shape[2]
        unpad = _group_unpad_remap(groups, cout_g, op)
        y = _RemapFn.apply(y, unpad, (N, Ho, Wo, Cout), None)
        if want_stats and stats is not None and stats.numel():
            R = stats.shape[0]
            if groups == 1:
                # the real channels are a prefix: the BN finalize reads the padded rows in place
                stats = stats.view(R, 2, op)[:, :, :Cout]
            else:
                stats = unpad.apply(stats.contiguous()).view(R, 2, Cout)
    return to_nchw(y), (stats if want_stats and stats is not None and stats.numel() else None)


class _AddBias(torch.autograd.Function):
    @staticmethod
    def forward(ctx, y, bias):
        ctx.bias = bias
        return (y.float() + bias).to(y.dtype)

    @staticmethod
    def backward(ctx, dy):
        b = ctx.bias
        db_ret = None
        if b.requires_grad:
            bbuf = G.grad_buffer(b) if b.is_leaf else None
            if bbuf is not None:
                _C().bias_grad(dy.contiguous(), bbuf)
                G.fire(b)
            else:
                db = _C().bias_grad(dy.contiguous())
                if b.is_leaf:
                    G.accumulate(b, db)
                else:
                    db_ret = db
        return dy, db_ret


def add_bias(y_nhwc, bias):
    return _AddBias.apply(y_nhwc, bias)


# -------------------------------------------------------------------------- batch norm
class _BNCfg:
    __slots__ = ("bn", "bn2", "act", "training", "count", "src", "bacc", "faccs", "pilot", "pilot2",
                 "dest", "dslot", "padslot", "brec")

    def __init__(self, bn, bn2, act, training, count):
        self.bn, self.bn2, self.act, self.training, self.count = bn, bn2, act, training, count
        self.dest = None      # NHWC channel slice of a concat slab the output is written into
        self.dslot = None     # dense slab: GradSlot where the slab's gradient of the input waits
        self.pilot = self.pilot2 = None   # the producers' pilots (receive this batch's means)
        self.src = None
        self.bacc = None      # the BN's backward StatAcc (sharded sums of dz, dz*xhat[, dz*xhat2])
        self.faccs = ()       # forward StatAccs this BN consumed (cleared by its backward kernel)
        self.padslot = None   # zero-padded conv output read in place: its dY goes back padded
        self.brec = None      # BiasRec of the conv whose output only this BN reads


def _bn_aux(C, bn, y, stats, training, count, pilot=None, kin=None, zero=None):
    """Finalize: aux [mean | invstd | scale | shift]. ``kin``: the shift the sums are of (pilot /
    K row / centred pass); ``pilot``: receives the batch mean (the producer's next shift);
    ``zero``: a StatAcc (this BN's backward accumulator) the finalize kernel clears."""
    if isinstance(stats, StatAcc):
        # an accumulator the fused kernel cannot consume here: finalize from its shard rows
        aux = _bn_aux(C, bn, y, stats.slab(), training, count, pilot, stats.krow(), zero)
        stats.state = "used"
        return aux
    use_batch = training or bn.running_mean is None
    rm = bn.running_mean
    rv = bn.running_var
    if rm is None:
        rm = torch.zeros(y.shape[-1], device=y.device)
        rv = torch.ones(y.shape[-1], device=y.device)
    update = training and bn.running_mean is not None
    if use_batch and stats is None:
        # no producer delivered sums: one centred pass (sums of y - y[0]; robust variance)
        stats, kin = C.bn_stats_centered(y if y.is_contiguous() or y.shape[-1] % 8 == 0
                                         else y.contiguous())
    elif use_batch and kin is None:
        kin = getattr(stats, "_pca_kin", None)
    momentum = bn.momentum if bn.momentum is not None else 0.1
    w = bn.weight.detach() if bn.weight is not None else None
    b = bn.bias.detach() if bn.bias is not None else None
    aux = C.bn_finalize(stats if use_batch else None, float(count), w, b, rm, rv,
                        bn.num_batches_tracked if update else None, momentum, bn.eps, use_batch, update,
                        kin if use_batch else None, pilot if use_batch else None,
                        zero.buf if zero is not None else None)
    if zero is not None:
        zero.state = "clean"
    return aux


class _BatchNormAct(torch.autograd.Function):
    """out = act(BN(y) [+ residual | + BN2(y2)]) with stats from the conv epilogue when given."""

    @staticmethod
    def forward(ctx, y, gamma, beta, res, y2, gamma2, beta2, stats, stats2, cfg, slot=None):
        C = _C()
        ctx.slot = slot
        relu = ACT[cfg.act] == 1
        bn, bn2 = cfg.bn, cfg.bn2
        fused = (cfg.training and isinstance(stats, StatAcc) and
                 (y2 is None or isinstance(stats2, StatAcc)) and
                 _bn_fusable(y.shape[-1], cfg.act, res is not None, y2 is not None, bn, bn2))
        if fused:
            def mom(b):
                return b.momentum if b.momentum is not None else 0.1

            a2 = stats2 if y2 is not None else None
            out, mask, aux, aux2 = C.bn_apply_acc(
                y, stats.buf, stats.R, float(cfg.count),
                bn.weight.detach() if bn.weight is not None else None,
                bn.bias.detach() if bn.bias is not None else None,
                bn.running_mean, bn.running_var, bn.num_batches_tracked, mom(bn), bn.eps,
                res, y2, a2.buf if a2 is not None else None, a2.R if a2 is not None else 0,
                bn2.weight.detach() if (a2 is not None and bn2.weight is not None) else None,
                bn2.bias.detach() if (a2 is not None and bn2.bias is not None) else None,
                bn2.running_mean if a2 is not None else None,
                bn2.running_var if a2 is not None else None,
                bn2.num_batches_tracked if a2 is not None else None,
                mom(bn2) if a2 is not None else 0.1, bn2.eps if a2 is not None else 1e-5,
                ACT[cfg.act], relu, cfg.bacc.buf if cfg.bacc is not None else None,
                stats.shifted, cfg.pilot, a2.shifted if a2 is not None else False,
                cfg.pilot2 if a2 is not None else None, cfg.dest,
                acc_off=stats.off if isinstance(stats, _SlabStats) else 0,
                acc_ld=stats.ld if isinstance(stats, _SlabStats) else 0)
            if cfg.bacc is not None:
                cfg.bacc.state = "clean"      # block 0 cleared this BN's backward accumulator
            stats.state = "used"
            cfg.faccs = (stats,) if a2 is None else (stats, a2)
            if isinstance(stats, _SlabStats):
                cfg.faccs = ()   # (the slab's cache is shared by the block's later BNs)
            if a2 is not None:
                a2.state = "used"
            if aux2 is not None and not aux2.numel():
                aux2 = None
            if mask is not None and not mask.numel():
                mask = None
        else:
            # (the finalize kernel's block 0 clears this BN's backward accumulator: no memset)
            aux = _bn_aux(C, bn, y, stats if isinstance(stats, StatAcc) or (stats is not None and stats.numel()) else None,
                          cfg.training, cfg.count, cfg.pilot, zero=cfg.bacc)
            aux2 = None
            if y2 is not None:
                aux2 = _bn_aux(C, bn2, y2, stats2 if isinstance(stats2, StatAcc) or (stats2 is not None and stats2.numel()) else None,
                               cfg.training, cfg.count, cfg.pilot2)
            out, mask = C.bn_apply(y, aux, res, y2, aux2, ACT[cfg.act], relu, cfg.dest)
            if cfg.bacc is not None:
                cfg.bacc.ensure_clean()
            cfg.faccs = tuple(a for a in (stats, stats2) if isinstance(a, StatAcc))
        ctx.cfg = cfg
        ctx.has_res = res is not None
        # ReLU backward needs only the sign of the output: keep the 1-bit mask when the kernel
        # produced one (C % 8 == 0), else the output itself
        has_mask = mask is not None and mask.numel() > 0
        ctx.save_for_backward(y, out if (relu and not has_mask) else None, mask if has_mask else None,
                              aux, y2, aux2)
        ctx.bnsrc = None
        if not y.is_contiguous() and not (y2 is None and y.shape[-1] % 8 == 0 and _nhwc_rows(y)
                                          and _STRIDED_BN_FUSE):
            # (the consumer dgrad's fused reduce reads a dense y, or a row-strided channel slice:
            # a DenseNet BatchNorm's slab suffix, the igemm / split-K dgrads only)
            cfg.src = None
        # (grad mode is off inside Function.forward: the caller decided it in cfg.src)
        if cfg.src is not None and relu and has_mask and y2 is None:
            ctx.bnsrc = cfg.src = _BNSrc(y, mask, aux, cfg.bacc)
        elif cfg.src is not None and relu and has_mask and _DUAL_BN_FUSE and \
                cfg.bacc is not None and cfg.bacc.NS >= 3 and aux2 is not None:
            # projection-shortcut tail: the consumer dgrad adds all three sums (dz, dz*xhat,
            # dz*xhat2) into the accumulator — no separate reduce + finalize launches
            ctx.bnsrc = cfg.src = _BNSrc(y, mask, aux, cfg.bacc, y2=y2, aux2=aux2)
        elif cfg.src is not None and ACT[cfg.act] == 2 and y2 is None and res is None and \
                cfg.bacc is not None and aux is not None and aux.numel() >= 4 * y.shape[-1]:
            # swish: only a depthwise consumer can fuse it (z recomputed from y, aux scale|shift)
            ctx.bnsrc = cfg.src = _BNSrc(y, None, aux, cfg.bacc, act=2)
        elif cfg.src is not None and ACT[cfg.act] == 0 and y2 is None and _FUSE_BN_NOACT and \
                cfg.bacc is not None and y.shape[-1] % 8 == 0 and not _DETERMINISTIC:
            # no activation: the consumer dgrad reduces dz = dout under an all-ones mask
            ctx.bnsrc = cfg.src = _BNSrc(y, _ones_mask(y.numel(), y.device), aux, cfg.bacc)
        else:
            cfg.src = None
        return out

    @staticmethod
    def backward(ctx, dout):
        C = _C()
        y, out, mask, aux, y2, aux2 = ctx.saved_tensors
        cfg = ctx.cfg
        bn, bn2 = cfg.bn, cfg.bn2
        dout = _rows_view(dout)        # (a concat slab's gradient slice stays a strided view)

        def acc(p):
            if p is None or not p.requires_grad or not p.is_leaf:
                return None
            return G.grad_buffer(p)

        g1, b1 = acc(bn.weight), acc(bn.bias)
        g2 = b2 = None
        if bn2 is not None:
            g2, b2 = acc(bn2.weight), acc(bn2.bias)
        part = None
        src = ctx.bnsrc
        acc = cfg.bacc if (cfg.training or bn.running_mean is None) else None
        if src is not None:
            if src.part is not None and src.dx is not None and dout.data_ptr() == src.dx.data_ptr() \
                    and dout.shape == src.dx.shape:
                part = src.part           # reduced by the consumer conv's dgrad epilogue
            src.part = src.dx = None
            ctx.bnsrc = None
        filled = False
        zeros = [None, None]
        if acc is not None:
            if part is not None and part.data_ptr() == acc.buf.data_ptr():
                filled = True             # the dgrad epilogue added into the accumulator
            else:
                acc.ensure_clean()        # filled by a dgrad whose output is not dout: discard
            part = None
            # unfilled: tensors up to bn_acc_max_elems() are reduced into the accumulator by a
            # separate pass (then consumed: "used"), larger ones take the slab path and leave it
            # untouched ("clean": no memset before the next forward)
            if filled or y.numel() <= _acc_max_elems():
                acc.state = "used"
            else:
                acc.state = "clean"
            # the forward accumulators this BN consumed are cleared by the backward kernel
            for i, fa in enumerate(cfg.faccs):
                if fa.state == "used":
                    zeros[i] = fa.buf
                    fa.state = "clean"
            cfg.faccs = ()
        # dense-block slab input: the slab's gradient of y (deposited by the append that also read
        # y) is the destination, and this backward adds into it (no autograd sum of the two)
        dgx = cfg.dslot.take() if cfg.dslot is not None else None
        if dgx is not None:
            dgx = _rows_view(dgx)
        dbias = None
        rec = cfg.brec
        if rec is not None and rec.armed and cfg.training and ctx.needs_input_grad[0]:
            cb = rec.bias
            if cb.requires_grad and cb.is_leaf:
                dbias = G.grad_buffer(cb)
        dy, dres, dy2, dg, db, dg2, db2 = C.bn_backward(
            dout, out, mask, y, aux,
            bn.weight.detach() if bn.weight is not None else None,
            y2, aux2,
            bn2.weight.detach() if (bn2 is not None and bn2.weight is not None) else None,
            ACT[cfg.act], cfg.training or bn.running_mean is None, ctx.has_res, g1, b1, g2, b2, part,
            acc.buf if acc is not None else None, acc.R if acc is not None else 0, filled,
            zeros[0], zeros[1], dgx, dgx is not None, dbias)
        if dbias is not None:
            rec.done = True
            G.fire(rec.bias)
        ps = cfg.padslot
        if ps is not None and dy is not None and not dy.is_contiguous() and dy.dim() == 4:
            # dY written into zero-padded rows (the binding's pad_dy): the producer conv takes
            # the whole padded tensor
            n, h, w, _ = dy.shape
            ld = dy.stride(2)
            ps.base = dy.as_strided((n, h, w, ld), (h * w * ld, w * ld, ld, 1))
            ps.dy = dy
        ret = {}

        def deliver(p, buf, val, slot):
            if p is None or not p.requires_grad:
                return
            if not p.is_leaf:          # replicated / functional parameter: hand to autograd
                ret[slot] = val
            elif buf is not None:
                G.fire(p)
            else:
                G.accumulate(p, val)

        deliver(bn.weight, g1, dg, 1)
        deliver(bn.bias, b1, db, 2)
        if bn2 is not None:
            deliver(bn2.weight, g2, dg2, 5)
            deliver(bn2.bias, b2, db2, 6)
        if ctx.has_res and ctx.slot is not None and ctx.slot.offer(dres):
            dres = None                      # summed into the block input's dX by its owner conv
        return (dy, ret.get(1), ret.get(2), dres if ctx.has_res else None,
                dy2 if y2 is not None else None, ret.get(5), ret.get(6), None, None, None, None)


def _ref_bn(bn, x, training):
    return F.batch_norm(x, bn.running_mean, bn.running_var, bn.weight, bn.bias,
                        training or bn.running_mean is None,
                        bn.momentum if bn.momentum is not None else 0.1, bn.eps)


def _ref_act(x, act):
    if act in (None, "none"):
        return x
    if act == "relu":
        return F.relu(x)
    if act in ("swish", "silu"):
        return x * torch.sigmoid(x)
    if act == "sigmoid":
        return torch.sigmoid(x)
    raise ValueError(act)


def _bn_input(x):
    """NHWC view of a BatchNorm input: a dense-block slab suffix stays a row-strided view
    (the BN kernels take the row stride), anything else as ``to_nhwc``."""
    v = x.permute(0, 2, 3, 1)
    if not v.is_contiguous() and getattr(x, "_pca_dense_slot", None) is not None:
        r = _rows_view(v)
        if r is v:
            return v
    if not v.is_contiguous() and getattr(x, "_pca_padslot", None) is not None:
        return v           # (a zero-padded conv's output prefix: the BN kernels take its rows)
    return to_nhwc(x)


def batch_norm_act(bn, x, act=None, residual=None, residual_bn=None, stats=None, out=None):
    """act(BN(x) [+ residual] [+ BN_b(x_b)]) — the fused block tail of the model zoo.

    ``residual_bn=(bn_b, x_b, stats_b)`` fuses a projection-shortcut BatchNorm into the same pass
    (resnet.py:47-51 with the 1x1 conv shortcut of resnet.py:31-36).
    ``out``: a :class:`ChannelSlab` destination (``slab.dest(i)``) the result is written into
    (zero-copy concatenation); ignored on the CPU reference path.
    """
    training = bn.training
    if bn.training and bn.track_running_stats and bn.num_batches_tracked is not None and _ref(x):
        bn.num_batches_tracked.add_(1)
        if residual_bn is not None and residual_bn[0].num_batches_tracked is not None:
            residual_bn[0].num_batches_tracked.add_(1)
    if _ref(x):
        out = _ref_bn(bn, x, training)
        if residual is not None:
            out = out + residual
        if residual_bn is not None:
            out = out + _ref_bn(residual_bn[0], residual_bn[1], residual_bn[0].training)
        return _ref_act(out, act)
    if ACT[act] >= 2 and (residual is not None or residual_bn is not None):
        # swish/sigmoid backward recomputes z from y alone: keep the residual out of the fusion
        out = batch_norm_act(bn, x, None, residual, residual_bn, stats)
        return activation(out, act)
    N, Cc, H, W = x.shape
    y = _bn_input(x)
    res = to_nhwc(residual) if residual is not None else None
    y2 = st2 = bn2 = None
    if residual_bn is not None:
        bn2, xb = residual_bn[0], residual_bn[1]
        st2 = residual_bn[2] if len(residual_bn) > 2 else None
        y2 = to_nhwc(xb)
    cfg = _BNCfg(bn, bn2, act, training, N * H * W)
    if out is not None:
        cfg.dest = out
    cfg.dslot = getattr(x, "_pca_dense_slot", None)
    cfg.padslot = getattr(x, "_pca_padslot", None) if not y.is_contiguous() else None
    if training and residual is None and residual_bn is None and getattr(x, "_pca_bias_sole", False):
        cfg.brec = getattr(x, "_pca_bias_rec", None)
    if cfg.dslot is not None and torch.is_grad_enabled():
        cfg.dslot.claimed = True
    if training and bn.running_mean is not None:
        # the producing MFMA conv(s) subtract this BN's pilot mean from their sums from now on
        p1 = getattr(x, "_pca_stats_src", None)
        if p1 is not None:
            cfg.pilot = link_pilot(p1, Cc, y.device)
        if bn2 is not None and bn2.running_mean is not None:
            p2 = getattr(residual_bn[1], "_pca_stats_src", None)
            if p2 is not None:
                cfg.pilot2 = link_pilot(p2, Cc, y.device)
    if _FUSE_BN_BWD and torch.is_grad_enabled() and training:
        cfg.src = True                # request: forward replaces it with the _BNSrc record
    if (stats is None and training and residual is None and bn2 is None
            and bn.running_mean is not None and act in ("relu", None)):
        ds = getattr(x, "_pca_dense_stats", None)
        if ds is not None and ds.C == Cc and _bn_fusable(Cc, act, False, False, bn):
            stats = ds                # the dense slab's cached sums of this suffix
    if training and acc_enabled(Cc, y.device) and \
            _bn_fusable(Cc, act, residual is not None, bn2 is not None, bn, bn2):
        # (also without grad: the forward kernel then just keeps it clear)
        cfg.bacc = stat_acc(bn, "bwd", Cc, 3 if bn2 is not None else 2, y.device)
        # no producing conv delivered statistics (depthwise / concat / pooled inputs): a
        # separate statistics pass adds them into this BN's own accumulator (small tensors), so
        # the fused finalize+apply kernel still serves it
        if _BN_OWN_STATS:
            stats = _own_stats(bn, "fwdstat", y, stats)
            if bn2 is not None:
                st2 = _own_stats(bn2, "fwdstat", y2, st2)
        # the producing conv(s) may deliver their statistics through accumulators from now on
        p1 = getattr(x, "_pca_stats_src", None)
        p2 = getattr(residual_bn[1], "_pca_stats_src", None) if residual_bn is not None else None
        if p1 is not None and (bn2 is None or p2 is not None):
            p1._pca_acc_ok = True
            if p2 is not None:
                p2._pca_acc_ok = True
    out = _BatchNormAct.apply(y, bn.weight, bn.bias, res, y2,
                              bn2.weight if bn2 is not None else None,
                              bn2.bias if bn2 is not None else None, stats, st2, cfg,
                              _slot_for_residual(residual))
    v = to_nchw(out)
    if cfg.src is not None:
        v._pca_bnsrc = cfg.src        # the consumer conv fuses this BN's backward reduce
    return v


# ------------------------------------------- BN(+act) applied inside the depthwise consumer
# act(BN(y)) -> depthwise conv as ONE node (mobilenetv2.py:31-35 conv1 -> bn1 -> relu -> conv2,
# efficientnet.py:96-98 with swish, mobilenet.py's pointwise BN -> next block's depthwise): the
# BN's batch statistics are folded by one small finalize launch, and its affine + activation are
# applied on the depthwise kernels' input loads (csrc/dwconv.hip "input transform") — in the
# forward and again in the weight gradient — so the BN output is never written, and read back by
# neither. The backward recomputes the activation derivative from y (ACT_RELU_Y / swish from the
# aux scale | shift) instead of a stored mask, reduces the BN-backward sums of the depthwise
# dgrad's output and applies them in one pass (whose finalize also clears the forward
# accumulator the BN consumed). Opt-in (PCA_DW_IN_FUSE=1): measured slower than the separate BN
# apply pass + plain depthwise (MobileNetV2 bs1024 15.40 vs 14.14 ms, EfficientNet-B0 bs128 4.19
# vs 3.98 ms; README "round 4") - the transform's per-load scale/shift/act costs the depthwise
# kernels more VALU time than the apply pass's HBM round trip.
_DW_IN_FUSE = os.environ.get("PCA_DW_IN_FUSE", "0") == "1"
_ACT_RELU_Y = 4


class _BNActDW(torch.autograd.Function):
    @staticmethod
    def forward(ctx, y, gamma, beta, weight, stats, cfg, stride, padding):
        C = _C()
        bn = cfg.bn
        aux = _bn_aux(C, bn, y, stats, cfg.training, cfg.count, cfg.pilot)
        cfg.faccs = (stats,) if isinstance(stats, StatAcc) else ()
        KH, KW = weight.shape[2], weight.shape[3]
        wT = _dw_weight(weight)
        out = C.dw_fwd_in(y, wT, KH, KW, stride, padding, aux, ACT[cfg.act])
        ctx.save_for_backward(y, wT, aux)
        ctx.cfg = cfg
        ctx.geom = (stride, padding, KH, KW)
        ctx.weight = weight
        return out

    @staticmethod
    def backward(ctx, dout):
        C = _C()
        y, wT, aux = ctx.saved_tensors
        cfg, bn = ctx.cfg, ctx.cfg.bn
        stride, padding, KH, KW = ctx.geom
        dout = dout.contiguous()
        H, W, Cx = y.shape[1], y.shape[2], y.shape[3]
        act = ACT[cfg.act]
        w = ctx.weight
        dw_ret = None
        if w.requires_grad:
            buf = G.grad_buffer(w) if w.is_leaf else None
            if buf is not None and buf.is_contiguous():
                C.dw_wgrad_in(y, dout, KH, KW, stride, padding, aux, act, buf.view(-1))
                G.fire(w)
            else:
                dwt = C.dw_wgrad_in(y, dout, KH, KW, stride, padding, aux, act)
                if w.is_leaf:
                    G.accumulate(w, dwt.view(w.shape[0], KH, KW, 1))
                else:
                    dw_ret = dwt.view(w.shape)
        # gradient w.r.t. act(BN(y)), then the BN(+act) backward with the derivative from y
        dz = C.dw_dgrad(dout, wT, H, W, Cx, KH, KW, stride, padding)

        def acc(p):
            if p is None or not p.requires_grad or not p.is_leaf:
                return None
            return G.grad_buffer(p)

        g1, b1 = acc(bn.weight), acc(bn.bias)
        zero1 = None
        for fa in cfg.faccs:
            if fa.state == "used":
                zero1 = fa.buf            # cleared by the backward finalize's block 0
                fa.state = "clean"
        cfg.faccs = ()
        dy, _, _, dg, db, _, _ = C.bn_backward(
            dz, None, None, y, aux, bn.weight.detach() if bn.weight is not None else None,
            None, None, None, _ACT_RELU_Y if act == 1 else act,
            cfg.training or bn.running_mean is None, False, g1, b1, None, None, None, None, 0,
            False, zero1, None)
        ret = {}
        for p, buf, val, slot in ((bn.weight, g1, dg, 1), (bn.bias, b1, db, 2)):
            if p is None or not p.requires_grad:
                continue
            if not p.is_leaf:
                ret[slot] = val
            elif buf is not None:
                G.fire(p)
            else:
                G.accumulate(p, val)
        return dy, ret.get(1), ret.get(2), dw_ret, None, None, None, None


def bn_act_dwconv(bn, x, act, conv):
    """``conv(act(bn(x)))`` for a depthwise ``conv`` (groups == channels, multiplier 1, no bias):
    one fused node on the GPU (BN applied on the depthwise kernels' loads), the plain composition
    elsewhere (CPU reference path, unsupported geometry / activation, PCA_DW_IN_FUSE unset)."""
    Cc = x.shape[1]
    ks, st, pd = conv.kernel_size, conv.stride, conv.padding
    simple = (conv.groups == Cc and conv.out_channels == Cc and conv.bias is None
              and ks[0] == ks[1] and st[0] == st[1] and pd[0] == pd[1])
    if (not _DW_IN_FUSE or _ref(x) or not simple or act not in ("relu", "swish", "silu")
            or bn.running_mean is None or torch.is_autocast_enabled() or Cc % 8
            or not _C().dw_in_supported(to_nhwc(x), Cc, ks[0], ks[1], st[0], pd[0], ACT[act])):
        return conv(bn(x, act=act))
    training = bn.training
    stats = getattr(x, "_pca_stats", None) if training else None
    y = to_nhwc(x)
    N, _, H, W = x.shape
    cfg = _BNCfg(bn, None, act, training, N * H * W)
    if training:
        p1 = getattr(x, "_pca_stats_src", None)
        if p1 is not None:
            cfg.pilot = link_pilot(p1, Cc, y.device)
            if acc_enabled(Cc, y.device):
                p1._pca_acc_ok = True     # the producer delivers into its accumulator from now on
    out = _BNActDW.apply(y, bn.weight, bn.bias, conv.weight, stats, cfg, st[0], pd[0])
    v = to_nchw(out)
    if training:
        v._pca_stats_src = conv
    return v


# ------------------------------------------- BN+ReLU applied inside the consumer 3x3 conv
# conv2(relu(bn1(y1))) of a ResNet BasicBlock (reference models/resnet.py:47: the mid-block BN
# whose output only conv2 reads) as ONE node: the BN's batch statistics are folded by one small
# finalize launch, and relu(y1 * scale + shift) is applied by the consumer itself — the layer-1
# c64 forward transforms each halo piece in LDS as it lands and writes the ReLU mask of its tile
# interiors (csrc/conv3x3_c64.hip XF), the halo weight gradient transforms its X stages the same
# way (conv_halo.hip XF). The BN output x1 is never written and never read back: the apply pass
# (read y1, write x1 + mask: ~276 MB at bs1024) is gone. The backward is the unfused one: the c64
# dgrad reduces the BN-backward sums from y1 + mask in its epilogue, one fused finalize+apply
# pass produces dy1. Bitwise the unfused forward (same arithmetic, same kernels otherwise).
# PCA_BN_CONV_FUSE=0: separate BN apply pass + plain conv (A/B).
_BN_CONV_FUSE = os.environ.get("PCA_BN_CONV_FUSE", "0") == "1"
_BN_CONV_USED = [0]   # fused nodes built (tests check the fused path ran)


class _BNActConv(torch.autograd.Function):
    @staticmethod
    def forward(ctx, y, gamma, beta, weight, stats, cfg, acc2, pilot2):
        C = _C()
        bn = cfg.bn
        aux = _bn_aux(C, bn, y, stats, cfg.training, cfg.count, cfg.pilot, zero=cfg.bacc)
        cfg.faccs = (stats,) if isinstance(stats, StatAcc) else ()
        w_phys = G.physical(weight)
        if not w_phys.is_contiguous():
            w_phys = w_phys.contiguous()
        wb, wt = _prepped_weight(weight, 1, w_phys, True)
        mask = torch.empty((y.numel() + 7) // 8, dtype=torch.uint8, device=y.device)
        if acc2 is not None:
            acc2.begin()
            y2, _ = C.conv_fwd(y, wb, None, 1, 1, 1, True, acc2.buf, acc2.R, pilot2, xf=aux,
                               xf_mask=mask)
            acc2.shifted = pilot2 is not None
            stats2 = None
        else:
            y2, stats2 = C.conv_fwd(y, wb, None, 1, 1, 1, True, None, 0, pilot2, xf=aux,
                                    xf_mask=mask)
            if pilot2 is not None and stats2.numel():
                stats2._pca_kin = pilot2.clone()   # (as _ConvMFMA: the K these sums are of)
        ctx.save_for_backward(y, wt, mask, aux)
        ctx.cfg = cfg
        ctx.weight = weight
        if stats2 is None:
            stats2 = torch.empty(0, device=y.device)
        ctx.mark_non_differentiable(stats2)
        ctx.set_materialize_grads(False)
        return y2, stats2

    @staticmethod
    def backward(ctx, dy2, _dstats):
        if dy2 is None:
            return (None,) * 8
        C = _C()
        y, wt, mask, aux = ctx.saved_tensors
        cfg, bn = ctx.cfg, ctx.cfg.bn
        dy2 = dy2.contiguous()
        H, W = y.shape[1], y.shape[2]
        # dX1 with the BN-backward sums reduced in the dgrad epilogue (into the BN's accumulator)
        src = _BNSrc(y, mask, aux, cfg.bacc)
        dx1 = _dgrad_bn(C, src, dy2, wt, H, W, 1, 1, 1, None)
        # dW2 from relu(BN(y1)) applied on the halo wgrad's X loads
        w = ctx.weight
        dw_ret = None
        if w.requires_grad:
            buf = G.grad_buffer(w) if w.is_leaf else None
            if buf is not None:
                piggy = _WGRAD_PIGGY and not _WGRAD_DEFER
                if _piggy_set[0] != piggy:
                    C.wgrad_piggy(piggy)
                    _piggy_set[0] = piggy
                C.conv_wgrad(y, dy2, 3, 3, 1, 1, 1, buf, defer=_WGRAD_DEFER or piggy, xf=aux)
                if (_WGRAD_DEFER or piggy) and C.wgrad_deferred():
                    _after_deferred_wgrad()
                G.fire(w)
            else:
                dw = C.conv_wgrad(y, dy2, 3, 3, 1, 1, 1, None, xf=aux)
                if w.is_leaf:
                    G.accumulate(w, dw)
                else:
                    dw_ret = dw.permute(0, 3, 1, 2)

        def gbuf(p):
            if p is None or not p.requires_grad or not p.is_leaf:
                return None
            return G.grad_buffer(p)

        g1, b1 = gbuf(bn.weight), gbuf(bn.bias)
        acc = cfg.bacc if (cfg.training or bn.running_mean is None) else None
        part = src.part if (src.part is not None and src.dx is dx1) else None
        filled = False
        zero1 = None
        if acc is not None:
            filled = part is not None and part.data_ptr() == acc.buf.data_ptr()
            if not filled:
                acc.ensure_clean()
            part = None
            acc.state = "used" if (filled or y.numel() <= _acc_max_elems()) else "clean"
            for fa in cfg.faccs:
                if fa.state == "used":
                    zero1 = fa.buf          # cleared by the backward kernel's block 0
                    fa.state = "clean"
            cfg.faccs = ()
        src.part = src.dx = None
        dy, _, _, dg, db, _, _ = C.bn_backward(
            dx1, None, mask, y, aux, bn.weight.detach() if bn.weight is not None else None,
            None, None, None, ACT["relu"], cfg.training or bn.running_mean is None, False, g1, b1,
            None, None, part, acc.buf if acc is not None else None, acc.R if acc is not None else 0,
            filled, zero1, None, None, False, None)
        ret = {}
        for p, buf, val, slot in ((bn.weight, g1, dg, 1), (bn.bias, b1, db, 2)):
            if p is None or not p.requires_grad:
                continue
            if not p.is_leaf:
                ret[slot] = val
            elif buf is not None:
                G.fire(p)
            else:
                G.accumulate(p, val)
        return dy, ret.get(1), ret.get(2), dw_ret, None, None, None, None


def bn_act_conv(bn, x, act, conv):
    """``conv(act(bn(x)))`` for a 3x3 / stride-1 conv whose input only this BN+ReLU produces:
    one fused node where the consumer applies the BN on its loads (layer-1 c64 geometry, training
    mode), the plain composition elsewhere. Returns what ``conv`` returns (statistics attached)."""
    from ..nn.modules import _STATS_ATTR

    Cc = x.shape[1]
    ks, st, pd = conv.kernel_size, conv.stride, conv.padding
    training = bn.training
    if (not _BN_CONV_FUSE or _ref(x) or not training or act != "relu" or bn.running_mean is None
            or not conv.training or conv.bias is not None or conv.groups != 1
            or ks != (3, 3) or st != (1, 1) or pd != (1, 1) or conv.in_channels != Cc
            or torch.is_autocast_enabled() or x.dim() != 4 or x.dtype != COMPUTE_DTYPE
            or not acc_enabled(Cc, x.device)):
        return conv(bn(x, act=act))
    stats = getattr(x, _STATS_ATTR, None)
    p1 = getattr(x, "_pca_stats_src", None)
    y = to_nhwc(x)
    if not (isinstance(stats, StatAcc) and p1 is not None and y.is_contiguous()
            and _C().conv_xf_supported(y, G.physical(conv.weight), 1, 1, 1)):
        return conv(bn(x, act=act))
    N, _, H, W = x.shape
    cfg = _BNCfg(bn, None, act, training, N * H * W)
    cfg.pilot = link_pilot(p1, Cc, y.device)
    cfg.bacc = stat_acc(bn, "bwd", Cc, 2, y.device)
    acc2 = None
    if conv.__dict__.get("_pca_acc_ok") and acc_enabled(conv.out_channels, y.device):
        acc2 = stat_acc(conv, "fwd", conv.out_channels, 2, y.device)
    pilot2 = conv_pilot(conv, y.device)
    _BN_CONV_USED[0] += 1
    out, stats2 = _BNActConv.apply(y, bn.weight, bn.bias, conv.weight, stats, cfg, acc2, pilot2)
    v = to_nchw(out)
    setattr(v, _STATS_ATTR, acc2 if acc2 is not None else stats2)
    v._pca_stats_src = conv
    return v


# ------------------------------------------------------------------------ activations
class _Act(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, act):
        ctx.act = act
        ctx.save_for_backward(x)
        return _C().act_fwd(x, act)

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        return _C().act_bwd(dy.contiguous(), x, ctx.act), None


def activation(x, act):
    if act in (None, "none"):
        return x
    if _ref(x) or x.dim() != 4:  # classifier-head [N, F] activations: tiny, library elementwise
        return _ref_act(x, act)
    return to_nchw(_Act.apply(to_nhwc(x), ACT[act]))


def relu(x):
    return activation(x, "relu")


class _AddAct(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, b, act):
        y = _C().add_act(a, b, act)
        ctx.act = act
        ctx.save_for_backward(y if act == 1 else None)
        return y

    @staticmethod
    def backward(ctx, dy):
        dy = dy.contiguous()
        if ctx.act == 0:
            return dy, dy, None
        (y,) = ctx.saved_tensors
        d = _C().act_bwd(dy, y, 1)
        return d, d, None


def add_act(a, b, act=None):
    """act(a + b) — the un-fused residual join (PNASNet cells, DPN, ShuffleNet)."""
    if _ref(a):
        return _ref_act(a + b, act)
    if ACT[act] not in (0, 1):
        return activation(add_act(a, b, None), act)
    return to_nchw(_AddAct.apply(to_nhwc(a), to_nhwc(b), ACT[act]))


class _DPNMerge(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, o, d, slot=None):
        y = _C().dpn_merge_fwd(x, o, d)
        ctx.save_for_backward(y)
        ctx.geom = (x.shape[-1], o.shape[-1], d)
        ctx.slot = slot
        return y

    @staticmethod
    def backward(ctx, dy):
        (y,) = ctx.saved_tensors
        dx, do = _C().dpn_merge_bwd(dy.contiguous(), y, *ctx.geom)
        if ctx.slot is not None and ctx.slot.offer(dx):
            dx = None        # the block input's conv1 dgrad adds it in its epilogue
        return dx, do, None, None


def dpn_merge(x, out, d):
    """DPN dual-path join relu(cat[x[:, :d] + out[:, :d], x[:, d:], out[:, d:]]) (dpn.py:29-31)
    as one native pass each way (no channel-slice copies / separate add, ReLU and concat).
    With an identity shortcut ``x`` is the block input, also read by conv1: its gradient from
    the join is handed to conv1's dgrad epilogue (GradSlot) instead of an autograd add."""
    if _ref(x) or d % 8 or x.shape[1] % 8 or out.shape[1] % 8:
        return torch.cat([add_act(x[:, :d], out[:, :d], "relu"), relu(x[:, d:]), relu(out[:, d:])], 1)
    return to_nchw(_DPNMerge.apply(to_nhwc(x), to_nhwc(out), d, _slot_for_residual(x)))


# ---------------------------------------------------------------------------- pooling
class _GAP(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        ctx.hw = (x.shape[1], x.shape[2])
        return _C().gap_fwd(x)

    @staticmethod
    def backward(ctx, dy):
        return _C().gap_bwd(dy.contiguous().float(), *ctx.hw)


def global_avg_pool(x):
    """[N,C,H,W] -> fp32 [N,C,1,1] (head / SE squeeze)."""
    if _ref(x):
        return F.adaptive_avg_pool2d(x, 1)
    return _GAP.apply(to_nhwc(x)).view(x.shape[0], x.shape[1], 1, 1)


# PCA_HEAD_BN_FUSE_BIG=1: the head backward adds the block-tail BN's backward sums at every batch
# size (the kernel then groups ceil(N / 64R) samples per block). Off by default: at bs1024 it does
# not beat the separate reduce + finalize + apply (same box 6.50-6.52 vs 6.48-6.51 ms,
# profiles/bench/r6b/ab_head_bn_fuse_big.log); the fused form is used while N / R <= 64
_HEAD_BN_FUSE_BIG = os.environ.get("PCA_HEAD_BN_FUSE_BIG", "0") == "1"


class _PoolLinear(torch.autograd.Function):
    """Global average pool [+ dropout] + Linear in one kernel each way (csrc/misc.hip head_*)."""

    @staticmethod
    def forward(ctx, x, weight, bias, p=0.0, rng=None, bnsrc=None):
        logits, pooled, dmask = _C().head_fwd(x, weight, bias, p, rng)
        ctx.save_for_backward(weight, pooled, dmask if p > 0 else None)
        ctx.hw = (x.shape[1], x.shape[2])
        ctx.params = (weight, bias)
        ctx.p = p
        # the producing BN+ReLU (block tail): its backward sums are added by the head backward
        C = x.shape[-1]
        # (sample blocks add into the R shard rows; the kernel gives each block enough samples to
        # keep <= 64 blocks per shard row — one block per sample at bs1024 ran the head 20 -> 74 us
        # on same-address atomics)
        ok = (bnsrc is not None and bnsrc.act == 1 and bnsrc.mask is not None and bnsrc.y2 is None
              and bnsrc.acc is not None and C % 8 == 0 and 256 % (C // 8) == 0
              and bnsrc.y.is_contiguous()
              and (_HEAD_BN_FUSE_BIG or x.shape[0] <= 64 * bnsrc.acc.R))
        ctx.bnsrc = bnsrc if ok else None
        return logits

    @staticmethod
    def backward(ctx, dl):
        weight, pooled, dmask = ctx.saved_tensors
        w, b = ctx.params
        ctx.params = None
        wbuf = G.grad_buffer(w) if (w.requires_grad and w.is_leaf) else None
        bbuf = G.grad_buffer(b) if (b is not None and b.requires_grad and b.is_leaf) else None
        src = ctx.bnsrc
        ctx.bnsrc = None
        if src is not None:
            src.acc.begin()
            dx, dw, db = _C().head_bwd(dl.float().contiguous(), weight, pooled, ctx.hw[0],
                                       ctx.hw[1], wbuf, bbuf, b is not None, ctx.p, dmask,
                                       src.y, src.mask, src.aux, src.acc.buf, src.acc.R)
            src.part, src.dx = src.acc.buf, dx   # the BN backward finds its sums filled
        else:
            dx, dw, db = _C().head_bwd(dl.float().contiguous(), weight, pooled, ctx.hw[0],
                                       ctx.hw[1], wbuf, bbuf, b is not None, ctx.p, dmask)
        dw_ret = db_ret = None
        if w.requires_grad:
            if wbuf is not None:
                G.fire(w)
            elif w.is_leaf:
                G.accumulate(w, dw)
            else:
                dw_ret = dw
        if b is not None and b.requires_grad:
            if bbuf is not None:
                G.fire(b)
            elif b.is_leaf:
                G.accumulate(b, db)
            else:
                db_ret = db
        return dx, dw_ret, db_ret, None, None, None


def rng_state(owner, device):
    """The persistent Philox state int64[3] {seed, step, tickets} of ``owner``'s dropout on
    ``device`` (kept in the module ``__dict__``: not a buffer, so state_dict keys stay the
    reference's). The kernels advance ``step`` themselves — eager and hipGraph replay alike."""
    d = owner.__dict__.setdefault("_pca_rng", {})
    key = device.index if device.index is not None else torch.cuda.current_device()
    t = d.get(key)
    if t is None:
        # seeded from torch's seed (torch.manual_seed reproduces it) and the creation order
        _RNG_SEQ[0] += 1
        seed = (torch.initial_seed() * 0x9E3779B97F4A7C15 + _RNG_SEQ[0] * 0xBF58476D1CE4E5B9) % (1 << 62)
        t = d[key] = torch.tensor([seed, 0, 0], dtype=torch.int64, device=device)
    return t


_RNG_SEQ = [0]


class _OrphanRng:
    """Holder of the Philox states of dropout / drop-connect calls made without an owner module
    (one process-wide object: those calls share it, and :func:`rng_states` always reports it, so
    a training-step snapshot covers them too)."""


_ORPHAN_RNG = _OrphanRng()


def rng_states(model):
    """Every dropout rng state tensor attached to ``model``'s modules (training-step state), plus
    the owner-less calls' states."""
    out = []
    for m in model.modules():
        out += list(m.__dict__.get("_pca_rng", {}).values())
    out += list(_ORPHAN_RNG.__dict__.get("_pca_rng", {}).values())
    return out


def pool_linear(x, kernel_size, linear, dropout_p=0.0, training=False):
    """``linear(dropout(avg_pool2d(x, kernel_size).flatten(1)))`` — the classifier head of the zoo
    (dropout only where the reference has it: efficientnet.py:147-149, p = 0.2 in training).

    ``kernel_size=None`` means a global (adaptive 1x1) pool. When the pool is global and the
    shapes allow (C % 8 == 0, <= 16 classes, fp32 weights), the pool, the dropout (Philox, keep
    mask kept as bytes for the backward) and the Linear run as one fused kernel forward and one
    backward (its weight gradient is added with fp32 atomics); otherwise (CPU reference path,
    non-global pools, deterministic mode) it is exactly the unfused composition.
    """
    N, C, H, W = x.shape
    glob = kernel_size is None or (_pair1(kernel_size) == H == W)
    w, b = linear.weight, linear.bias
    p = float(dropout_p) if training else 0.0
    if (_ref(x) or not glob or w.dtype != torch.float32 or torch.is_autocast_enabled()
            or not _C().head_supported(N, C, w.shape[0]) or _C().deterministic()):
        out = adaptive_avg_pool2d(x, 1) if kernel_size is None else avg_pool2d(x, kernel_size)
        out = out.reshape(N, -1)
        if p > 0:
            out = dropout(out, p, True, owner=linear)
        return linear(out)
    rng = rng_state(linear, x.device) if p > 0 else None
    src = getattr(x, "_pca_bnsrc", None) if torch.is_grad_enabled() else None
    return _PoolLinear.apply(to_nhwc(x), w, b, p, rng, src)


class _AvgPool(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, s, p):
        ctx.cfg = (x.shape[1], x.shape[2], k, s, p)
        return _C().avgpool_fwd(x, k, s, p)

    @staticmethod
    def backward(ctx, dy):
        H, W, k, s, p = ctx.cfg
        return _C().avgpool_bwd(dy.contiguous(), H, W, k, s, p), None, None, None


class _MaxPool(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, s, p, slot=None):
        y, arg = _C().maxpool_fwd(x, k, s, p)
        ctx.cfg = (x.shape[1], x.shape[2], k, s, p)
        ctx.slot = slot
        ctx.save_for_backward(arg)
        ctx.mark_non_differentiable(arg)
        return y

    @staticmethod
    def backward(ctx, dy):
        (arg,) = ctx.saved_tensors
        H, W, k, s, p = ctx.cfg
        dx = _C().maxpool_bwd(dy.contiguous(), arg, H, W, k, s, p)
        if ctx.slot is not None and ctx.slot.offer(dx):
            # (GoogLeNet's Inception pool branch, googlenet.py:41-45: its input gradient joins the
            # sibling convs' dgrad epilogues instead of an autograd add)
            dx = None
        return dx, None, None, None, None


def _pair1(v):
    if isinstance(v, (tuple, list)):
        assert v[0] == v[1], "only square pooling windows"
        return v[0]
    return v


def avg_pool2d(x, kernel_size, stride=None, padding=0):
    k = _pair1(kernel_size)
    s = _pair1(stride) if stride is not None else k
    p = _pair1(padding)
    if _ref(x):
        return F.avg_pool2d(x, k, s, p)
    H, W = x.shape[2], x.shape[3]
    if k == 1 and s == 1 and p == 0:
        return x           # (vgg.py:33's AvgPool2d(1, 1): identity, no pass — also on a 1x1 map)
    if p == 0 and k == H and k == W:
        return global_avg_pool(x)
    return to_nchw(_AvgPool.apply(to_nhwc(x), k, s, p))


def max_pool2d(x, kernel_size, stride=None, padding=0):
    k = _pair1(kernel_size)
    s = _pair1(stride) if stride is not None else k
    p = _pair1(padding)
    if _ref(x):
        return F.max_pool2d(x, k, s, p)
    return to_nchw(_MaxPool.apply(to_nhwc(x), k, s, p, _slot_for_residual(x)))


def adaptive_avg_pool2d(x, output_size):
    o = _pair1(output_size)
    assert o == 1, "only global adaptive pooling is used by the zoo"
    return global_avg_pool(x)


# ------------------------------------------------------------------------ squeeze-excite
class _SEScale(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, s):
        ctx.save_for_backward(x, s)
        return _C().se_scale_fwd(x, s)

    @staticmethod
    def backward(ctx, dy):
        x, s = ctx.saved_tensors
        dx, ds = _C().se_scale_bwd(dy.contiguous(), x, s)
        return dx, ds


def se_excite(x, s_logits):
    """x * sigmoid(s) with s = per-(n, c) excitation logits [N, C] (fp32)."""
    if _ref(x):
        return x * torch.sigmoid(s_logits).view(x.shape[0], x.shape[1], 1, 1)
    s = s_logits.reshape(x.shape[0], x.shape[1]).float().contiguous()
    return to_nchw(_SEScale.apply(to_nhwc(x), s))


# PCA_SE_FUSED=1: the fused squeeze-excite kernels — pool + both MLP layers in one launch (+ the
# scale: 2 forward launches), excitation reduce + MLP data path in one (+ parameters + dx: 3
# backward) — reading W2 transposed from the weight-prep plan. Off by default: even with the
# coalesced W2^T reads (fused backward at C 1152 / R 48: 65.7 -> 45.8 us per call) the per-sample
# blocks serialise pool -> MLP -> MLP latency, and the split kernels win the step, same box:
# EfficientNet-B0 bs128 3.865-3.867 vs 3.991-3.992 ms, bs1024 8.31 vs 9.12 ms
# (profiles/bench/r6b/ab_se_fused.log, tools/se_bench.py per shape: se_bench_r6.jsonl)
_SE_FUSED = os.environ.get("PCA_SE_FUSED", "0") == "1"


class _SqueezeExcite(torch.autograd.Function):
    """The whole squeeze-excite block on NHWC bf16 x (csrc/misc.hip se_*): 3 launches forward
    (pool, MLP, scale) and 4 backward (excitation reduce, MLP data, MLP parameters with fp32
    atomics into the gradient arena, combined dx) instead of the 5 + 10 of the library-GEMM
    composition."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2, act):
        # W2 transposed [R][C] for the fused kernels: the weight-prep plan's fp32 copy (refreshed
        # by its one batched launch per forward / by the fused SGD step), like a depthwise weight
        w2t = _dw_weight(w2) if _SE_FUSED else None
        out, pooled, hpre, s = _C().se_forward(x, w1, b1, w2, b2, act, w2t)
        ctx.w2t = w2t
        ctx.save_for_backward(x, pooled, hpre, s, w1, w2)
        ctx.act = act
        ctx.params = (w1, b1, w2, b2)
        return out

    @staticmethod
    def backward(ctx, dout):
        x, pooled, hpre, s, w1s, w2s = ctx.saved_tensors
        params = ctx.params
        ctx.params = None

        def buf(p):
            return G.grad_buffer(p) if (p is not None and p.requires_grad and p.is_leaf) else None

        bufs = [buf(p) for p in params]
        w2t, ctx.w2t = ctx.w2t, None
        dx, dw1, db1, dw2, db2 = _C().se_backward(
            dout.contiguous(), x, pooled, hpre, s, w1s, w2s, ctx.act,
            *[b.view(-1) if b is not None else None for b in bufs],
            params[1] is not None, params[3] is not None, w2t)
        ret = []
        for p, b, g in zip(params, bufs, (dw1, db1, dw2, db2)):
            r = None
            if p is not None and p.requires_grad:
                if b is not None:
                    G.fire(p)
                elif p.is_leaf:
                    G.accumulate(p, g.view(p.shape))
                else:
                    r = g.view(p.shape)
            ret.append(r)
        return (dx, *ret, None)


def squeeze_excite(x, w1, b1, w2, b2, act):
    """x * sigmoid(W2 act(W1 mean_hw(x) + b1) + b2) as one native block, or None when the
    shapes / mode need the composed path (CPU reference, deterministic mode: the parameter
    gradients are fp32 atomics)."""
    if (_ref(x) or act not in ("relu", "swish", "silu") or w1.dtype != torch.float32
            or w2.dtype != torch.float32 or torch.is_autocast_enabled()
            or _DETERMINISTIC or _C().deterministic()
            or not _C().se_supported(x.shape[1], w1.shape[0])):
        return None
    return to_nchw(_SqueezeExcite.apply(to_nhwc(x), w1, b1, w2, b2, ACT[act]))


# ------------------------------------------------------------------------ cross-entropy
_UNIT = {}


def unit_grad(loss: torch.Tensor) -> torch.Tensor:
    """A persistent ones tensor shaped like ``loss`` for ``loss.backward(unit_grad(loss))``.

    ``loss.backward()`` makes autograd launch a fill for the implicit 1.0 seed, and the CE
    backward then scales dlogits by it (a second launch). Seeding with this never-written tensor
    lets the CE backward recognise the unit seed by address and hand dlogits through as they are.
    """
    key = (loss.device, loss.dtype, tuple(loss.shape))
    t = _UNIT.get(key)
    if t is None:
        t = torch.ones(loss.shape, dtype=loss.dtype, device=loss.device)
        _UNIT[key] = t
    return t


def _is_unit(g: torch.Tensor) -> bool:
    t = _UNIT.get((g.device, g.dtype, tuple(g.shape)))
    return t is not None and t.data_ptr() == g.data_ptr()


class _CrossEntropy(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, target, metrics):
        loss, dl = _C().ce_fused(logits, target, metrics, True)
        ctx.save_for_backward(dl)
        return loss

    @staticmethod
    def backward(ctx, dloss):
        (dl,) = ctx.saved_tensors
        if _is_unit(dloss):
            return dl, None, None
        return _C().scale_by_scalar(dl, dloss.float().reshape(1).contiguous()), None, None


def cross_entropy(logits, target, metrics=None):
    """Mean CE; ``metrics`` (fp64 [3] on device) accumulates (loss, correct, count) with no sync."""
    if _ref(logits):
        loss = F.cross_entropy(logits.float(), target)
        if metrics is not None:
            with torch.no_grad():
                metrics[0] += loss.double()
                metrics[1] += (logits.argmax(1) == target).sum().double()
                metrics[2] += target.numel()
        return loss
    logits = logits.float().contiguous()
    from .. import _native

    if _native._debug:   # --debug_sync: name a bad label on the host (the kernel NaN-poisons it)
        bad = (target < 0) | (target >= logits.shape[1])
        if bool(bad.any()):
            i = int(bad.nonzero()[0, 0])
            raise IndexError(f"cross_entropy: target {int(target[i])} at position {i} is outside "
                             f"[0, {logits.shape[1]})")
    if torch.is_grad_enabled() and logits.requires_grad:
        return _CrossEntropy.apply(logits, target, metrics)
    loss, _ = _C().ce_fused(logits, target, metrics, False)
    return loss


class _Dropout(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, p, unit_len, rng):
        y, mask = _C().dropout_fwd(x, p, unit_len, rng)
        ctx.save_for_backward(mask)
        ctx.cfg = (p, unit_len)
        return y

    @staticmethod
    def backward(ctx, dy):
        (mask,) = ctx.saved_tensors
        p, unit_len = ctx.cfg
        return _C().dropout_bwd(dy.contiguous(), mask, p, unit_len), None, None, None


def _dropout_units(x, unit_len, p, owner):
    # NCHW-shaped channels_last activations are contiguous as NHWC: a per-sample unit is still a
    # contiguous run of C*H*W elements, an elementwise one ignores the layout
    flat = x.permute(0, 2, 3, 1) if (x.dim() == 4 and not x.is_contiguous()) else x
    if not flat.is_contiguous():
        flat = flat.contiguous()
    y = _Dropout.apply(flat, float(p), int(unit_len), rng_state(owner, x.device))
    return y.permute(0, 3, 1, 2) if flat is not x else y


def dropout(x, p, training, owner=None):
    """Training-mode dropout (efficientnet.py:147-149): Philox keep mask, 1/(1-p) scaling."""
    if not training or p == 0:
        return x
    if _ref(x):
        return F.dropout(x, p=p, training=True)
    return _dropout_units(x, 1, p, owner if owner is not None else _ORPHAN_RNG)


def drop_connect(x, drop_ratio, owner=None):
    """Per-sample drop-connect (efficientnet.py:16-22): the whole sample kept with probability
    1 - drop_ratio and scaled by 1/(1 - drop_ratio) — one keep byte per sample."""
    if drop_ratio <= 0:
        return x
    if _ref(x):
        keep = 1.0 - drop_ratio
        mask = torch.empty([x.shape[0], 1, 1, 1], dtype=x.dtype, device=x.device).bernoulli_(keep)
        return x / keep * mask
    return _dropout_units(x, x[0].numel(), drop_ratio, owner if owner is not None else _ORPHAN_RNG)


class Remap:
    """An injective channel remap ``out[q][j] = in[src(q)][cmap[j]]`` (-1 = zero) and its adjoint.

    ``cmap`` has J entries indexing the Cin input channels; ``rmap`` (optional) maps output rows
    to input rows of K-row blocks (conv weights [Cout][KH*KW][Cg], K = KH*KW). The adjoint of an
    injective remap is the remap with the inverse maps, so forward and backward are both one
    launch of ``chan_remap`` (csrc/misc.hip). Device maps are built once per (key, device) — before
    hipGraph capture, on the warm-up steps — and reused by every replay."""

    _cache = {}
    flat = False      # True: maps whole flattened tensors (one row of ``cin`` elements)

    def __init__(self, cmap, cin, rmap=None, rin=None, K=1):
        self.cmap, self.cin, self.rmap, self.rin, self.K = list(cmap), cin, rmap, rin, K
        inv = [-1] * cin
        for j, c in enumerate(self.cmap):
            if c >= 0:
                inv[c] = j
        self.icmap = inv
        self.irmap = None
        if rmap is not None:
            inv_r = [-1] * rin
            for r, s in enumerate(rmap):
                if s >= 0:
                    inv_r[s] = r
            self.irmap = inv_r
        self._dev = {}

    @classmethod
    def get(cls, key, build):
        m = cls._cache.get(key)
        if m is None:
            m = build()
            cls._cache[key] = m
        return m

    def maps(self, device):
        d = self._dev.get(device)
        if d is None:
            def t(v):
                return None if v is None else torch.tensor(v, dtype=torch.int32, device=device)
            d = (t(self.cmap), t(self.rmap), t(self.icmap), t(self.irmap))
            self._dev[device] = d
        return d

    def apply(self, x, inverse=False, acc=None, clear_src=False):
        """Remap the contiguous ``x`` (last dim = channels) -> flat [Q, J] (or add into ``acc``);
        ``clear_src`` zeroes the elements of ``x`` it read (fp32)."""
        cm, rm, icm, irm = self.maps(x.device)
        if inverse:
            cm, rm = icm, irm
        return _C().chan_remap(x, cm, rm, self.K, acc, clear_src)


class _RemapFn(torch.autograd.Function):
    """Differentiable channel remap of a physical-order tensor; ``leaf`` (a parameter whose
    physical view is ``x``) gets its gradient added straight into its arena buffer."""

    @staticmethod
    def forward(ctx, x, remap, out_shape, leaf):
        ctx.remap, ctx.in_shape, ctx.leaf = remap, x.shape, leaf
        return remap.apply(x.reshape(-1) if remap.flat else x).view(out_shape)

    @staticmethod
    def backward(ctx, dy):
        dy = dy.contiguous()
        if ctx.remap.flat:
            dy = dy.view(-1)
        leaf = ctx.leaf
        if leaf is not None:
            buf = G.grad_buffer(leaf)
            if buf is not None and tuple(buf.shape) == tuple(ctx.in_shape):
                ctx.remap.apply(dy, inverse=True, acc=buf.view(-1) if ctx.remap.flat else buf)
                G.fire(leaf)
                return None, None, None, None
        return ctx.remap.apply(dy, inverse=True).view(ctx.in_shape), None, None, None


class _PadInput(torch.autograd.Function):
    """Zero-pad the channels of an activation (one remap launch); the backward's unpad adds the
    gradient another consumer left in ``slot`` (its owner is this conv) in the same launch —
    no autograd add (csrc/misc.hip chan_remap_rows_kernel ACC)."""

    @staticmethod
    def forward(ctx, x, remap, out_shape, slot):
        ctx.remap, ctx.in_shape, ctx.slot = remap, x.shape, slot
        return remap.apply(x).view(out_shape)

    @staticmethod
    def backward(ctx, dy):
        dy = dy.contiguous()
        slot, ctx.slot = ctx.slot, None
        other = slot.take() if slot is not None else None
        if (other is not None and other.dtype == dy.dtype and other.is_contiguous()
                and tuple(other.shape) == tuple(ctx.in_shape)):
            ctx.remap.apply(dy, inverse=True, acc=other)     # other += unpad(dy)
            return other, None, None, None
        dx = ctx.remap.apply(dy, inverse=True).view(ctx.in_shape)
        if other is not None:
            dx = dx + other.reshape(dx.shape)
        return dx, None, None, None


def _remap_param(p, remap, phys_shape):
    """Remapped copy of parameter ``p`` in physical order; its gradient flows back natively."""
    phys = G.physical(p)
    leaf = p if (p.is_leaf and p.requires_grad and phys.is_contiguous()) else None
    if not phys.is_contiguous():
        phys = phys.contiguous()
    return _RemapFn.apply(phys, remap, phys_shape, leaf)


def _shuffle_remap(C, groups):
    # out channel j = i * groups + g  <-  in channel g * (C / groups) + i
    def build():
        cpg = C // groups
        return Remap([(j % groups) * cpg + j // groups for j in range(C)], C)
    return Remap.get(("shuffle", C, groups), build)


def channel_shuffle(x, groups):
    """[N,C,H,W] -> [N,g,C/g,H,W] -> transpose -> [N,C,H,W] (shufflenet*.py ShuffleBlock): on the
    GPU one native channel-remap pass each way (NHWC, the channel dim is innermost) instead of a
    transposing stock copy."""
    N, C, H, W = x.shape
    if _ref(x) or x.dtype != COMPUTE_DTYPE:
        out = x.reshape(N, groups, C // groups, H, W).transpose(1, 2).reshape(N, C, H, W)
        if not _ref(out):
            out = out.contiguous(memory_format=torch.channels_last)
        return out
    xn = to_nhwc(x)
    return to_nchw(_RemapFn.apply(xn, _shuffle_remap(C, groups), xn.shape, None))


class _CatNHWC(torch.autograd.Function):
    @staticmethod
    def forward(ctx, *xs):
        ctx.sizes = [x.shape[-1] for x in xs]
        return _C().cat_nhwc(list(xs))

    @staticmethod
    def backward(ctx, dy):
        return tuple(_C().split_nhwc(dy.contiguous(), ctx.sizes))


class _SplitChannels(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, c):
        ctx.sizes = [c, x.shape[-1] - c]
        a, b = _C().split_nhwc(x, ctx.sizes)
        return a, b

    @staticmethod
    def backward(ctx, da, db):
        ref = da if da is not None else db
        shp = list(ref.shape[:-1])
        da = da.contiguous() if da is not None else ref.new_zeros(shp + [ctx.sizes[0]])
        db = db.contiguous() if db is not None else ref.new_zeros(shp + [ctx.sizes[1]])
        return _C().cat_nhwc([da, db]), None


def split_channels(x, c):
    """(x[:, :c], x[:, c:]) as two dense tensors (shufflenetv2.py:22-29 SplitBlock): one native
    pass, backward one native concat — instead of strided slice copies whose autograd backward
    zero-fills and adds two full-size tensors."""
    if _ref(x) or x.dtype != COMPUTE_DTYPE or x.dim() != 4:
        return x[:, :c], x[:, c:]
    a, b = _SplitChannels.apply(to_nhwc(x), c)
    return to_nchw(a), to_nchw(b)


class _Interleave2(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, b):
        return _C().interleave2(a, b)

    @staticmethod
    def backward(ctx, dy):
        da, db = _C().deinterleave2(dy.contiguous())
        return da, db


def cat_shuffle2(a, b):
    """channel_shuffle(cat([a, b], 1), groups=2) for equal widths (ShuffleNetV2 joins,
    shufflenetv2.py:49/73 + ShuffleBlock 10-19): a single channel interleave each way."""
    if _ref(a) or a.shape != b.shape or a.dtype != COMPUTE_DTYPE or b.dtype != COMPUTE_DTYPE:
        return channel_shuffle(cat([a, b], 1), 2)
    return to_nchw(_Interleave2.apply(to_nhwc(a), to_nhwc(b)))


def _nhwc_rows(t):
    """Dense NHWC rows, possibly wider than C (row stride >= C, dense outer strides): the layout
    the row-strided native kernels accept, at any channel count."""
    return (t.dim() == 4 and t.stride(3) == 1 and t.stride(2) >= t.shape[3]
            and t.stride(1) == t.shape[2] * t.stride(2) and t.stride(0) == t.shape[1] * t.stride(1))


class _Interleave2Split(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, b, pad_hi):
        lo, hi = _C().interleave2_split(a, b, pad_hi)
        return lo, hi

    @staticmethod
    def backward(ctx, dlo, dhi):
        ref = dlo if dlo is not None else dhi
        dlo = dlo.contiguous() if dlo is not None else torch.zeros_like(ref)
        if dhi is None:
            dhi = torch.zeros_like(ref)
        elif not _nhwc_rows(dhi):
            dhi = dhi.contiguous()
        # (a row-strided NHWC view — at the odd half widths 58 / 116 the prefix of the padded
        # conv's dX — is read in place: the kernel takes any row stride >= C)
        da, db = _C().deinterleave2_split(dlo, dhi)
        return da, db, None


def cat_shuffle2_split(a, b, pad_hi=0):
    """The two channel halves of channel_shuffle(cat([a, b], 1), 2) — a ShuffleNetV2 join followed
    by the next block's SplitBlock (shufflenetv2.py:22-29, 49) — as ONE native interleave pass
    writing both halves (backward: one pass reading both half-gradients): no concatenated
    tensor is formed, and the split / concat passes of the two-step form disappear.
    ``pad_hi`` (a multiple of 8 above the half width): the second half — the next block's
    branch input — is the channel prefix of a zero-padded buffer of that width, which its
    odd-width 1x1 conv then reads in place (``_pca_zpad``) instead of a pad pass."""
    if (_ref(a) or a.shape != b.shape or a.dtype != COMPUTE_DTYPE or b.dtype != COMPUTE_DTYPE
            or a.dim() != 4 or a.shape[1] % 2):
        y = cat_shuffle2(a, b)
        c = y.shape[1] // 2
        return y[:, :c], y[:, c:]
    C = a.shape[1]
    pad = pad_hi if (pad_hi > C and pad_hi % 8 == 0 and _GROUP_PAD) else 0
    lo, hi = _Interleave2Split.apply(to_nhwc(a), to_nhwc(b), pad)
    hi = to_nchw(hi)
    if pad:
        hi._pca_zpad = pad
    return to_nchw(lo), hi


class _ZeroPadView(torch.autograd.Function):
    """The whole zero-padded buffer [N,H,W,cp] behind a channel-prefix view (its padding channels
    written as zeros by their producer); backward: the gradient's channel prefix, a view."""

    @staticmethod
    def forward(ctx, xn, cp):
        N, H, W, C = xn.shape
        ctx.C = C
        return xn.as_strided((N, H, W, cp), (H * W * cp, W * cp, cp, 1))

    @staticmethod
    def backward(ctx, dxp):
        return dxp[..., : ctx.C], None


class _PadSlot:
    """Hand-off between a zero-padded conv's output prefix (_UnpadView) and the BatchNorm that
    reads it in place: the BN backward deposits its dY, written into zero-padded rows, here."""
    __slots__ = ("base", "dy")

    def __init__(self):
        self.base = self.dy = None


class _UnpadView(torch.autograd.Function):
    """The real channels of a zero-padded conv output [N,H,W,op] as a row-strided view (no slice
    pass). Backward: the padded gradient the consuming BatchNorm left in the slot (same tensor:
    no pad pass), else the gradient padded with zeros here."""

    @staticmethod
    def forward(ctx, yp, C, slot):
        ctx.C, ctx.slot, ctx.op = C, slot, yp.shape[-1]
        return yp[..., :C]

    @staticmethod
    def backward(ctx, dy):
        slot = ctx.slot
        base, dyv = slot.base, slot.dy
        slot.base = slot.dy = None
        if base is not None and dyv is not None and dy.data_ptr() == dyv.data_ptr() and \
                dy.shape == dyv.shape and dy.stride() == dyv.stride():
            return base, None, None
        out = dy.new_zeros(dy.shape[:-1] + (ctx.op,))
        out[..., : ctx.C] = dy
        return out, None, None


# ------------------------------------------------------------- zero-copy concatenation
# a concatenation is a preallocated NHWC slab whose channel slices the producers
# write directly (their BatchNorm+activation kernel takes the slice as a row-strided output:
# batchnorm.hip BnLd), and whose gradient reaches each producer's backward as a row-strided view
# of the slab's gradient — no gather copy forward, no split copy backward (reference
# googlenet.py:53 torch.cat([y1, y2, y3, y4], 1), ...).
def _rows_view(t):
    """``t`` itself when it is a contiguous or row-strided NHWC [N,H,W,C] bf16 tensor whose channel
    count allows the strided BatchNorm kernels (C % 8 == 0), else a contiguous copy."""
    if t.is_contiguous():
        return t
    if (t.dim() == 4 and t.is_cuda and t.dtype == COMPUTE_DTYPE and t.stride(3) == 1 and
            t.shape[3] % 8 == 0 and t.stride(2) >= t.shape[3] and
            t.stride(1) == t.shape[2] * t.stride(2) and t.stride(0) == t.shape[1] * t.stride(1)):
        return t
    return t.contiguous()


@functools.lru_cache(maxsize=None)
def _bn_rows_max_c():
    """Widest channel count the native row-tiled BatchNorm kernels take (0 with PCA_BN_ROWS=0):
    the only BN kernels that read / write row-strided (slab) operands."""
    lib = _C()
    return int(lib.bn_rows_max_c()) if hasattr(lib, "bn_rows_max_c") else 0


def _slab_alias(buf, c0, c1):
    """A fresh tensor over channels [c0, c1) of the NHWC slab ``buf`` — not an autograd view of
    it: slices are written by native kernels (no in-place op autograd could see), and each slice
    is an independent output of its producer."""
    t = torch.empty(0, dtype=buf.dtype, device=buf.device)
    t.set_(buf.untyped_storage(), buf.storage_offset() + c0,
           (buf.shape[0], buf.shape[1], buf.shape[2], c1 - c0), buf.stride())
    return t


class ChannelSlab:
    """Destination of a channel concatenation: ``dest(i)`` is producer i's slice (pass it as the
    ``out=`` of its final BatchNorm), ``cat(parts)`` returns the whole slab as the concat result."""

    def __init__(self, like, widths, hw=None):
        N, _, H, W = like.shape
        if hw is not None:
            H, W = hw          # the producers' output size (they may stride their input)
        self.widths = list(widths)
        self.offs = [0]
        for w in self.widths:
            self.offs.append(self.offs[-1] + w)
        self.buf = torch.empty((N, H, W, self.offs[-1]), dtype=COMPUTE_DTYPE, device=like.device)

    @staticmethod
    def usable(x, widths):
        # (the BatchNorms reading / writing the slices row-strided need the row-tiled kernels:
        # slab width within their reach, and PCA_BN_ROWS not disabled)
        return (not _ref(x) and x.dim() == 4 and all(w % 8 == 0 for w in widths)
                and sum(widths) <= _bn_rows_max_c()
                and os.environ.get("PCA_ZERO_COPY_CAT", "1") != "0")

    def dest(self, i):
        return _slab_alias(self.buf, self.offs[i], self.offs[i + 1])

    def cat(self, parts):
        pns = [p.permute(0, 2, 3, 1) for p in parts]
        for pn, o, w in zip(pns, self.offs, self.widths):
            if (pn.untyped_storage().data_ptr() != self.buf.untyped_storage().data_ptr()
                    or pn.storage_offset() != self.buf.storage_offset() + o or pn.shape[-1] != w):
                raise RuntimeError("ChannelSlab.cat: part was not produced into its slab slice")
        self.junctions = [getattr(p, "_pca_junction", None) for p in parts]
        return to_nchw(_SlabCat.apply(self, *pns))


class _Junction(GradSlot):
    """Gradient junction of a slab slice that also fed a dense copy (DLA / SimpleDLA Root: the left
    child's output is read by the root conv through the slab and by the right child through
    ``dense_copy``). The slab's backward (it runs first: the root is later in the forward) leaves
    the slice's gradient here instead of returning it; the copy's backward adds its own gradient
    in one native pass (``add_rows``) and returns the sum — no autograd add."""
    __slots__ = ()


class _CopyRows(torch.autograd.Function):
    """Dense copy of a row-strided NHWC slab slice (one native pass; identity backward, or the
    junction sum when the slab left the slice's gradient in ``junction``)."""

    @staticmethod
    def forward(ctx, x, junction=None):
        out = torch.empty(x.shape, dtype=x.dtype, device=x.device)
        _C().copy_rows(x, out)
        ctx.junction = junction
        return out

    @staticmethod
    def backward(ctx, g):
        j = ctx.junction
        if j is not None:
            other = j.take()
            if other is not None and g is not None and g.dtype == other.dtype:
                gv = g if _nhwc_rows(g) else g.contiguous()
                out = torch.empty(g.shape, dtype=g.dtype, device=g.device)
                _C().add_rows(other, gv, out)
                return out, None
            if other is not None:
                g = other if g is None else g + other
        return g, None


def dense_copy(x):
    """A dense NHWC-stored copy of ``x`` (an NCHW-shaped view of a concat slab slice) for
    consumers that need dense operands (the MFMA convs' A side, residual adds)."""
    if _ref(x):
        return x
    j = None
    if torch.is_grad_enabled() and x.requires_grad and x.shape[1] % 8 == 0:
        j = _Junction()
        x._pca_junction = j
    return to_nchw(_CopyRows.apply(x.permute(0, 2, 3, 1), j))


class _SlabCat(torch.autograd.Function):
    @staticmethod
    def forward(ctx, slab, *parts):
        ctx.offs = slab.offs
        ctx.junctions = getattr(slab, "junctions", None) or [None] * len(parts)
        return _slab_alias(slab.buf, 0, slab.offs[-1])

    @staticmethod
    def backward(ctx, dy):
        # dy: NHWC-shaped gradient of the slab; producer i gets its channel range as a view —
        # or, when part i also fed a dense copy, the view waits in that junction for the copy's
        # gradient (summed there in one native pass)
        o = ctx.offs
        out = []
        for i in range(len(o) - 1):
            v = dy[..., o[i]:o[i + 1]]
            j = ctx.junctions[i]
            if (j is not None and v.dtype == COMPUTE_DTYPE and _nhwc_rows(v)
                    and v.shape[-1] % 8 == 0 and j.offer(v)):
                v = None
            out.append(v)
        return (None,) + tuple(out)


class DenseSlab:
    """One dense block's concatenations as a single slab (densenet.py:20 ``cat([out, x], 1)``,
    new features first): x_0 sits at the slab's right end and layer l's g new channels go just
    left of x_l, so every x_l is a channel suffix of the slab — read in place (row-strided) by the
    next layer's BatchNorm, never re-copied: the block moves O(g) bytes per layer instead of the
    O(C_l) gather + split of a copying concat. Gradients: x_l's gradient is a suffix view of the
    slab gradient; the append deposits it in x_l's GradSlot and the BatchNorm that also read x_l
    adds its own contribution into that memory (bn_backward dx_acc), so nothing is summed or split
    by copies either."""

    def __init__(self, x0, growth, layers, training=False):
        N, C0, H, W = x0.shape
        self.g = growth
        self.C = C0 + growth * layers
        self.buf = torch.empty((N, H, W, self.C), dtype=COMPUTE_DTYPE, device=x0.device)
        self.c0 = self.C - C0      # first channel of the current suffix
        # statistics cache (training): every channel's centred batch sums, added as the channel is
        # copied into the slab (bn_stats_copy), so each layer's BatchNorm folds its suffix of the
        # cache in its apply kernel instead of a stats + finalize pass over the whole suffix (the
        # O(L^2) reduction of the block); zeroed once per step before the first producer
        self.sbuf = None
        if training and _SLAB_STATS and acc_enabled(self.C, x0.device):
            self.R = acc_shards(self.C)
            self.sbuf = torch.empty(self.R * 2 * self.C + self.C, dtype=torch.float32,
                                    device=x0.device)

    @staticmethod
    def usable(x0, growth, layers):
        # every suffix BatchNorm reads up to the whole slab row-strided: the final width must be
        # within the row-tiled kernels' reach (DenseNet161's dense3 / dense4 reach 2112 / 2208
        # channels and keep the copying concat)
        return (not _ref(x0) and x0.dim() == 4 and x0.dtype == COMPUTE_DTYPE and growth % 8 == 0
                and x0.shape[1] % 8 == 0 and x0.shape[1] + growth * layers <= _bn_rows_max_c()
                and os.environ.get("PCA_ZERO_COPY_CAT", "1") != "0")

    def _suffix(self, t_nhwc, slot):
        v = to_nchw(t_nhwc)
        v._pca_dense_slot = slot
        if self.sbuf is not None:
            v._pca_dense_stats = _SlabStats(self.sbuf, self.R, self.c0, self.C, self.C - self.c0)
        return v

    def start(self, x0):
        return self._suffix(_SlabPut.apply(to_nhwc(x0), self, self.c0), _DenseSlot())

    def append(self, out, x):
        """cat([out, x], 1) where x is this slab's current suffix."""
        self.c0 -= self.g
        xs, ys = x._pca_dense_slot, _DenseSlot()
        return self._suffix(_DenseAppend.apply(to_nhwc(out), x.permute(0, 2, 3, 1), self, self.c0,
                                               xs if xs.claimed else None, ys), ys)


class _SlabPut(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, slab, c0):
        dst = _slab_alias(slab.buf, c0, slab.C)
        if slab.sbuf is not None:
            _C().zero_(slab.sbuf)
            _C().bn_stats_copy(x, dst, slab.sbuf, c0, slab.C, slab.R)
        else:
            _C().copy_rows(x, dst)
        return dst

    @staticmethod
    def backward(ctx, dy):
        dx = torch.empty(dy.shape, dtype=dy.dtype, device=dy.device)
        _C().copy_rows(_rows_view(dy), dx)
        return dx, None, None


class _DenseAppend(torch.autograd.Function):
    @staticmethod
    def forward(ctx, out, x, slab, c0, xslot, yslot):
        ctx.g = out.shape[-1]
        ctx.xslot, ctx.yslot = xslot, yslot
        if slab.sbuf is not None:
            _C().bn_stats_copy(out, _slab_alias(slab.buf, c0, c0 + ctx.g), slab.sbuf, c0, slab.C,
                               slab.R)
        else:
            _C().copy_rows(out, _slab_alias(slab.buf, c0, c0 + ctx.g))
        return _slab_alias(slab.buf, c0, slab.C)

    @staticmethod
    def backward(ctx, dy):
        g = ctx.g
        if not ctx.yslot.claimed:
            # dy came from outside (not a dense-block BatchNorm's fresh / slab-gradient tensor):
            # it may be held elsewhere, so the in-place accumulation below works on a private copy
            dy = dy.clone(memory_format=torch.contiguous_format)
        dout = torch.empty(dy.shape[:-1] + (g,), dtype=dy.dtype, device=dy.device)
        _C().copy_rows(_rows_view(dy[..., :g]), dout)     # dense copy for the conv's backward
        dx = dy[..., g:]
        if ctx.xslot is not None and ctx.xslot.offer(dx):
            dx = None          # the BatchNorm that read x adds its gradient into this memory
        return dout, dx, None, None, None, None


def cat(xs, dim=1):
    """Channel concatenation (densenet.py:20, dla*.py Root, googlenet.py:53, dpn.py:31): on the
    GPU one native NHWC pass each way (the channel dim is innermost, so torch.cat / its
    backward's narrow copies are strided gathers)."""
    xs = list(xs)
    if (dim == 1 and 1 < len(xs) <= 8 and not _ref(xs[0]) and xs[0].dim() == 4
            and all(x.dtype == COMPUTE_DTYPE for x in xs)):
        return to_nchw(_CatNHWC.apply(*[to_nhwc(x) for x in xs]))
    out = torch.cat(xs, dim)
    if not _ref(out) and out.dim() == 4:
        out = out.contiguous(memory_format=torch.channels_last)
    return out


def kaiming_fan_in_bound(fan_in: int) -> float:
    return 1.0 / math.sqrt(fan_in) if fan_in > 0 else 0.0
