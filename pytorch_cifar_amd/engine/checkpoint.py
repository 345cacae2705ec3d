"""Checkpoint save/resume in the reference layout (main.py:137-148, main_dist.py:239-252).

Payload ``{'net': wrapped.state_dict(), 'acc': float percent, 'epoch': int}`` — the same keys,
``module.``-prefixed parameter names when the net is wrapped, fp32 tensors in the reference's
NCHW parameter shapes — so reference checkpoints load here and vice versa. Additions (extra keys
are ignored by reference loaders): optional ``optimizer`` / ``scheduler`` state
so a resumed run continues the momentum buffers and the cosine schedule.

Writes are atomic (temp file + rename) and done by one rank. Loads use ``weights_only=True``.
Resume tolerates a ``module.`` prefix mismatch (the reference's resume fails on a bare model).
"""
from __future__ import annotations

import os
import warnings

import torch


def _unwrap_keys(sd, want_prefix: bool):
    has = all(k.startswith("module.") for k in sd) and len(sd) > 0
    if want_prefix and not has:
        return {"module." + k: v for k, v in sd.items()}
    if not want_prefix and has:
        return {k[len("module."):]: v for k, v in sd.items()}
    return sd


def save_checkpoint(path, net, acc, epoch, optimizer=None, scheduler=None, extra=None,
                    scheduler_stepped=False):
    """``scheduler_stepped``: whether ``scheduler.step()`` already ran for ``epoch`` when this was
    saved (main.py / main_dist.py save inside the epoch, before stepping: False). Recorded in the
    payload so a resume advances the schedule only when the saved state is one step behind."""
    if hasattr(net, "finish"):
        net.finish()       # DDP: join a buffer broadcast still in flight on the comm stream
    state = {"net": net.state_dict(), "acc": float(acc), "epoch": int(epoch)}
    if optimizer is not None:
        state["optimizer"] = optimizer.state_dict()
    if scheduler is not None:
        state["scheduler"] = scheduler.state_dict()
        state["scheduler_stepped"] = bool(scheduler_stepped)
    if extra:
        state.update(extra)
    d = os.path.dirname(os.path.abspath(path))
    os.makedirs(d, exist_ok=True)
    tmp = path + ".tmp"
    torch.save(state, tmp)
    os.replace(tmp, path)
    return path


def load_checkpoint(path, net, optimizer=None, scheduler=None, map_location="cpu"):
    """Restore ``net`` (and optionally optimizer/scheduler); returns (best_acc, epoch)."""
    ck = torch.load(path, map_location=map_location, weights_only=True)
    sd = ck["net"]
    want_prefix = all(k.startswith("module.") for k in net.state_dict())
    net.load_state_dict(_unwrap_keys(sd, want_prefix))
    if optimizer is not None and "optimizer" in ck:
        optimizer.load_state_dict(ck["optimizer"])
    if scheduler is not None and "scheduler" in ck:
        scheduler.load_state_dict(ck["scheduler"])
        # A resumed run starts at epoch e + 1. A checkpoint taken inside epoch e before that
        # epoch's scheduler.step() (the entry points' order) is one step behind: advance it once
        # so e + 1 trains at lr(e + 1). One saved after stepping is already there.
        if not ck.get("scheduler_stepped", False):
            with warnings.catch_warnings():
                warnings.simplefilter("ignore")   # "scheduler.step() before optimizer.step()"
                scheduler.step()
    return float(ck.get("acc", 0.0)), int(ck.get("epoch", 0))
