"""Helpers with the reference's names and output formats (parity: reference utils.py:16-141).

Reference defects fixed: ``progress_bar`` no longer runs ``stty size`` at
import (crashed every headless run) — the terminal width comes from ``shutil`` with an 80-column
fallback; ``get_mean_and_std`` and ``init_params`` work (the reference's referenced an unimported
``torch`` and deprecated non-underscore init functions / ambiguous tensor truth tests).
"""
from __future__ import annotations

import logging
import shutil
import sys
import time

import torch
import torch.nn as nn
import torch.nn.init as init

TOTAL_BAR_LENGTH = 65.0
_last_time = time.time()
_begin_time = _last_time


def _term_width() -> int:
    return shutil.get_terminal_size(fallback=(80, 24)).columns


def get_mean_and_std(dataset):
    """Per-channel mean/std averaged over per-image statistics (utils.py:16-28 semantics).

    ``dataset`` yields (image [3,H,W] tensor, label) pairs, or is a uint8 [N,H,W,3] array.
    """
    if hasattr(dataset, "shape") and len(getattr(dataset, "shape")) == 4:
        x = torch.as_tensor(dataset).float().div_(255.0).permute(0, 3, 1, 2)
        return x.mean(dim=(2, 3)).mean(0), x.std(dim=(2, 3)).mean(0)
    mean = torch.zeros(3)
    std = torch.zeros(3)
    n = 0
    for inputs, _ in dataset:
        inputs = torch.as_tensor(inputs)
        for i in range(3):
            mean[i] += inputs[i, :, :].mean()
            std[i] += inputs[i, :, :].std()
        n += 1
    return mean.div_(n), std.div_(n)


def init_params(net):
    """Kaiming-normal (fan_out) convs, BN weight 1 / bias 0, Linear N(0, 1e-3) (utils.py:30-43)."""
    for m in net.modules():
        if isinstance(m, nn.Conv2d):
            init.kaiming_normal_(m.weight, mode="fan_out")
            if m.bias is not None:
                init.constant_(m.bias, 0)
        elif isinstance(m, nn.BatchNorm2d):
            init.constant_(m.weight, 1)
            init.constant_(m.bias, 0)
        elif isinstance(m, nn.Linear):
            init.normal_(m.weight, std=1e-3)
            if m.bias is not None:
                init.constant_(m.bias, 0)


def format_time(seconds):
    """Two most significant units among D/h/m/s/ms (utils.py:95-125 format)."""
    days = int(seconds / 3600 / 24)
    seconds = seconds - days * 3600 * 24
    hours = int(seconds / 3600)
    seconds = seconds - hours * 3600
    minutes = int(seconds / 60)
    seconds = seconds - minutes * 60
    secondsf = int(seconds)
    seconds = seconds - secondsf
    millis = int(seconds * 1000)
    parts = [(days, "D"), (hours, "h"), (minutes, "m"), (secondsf, "s"), (millis, "ms")]
    out = "".join(f"{v}{u}" for v, u in [p for p in parts if p[0] > 0][:2])
    return out or "0ms"


def progress_bar(current, total, msg=None, stream=None):
    """xlua-style bar ``[=====>....]  Step: .. | Tot: .. | msg  cur/total`` (utils.py:49-93).

    Written as one string per call (the reference wrote char by char); on a non-TTY stream only
    the final step of a bar is printed, as a single plain line, so logs stay readable.
    """
    global _last_time, _begin_time
    stream = stream or sys.stdout
    if current == 0:
        _begin_time = time.time()
    cur_time = time.time()
    step_time = cur_time - _last_time
    _last_time = cur_time
    tot_time = cur_time - _begin_time
    parts = [f"  Step: {format_time(step_time)}", f" | Tot: {format_time(tot_time)}"]
    if msg:
        parts.append(" | " + msg)
    info = "".join(parts)
    tty = hasattr(stream, "isatty") and stream.isatty()
    if not tty:
        if current >= total - 1:
            stream.write(f" {current + 1}/{total}{info}\n")
            stream.flush()
        return
    cur_len = int(TOTAL_BAR_LENGTH * current / total)
    rest_len = int(TOTAL_BAR_LENGTH - cur_len) - 1
    bar = " [" + "=" * cur_len + ">" + "." * rest_len + "]"
    width = _term_width()
    line = bar + info
    line += " " * max(0, width - int(TOTAL_BAR_LENGTH) - len(info) - 3)
    line += f" {current + 1}/{total} "
    stream.write(line[: max(width - 1, 20)] + ("\r" if current < total - 1 else "\n"))
    stream.flush()


def set_logger(log_path, rank: int = 0):
    """Root logger at INFO: file '%(asctime)s:%(levelname)s: %(message)s' + console '%(message)s'
    (utils.py:128-141). Only rank 0 attaches the file handler (the reference had every rank append
    to the same train.log)."""
    logger = logging.getLogger()
    logger.setLevel(logging.INFO)
    if not logger.handlers:
        if rank == 0 and log_path:
            fh = logging.FileHandler(log_path)
            fh.setFormatter(logging.Formatter("%(asctime)s:%(levelname)s: %(message)s"))
            logger.addHandler(fh)
        sh = logging.StreamHandler()
        sh.setFormatter(logging.Formatter("%(message)s"))
        logger.addHandler(sh)
    return logger
