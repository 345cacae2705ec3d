"""Kernel-selection tables: the shipped MI355X tune table, rank-consistent selection, selection hash.

The reference sets ``cudnn.benchmark = True`` (main.py:75, main_dist.py:147), so every process
times its own conv algorithms. Here the per-geometry autotuner (csrc/bindings.cpp autotune_conv)
is that analogue, with two additions:

* a validated table for the BASELINE configurations ships with the package
  (``tune/mi355x.json``, written by ``tools/tune_table.py`` on a GPU box) and is imported at load,
  so a fresh box starts from the measured selection and the autotuner only fills misses — box to
  box the same kernels run (``PCA_TUNE_TABLE=0`` ignores the table);
* under data parallelism rank 0's selection is broadcast after the first (tuning) step and every
  rank adopts it, so the replicas run identical kernels: no per-rank step-time skew from
  different tile / split / slab-vs-atomic picks gating every bucket all-reduce, and bitwise-equal
  per-rank gradient arithmetic (reference main_dist.py:140-147: replicated model).

Rows are ``tune_export()``'s ``[table, key[13], cfg, split]`` integers.
"""
from __future__ import annotations

import hashlib
import json
import os

TABLE_PATH = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tune", "mi355x.json")


def selection_rows(lib) -> list[list[int]]:
    return sorted(list(map(int, r)) for r in lib.tune_export())


def selection_hash(rows) -> str:
    """Order-independent digest of a selection (printed by bench.py)."""
    h = hashlib.sha256()
    for r in sorted(list(map(int, r)) for r in rows):
        h.update((",".join(map(str, r)) + "\n").encode())
    return h.hexdigest()[:16]


_loaded = {"rows": 0}


def table_rows_loaded() -> int:
    return _loaded["rows"]


def load_table(lib, path: str = TABLE_PATH) -> int:
    """Import the shipped table if it was made for this kernel candidate set; returns rows taken."""
    if os.environ.get("PCA_TUNE_TABLE", "1") == "0" or not hasattr(lib, "tune_version"):
        return 0
    try:
        with open(path) as fh:
            tab = json.load(fh)
    except (OSError, ValueError):
        return 0
    if tab.get("version") != lib.tune_version():
        _skip(f"candidate-set version {tab.get('version')} != {lib.tune_version()}")
        return 0   # candidate set changed since the table was measured: tune afresh
    why = device_mismatch(tab)
    if why:
        _skip(why)
        return 0
    _loaded["rows"] = int(lib.tune_import(tab.get("rows", [])))
    return _loaded["rows"]


def _skip(why: str) -> None:
    import sys

    print(f"pytorch_cifar_amd: shipped tune table not used ({why}); autotuning every geometry",
          file=sys.stderr)


def device_mismatch(tab: dict) -> str:
    """Why the table does not describe the current device ('' = it does). The selections are
    timings of one part: another architecture or CU count must re-tune. Checked only once the
    process already holds a GPU context (the table is imported when the extension loads, and
    asking for device properties earlier would initialise HIP in launcher parents)."""
    import torch

    if not (torch.cuda.is_available() and torch.cuda.is_initialized()):
        return ""
    props = torch.cuda.get_device_properties(torch.cuda.current_device())
    arch = str(getattr(props, "gcnArchName", "") or "").split(":")[0]
    if tab.get("arch") and arch and arch != tab["arch"]:
        return f"table arch {tab['arch']}, device {arch}"
    cus = tab.get("cus")
    if cus and props.multi_processor_count != cus:
        return f"table measured on {cus} CUs, device has {props.multi_processor_count}"
    return ""


def sync_selection(ctx, lib=None, export=None, import_=None, clear=None) -> str:
    """Adopt rank 0's kernel selection on every rank (call after the first, tuning, step; every
    rank must call it). Returns the selection hash, equal on all ranks afterwards."""
    import torch.distributed as dist

    if lib is not None:
        export = export or lib.tune_export
        import_ = import_ or lib.tune_import
        clear = clear or lib.conv_clear_tuned
    rows = [sorted(list(map(int, r)) for r in export())] if ctx.rank == 0 else [None]
    if ctx.world > 1:
        dist.broadcast_object_list(rows, src=0)
    if ctx.rank != 0:
        clear()
        import_(rows[0])
    return selection_hash(rows[0])
