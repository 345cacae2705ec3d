"""Kernel-selection tables on the GPU (engine/tuning.py): the shipped MI355X table matches the
built candidate set and is imported, and tune_export -> conv_clear_tuned -> tune_import
round-trips a live selection (including the rows a real training step tuned)."""
import json

import pytest
import torch

pytestmark = pytest.mark.gpu


def _rows(lib):
    return sorted(list(map(int, r)) for r in lib.tune_export())


def test_shipped_table_matches_build_and_loads():
    from pytorch_cifar_amd import _native
    from pytorch_cifar_amd.engine import tuning

    lib = _native.lib()
    with open(tuning.TABLE_PATH) as fh:
        tab = json.load(fh)
    assert tab["version"] == lib.tune_version(), "shipped table made for another candidate set"
    assert tab["hash"] == tuning.selection_hash(tab["rows"])
    lib.conv_clear_tuned()
    assert tuning.load_table(lib) == len(tab["rows"])
    have = {tuple(r) for r in _rows(lib)}
    assert all(tuple(map(int, r)) in have for r in tab["rows"])


def test_export_import_round_trip_after_a_step():
    from pytorch_cifar_amd import _native, models
    from pytorch_cifar_amd.engine import tuning
    from pytorch_cifar_amd.ops.functional import cross_entropy

    lib = _native.lib()
    torch.manual_seed(0)
    m = models.ResNet18().cuda()
    x = torch.randn(24, 3, 32, 32, device="cuda")
    y = torch.randint(0, 10, (24,), device="cuda")
    cross_entropy(m(x), y).backward()          # tunes any geometry the table does not hold
    torch.cuda.synchronize()
    rows = _rows(lib)
    assert rows, "no selection rows after a step"
    h = tuning.selection_hash(rows)
    lib.conv_clear_tuned()
    assert _rows(lib) == []
    assert lib.tune_import(rows) == len(rows)
    assert _rows(lib) == rows and tuning.selection_hash(_rows(lib)) == h
