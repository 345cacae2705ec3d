"""Host-side AddressSanitizer + UBSan run of the kernel library's launch planners (SURVEY §5:
race / fault detection; the reference has none). GPU ASan and XNACK runs are not available on the
MI355X pool, so the host logic that sizes workspaces, BatchNorm slab rows and persistent grids,
and the autotuner's candidate lists, is built with the address + undefined-behaviour sanitizers (host side only)
and driven over the zoo's conv census at batch 1-1024 and every tuning candidate
(tools/sanitize/host_plan_check.cpp). CPU only; takes ~3 minutes (the kernels' device code is
compiled too). PCA_SKIP_SANITIZE=1 skips it."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(os.environ.get("PCA_SKIP_SANITIZE") == "1" or shutil.which("/opt/rocm/bin/hipcc") is None,
                    reason="sanitizer build skipped / no hipcc")
def test_host_planners_under_asan_ubsan(tmp_path):
    r = subprocess.run(["bash", os.path.join(ROOT, "tools", "sanitize", "run.sh")],
                       env=dict(os.environ, SAN_OUT=str(tmp_path)), capture_output=True, text=True,
                       timeout=900)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "ERROR: AddressSanitizer" not in out and "runtime error:" not in out, out[-4000:]
    assert "failures: 0" in out
