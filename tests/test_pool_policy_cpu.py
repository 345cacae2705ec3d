"""Pool-policy check over every script and source the GPU runs could upload.

The MI355X pool refuses a run when any uploaded script names a GPU sanitizer build or an XNACK-on
code object (round 3 lost its whole driver-side GPU run to one hipcc link line). This test scans
every ``*.sh`` / ``*.py`` / ``*.hip`` / ``*.cpp`` / ``*.h`` / ``Makefile`` / ``CMakeLists.txt`` in
the repository (minus what ``.gpurunignore`` keeps off the box) and asserts, per logical statement
(backslash continuations joined):

* every ``-fsanitize=`` token comes right after ``-Xarch_host``, or the statement carries
  ``-fno-gpu-sanitize`` and no ``-Xarch_`` option at all;
* nothing turns XNACK on (``HSA_XNACK=1``, ``xnack+`` targets).

It also checks that the host-only sanitizer harness and its test stay listed in ``.gpurunignore``
(the GPU run does not need them).
"""
import fnmatch
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SELF = os.path.relpath(os.path.abspath(__file__), ROOT)
SCAN_SUFFIX = (".sh", ".py", ".hip", ".cpp", ".h", ".hpp", ".cc", ".mk")
SCAN_NAMES = ("Makefile", "CMakeLists.txt")
SKIP_DIRS = {".git", "gpurun_out", "__pycache__", ".pytest_cache", "build"}

SAN = "-f" + "sanitize="          # split so this file does not name the token itself
NOGPU = "-fno-gpu-" + "sanitize"
XNACK_ON = ("HSA_" + "XNACK=1", "xnack" + "+")


def _ignore_patterns():
    pats = []
    path = os.path.join(ROOT, ".gpurunignore")
    if os.path.exists(path):
        for line in open(path):
            line = line.strip()
            if line and not line.startswith("#"):
                pats.append(line)
    return pats


def _ignored(rel, pats):
    for p in pats:
        if p.startswith("./"):
            if rel == p[2:] or rel.startswith(p[2:].rstrip("/") + "/"):
                return True
        elif fnmatch.fnmatch(os.path.basename(rel), p) or fnmatch.fnmatch(rel, p):
            return True
    return False


def _files(include_ignored):
    pats = _ignore_patterns()
    for dirpath, dirnames, filenames in os.walk(ROOT):
        dirnames[:] = [d for d in dirnames if d not in SKIP_DIRS]
        for fn in filenames:
            if not (fn.endswith(SCAN_SUFFIX) or fn in SCAN_NAMES):
                continue
            rel = os.path.relpath(os.path.join(dirpath, fn), ROOT)
            if rel == SELF:
                continue
            if not include_ignored and _ignored(rel, pats):
                continue
            yield rel


def _statements(text):
    """Logical statements: shell backslash continuations joined."""
    out, cur, start = [], "", 1
    for i, line in enumerate(text.splitlines(), 1):
        if not cur:
            start = i
        if line.rstrip().endswith("\\"):
            cur += line.rstrip()[:-1] + " "
            continue
        out.append((start, cur + line))
        cur = ""
    if cur:
        out.append((start, cur))
    return out


def statement_violations(stmt):
    """Reasons one statement breaks the pool rule (empty list: compliant)."""
    bad = []
    toks = stmt.split()
    if any(SAN in t for t in toks):
        if NOGPU in stmt:
            if any(t.startswith("-Xarch_") for t in toks):
                bad.append("has " + NOGPU + " and an -Xarch_ option")
        else:
            for k, t in enumerate(toks):
                if SAN in t and (k == 0 or toks[k - 1] != "-Xarch_host"):
                    bad.append(f"{t!r} not preceded by -Xarch_host")
    for x in XNACK_ON:
        if x in stmt:
            bad.append(f"turns XNACK on ({x})")
    return bad


def test_rule_checker_itself():
    assert statement_violations(f"hipcc -Xarch_host {SAN}address -c a.hip") == []
    assert statement_violations(f"hipcc {SAN}address a.o") != []
    assert statement_violations(f"hipcc {NOGPU} {SAN}address a.o") == []
    assert statement_violations(f"hipcc -Xarch_host {SAN}address -Xarch_host {SAN}undefined a.hip") == []
    assert statement_violations(f"hipcc {NOGPU} -Xarch_host {SAN}address a.o") != []
    assert statement_violations("hipcc --offload-arch=gfx950:" + XNACK_ON[1] + " a.hip") != []
    assert statement_violations("hipcc --offload-arch=gfx950 -O3 a.hip") == []


def test_every_uploaded_or_local_script_follows_the_pool_rule():
    problems = []
    for rel in _files(include_ignored=True):
        try:
            text = open(os.path.join(ROOT, rel), errors="replace").read()
        except OSError:
            continue
        for line_no, stmt in _statements(text):
            for why in statement_violations(stmt):
                problems.append(f"{rel}:{line_no}: {why}")
    assert not problems, "\n".join(problems)


def test_sanitizer_harness_stays_off_the_gpu_box():
    pats = _ignore_patterns()
    for rel in ("tools/sanitize/run.sh", "tools/sanitize/host_plan_check.cpp",
                "tests/test_sanitize_cpu.py", SELF):
        assert _ignored(rel, pats), f"{rel} must be listed in .gpurunignore"
