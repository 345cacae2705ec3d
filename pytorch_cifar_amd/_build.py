"""In-tree native build of the gfx950 kernel library (``pytorch_cifar_amd._C``).

No hipify, no torch JIT cache: every ``csrc/*.hip`` kernel file and ``csrc/*.cpp`` host file is
compiled explicitly with ``hipcc --offload-arch=gfx950`` into ``build/obj`` and linked into an
extension module that lives next to this file, so the built ``.so`` travels with the repository
snapshot to the GPU box.  Objects are rebuilt only when a source or header is newer.

Usage:  python -m pytorch_cifar_amd._build [--force] [-v]
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
import sysconfig

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
REPO_DIR = os.path.dirname(PKG_DIR)
CSRC = os.path.join(PKG_DIR, "csrc")
OBJ_DIR = os.path.join(REPO_DIR, "build", "obj")
ARCH = os.environ.get("PCA_OFFLOAD_ARCH", "gfx950")
EXT_NAME = "_C"


def ext_path() -> str:
    suffix = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
    return os.path.join(PKG_DIR, EXT_NAME + suffix)


def _hipcc() -> str:
    rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
    cand = os.path.join(rocm, "bin", "hipcc")
    return cand if os.path.exists(cand) else (shutil.which("hipcc") or "hipcc")


def _torch_paths():
    import torch
    import torch.utils.cpp_extension as ce

    tdir = os.path.dirname(torch.__file__)
    incs = ce.include_paths()
    incs = [p for p in incs if os.path.isdir(p)]
    libdir = os.path.join(tdir, "lib")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return incs, libdir, abi


def _common_flags(incs, abi):
    py_inc = sysconfig.get_paths()["include"]
    flags = [
        "-O3",
        "-std=c++17",
        "-fPIC",
        "-DUSE_ROCM",
        "-D__HIP_PLATFORM_AMD__=1",
        f"-DTORCH_EXTENSION_NAME={EXT_NAME}",
        "-DTORCH_API_INCLUDE_EXTENSION_H",
        f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
        "-Wno-unused-result",
        "-Wno-deprecated-declarations",
        "-Wno-unused-command-line-argument",
        f"-I{CSRC}",
        f"-I{py_inc}",
    ]
    # build-time kernel variants for same-box A/B trees (e.g. -DPCA_IGEMM_DMA_SPREAD=1)
    flags += os.environ.get("PCA_EXTRA_HIPCC_FLAGS", "").split()
    flags += [f"-I{p}" for p in incs]
    return flags


def source_digest() -> str:
    """sha256 over every csrc source/header (name + bytes): identifies what a built .so is of."""
    import hashlib

    h = hashlib.sha256()
    for f in sorted(os.listdir(CSRC)):
        if f.endswith((".hip", ".cpp", ".h")):
            h.update(f.encode())
            with open(os.path.join(CSRC, f), "rb") as fh:
                h.update(fh.read())
    return h.hexdigest()


def digest_path() -> str:
    return ext_path() + ".srchash"


def is_stale():
    """True when the in-tree .so is missing or was built from different csrc contents, False when
    its recorded digest matches, None when unknown (the .so exists but its git-ignored ``.srchash``
    does not, e.g. a fresh checkout next to a shipped .so): the loader then compares the digest the
    .so carries itself (``_C.src_digest()``) after import."""
    if not os.path.exists(ext_path()):
        return True
    try:
        with open(digest_path()) as fh:
            return fh.read().strip() != source_digest()
    except OSError:
        return None


def _digest_object(flags, verbose):
    """A one-symbol object carrying the source digest, linked into the .so (see is_stale)."""
    src = os.path.join(OBJ_DIR, "srcdigest.cpp")
    with open(src, "w") as fh:
        fh.write('extern "C" const char pca_src_digest[] = "%s";\n' % source_digest())
    return _compile(src, src + ".o", flags, verbose)


def _headers():
    return [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]


def _needs_build(src: str, obj: str, deps) -> bool:
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    return any(os.path.getmtime(d) > t for d in [src, *deps])


def _compile(src, obj, flags, verbose):
    cmd = [_hipcc()] + flags
    if src.endswith(".hip"):
        cmd += ["-x", "hip", f"--offload-arch={ARCH}"]
    cmd += ["-c", src, "-o", obj]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {os.path.basename(src)}:\n{r.stderr[-6000:]}")
    return obj


def build(force: bool = False, verbose: bool = False, jobs: int | None = None) -> str:
    """Compile and link the extension; returns the path of the built module."""
    incs, libdir, abi = _torch_paths()
    flags = _common_flags(incs, abi)
    os.makedirs(OBJ_DIR, exist_ok=True)
    srcs = sorted(
        os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith((".hip", ".cpp"))
    )
    hdrs = _headers()
    todo, objs = [], []
    for s in srcs:
        o = os.path.join(OBJ_DIR, os.path.basename(s) + ".o")
        objs.append(o)
        if force or _needs_build(s, o, hdrs):
            todo.append((s, o))
    jobs = jobs or min(len(todo) or 1, int(os.environ.get("MAX_JOBS", os.cpu_count() or 4)), 8)
    if todo:
        with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
            futs = [ex.submit(_compile, s, o, flags, verbose) for s, o in todo]
            for f in futs:
                f.result()
    objs.append(_digest_object(flags, verbose))
    out = ext_path()
    if todo or not os.path.exists(out) or any(os.path.getmtime(o) > os.path.getmtime(out) for o in objs):
        cmd = [_hipcc(), "-shared", "-fPIC", f"--offload-arch={ARCH}", *objs, "-o", out,
               f"-L{libdir}", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip",
               "-ltorch_python", "-lamdhip64", "-lrccl", f"-Wl,-rpath,{libdir}"]
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr[-6000:]}")
    with open(digest_path(), "w") as fh:
        fh.write(source_digest() + "\n")
    return out


def build_locked(**kw) -> str:
    """``build`` under an exclusive file lock, so concurrent ranks build once and then reuse."""
    import fcntl

    os.makedirs(os.path.dirname(OBJ_DIR), exist_ok=True)
    with open(os.path.join(os.path.dirname(OBJ_DIR), ".build.lock"), "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        try:
            if is_stale() is False and not kw.get("force"):
                return ext_path()
            return build(**kw)
        finally:
            fcntl.flock(lk, fcntl.LOCK_UN)


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=None)
    a = ap.parse_args(argv)
    print(build(force=a.force, verbose=a.verbose, jobs=a.jobs))


if __name__ == "__main__":
    sys.exit(main())
