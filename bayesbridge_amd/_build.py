"""Build BayesBridge.so (gfx950) in-tree with hipcc.

The shared object is the drop-in for the reference's R package library
(`useDynLib("BayesBridge")`, Code/BBPackage/BayesBridge/NAMESPACE:1-3): it exports
the reference's .C symbols plus the bb_* extensions of include/bayesbridge.h.
"""
from __future__ import annotations

import os
import shutil
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
SO_PATH = os.path.join(HERE, "BayesBridge.so")
OBJ_DIR = os.path.join(HERE, "build")  # per-source objects (kept: tests relink them)
SOURCES = ["bb_kernels.hip", "bb_ozaki.hip", "bb_tri.hip", "bb_sparse.hip", "bb_logit.hip", "bb_nid.hip",
           "bb_small.hip", "bb_engine.cpp"]
HEADERS = ["bb_kernels.h", "bb_sampler.h", "bb_ozaki.h", "bb_sparse.h", "bb_pg.h", "bb_chol4.h"]
ARCH = os.environ.get("BB_OFFLOAD_ARCH", "gfx950")


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found: the HIP extension cannot be built")


def source_sha(root: str | None = None) -> str:
    """sha256 (first 16 hex digits) of every source and header the library is built from (of
    this tree, or of the tree at root): the committed profiles record it; bench.py uses a
    profile for a kernel whose code it recorded (bayesbridge_amd/_kernel_code.py) if that code
    is unchanged, otherwise only if the tree matches."""
    import hashlib

    root = root or ROOT
    csrc = os.path.join(root, "bayesbridge_amd", "csrc")
    h = hashlib.sha256()
    files = [os.path.join(csrc, f) for f in sorted(SOURCES + HEADERS)]
    files.append(os.path.join(root, "include", "bayesbridge.h"))
    for f in files:
        h.update(os.path.basename(f).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def _stale() -> bool:
    if not os.path.exists(SO_PATH):
        return True
    so_m = os.path.getmtime(SO_PATH)
    deps = [os.path.join(CSRC, f) for f in SOURCES + HEADERS]
    deps.append(os.path.join(ROOT, "include", "bayesbridge.h"))
    deps.append(os.path.abspath(__file__))
    return any(os.path.getmtime(d) > so_m for d in deps)


LINK_LIBS = ["-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,/opt/rocm/lib", "-ldl", "-pthread"]


def objects(force: bool = False, verbose: bool = False) -> list:
    """Compile every translation unit of SOURCES into OBJ_DIR (in parallel; only the stale
    ones unless force) and return the object paths in SOURCES order."""
    os.makedirs(OBJ_DIR, exist_ok=True)
    flags = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
             "-Wall", "-Wno-unused-result", "-pthread", f"-I{os.path.join(ROOT, 'include')}"]
    hdrs = [os.path.join(CSRC, h) for h in HEADERS]
    hdrs.append(os.path.join(ROOT, "include", "bayesbridge.h"))
    newest_dep = max(os.path.getmtime(h) for h in hdrs + [os.path.abspath(__file__)])
    objs, procs = [], []
    for src in SOURCES:  # translation units compile in parallel
        path = os.path.join(CSRC, src)
        obj = os.path.join(OBJ_DIR, src.rsplit(".", 1)[0] + ".o")
        objs.append(obj)
        if (not force and os.path.exists(obj)
                and os.path.getmtime(obj) >= max(newest_dep, os.path.getmtime(path))):
            continue
        cmd = [hipcc(), *flags, "-c", path, "-o", obj]
        if verbose:
            print(" ".join(cmd))
        procs.append((cmd, subprocess.Popen(cmd)))
    failed = [cmd for cmd, pr in procs if pr.wait() != 0]
    if failed:
        raise subprocess.CalledProcessError(1, failed[0])
    return objs


def link(objs: list, out: str, verbose: bool = False) -> str:
    tmp = out + ".tmp"
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp, *objs, *LINK_LIBS]
    if verbose:
        print(" ".join(cmd))
    subprocess.check_call(cmd)
    os.replace(tmp, out)
    return out


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and not _stale():
        return SO_PATH
    return link(objects(force=force, verbose=verbose), SO_PATH, verbose=verbose)


if __name__ == "__main__":
    print(build(force=True, verbose=True))
