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
SOURCES = ["bb_kernels.hip", "bb_ozaki.hip", "bb_tri.hip", "bb_sparse.hip", "bb_logit.hip", "bb_nid.hip",
           "bb_small.hip", "bb_engine.cpp"]
HEADERS = ["bb_kernels.h", "bb_sampler.h", "bb_ozaki.h", "bb_sparse.h", "bb_pg.h"]
ARCH = os.environ.get("BB_OFFLOAD_ARCH", "gfx950")


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found: the HIP extension cannot be built")


def _stale() -> bool:
    if not os.path.exists(SO_PATH):
        return True
    so_m = os.path.getmtime(SO_PATH)
    deps = [os.path.join(CSRC, f) for f in SOURCES + HEADERS]
    deps.append(os.path.join(ROOT, "include", "bayesbridge.h"))
    deps.append(os.path.abspath(__file__))
    return any(os.path.getmtime(d) > so_m for d in deps)


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and not _stale():
        return SO_PATH
    objs = []
    flags = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
             "-Wall", "-Wno-unused-result", "-pthread", f"-I{os.path.join(ROOT, 'include')}"]
    procs = []
    for src in SOURCES:  # translation units compile in parallel
        obj = os.path.join(CSRC, src.rsplit(".", 1)[0] + ".o")
        cmd = [hipcc(), *flags, "-c", os.path.join(CSRC, src), "-o", obj]
        if verbose:
            print(" ".join(cmd))
        procs.append((cmd, subprocess.Popen(cmd)))
        objs.append(obj)
    failed = [cmd for cmd, pr in procs if pr.wait() != 0]
    if failed:
        raise subprocess.CalledProcessError(1, failed[0])
    tmp = SO_PATH + ".tmp"
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp, *objs,
           "-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,/opt/rocm/lib", "-ldl", "-pthread"]
    if verbose:
        print(" ".join(cmd))
    subprocess.check_call(cmd)
    os.replace(tmp, SO_PATH)
    for o in objs:
        os.remove(o)
    return SO_PATH


if __name__ == "__main__":
    print(build(force=True, verbose=True))
