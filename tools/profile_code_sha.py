"""Record, in committed profile summaries, the code identity of every kernel they measured.

    python tools/profile_code_sha.py --tree /path/to/checkout profiles/r05_pmc.json ...

--tree is a checkout of the sources the profiles were taken from, built in place
(`python -c "from bayesbridge_amd import _build; _build.build()"` inside it; hipcc is
deterministic, so its library is the one the GPU box ran).  A profile is annotated only if its
source_sha equals that tree's: each bb:: kernel entry then gets "code_sha"
(bayesbridge_amd/_kernel_code.py: its gfx950 code bytes + kernel descriptor), and the summary
records where the identities came from.  bench.py uses a profile's entry for a later build when
the kernel's code_sha is unchanged -- a change elsewhere in the library no longer retires the
evidence of kernels it did not touch, and any change of the kernel itself still does.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from bayesbridge_amd import _build, _kernel_code  # noqa: E402


def kernel_maps(d):
    """The {instance: entry} maps of a profile summary (pmc: kernels; valu / mfma: configs)."""
    if isinstance(d.get("kernels"), dict):
        yield d["kernels"]
    for cfg in (d.get("configs") or {}).values():
        if isinstance(cfg.get("kernels"), dict):
            yield cfg["kernels"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tree", required=True)
    ap.add_argument("profiles", nargs="+")
    a = ap.parse_args()
    tree_sha = _build.source_sha(a.tree)
    so = os.path.join(a.tree, "bayesbridge_amd", "BayesBridge.so")
    shas = _kernel_code.code_shas(so)
    for f in a.profiles:
        d = json.load(open(f))
        if d.get("source_sha") != tree_sha:
            print(f"{f}: profiled source {d.get('source_sha')}, tree {tree_sha}: skipped")
            continue
        k = sum(_kernel_code.annotate(m, shas) for m in kernel_maps(d))
        d["code_sha_from"] = (f"library rebuilt from the profiled sources (source_sha {tree_sha}) "
                              "by tools/profile_code_sha.py")
        json.dump(d, open(f, "w"), indent=1)
        print(f"{f}: {k} kernel entries annotated")


if __name__ == "__main__":
    main()
