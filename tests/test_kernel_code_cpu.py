"""Kernel code identity (bayesbridge_amd/_kernel_code.py) and its use by bench.py's evidence
lookups: a committed profile entry describes this build's kernel iff the recorded code_sha
(gfx950 code bytes + kernel descriptor) equals the library's.  CPU only: the library's code
objects are parsed from the file, nothing runs on a device."""
import json

import pytest

import bench
from bayesbridge_amd import _build, _kernel_code

DOMINANT = ["bb::k_lambda_xu<8, 8>", "bb::k_lambda_cb_in<8>", "bb::k_eapply<8, 0>",
            "bb::k_eapply<8, 2>", "bb::k_beta_wb_xb<16, true>", "bb::k_chol_persistent<1>",
            "bb::k_oz_gemm16u<0>", "bb::k_pre", "bb::k_scalars", "bb::k_nid_reduce"]


def test_mangled_prefix_forms():
    assert _kernel_code.mangled_prefix("bb::k_lambda_xu<8, 8>") == "_ZN2bb11k_lambda_xuILi8ELi8EEEv"
    assert _kernel_code.mangled_prefix("bb::k_beta_wb_xb<16, true>") == \
        "_ZN2bb12k_beta_wb_xbILi16ELb1EEEv"
    assert _kernel_code.mangled_prefix("bb::k_pre") == "_ZN2bb5k_preE"
    with pytest.raises(ValueError):
        _kernel_code.mangled_prefix("__amd_rocclr_copyBuffer")


def test_every_dominant_kernel_has_a_unique_code_identity():
    _build.build()
    shas = _kernel_code.code_shas()
    assert len(shas) > 100  # every kernel of the seven HIP translation units
    got = {k: _kernel_code.code_sha(k) for k in DOMINANT}
    assert all(v and len(v) == 16 for v in got.values()), got
    # distinct kernels, distinct code (the KIND instances of the E-apply differ)
    assert got["bb::k_eapply<8, 0>"] != got["bb::k_eapply<8, 2>"]
    assert _kernel_code.code_sha("bb::k_no_such_kernel") is None


def test_annotate_marks_only_unique_bb_kernels():
    shas = {"_ZN2bb5k_preEPKd": "a" * 16, "_ZN2bb6k_gramEPKd": "b" * 16}
    m = {"bb::k_pre": {}, "bb::k_gram": {}, "__amd_rocclr_copyBuffer": {}, "bb::k_none": {}}
    assert _kernel_code.annotate(m, shas) == 2
    assert m["bb::k_pre"]["code_sha"] == "a" * 16 and "code_sha" not in m["bb::k_none"]
    assert "code_sha" not in m["__amd_rocclr_copyBuffer"]


def test_stale_note_follows_the_kernel_code_not_the_tree(monkeypatch):
    inst = "bb::k_lambda_xu<8, 8>"
    cur = _kernel_code.code_sha(inst)
    other_tree = {"source_sha": "0" * 16}
    # the profiled tree differs, the kernel's code does not: the entry is this build's
    assert bench._stale_note(other_tree, "p.json", {"code_sha": cur}, inst) is None
    # the kernel's code differs: not used, whatever the tree
    note = bench._stale_note({"source_sha": bench.tree_sha()}, "p.json", {"code_sha": "f" * 16}, inst)
    assert note and "not used" in note
    # an entry without a code identity falls back to the tree's source_sha
    assert bench._stale_note({"source_sha": bench.tree_sha()}, "p.json", {}, inst) is None
    assert "not used" in bench._stale_note(other_tree, "p.json", {}, inst)


def test_pmc_lookups_use_code_identity(tmp_path, monkeypatch):
    """pmc_traffic / pmc_valu take a profile of another tree when the kernel's code matches
    and refuse it when it does not."""
    inst = "bb::k_lambda_xu<8, 8>"
    cur = _kernel_code.code_sha(inst)
    prof = tmp_path / "profiles"
    prof.mkdir()
    for tag, cs in (("ok", cur), ("bad", "f" * 16)):
        d = {"source_sha": "0" * 16, "workload": {"n": 7, "p": 11 if tag == "ok" else 13},
             "window": {"steps": 20, "warmup": 5},
             "kernels": {inst: {"hbm_bytes": 123.0, "code_sha": cs}}}
        (prof / f"r99{tag}_pmc.json").write_text(json.dumps(d))
        v = {"source_sha": "0" * 16, "configs": {"c": {
            "n": 7, "p": 11 if tag == "ok" else 13, "window": {"steps": 20, "warmup": 5},
            "kernels": {inst: {"SQ_INSTS_VALU": 1.0, "code_sha": cs}}}}}
        (prof / f"r99{tag}_pmc_valu.json").write_text(json.dumps(v))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    b, src, note = bench.pmc_traffic(7, 11, 1, inst, (20, 5))
    assert b == 123.0 and note is None
    b, src, note = bench.pmc_traffic(7, 13, 1, inst, (20, 5))
    assert b is None and "not used" in note
    e, note = bench.pmc_valu(7, 11, 1, inst, (20, 5))
    assert e and e["SQ_INSTS_VALU"] == 1.0
    e, note = bench.pmc_valu(7, 13, 1, inst, (20, 5))
    assert e is None and "not used" in note


def test_eapply_family_traffic_is_dispatch_weighted(tmp_path, monkeypatch):
    """The mixed plan's E-apply phase launches three instances; its traffic per launch is
    their dispatch-weighted mean in the profile of the same window, and a changed kernel
    retires the whole family's evidence."""
    fam = ["bb::k_eapply<8, 0>", "bb::k_eapply<8, 2>", "bb::k_eapply<8, 3>"]
    cs = {k: _kernel_code.code_sha(k) for k in fam}
    prof = tmp_path / "profiles"
    prof.mkdir()
    ks = {fam[0]: {"hbm_bytes": 400.0, "dispatches": 3, "code_sha": cs[fam[0]]},
          fam[1]: {"hbm_bytes": 800.0, "dispatches": 1, "code_sha": cs[fam[1]]},
          fam[2]: {"hbm_bytes": 400.0, "dispatches": 4, "code_sha": cs[fam[2]]}}
    d = {"source_sha": "0" * 16, "workload": {"n": 5, "p": 9}, "window": {"steps": 10, "warmup": 1},
         "kernels": ks}
    (prof / "r99a_pmc.json").write_text(json.dumps(d))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    b, src, note, per = bench.pmc_traffic_family(5, 9, 1, fam, (10, 1))
    assert b == (3 * 400 + 800 + 4 * 400) / 8 and note is None and per[fam[1]]["dispatches"] == 1
    ks[fam[1]]["code_sha"] = "f" * 16
    (prof / "r99a_pmc.json").write_text(json.dumps(d))
    b, src, note, per = bench.pmc_traffic_family(5, 9, 1, fam, (10, 1))
    assert b is None and "not used" in note


def _build_so(tmp_path, name, src):
    import subprocess
    f = tmp_path / f"{name}.hip"
    f.write_text(src)
    so = tmp_path / f"{name}.so"
    subprocess.check_call([_build.hipcc(), "--offload-arch=gfx950", "-O3", "-shared", "-fPIC",
                           "-o", str(so), str(f)])
    return str(so)


def test_identity_follows_code_not_layout(tmp_path):
    """Two libraries built here: the second adds a kernel before `keep` (its code moves in
    the code object) and changes `edit`.  `keep` keeps its identity (the descriptor's entry
    offset is left out), `edit` gets a new one."""
    base = """#include <hip/hip_runtime.h>
namespace bb {
__global__ void keep(double *x) { x[threadIdx.x] = x[threadIdx.x] * 2.0 + 1.0; }
__global__ void edit(double *x) { x[threadIdx.x] += 3.0; }
}
"""
    moved = """#include <hip/hip_runtime.h>
namespace bb {
__global__ void added(double *x, int n) { for (int i = 0; i < n; ++i) x[i] = x[i] * x[i] + 0.5; }
__global__ void keep(double *x) { x[threadIdx.x] = x[threadIdx.x] * 2.0 + 1.0; }
__global__ void edit(double *x) { x[threadIdx.x] += 4.0; }
}
"""
    a = _kernel_code.code_shas(_build_so(tmp_path, "a", base))
    b = _kernel_code.code_shas(_build_so(tmp_path, "b", moved))
    k = [m for m in a if "4keep" in m][0]
    e = [m for m in a if "4edit" in m][0]
    assert a[k] == b[k]
    assert a[e] != b[e]
    assert any("5added" in m for m in b) and not any("5added" in m for m in a)


def test_identity_follows_out_of_line_callees(tmp_path):
    """A kernel that calls a __noinline__ helper gets a new identity when only the helper
    changes (the callee's code is part of the caller's identity)."""
    src = """#include <hip/hip_runtime.h>
namespace bb {
__device__ __noinline__ double helper(double v) { return v * v + %s; }
__global__ void caller(double *x) { x[threadIdx.x] = helper(x[threadIdx.x]); }
}
"""
    a = _kernel_code.code_shas(_build_so(tmp_path, "ca", src % "0.25"))
    b = _kernel_code.code_shas(_build_so(tmp_path, "cb", src % "0.75"))
    k = [m for m in a if "6caller" in m][0]
    assert a[k] != b[k]


def test_round5_profiles_carry_code_identities():
    """Every committed round-5 PMC / VALU / MFMA summary stamps its bb:: kernel entries with
    the kernel's code identity (what bench.py matches a later build against)."""
    import glob
    import os

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    files = glob.glob(os.path.join(root, "profiles", "r05*_pmc*.json"))
    assert files
    for f in files:
        d = json.load(open(f))
        maps = [d["kernels"]] if isinstance(d.get("kernels"), dict) else []
        maps += [c["kernels"] for c in d.get("configs", {}).values() if "kernels" in c]
        for m in maps:
            for k, v in m.items():
                if k.startswith("bb::") and isinstance(v, dict):
                    assert v.get("code_sha"), (f, k)
