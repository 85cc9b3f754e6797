"""CPU tests of the drop-in boundary: BayesBridge.so loads and exports every symbol that
include/bayesbridge.h declares (no compute calls -- there is no GPU here)."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

import bayesbridge_amd as bb

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    src = open(os.path.join(ROOT, "include", "bayesbridge.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"\b([A-Za-z_][A-Za-z0-9_]*)\s*\([^;{]*\)\s*;", src)
    return sorted(set(n for n in names if n not in ("if", "while", "sizeof")))


def test_header_declares_reference_entry_points():
    names = declared_functions()
    # the reference's .C symbols for this path (BridgeWrapper.h:205-226, :244)
    assert "bridge_reg_stable" in names and "retstable_LD" in names
    assert len(names) >= 30


def test_library_exports_every_declared_symbol():
    L = bb.library()
    missing = [n for n in declared_functions() if not hasattr(L, n)]
    assert not missing, missing
    assert set(bb.EXPORTED_SYMBOLS) <= set(declared_functions())


def test_symbols_are_unmangled_c_linkage():
    out = subprocess.check_output(["nm", "-D", "--defined-only", bb._build.SO_PATH], text=True)
    exported = {ln.split()[-1] for ln in out.splitlines() if " T " in ln}
    for n in declared_functions():
        assert n in exported, n


def test_library_is_named_for_r_dyn_load():
    # useDynLib("BayesBridge") (Code/BBPackage/BayesBridge/NAMESPACE:3) loads BayesBridge.so
    assert os.path.basename(bb._build.SO_PATH) == "BayesBridge.so"


def test_library_is_gfx950_code_object():
    blob = open(bb._build.SO_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob


def test_info_calls_without_gpu():
    L = bb.library()
    assert b"gfx950" in L.bb_version()
    assert L.bb_device_count() >= 0
    bb.set_seed(123)
    assert bb.get_rng_state() == (123, 0)
    bb.set_rng_state(5, 9)
    assert bb.get_rng_state() == (5, 9)


def test_tuning_keys_report_defaults_without_gpu():
    """bb_set_tuning with a negative value changes nothing and returns the setting; the keys
    include/bayesbridge.h documents (11: polled decision tag, 12: XCD-aware row blocks, 10: the
    mixed plan) answer with their defaults, an unknown key with -1."""
    for key, want in ((10, 1), (11, 1), (12, 1), (13, 1), (15, 1), (9, 0), (8, 1), (16, 0), (17, 1), (20, 1)):
        assert bb.set_tuning(key, -1) == want, key
    assert bb.set_tuning(99, 1) == -1
    old = bb.set_tuning(12, 0)
    try:
        assert bb.set_tuning(12, -1) == 0
    finally:
        bb.set_tuning(12, old)


def test_config_struct_layout_matches_header():
    L = bb.library()
    c = bb.bb_config()
    L.bb_config_default(ctypes.byref(c))
    assert c.world == 1 and c.nu_shape == 2.0 and c.nu_rate == 2.0 and c.true_alpha == 0.5
    assert c.seed == 0xB4E5B41D6E


def test_no_gpu_fails_loudly():
    if bb.device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(RuntimeError):
        bb.retstable_ld(3, 0.5, 1.0, 1.0)


def test_dot_c_controls_take_pointers():
    """Every control R must call has a pointer-only `.C` form (R's .C passes pointers,
    BridgeWrapper.h:164-245): .C("bb_set_device_count_C", k) stores k itself -- the by-value
    bb_set_device_count(int) would receive the address of R's integer."""
    try:
        for k in (0, 1, 3):
            bb.dot_c("bb_set_device_count_C", k)
            (got,) = bb.dot_c("bb_get_device_count_C", 0)
            assert int(got[0]) == k
        # seed / stream / byte counts travel as R doubles (exact integers up to 2^53)
        bb.dot_c("bb_set_rng_state_C", float(2 ** 52 + 7), 11.0)
        assert bb.get_rng_state() == (2 ** 52 + 7, 11)
        bb.dot_c("bb_set_seed_C", 4242.0)
        s, t = bb.dot_c("bb_get_rng_state_C", 0.0, 0.0)
        assert (s[0], t[0]) == (4242.0, 0.0)
        # a negative, NaN, fractional or > 2^53 double is refused, not cast (UB in C++)
        for bad in (-1.0, float("nan"), float("inf"), 2.5, 2.0 ** 60):
            bb.dot_c("bb_set_seed_C", bad)
            assert bb.get_rng_state() == (4242, 0), bad
            assert "ignored" in bb._err()
            bb.dot_c("bb_set_rng_state_C", 5.0, bad)
            assert bb.get_rng_state() == (4242, 0), bad
        bb.dot_c("bb_set_verbose_C", 0)
        d, c, i = bb.dot_c("bb_last_call_info_C", 0, 0, 0)
        assert d.dtype == np.int32 and c.dtype == np.int32 and i[0] in (0, 1)
    finally:
        bb.set_device_count(1)
        bb.set_verbose(1)


@pytest.mark.parametrize("setting,nvis,n,p,ortho,want", [
    (1, 8, 2000, 50000, 0, 1),   # the default: one device
    (0, 8, 2000, 50000, 0, 8),   # 0 = every visible device
    (0, 1, 2000, 50000, 0, 1),
    (4, 8, 2000, 50000, 0, 4),   # k
    (16, 8, 2000, 50000, 0, 8),  # capped by the visible devices
    (0, 8, 2000, 20000, 0, 4),   # >= 4096 columns per device
    (0, 8, 1000, 900, 0, 1),     # p <= n: replicas only, never sharded
    (2, 8, 200, 10000, 1, 2),    # the orthogonal design shards too
])
def test_dot_c_device_plan(setting, nvis, n, p, ortho, want):
    """The device count a .C sampler call takes after .C("bb_set_device_count_C", k) for k =
    0, 1 and k > 1 (bb_plan_devices_C evaluates the driver's own rule for a given number of
    visible devices, so it runs without a GPU)."""
    try:
        bb.dot_c("bb_set_device_count_C", setting)
        (dev,) = bb.dot_c("bb_plan_devices_C", n, p, ortho, nvis, 0)[-1:]
        assert int(dev[0]) == want
    finally:
        bb.set_device_count(1)


def _documented_makevars_objects():
    """The OBJECTS line of INTEGRATION.md's package Makevars (Option B)."""
    txt = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    m = re.search(r"^OBJECTS\s*=\s*(.+)$", txt, flags=re.M)
    assert m, "INTEGRATION.md has no Makevars OBJECTS line"
    return m.group(1).split()


def test_documented_makevars_objects_match_build_sources():
    # Code/C/Makevars:1-6 is the reference's recipe; ours must name every translation unit
    # the in-tree build compiles, or R's dyn.load fails on unresolved bb:: symbols
    objs = _documented_makevars_objects()
    want = [s.rsplit(".", 1)[0] + ".o" for s in bb._build.SOURCES]
    assert sorted(objs) == sorted(want), (objs, want)
    assert len(set(objs)) == len(objs)


def test_documented_makevars_links_without_unresolved_engine_symbols(tmp_path):
    """Link a .so from exactly the documented object list and check that nothing of the
    engine (namespace bb, mangled _ZN2bb) is left undefined."""
    built = {os.path.basename(o): o for o in bb._build.objects()}
    objs = [built[o] for o in _documented_makevars_objects()]
    so = bb._build.link(objs, str(tmp_path / "BayesBridge.so"))
    out = subprocess.check_output(["nm", "-D", "--undefined-only", so], text=True)
    bad = [ln.split()[-1] for ln in out.splitlines() if "_ZN2bb" in ln or " bb::" in ln]
    assert not bad, bad[:10]
    # and it exports the reference's .C symbols
    exp = subprocess.check_output(["nm", "-D", "--defined-only", so], text=True)
    names = {ln.split()[-1] for ln in exp.splitlines()}
    assert {"bridge_reg_stable", "retstable_LD", "bridge_EM"} <= names
