"""CPU tests of the drop-in boundary: BayesBridge.so loads and exports every symbol that
include/bayesbridge.h declares (no compute calls -- there is no GPU here)."""
import ctypes
import os
import re
import subprocess

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
