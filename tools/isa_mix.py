"""Static VALU instruction mix of a kernel (gfx950 assembly from hipcc --cuda-device-only -S),
priced with the issue costs measured by tools/valu_rate.hip: the weights bench.py uses for the
two rocprofv3 VALU classes whose members differ in cost (SQ_INSTS_VALU_INT32: v_add_u32 2
cycles, v_mul_lo_u32 / v_bfe_u32 4; and the instructions no class counts -- v_cndmask_b32,
v_mov_b32, v_and_b32 at 2, 64-bit and f64 ops such as v_ldexp_f64, v_lshlrev_b64, v_cmp_*_f64
at 4).  Membership as measured (profiles/r05_valu_costs.json).

    python tools/isa_mix.py <file.s> <mangled-name-prefix> [...]
"""
import collections
import json
import re
import sys

TRANS_F64 = {"v_rcp_f64", "v_sqrt_f64", "v_rsq_f64"}
TRANS_F32 = {"v_exp_f32", "v_log_f32", "v_rcp_f32", "v_rsq_f32", "v_sqrt_f32", "v_sin_f32",
             "v_cos_f32", "v_rcp_iflag_f32", "v_exp_legacy_f32", "v_log_legacy_f32"}
INT32_QUARTER = {"v_mul_lo_u32", "v_mul_hi_u32", "v_mul_hi_i32", "v_bfe_u32", "v_bfe_i32",
                 "v_mad_u32_u24", "v_mul_u32_u24", "v_mad_i32_i24", "v_mul_i32_i24",
                 "v_mul_lo_i32"}
INT32_FULL = {"v_add_u32", "v_sub_u32", "v_subrev_u32", "v_add_co_u32", "v_sub_co_u32",
              "v_addc_co_u32", "v_subb_co_u32", "v_subrev_co_u32", "v_add3_u32",
              "v_add_lshl_u32", "v_lshl_add_u32", "v_add_i32", "v_sub_i32"}


def wide(m):
    return bool(re.search(r"_(f64|b64|i64|u64)\b", m)) or m.endswith(("_f64", "_b64", "_i64",
                                                                       "_u64"))


def classify(m):
    """(class, issue cycles per wave64 instruction) of a VALU mnemonic."""
    if m.startswith("v_mfma"):
        return "MFMA", None
    if m in ("v_fma_f64", "v_fmac_f64"):
        return "FMA_F64", 4
    if m == "v_mul_f64":
        return "MUL_F64", 4
    if m == "v_add_f64":
        return "ADD_F64", 4
    if m in TRANS_F64:
        return "TRANS_F64", 16
    if m in TRANS_F32:
        return "TRANS_F32", 8
    if m in ("v_fma_f32", "v_fmac_f32", "v_mac_f32", "v_fmaak_f32", "v_fmamk_f32"):
        return "FMA_F32", 2
    if m in ("v_add_f32", "v_sub_f32", "v_subrev_f32"):
        return "ADD_F32", 2
    if m == "v_mul_f32":
        return "MUL_F32", 2
    if m in ("v_mad_u64_u32", "v_mad_i64_i32"):
        return "INT64", 4
    if m.startswith("v_cvt_"):
        return "CVT", 4 if wide(m) else 2
    if m in INT32_QUARTER:
        return "INT32", 4
    if m in INT32_FULL:
        return "INT32", 2
    return "OTHER", 4 if wide(m) else 2


def mix(asm, prefix):
    lines = asm.splitlines()
    start = None
    for i, ln in enumerate(lines):
        if ln.startswith(prefix) and ln.split(";")[0].rstrip().endswith(":"):
            start = i
            break
    if start is None:
        raise SystemExit(f"{prefix}: not found")
    cnt = collections.Counter()
    for ln in lines[start + 1:]:
        s = ln.strip()
        if s.startswith(".Lfunc_end"):
            break
        if s.startswith("v_"):
            cnt[s.split()[0].replace("_e32", "").replace("_e64", "").replace("_sdwa", "")
                .replace("_dpp", "")] += 1
    per = collections.defaultdict(lambda: [0, 0])
    for m, c in cnt.items():
        k, cyc = classify(m)
        if cyc is None:
            continue
        per[k][0] += c
        per[k][1] += c * cyc
    return {k: {"static_count": v[0], "avg_cycles": v[1] / v[0]} for k, v in sorted(per.items())}, cnt


def main():
    asm = open(sys.argv[1]).read()
    out = {}
    for prefix in sys.argv[2:]:
        out[prefix], cnt = mix(asm, prefix)
        print(prefix, json.dumps(out[prefix], indent=1))
        print("  top:", cnt.most_common(25))
    return out


if __name__ == "__main__":
    main()
