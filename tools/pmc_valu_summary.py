"""Summarise tools/pmc_valu.sh into profiles/<round>_pmc_valu.json, and tools/pmc_valu_classes.sh
into profiles/<round>_valu_costs.json (--classes).

Per kernel and config, averages over the TIMED dispatches (the last `steps` dispatches of the
kernel in the profiled bench run, whose sweeps are the ones bench.py times) of SQ_INSTS_VALU
(VALU instructions issued, summed over waves), SQ_ACTIVE_INST_VALU, GRBM_GUI_ACTIVE and the
per-class counts SQ_INSTS_VALU_{FMA,MUL,ADD,TRANS}_{F64,F32}, _INT32, _INT64, _CVT, and

  issue_cycles = sum over classes of count x cycles per wave64 instruction on one SIMD
                 (measured, tools/valu_rate.hip: f64 FMA/MUL/ADD 4, f64 transcendental 16,
                 f32 transcendental 8, f32 FMA/MUL/ADD 2, INT64 4; INT32, CVT and the
                 instructions no class counts (OTHER = SQ_INSTS_VALU - sum of the classes) at
                 the average cost of their members in the kernel's own ISA, tools/isa_mix.py),
                 with issue_cycles_low / _high pricing INT32, CVT and OTHER at 2 and at 4;
  valu_issue_frac_nominal = issue_cycles / (1024 SIMDs x 2.4 GHz x the dispatch duration).

Every summary carries the source_sha of the tree that was profiled; bench.py uses it only
for the same tree.
Usage: python tools/pmc_valu_summary.py r05 [asm]     (asm: hipcc -S output of bb_kernels.hip;
                                                        compiled here when omitted)
       python tools/pmc_valu_summary.py --classes r05
"""
import csv
import glob
import json
import os
import re
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_mfma_summary import ROOT, SIMDS, short  # noqa: E402

CLASSES = ("FMA_F64", "MUL_F64", "ADD_F64", "TRANS_F64", "FMA_F32", "MUL_F32", "ADD_F32",
           "TRANS_F32", "INT32", "INT64", "CVT")
# measured issue cycles per wave64 instruction on one SIMD (profiles/r05_valu_costs.json)
FIXED_COST = {"FMA_F64": 4, "MUL_F64": 4, "ADD_F64": 4, "TRANS_F64": 16, "FMA_F32": 2,
              "MUL_F32": 2, "ADD_F32": 2, "TRANS_F32": 8, "INT64": 4}
MIXED = ("INT32", "CVT", "OTHER")


def read_sha(d):
    f = os.path.join(d, "source_sha.txt")
    return open(f).read().strip() if os.path.exists(f) else None


def dispatches(d, counter):
    """{kernel: [(value, duration s), ...] in dispatch order}"""
    out = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        rows = [r for r in csv.DictReader(open(f)) if r.get("Counter_Name") == counter]
        rows.sort(key=lambda r: int(r["Dispatch_Id"]))
        for r in rows:
            out.setdefault(short(r["Kernel_Name"]), []).append(
                (float(r["Counter_Value"]),
                 (float(r["End_Timestamp"]) - float(r["Start_Timestamp"])) * 1e-9))
    return out


def bench_line(d):
    for f in sorted(glob.glob(os.path.join(d, "*.json"))):
        for line in open(f):
            if line.startswith("{"):
                return json.loads(line)
    return {}


def mangled_prefix(name):
    """bb::k_lambda_xu<8, 8> -> _ZN2bb11k_lambda_xuILi8ELi8EE (int / bool template args)"""
    m = re.match(r"bb::(\w+)(?:<(.*)>)?$", name)
    base, args = m.group(1), m.group(2)
    s = f"_ZN2bb{len(base)}{base}"
    if args:
        s += "I"
        for a in (x.strip() for x in args.split(",")):
            s += {"true": "Lb1E", "false": "Lb0E"}.get(a, f"Li{a}E")
        s += "E"
    return s


def static_costs(asm_text, kernel):
    import isa_mix

    mix, _ = isa_mix.mix(asm_text, mangled_prefix(kernel))
    return {k: mix[k]["avg_cycles"] for k in MIXED if k in mix}


def main_counts(rnd, asm_path):
    src = os.path.join(ROOT, "gpurun_out", f"pmc_valu_{rnd}")
    if asm_path is None:
        # the kernels live in bb_kernels.hip and bb_nid.hip (the split lambda launch)
        parts = []
        for src_name in ("bb_kernels.hip", "bb_nid.hip"):
            path = f"/tmp/{src_name}_isa.s"
            subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3",
                                   "-std=c++17", "-ffp-contract=off",
                                   f"-I{os.path.join(ROOT, 'include')}", "--cuda-device-only",
                                   "-S", "-o", path,
                                   os.path.join(ROOT, "bayesbridge_amd", "csrc", src_name)])
            parts.append(open(path).read())
        asm = "\n".join(parts)
    else:
        asm = open(asm_path).read()
    out = {"round": rnd, "source": "tools/pmc_valu.sh (one counter per rocprofv3 --pmc pass)",
           "source_sha": read_sha(src), "cost_model": {
               "fixed_cycles": FIXED_COST,
               "mixed": "INT32, CVT, OTHER at the average cycles of their members in the "
                        "kernel's ISA (tools/isa_mix.py); _low / _high at 2 / 4",
               "peak": "1024 SIMDs x 2.4 GHz issue cycles"}, "configs": {}}
    for cfg in sorted(os.listdir(src)):
        d = os.path.join(src, cfg)
        if not os.path.isdir(d):
            continue
        bl = bench_line(d)
        steps = int(bl.get("steps", 0)) or None
        ent = {"workload": bl.get("config", {}).get("workload"), "n": bl.get("config", {}).get("n"),
               "p": bl.get("config", {}).get("p"), "timed_dispatches": steps,
               "window": {"steps": bl.get("steps"), "warmup": bl.get("warmup")}, "kernels": {}}
        per = {}
        for cd in sorted(os.listdir(d)):
            if os.path.isdir(os.path.join(d, cd)):
                for k, v in dispatches(os.path.join(d, cd), cd).items():
                    per.setdefault(k, {})[cd] = v[-steps:] if steps else v
        for k, ctrs in sorted(per.items()):
            if not k.startswith("bb::k_lambda"):
                continue
            e = {}
            for c, v in ctrs.items():
                e[c] = sum(x for x, _ in v) / len(v)
                e["dispatches_averaged"] = len(v)
            dur = [t for _, t in ctrs.get("SQ_INSTS_VALU", [])]
            if not dur:
                continue
            e["duration_ms_profiled"] = 1e3 * sum(dur) / len(dur)
            counted = {c: e.get("SQ_INSTS_VALU_" + c) for c in CLASSES}
            if any(v is None for v in counted.values()):
                ent["kernels"][k] = e
                continue
            other = e["SQ_INSTS_VALU"] - sum(counted.values())
            counted["OTHER"] = other
            sc = static_costs(asm, k)
            cyc = {c: (FIXED_COST[c] if c in FIXED_COST else sc.get(c, 3.0)) for c in counted}
            e["class_counts"] = counted
            e["class_cycles"] = cyc
            e["issue_cycles"] = sum(counted[c] * cyc[c] for c in counted)
            e["issue_cycles_low"] = sum(counted[c] * (FIXED_COST.get(c) or 2) for c in counted)
            e["issue_cycles_high"] = sum(counted[c] * (FIXED_COST.get(c) or 4) for c in counted)
            sec = e["duration_ms_profiled"] * 1e-3
            e["valu_issue_frac_nominal"] = e["issue_cycles"] / (SIMDS * 2.4e9 * sec)
            if e.get("GRBM_GUI_ACTIVE"):
                e["valu_issue_frac_busy_clock"] = e["issue_cycles"] / (SIMDS * e["GRBM_GUI_ACTIVE"] / 8)
            if e.get("SQ_ACTIVE_INST_VALU") and e.get("GRBM_GUI_ACTIVE"):
                e["valu_busy_frac"] = 4.0 * e["SQ_ACTIVE_INST_VALU"] / (SIMDS * e["GRBM_GUI_ACTIVE"] / 8)
            ent["kernels"][k] = e
        out["configs"][cfg] = ent
    # the code identity of every profiled kernel (kernel_code.json, written on the GPU box
    # from the library it ran): bench.py uses an entry while the kernel's code is unchanged
    kcf = os.path.join(src, "kernel_code.json")
    if os.path.exists(kcf):
        sys.path.insert(0, ROOT)
        from bayesbridge_amd import _kernel_code
        shas = json.load(open(kcf))
        maps = [out["kernels"]] if isinstance(out.get("kernels"), dict) else []
        maps += [c["kernels"] for c in out.get("configs", {}).values() if "kernels" in c]
        for m in maps:
            _kernel_code.annotate(m, shas)
        out["code_sha_from"] = "kernel_code.json written on the GPU box from the profiled library"
    dst = os.path.join(ROOT, "profiles", f"{rnd}_pmc_valu.json")
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps(out, indent=1))


def main_classes(rnd):
    src = os.path.join(ROOT, "gpurun_out", f"valu_classes_{rnd}")
    rates = {}
    names = []
    for ln in open(os.path.join(src, "rates.txt")):
        m = re.match(r"(\S+)\s+W=(\d+)\s+([\d.]+) cyc", ln)
        if m:
            if m.group(2) not in ("1", "2", "4"):
                continue
            if m.group(1) not in rates:
                names.append(m.group(1))
            rates.setdefault(m.group(1), {})[f"W{m.group(2)}"] = float(m.group(3))
    tot = {}
    for d in sorted(glob.glob(os.path.join(src, "SQ_INSTS_VALU*"))):
        if not os.path.isdir(d):
            continue
        ctr = os.path.basename(d)
        agg = {}
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                m = re.search(r"k_rate<(\d+)>", r["Kernel_Name"])
                if m:
                    agg[int(m.group(1))] = agg.get(int(m.group(1)), 0.0) + float(r["Counter_Value"])
        tot[ctr] = agg
    out = {"round": rnd, "source": "tools/valu_rate.hip + tools/pmc_valu_classes.sh",
           "source_sha": read_sha(src),
           "cycles": "per wave64 instruction per SIMD (workgroup span of W waves per SIMD on "
                     "every CU, 8 independent chains per wave; includes the loop's own overhead, "
                     "~0.5 cycles)", "instructions": {}}
    for i, nm in enumerate(names):
        v = tot.get("SQ_INSTS_VALU", {}).get(i, 0.0)
        fr = {c.replace("SQ_INSTS_VALU_", ""): round(t.get(i, 0.0) / v, 3)
              for c, t in tot.items() if c != "SQ_INSTS_VALU" and v}
        cls = [c for c, x in fr.items() if x > 0.5]
        out["instructions"][nm] = {"cycles": rates.get(nm), "class": cls[0] if cls else "OTHER",
                                   "class_fractions": fr}
    dst = os.path.join(ROOT, "profiles", f"{rnd}_valu_costs.json")
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    if sys.argv[1] == "--classes":
        main_classes(sys.argv[2])
    else:
        main_counts(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
