"""Summarise tools/pmc_mfma.sh into profiles/<round>_pmc_mfma.json.

Per kernel and config: the average over dispatches of SQ_VALU_MFMA_BUSY_CYCLES (MFMA-busy
cycles summed over every SIMD), GRBM_GUI_ACTIVE (GPU-busy cycles summed over the 8 XCDs,
MI355X_MICROARCH.md "DVFS give-back") and SQ_BUSY_CU_CYCLES, and
  kernel_cycles   = GRBM_GUI_ACTIVE / 8
  mfma_busy_frac  = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x kernel_cycles)
i.e. the fraction of the SIMDs' cycles (at whatever clock the chip ran) in which an MFMA
executed, and mfma_busy_frac_nominal_clock, the same busy cycles over 1024 x 2.4 GHz x the
dispatch's duration (the MFMA pass's timestamps) -- comparable with an ops fraction of the
nominal peak.  For k_oz_gemm16u the MFMA count is known exactly (16 n_oz-row residue Grams,
v_mfma_i32_16x16x64_i8 = 16 cycles each), which checks the counter's normalisation.
Usage: python tools/pmc_mfma_summary.py r04
"""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SIMDS = 1024
XCDS = 8


def short(name):
    return name.split("(")[0].replace("void ", "").strip()


def avgs(d, counter):
    """{kernel: (average counter value, dispatches, average duration in s)}"""
    tot, cnt, dur = {}, {}, {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != counter:
                continue
            k = short(r["Kernel_Name"])
            tot[k] = tot.get(k, 0.0) + float(r["Counter_Value"])
            cnt[k] = cnt.get(k, 0) + 1
            dur[k] = dur.get(k, 0.0) + (float(r["End_Timestamp"]) - float(r["Start_Timestamp"])) * 1e-9
    return {k: (tot[k] / cnt[k], cnt[k], dur[k] / cnt[k]) for k in tot}


def bench_line(d):
    for f in glob.glob(os.path.join(d, "*.json")):
        for line in open(f):
            if line.startswith("{"):
                return json.loads(line)
    return {}


def main():
    rnd = sys.argv[1]
    src = os.path.join(ROOT, "gpurun_out", f"pmc_mfma_{rnd}")
    shaf = os.path.join(src, "source_sha.txt")
    out = {"round": rnd, "source": "tools/pmc_mfma.sh (one counter per rocprofv3 --pmc pass)",
           "source_sha": open(shaf).read().strip() if os.path.exists(shaf) else None,
           "formula": "mfma_busy_frac = SQ_VALU_MFMA_BUSY_CYCLES / (1024 x GRBM_GUI_ACTIVE / 8)",
           "configs": {}}
    for cfg in sorted(os.listdir(src)):
        d = os.path.join(src, cfg)
        if not os.path.isdir(d):
            continue
        mf = avgs(os.path.join(d, "SQ_VALU_MFMA_BUSY_CYCLES"), "SQ_VALU_MFMA_BUSY_CYCLES")
        gr = avgs(os.path.join(d, "GRBM_GUI_ACTIVE"), "GRBM_GUI_ACTIVE")
        cu = avgs(os.path.join(d, "SQ_BUSY_CU_CYCLES"), "SQ_BUSY_CU_CYCLES")
        bl = bench_line(d)
        c = bl.get("config", {})
        ent = {"workload": c.get("workload"), "n": c.get("n"), "p": c.get("p"),
               "gram": c.get("gram"), "kernels": {}}
        for k in sorted(set(mf) | set(gr)):
            e = {"dispatches": (mf.get(k) or gr.get(k))[1]}
            if k in mf:
                e["SQ_VALU_MFMA_BUSY_CYCLES"] = mf[k][0]
            if k in gr:
                e["GRBM_GUI_ACTIVE"] = gr[k][0]
                e["kernel_cycles"] = gr[k][0] / XCDS
                # the dispatch's own duration in the profiled pass (counter-collection
                # timestamps) and the clock it implies (MI355X_MICROARCH.md: reads high for
                # dispatches shorter than ~0.3 ms)
                e["duration_ms_profiled"] = gr[k][2] * 1e3
                e["effective_clock_GHz"] = gr[k][0] / XCDS / gr[k][2] / 1e9
            if k in cu:
                e["SQ_BUSY_CU_CYCLES"] = cu[k][0]
            if k in mf and k in gr and gr[k][0] > 0:
                e["mfma_busy_frac"] = mf[k][0] / (SIMDS * gr[k][0] / XCDS)
                # the same busy cycles against the nominal 2.4 GHz over the MFMA pass's own
                # duration: comparable with the roofline's ops fraction at nominal peak
                e["mfma_busy_frac_nominal_clock"] = mf[k][0] / (SIMDS * 2.4e9 * mf[k][2])
            if k.startswith("bb::k_oz_gemm16u") and c.get("n"):
                n, p = int(c["n"]), int(c["p"])
                n_oz = -(-(-(-n // 128) * 128) // 256) * 256
                p_pad = -(-p // 256) * 256
                nt = n_oz // 256
                # tiles computed: off-diagonal full + diagonal lower halves, 16 moduli
                macs = 16 * (nt * (nt - 1) / 2 * 256 * 256 + nt * 256 * 128 + nt * 256 * 8) * p_pad
                e["mfma_instructions_model"] = macs / (16 * 16 * 64)
                e["busy_cycles_model_16_per_mfma"] = 16 * macs / (16 * 16 * 64)
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
    dst = os.path.join(ROOT, "profiles", f"{rnd}_pmc_mfma.json")
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
