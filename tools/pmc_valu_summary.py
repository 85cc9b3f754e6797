"""Summarise tools/pmc_valu.sh into profiles/<round>_pmc_valu.json.

Per kernel and config, averages over dispatches of SQ_INSTS_VALU (VALU instructions issued,
summed over waves), SQ_ACTIVE_INST_VALU (quad-cycles waves spend executing VALU
instructions, MI355X_MICROARCH.md), SQ_WAVE_CYCLES, SQ_BUSY_CYCLES and GRBM_GUI_ACTIVE (GPU
cycles summed over the 8 XCDs), the dispatch duration from the counter-collection
timestamps, and
  kernel_cycles        = GRBM_GUI_ACTIVE / 8
  valu_busy_frac       = 4 SQ_ACTIVE_INST_VALU / (1024 SIMDs x kernel_cycles)
  valu_issue_frac      = SQ_INSTS_VALU / (1024 SIMDs x kernel_cycles / 4)
                         (one wave64 VALU instruction per 4 cycles per SIMD)
  valu_issue_frac_nominal = the same at 2.4 GHz over the dispatch duration.
Usage: python tools/pmc_valu_summary.py r04
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_mfma_summary import ROOT, SIMDS, XCDS, avgs, bench_line  # noqa: E402

COUNTERS = ("SQ_INSTS_VALU", "SQ_ACTIVE_INST_VALU", "GRBM_GUI_ACTIVE", "SQ_WAVE_CYCLES",
            "SQ_BUSY_CYCLES")


def main():
    rnd = sys.argv[1]
    src = os.path.join(ROOT, "gpurun_out", f"pmc_valu_{rnd}")
    out = {"round": rnd, "source": "tools/pmc_valu.sh (one counter per rocprofv3 --pmc pass)",
           "configs": {}}
    for cfg in sorted(os.listdir(src)):
        d = os.path.join(src, cfg)
        if not os.path.isdir(d):
            continue
        c = {k: avgs(os.path.join(d, k), k) for k in COUNTERS}
        bl = bench_line(d).get("config", {})
        ent = {"workload": bl.get("workload"), "n": bl.get("n"), "p": bl.get("p"), "kernels": {}}
        names = set()
        for v in c.values():
            names |= set(v)
        for k in sorted(names):
            e = {}
            for ctr, v in c.items():
                if k in v:
                    e[ctr] = v[k][0]
                    e["dispatches"] = v[k][1]
            g = c["GRBM_GUI_ACTIVE"].get(k)
            if g and g[0] > 0:
                cyc = g[0] / XCDS
                e["kernel_cycles"] = cyc
                e["duration_ms_profiled"] = g[2] * 1e3
                e["effective_clock_GHz"] = cyc / g[2] / 1e9
                if "SQ_ACTIVE_INST_VALU" in e:
                    e["valu_busy_frac"] = 4.0 * e["SQ_ACTIVE_INST_VALU"] / (SIMDS * cyc)
                if "SQ_INSTS_VALU" in e:
                    e["valu_issue_frac"] = e["SQ_INSTS_VALU"] / (SIMDS * cyc / 4.0)
                    dur = c["SQ_INSTS_VALU"][k][2]
                    e["valu_issue_frac_nominal"] = e["SQ_INSTS_VALU"] / (SIMDS * 2.4e9 * dur / 4.0)
            ent["kernels"][k] = e
        out["configs"][cfg] = ent
    dst = os.path.join(ROOT, "profiles", f"{rnd}_pmc_valu.json")
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
