"""Turn a tools/profile_round.sh output directory into the committed round summaries:
  profiles/<round>_kernel_stats.csv   rocprofv3 --stats table (copied as is)
  profiles/<round>_kernel_stats.txt   the same, sorted, with % of GPU time
  profiles/<round>_pmc.json           per-kernel average FETCH_SIZE / WRITE_SIZE per dispatch

FETCH_SIZE / WRITE_SIZE are KB (x1024).  On gfx950 FETCH_SIZE reports 1/2 of the bytes of a
wide coalesced streaming read (MI355X_MICROARCH.md HBM section), so read bytes are taken as
2 x FETCH_SIZE x 1024; the fused beta pass (k_beta_wb_xb, or k_xv on the fp64-Gram path),
which streams X exactly once with known bytes, is reported beside it as an in-run
calibration of that factor.
Usage: python tools/profile_summary.py r01 [n] [p]
The workload (n, p, design) is read from the profiled bench line (kt_bench.json) when it is
there, so `ROUND=r02c5 bash tools/profile_round.sh --workload c5` followed by
`python tools/profile_summary.py r02c5` summarises C5 (bench.py picks the file by n, p).
"""
import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def one(pattern):
    hits = glob.glob(pattern, recursive=True)
    if not hits:
        raise SystemExit(f"missing {pattern}")
    return hits[0]


def short(name):
    return name.split("(")[0].replace("void ", "").strip()


def pmc_avgs(path, counter):
    tot, cnt = {}, {}
    for r in csv.DictReader(open(path)):
        if r.get("Counter_Name") != counter:
            continue
        k = short(r["Kernel_Name"])
        tot[k] = tot.get(k, 0.0) + float(r["Counter_Value"])
        cnt[k] = cnt.get(k, 0) + 1
    return {k: (tot[k] / cnt[k], cnt[k]) for k in tot}


def main():
    rnd = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 2000
    p = int(sys.argv[3]) if len(sys.argv) > 3 else 50000
    src = os.path.join(ROOT, "gpurun_out", f"prof_{rnd}")
    bench, cfg = {}, {}
    try:  # the bench line the kernel-trace pass printed
        line = [l for l in open(os.path.join(src, "kt_bench.json")) if l.startswith("{")][-1]
        bench = json.loads(line)
        cfg = dict(bench.get("config", {}))
        n, p = int(cfg.get("n", n)), int(cfg.get("p", p))
        cfg["_steps"] = f"--steps {bench.get('steps')} --warmup {bench.get('warmup')} "
    except (OSError, IndexError, ValueError):
        pass
    wl = cfg.get("workload", "")
    logit, sparse = "logistic" in wl, "sparse" in wl
    dst = os.path.join(ROOT, "profiles")
    os.makedirs(dst, exist_ok=True)
    ks = one(os.path.join(src, "kt", "**", "*kernel_stats.csv"))
    shutil.copy(ks, os.path.join(dst, f"{rnd}_kernel_stats.csv"))
    rows = list(csv.DictReader(open(ks)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    steps = cfg.get("_steps", "")
    lines = [f"# rocprofv3 --kernel-trace --stats of: python3 bench.py {steps}"
             f"--no-cpu-baseline ({wl or f'n={n}, p={p}'}, 1 GPU)",
             f"{'kernel':48s} {'calls':>6s} {'avg_us':>10s} {'min_us':>10s} {'tot_ms':>9s}  share"]
    avg_us = {}
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
        k = short(r["Name"])
        avg_us[k] = float(r["AverageNs"]) / 1e3
        lines.append(f"{k[:48]:48s} {r['Calls']:>6s} {float(r['AverageNs']) / 1e3:10.2f} "
                     f"{float(r['MinNs']) / 1e3:10.2f} {float(r['TotalDurationNs']) / 1e6:9.2f} "
                     f"{100 * float(r['TotalDurationNs']) / tot:5.1f}%")
    open(os.path.join(dst, f"{rnd}_kernel_stats.txt"), "w").write("\n".join(lines) + "\n")
    fetch = pmc_avgs(one(os.path.join(src, "fetch", "**", "*counter_collection.csv")), "FETCH_SIZE")
    write = pmc_avgs(one(os.path.join(src, "write", "**", "*counter_collection.csv")), "WRITE_SIZE")
    n_pad = -(-n // 128) * 128
    p_pad = -(-p // 256) * 256
    x_bytes = 8.0 * n_pad * p_pad
    shaf = os.path.join(src, "source_sha.txt")
    out = {"round": rnd, "source_sha": open(shaf).read().strip() if os.path.exists(shaf) else None,
           "workload": {"n": n, "p": p, "n_pad": n_pad, "p_pad": p_pad},
           # the profiled bench window (every pass ran it): bench.py matches the per-sweep
           # kernels' traffic on it; "fitted": the run included the fitted-regime sweeps
           "window": {"steps": bench.get("steps"), "warmup": bench.get("warmup"),
                      "fitted": bench.get("fitted_regime") is not None},
           "units": "bytes per dispatch (average over the profiled dispatches)",
           "correction": "read_bytes = 2 x FETCH_SIZE x 1024 (gfx950 1/2 reporting of wide "
                         "streaming reads); write_bytes = WRITE_SIZE x 1024",
           "kernels": {}}
    for k in sorted(set(fetch) | set(write)):
        f_kb, fc = fetch.get(k, (float("nan"), 0))
        w_kb, wc = write.get(k, (float("nan"), 0))
        out["kernels"][k] = {"fetch_kb": f_kb, "write_kb": w_kb, "dispatches": max(fc, wc),
                             "read_bytes": 2 * 1024 * f_kb, "write_bytes": 1024 * w_kb,
                             "hbm_bytes": 2 * 1024 * f_kb + 1024 * w_kb,
                             "avg_us": avg_us.get(k)}
    # the fused beta pass (k_beta_wb_xb<NR, nt>: whatever instance ran) or the fp64 path's k_xv
    cands = [k for k in out["kernels"] if k.startswith("bb::k_beta_wb_xb<")] + ["bb::k_xv"]
    for kname in cands:
        if kname in out["kernels"]:
            kx = out["kernels"][kname]
            out["calibration"] = {"kernel": kname, "algorithmic_read_bytes": x_bytes,
                                  "fetch_x1024": 1024 * kx["fetch_kb"],
                                  "ratio_algorithmic_over_fetch":
                                      x_bytes / (1024 * kx["fetch_kb"])}
            break
    # the Gram GEMM kernels: fp64 k_gram reads X (+D) and writes n_pad^2 partials per split;
    # k_oz_gemm reads the 16 int8 residue planes (16 n_oz p_pad bytes) and writes partials
    # (the logistic Gram X' diag(omega) X has rows = coefficients and K = observations)
    rows_pad, k_pad = (p_pad, n_pad) if logit else (n_pad, p_pad)
    n_oz = -(-rows_pad // 256) * 256
    algo = {"bb::k_gram": x_bytes + 8.0 * p_pad + 8.0 * n_pad ** 2,
            "bb::k_oz_residues": x_bytes + 16.0 * n_oz * k_pad}
    for k in out["kernels"]:  # production GEMM instantiation(s): dbg = 0
        if k.startswith("bb::k_oz_gemm") and "<0" in k:
            algo[k] = 16.0 * n_oz * k_pad
    if sparse:  # the pair-list Gram's algorithmic bytes as bench.py counts them
        rf = bench["roofline"] if bench["roofline"].get("phase") == "gram" else \
            (bench.get("roofline_secondary") or {})
        algo = {k: rf.get("algorithmic_bytes_per_launch") for k in out["kernels"]
                if k.startswith("bb::k_sp_gram_col") or k.startswith("bb::k_sp_gram_flat")}
    out["workload"]["name"] = wl or None
    out["gram_kernels"] = {}
    for k, a in algo.items():
        if k in out["kernels"]:
            g = out["kernels"][k]
            out["gram_kernels"][k] = {"hbm_bytes_per_launch": g["hbm_bytes"],
                                      "algorithmic_bytes_per_launch": a, "avg_us": g["avg_us"]}
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
    json.dump(out, open(os.path.join(dst, f"{rnd}_pmc.json"), "w"), indent=1)
    print("\n".join(lines[:16]))
    print(json.dumps({k: v for k, v in out.items() if k != "kernels"}, indent=1))


if __name__ == "__main__":
    main()
