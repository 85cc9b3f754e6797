"""The reference's published benchmark, replicated like for like.

Protocol (Notes/bbnotes.tex:893-965, Code/R/PublicBenchmark.R:140-310): for each design and
method, 10 simulations of 100 000 samples after 10 000 burn-in sweeps, alpha = 0.5, sig2
Jeffreys, nu = tau^-alpha ~ Ga(2, rate = 2); per simulation the coda effectiveSize of every
beta_j (sum.stat, :112-134); per coefficient the median over the simulations (table.info,
:276-305, `apply(info$stb.stat[,colnum,], 1, median)`); the table reports min / median /
max / sd of those per-coefficient values and the median runtime.  ESR = ESS / runtime.

Designs (the reference's data(diabetes), man/diabetes.Rd:22: "x has been standardized to
have unit L2 norm in each column and zero mean"):
  DB   = sklearn's load_diabetes(scaled=True) -- the same Efron et al. data, columns centred
         and scaled to unit L2 norm -- and y = the raw target, centred (:331-341);
  DBI  = x2: the 10 columns of DB, the 9 squares (sex is binary) and the 45 pairwise
         products, in lars' column order (main effects, squares, interactions), each
         centred and scaled to unit L2 norm (lars' quadratic model).  The order matters only
         for the orthogonalised runs (Q of the QR depends on it);
  orth = Q of the QR of the centred design, qr.Q(qr(X)) (unit columns, :485-488), run with
         ortho = TRUE.
The Boston Housing designs need mlbench's data, absent offline, so only DB / DBI are
compared with the published ESS.

Beside each GPU row: the compiled CPU chain (oracle/bb_cpu_chain.c, reference-literal
p x p dpotrf / the ortho draw, scipy OpenBLAS, 1 thread) on the same design, one simulation
of CPU_SAMPLES samples, for sweeps/s side by side.  Output: one JSON document on stdout.
Usage: python tools/published_ess.py OUT.json  (the library's .C drivers print to stdout,
so the document is written to the file named on the command line)
"""
import itertools
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bayesbridge_amd as bb  # noqa: E402
from bayesbridge_amd.diagnostics import effective_size  # noqa: E402

# Notes/bbnotes.tex:901-925 (general design) and :946-978 (orthogonal design):
# (time s, ESS min, med, max, sd)
PUBLISHED = {
    ("DB", "tri"): (1.51, 9744.17, 16583.07, 45168.14, 10901.50),
    ("DB", "stable"): (4.80, 28727.55, 54360.66, 98428.62, 24566.58),
    ("DBI", "tri"): (45.12, 227.78, 674.99, 1582.25, 232.56),
    ("DBI", "stable"): (68.68, 17924.24, 60873.07, 91261.17, 18936.41),
    ("DB", "tri_orth"): (1.20, 56884.02, 67798.11, 95013.04, 11393.50),
    ("DB", "stable_orth"): (4.06, 64337.74, 83198.38, 97460.85, 10473.23),
    ("DBI", "tri_orth"): (8.69, 20692.11, 66531.77, 100000.0, 24770.91),
    ("DBI", "stable_orth"): (25.30, 32037.12, 76789.69, 100000.0, 20687.61),
}


# Effective sampling rate, ESS / runtime (Notes/bbnotes.tex:913-925 general, :967-979
# orthogonal): (min, med, max, sd) over coefficients
PUBLISHED_ESR = {
    ("DB", "tri"): (6412.15, 10979.52, 29850.64, 7212.68),
    ("DB", "stable"): (6006.14, 11312.78, 20522.83, 5118.33),
    ("DBI", "tri"): (5.06, 14.98, 35.10, 5.16),
    ("DBI", "stable"): (261.86, 886.12, 1320.26, 276.42),
    ("DB", "tri_orth"): (47343.30, 56407.57, 79058.63, 9447.09),
    ("DB", "stable_orth"): (15842.58, 20500.59, 23991.48, 2581.22),
    ("DBI", "tri_orth"): (2377.19, 7675.35, 11531.89, 2848.33),
    ("DBI", "stable_orth"): (1267.65, 3029.24, 3965.43, 817.16),
}


def esr_stats(ess, rts):
    """Per coefficient the median over simulations of ESS_s / runtime_s; min / median / max /
    sd over coefficients (the published ESR rows, bbnotes.tex:1005-1012)."""
    per = np.median(np.array(ess) / np.array(rts)[:, None], axis=0)
    return {"min": float(per.min()), "median": float(np.median(per)), "max": float(per.max()),
            "sd": float(np.std(per, ddof=1))}


def unit_l2(Z):
    Z = Z - Z.mean(axis=0)
    return Z / np.linalg.norm(Z, axis=0)


def designs():
    from sklearn.datasets import load_diabetes
    d = load_diabetes(scaled=True)  # centred, unit L2 columns: the lars diabetes$x
    X = unit_l2(d.data)
    y = d.target - d.target.mean()
    cols = [X[:, i] for i in range(10)]
    cols += [X[:, i] ** 2 for i in range(10) if i != 1]  # sex is binary: no square
    cols += [X[:, i] * X[:, j] for i, j in itertools.combinations(range(10), 2)]
    X2 = unit_l2(np.column_stack(cols))
    assert X2.shape == (442, 64)
    return {"DB": (X, y), "DBI": (X2, y)}


def qr_q(X):
    return np.linalg.qr(X)[0]


def gpu_run(X, y, method, nsamp, burn, seed):
    bb.set_seed(seed)
    orth = method.endswith("_orth")
    if method.startswith("tri"):
        out = bb.bridge_reg_tri(y, X, nsamp=nsamp, burn=burn, ortho=orth)
    else:
        out = bb.bridge_reg_stb(y, X, nsamp=nsamp, burn=burn, ortho=orth)
    return out["beta"], out["runtime"]


def cpu_run(X, y, method, nsamp, burn):
    import oracle
    if method.startswith("tri"):
        return None
    r = oracle.cpu_chain(y, X, nsamp, burn=burn, method="ortho" if method.endswith("_orth")
                         else "chol", seed=1, threads=1, record=False)
    return nsamp / r["runtime"]


def cpu_protocol(X, y, method, nsamp, burn, nsim):
    """The compiled CPU chain (reference-literal, 1 core) under the full published protocol:
    its ESS and ESR beside the GPU's (stable methods only)."""
    import oracle
    if method.startswith("tri"):
        return None
    ess, rts = [], []
    for s in range(nsim):
        r = oracle.cpu_chain(y, X, nsamp, burn=burn, method="ortho" if method.endswith("_orth")
                             else "chol", seed=1000 + s, threads=1)
        ess.append(effective_size(r["beta"].T))
        rts.append(r["runtime"])
    per = np.median(np.array(ess), axis=0)
    return {"runtime_s": float(np.median(rts)), "threads": 1,
            "ess": {"min": float(per.min()), "median": float(np.median(per)),
                    "max": float(per.max()), "sd": float(np.std(per, ddof=1))},
            "esr": esr_stats(ess, rts)}


def main():
    nsamp = int(os.environ.get("NSAMP", "100000"))
    burn = int(os.environ.get("BURN", "10000"))
    nsim = int(os.environ.get("NSIM", "10"))
    cpu_samples = int(os.environ.get("CPU_SAMPLES", "20000"))
    only_m = os.environ.get("METHODS", "stable,tri,stable_orth,tri_orth").split(",")
    only_d = os.environ.get("DESIGNS", "DB,DBI").split(",")
    bb.set_verbose(0)
    rows = []
    for name, (X0, y) in designs().items():
        if name not in only_d:
            continue
        for method in only_m:
            X = qr_q(X0) if method.endswith("_orth") else X0
            ess, rts = [], []
            for s in range(nsim):
                t0 = time.perf_counter()
                beta, rt = gpu_run(X, y, method, nsamp, burn, seed=1000 + s)
                ess.append(effective_size(beta))
                rts.append(rt)
                print(f"[{name} {method}] sim {s}: runtime {rt:.2f} s (wall "
                      f"{time.perf_counter() - t0:.1f} s), ESS median {np.median(ess[-1]):.0f}",
                      file=sys.stderr, flush=True)
            per_coef = np.median(np.array(ess), axis=0)  # table.info: median over simulations
            rt = float(np.median(rts))
            rec = {"design": name, "method": method, "n": X.shape[0], "p": X.shape[1],
                   "simulations": nsim, "nsamp": nsamp, "burn": burn,
                   "runtime_s": rt, "sweeps_per_s": nsamp / rt,
                   "ess": {"min": float(per_coef.min()), "median": float(np.median(per_coef)),
                           "max": float(per_coef.max()), "sd": float(np.std(per_coef, ddof=1))},
                   "esr": esr_stats(ess, rts)}
            pub = PUBLISHED.get((name, method))
            if pub:
                rec["published"] = {"runtime_s": pub[0], "sweeps_per_s": 100000 / pub[0],
                                    "ess": dict(zip(("min", "median", "max", "sd"), pub[1:])),
                                    "esr": dict(zip(("min", "median", "max", "sd"),
                                                    PUBLISHED_ESR[(name, method)])),
                                    "source": "Notes/bbnotes.tex:901-978 (2011 laptop)"}
                rec["esr_over_published_median"] = (rec["esr"]["median"]
                                                    / PUBLISHED_ESR[(name, method)][1])
            if os.environ.get("CPU_PROTOCOL", "0") == "1":
                rec["cpu_compiled_protocol"] = cpu_protocol(X, y, method, nsamp, burn, nsim)
            cpu = cpu_run(X, y, method, cpu_samples, min(burn, cpu_samples // 10))
            if cpu:
                rec["cpu_compiled_1core_sweeps_per_s"] = cpu
            rows.append(rec)
            print(json.dumps(rec), file=sys.stderr, flush=True)
    out = sys.argv[1] if len(sys.argv) > 1 else "/dev/stdout"
    with open(out, "w") as fh:
        fh.write(json.dumps({"protocol": f"{nsim} simulations x {nsamp} samples after {burn} burn-in, "
                                  "alpha = 0.5, sig2 Jeffreys, nu ~ Ga(2, 2) "
                                  "(Notes/bbnotes.tex:893-965)",
                      "ess": "coda effectiveSize per beta_j, median over simulations; "
                             "min / median / max / sd over coefficients",
                      "results": rows}, indent=1) + "\n")


if __name__ == "__main__":
    main()
