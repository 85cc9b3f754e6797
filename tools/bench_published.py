"""The reference's published benchmark protocol on MI355X (Notes/bbnotes.tex
:893-965, Code/R/PublicBenchmark.R:112-190): 100 000 samples after 10 000 burn-in sweeps of
the normal-mixture (stable) and triangle samplers through the .C entry points, alpha = 0.5,
sig2 Jeffreys, nu = tau^-alpha ~ Ga(2, 2), reporting the post-burn runtime, sweeps/s and
coda-style ESS / ESR per coefficient (bayesbridge_amd.diagnostics).

Designs: DB = the diabetes data (sklearn's copy of Efron et al., the reference's
data(diabetes)); DBI = diabetes with interactions built like lars' x2 (10 main effects, 45
two-way interactions, 9 squares; 442 x 64); BH / BHI = synthetic Gaussian designs of the
Boston Housing shapes (506 x 13, 506 x 103) -- the dataset itself is not available offline.
"orth" = the design orthogonalised (X = Q R -> Q sqrt(n)), as the reference's orthogonal
runs.  Writes one JSON document to stdout.
"""
import itertools
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bayesbridge_amd as bb  # noqa: E402
from bayesbridge_amd.diagnostics import effective_size  # noqa: E402

PUBLISHED = {  # Notes/bbnotes.tex:901-965 (100k samples, seconds; ESR median)
    "DB": {"stable": 4.80, "stable_esr": 11313, "tri": 1.51, "stable_orth": 4.06},
    "DBI": {"stable": 68.68, "stable_esr": 886, "tri": 45.12, "stable_orth": 25.30},
    "BH": {"stable": 5.96, "stable_esr": 13226, "tri": 2.20, "stable_orth": 5.49},
    "BHI": {"stable": 197.59, "stable_esr": 251, "tri": 155.64, "stable_orth": 40.95},
}


def designs():
    from sklearn.datasets import load_diabetes
    d = load_diabetes(scaled=False)
    X = d.data - d.data.mean(axis=0)
    y = d.target - d.target.mean()
    out = {"DB": (X, y)}
    Z = (X - X.mean(0)) / X.std(0)
    cols = [Z[:, i] for i in range(10)]
    cols += [Z[:, i] * Z[:, j] for i, j in itertools.combinations(range(10), 2)]
    cols += [Z[:, i] ** 2 for i in range(10) if i != 1]  # sex is binary: no square
    Xi = np.column_stack(cols)
    Xi = (Xi - Xi.mean(0)) / Xi.std(0)
    out["DBI"] = (Xi, y)
    rng = np.random.default_rng(20240501)
    for name, p in (("BH", 13), ("BHI", 103)):
        Xs = rng.standard_normal((506, p))
        Xs -= Xs.mean(0)
        b = np.zeros(p)
        b[:6] = [3.0, -2.0, 1.5, -1.0, 2.5, 0.8]
        ys = Xs @ b + 2.0 * rng.standard_normal(506)
        out[name] = (Xs, ys - ys.mean())
    return out


def orth(X):
    Q, _ = np.linalg.qr(X)
    return Q * np.sqrt(X.shape[0])


def run(name, X, y, method, nsamp, burn):
    bb.set_seed(77)
    t0 = time.perf_counter()
    if method == "tri":
        out = bb.bridge_reg_tri(y, X, nsamp=nsamp, burn=burn, extras=True)
    else:
        out = bb.bridge_reg_stb(y, X, nsamp=nsamp, burn=burn, ortho=(method == "stable_orth"))
    wall = time.perf_counter() - t0
    rt = out["runtime"]
    ess = effective_size(out["beta"])
    rec = {"design": name, "n": X.shape[0], "p": X.shape[1], "method": method,
           "nsamp": nsamp, "burn": burn, "runtime_s": rt, "wall_s": wall,
           "sweeps_per_s": nsamp / rt if rt > 0 else None,
           "ess_median": float(np.median(ess)), "ess_min": float(ess.min()),
           "esr_median": float(np.median(ess) / rt) if rt > 0 else None}
    pub = PUBLISHED[name].get(method)
    if pub:
        rec["published_runtime_s"] = pub
        rec["speedup_vs_published"] = pub / rt * (nsamp / 100000) if rt > 0 else None
    if method == "stable":
        rec["published_esr_median"] = PUBLISHED[name]["stable_esr"]
    return rec


def main():
    nsamp = int(os.environ.get("NSAMP", "100000"))
    burn = int(os.environ.get("BURN", "10000"))
    bb.set_verbose(0)
    only_d = os.environ.get("DESIGNS", "DB,DBI,BH,BHI").split(",")
    only_m = os.environ.get("METHODS", "stable,tri,stable_orth").split(",")
    recs = []
    for name, (X, y) in designs().items():
        if name not in only_d:
            continue
        for method in only_m:
            Xm = orth(X) if method == "stable_orth" else X
            recs.append(run(name, Xm, y, method, nsamp, burn))
            print(json.dumps(recs[-1]), file=sys.stderr, flush=True)
    print(json.dumps({"protocol": "100k samples + 10k burn-in, alpha=0.5 (bbnotes.tex:893-965)",
                      "results": recs}, indent=1))


if __name__ == "__main__":
    main()
