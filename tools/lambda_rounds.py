"""Rounds per tilted-stable draw at the C3 steady state (tail analysis of k_lambda).

  --dump: (GPU) run bench.py's C3 problem for --sweeps sweeps, save beta, tau to --state.
  default: (CPU) replay the lambda draws of that state with the oracle's attempt counters
  and print the distribution of group rounds for G-lane inner speculation: a draw takes
  sum over its outer attempts of ceil(inner attempts / G) rounds."""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def dump(args):
    import bayesbridge_amd as bb
    import bench
    n, p = 2000, 50000
    X = bench.make_columns(n, 0, p)
    y, _ = bench.make_problem_y(n, p)
    cfg = bb.EngineConfig(n=n, p=p, p_local=p, true_alpha=0.5, method=2, trace_capacity=1,
                          seed=0xB4E5B41D6E, stream=0)
    eng = bb.Engine(cfg, X, y)
    del X
    eng.init_state()
    eng.run(1, args.sweeps, first_slot=-1)
    eng.sync()
    st = eng.state()
    np.savez(args.state, beta=st["beta"], tau=st["tau"])
    print("saved", args.state, "tau", st["tau"])


def analyze(args):
    import oracle
    d = np.load(args.state)
    beta, tau = d["beta"], float(d["tau"])
    h = beta * beta / (tau * tau)
    p = h.size
    idx = np.arange(p) if args.sample <= 0 else np.linspace(0, p - 1, args.sample).astype(int)
    rounds = {g: [] for g in (8, 16, 64)}
    outer = []
    for j in idx:
        # replay the draw attempt by attempt: per outer attempt, how many inner attempts
        x, no, ni = oracle.retstable(h[j], 0.25, 1.0, seed=1, stream=0, t=5, j=int(j),
                                     counts=True)
        outer.append(no)
        rounds_j = {g: 0 for g in rounds}
        # the oracle reports totals; per-outer inner counts need the per-attempt replay below
        rounds_j = None
        rounds[8].append((no, ni))
    no = np.array([r[0] for r in rounds[8]])
    ni = np.array([r[1] for r in rounds[8]])
    print(f"draws {len(no)}: outer attempts mean {no.mean():.2f} max {no.max()}, "
          f"inner attempts mean {ni.mean():.2f} max {ni.max()}")
    for q in (0.5, 0.9, 0.99, 0.999, 1.0):
        print(f"  quantile {q}: outer {np.quantile(no, q):.0f} inner {np.quantile(ni, q):.0f}")
    # lower bound on G=8 rounds: max(outer, ceil(inner/8))
    r8 = np.maximum(no, np.ceil(ni / 8))
    print(f"  G=8 rounds >= {r8.mean():.2f} mean, max {r8.max():.0f}; "
          f"share of draws with >= 5 rounds {np.mean(r8 >= 5):.4f}")


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--dump", action="store_true")
    ap.add_argument("--sweeps", type=int, default=300)
    ap.add_argument("--state", default="gpurun_out/c3_state.npz")
    ap.add_argument("--sample", type=int, default=0)
    a = ap.parse_args()
    dump(a) if a.dump else analyze(a)
