"""Dump chain states of a bench workload from the reference start (GPU engine, bench.py's X, y
and key) for the near-identity bound study: every sweep's certified eps and
Chebyshev iterate count K, and at the listed sweeps the state (lambda, tau, sig2) whose system
that sweep solved.  Output: gpurun_out/<workload>_states.npz.

    python tools/c3_states.py [--workload c3] [--sweeps 1100] [--at 20,100,...]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import bench
    import bayesbridge_amd as bb

    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c3")
    ap.add_argument("--sweeps", type=int, default=1100)
    ap.add_argument("--at", default="20,50,100,200,300,400,500,600,700,800,900,1000,1100")
    ap.add_argument("--tuning", action="append", default=[])
    a = ap.parse_args()
    for kv in a.tuning:
        k, v = kv.split("=")
        bb.set_tuning(int(k), int(v))
    n, p, alpha, kind = bench.WORKLOADS[a.workload]
    X = bench.make_columns(n, 0, p)
    y, _ = bench.make_problem_y(n, p)
    bb.set_verbose(0)
    e = bb.Engine(bb.EngineConfig(n=n, p=p, seed=0xB4E5B41D6E, stream=0, true_alpha=alpha,
                                  trace_capacity=1), X, y)
    e.init_state()
    at = sorted(int(s) for s in a.at.split(","))
    eps, mode, keep = [], [], {}
    for t in range(1, a.sweeps + 1):
        e.run(t, 1, first_slot=-1)
        st = e.nid_stats()
        eps.append(st["eps"])
        mode.append(st["mode"])
        if t in at:
            s = e.state()
            keep[t] = (s["lambda"].copy(), s["tau"], s["sig2"])
            print(f"sweep {t}: eps {st['eps']:.3e} K {st['mode']} tau {s['tau']:.3e} "
                  f"sig2 {s['sig2']:.4g}", flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    out = os.path.join(ROOT, "gpurun_out", f"{a.workload}_states.npz")
    ts = sorted(keep)
    np.savez_compressed(out, eps=np.array(eps), mode=np.array(mode), at=np.array(ts),
                        lam=np.array([keep[t][0] for t in ts]),
                        tau=np.array([keep[t][1] for t in ts]),
                        sig2=np.array([keep[t][2] for t in ts]),
                        lambda_x=e.nid_stats()["lambda_x"])
    print("wrote", out)
    e.close()


if __name__ == "__main__":
    main()
