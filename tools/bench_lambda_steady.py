"""Lambda-kernel group-size sweep on a steady-state C3 chain state (n=2000, p=50000).

The state comes from the GPU engine after `--sweeps` Gibbs sweeps (bench.py's synthetic
problem), so h = beta^2 / tau^2 has the distribution the timed loop meets.  One line per
group size G with the average launch time."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bayesbridge_amd as bb  # noqa: E402
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sweeps", type=int, default=200)
    args = ap.parse_args()
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
    beta, tau = st["beta"], st["tau"]
    print(f"state after {args.sweeps} sweeps: tau={tau:.3e}, "
          f"mean abs beta={float(abs(beta).mean()):.3e}", flush=True)
    # variant 0: inlined sampler; 1: sampler in non-inlined calls (fewer registers)
    for part in (p, p // 2, p // 4, p // 8):
        for var in (0, 1):
            for g in (2, 4, 8, 16):
                ms, _ = bb.bench_lambda(beta[:part], 0.5, tau, g, var, 20)
                print(f"p={part:6d} variant={var} G={g:2d}: {ms * 1e3:8.1f} us/launch",
                      flush=True)


if __name__ == "__main__":
    main()
