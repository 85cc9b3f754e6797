"""Host enqueue cost of one sweep against its device time.

An on-device shard group of N members (N column shards of C3 on ONE GPU, one host thread,
every member's phases interleaved) is the worst case for host launch overhead: N x ~12
launches per sweep from one thread.  RCCL groups (distinct devices) enqueue from one thread
per member (bb_group_run), so each thread issues one member's ~12 launches per sweep.
Prints, per configuration, host ms per sweep spent inside run() (enqueue only; HIP queues
are deep enough that run() returns before the device finishes) and device ms per sweep.
Usage: python tools/enqueue_probe.py [n p members sweeps]"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import bayesbridge_amd as bb  # noqa: E402


def note(msg):
    print(f"[enqueue_probe] {msg}", file=sys.stderr, flush=True)


def probe(engines, runner, sweeps):
    runner.run(1, 3, first_slot=-1)
    runner.sync()
    t0 = time.perf_counter()
    runner.run(4, sweeps, first_slot=-1)
    t1 = time.perf_counter()
    runner.sync()
    t2 = time.perf_counter()
    return 1e3 * (t1 - t0) / sweeps, 1e3 * (t2 - t0) / sweeps


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
    p = int(sys.argv[2]) if len(sys.argv) > 2 else 50000
    members = int(sys.argv[3]) if len(sys.argv) > 3 else 8
    sweeps = int(sys.argv[4]) if len(sys.argv) > 4 else 20
    bb.set_verbose(0)
    note(f"n={n} p={p} members={members}: building data")
    y, _ = bench.make_problem_y(n, p)
    out = {"n": n, "p": p, "sweeps": sweeps, "results": []}
    per = (p + members - 1) // members
    engines = []
    for r in range(members):
        j0, j1 = r * per, min(p, (r + 1) * per)
        cfg = bb.EngineConfig(n=n, p=p, p_local=j1 - j0, j0=j0, rank=r, world=members,
                              true_alpha=0.5, method=2, seed=0xB4E5B41D6E)
        engines.append(bb.Engine(cfg, bench.make_columns(n, j0, j1), y))
        note(f"engine {r} created")
    grp = bb.ShardGroup(engines)
    grp.init_state()
    note("on-device group ready")
    h, d = probe(engines, grp, sweeps)
    note(f"on-device group: host {h:.3f} ms, device {d:.3f} ms per sweep")
    out["results"].append({"config": f"on-device group, {members} members, one host thread",
                           "host_enqueue_ms_per_sweep": h, "device_ms_per_sweep": d})
    grp.close()
    for e in engines:
        e.close()
    cfg = bb.EngineConfig(n=n, p=p, true_alpha=0.5, method=2, seed=0xB4E5B41D6E)
    e = bb.Engine(cfg, bench.make_columns(n, 0, p), y)
    g1 = bb.ShardGroup([e], rccl=True)
    g1.init_state()
    note("RCCL group ready")
    h, d = probe([e], g1, sweeps)
    note(f"RCCL group: host {h:.3f} ms, device {d:.3f} ms per sweep")
    out["results"].append({"config": "RCCL group, 1 member (its own enqueue thread)",
                           "host_enqueue_ms_per_sweep": h, "device_ms_per_sweep": d})
    g1.close()
    e.close()
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
