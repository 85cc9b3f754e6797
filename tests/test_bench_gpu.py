"""bench.py end to end on the GPU, as the driver runs it (one JSON line on stdout).

The contract (task statement): metric / value / unit / n_gpus / steps / warmup /
ms_per_step / higher_is_better / scaling / dtype / data / config, plus `roofline` (the
dominant kernel's bound, achieved rate, peak, fraction and how it was timed) and
`cpu_baseline` (the oracle or the compiled reference-literal chain timed on the host).  Small
shapes (C2's n = 1000, p = 5000, and a 300 x 3000 design) keep each run to seconds.
"""
import json
import math

import pytest

from tests.test_bench_cpu import run_bench

pytestmark = pytest.mark.gpu

KEYS = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
        "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config", "roofline")


def _line(r):
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.strip().splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


def test_bench_c2_line_contract():
    d = _line(run_bench("--workload", "c2", "--steps", "8", "--warmup", "2",
                        "--no-cpu-baseline", "--no-fitted"))
    for k in KEYS:
        assert k in d, k
    assert d["unit"] == "sweeps/s" and d["n_gpus"] == 1 and d["steps"] == 8
    assert d["dtype"] == "f64" and d["higher_is_better"] is True
    assert d["value"] > 0 and math.isclose(d["value"] * d["ms_per_step"], 1000.0, rel_tol=1e-6)
    ro = d["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "kernel", "timing"):
        assert k in ro, k
    assert ro["peak"] > 0, ro
    # a VALU-bound kernel's rate needs the committed VALU PMC of the workload's shape (C3, C5:
    # profiles/r04_pmc_valu.json); without it achieved and frac are null
    if ro["bound"] == "valu" and ro["achieved"] is None:
        assert ro["frac"] is None, ro
    else:
        assert ro["achieved"] > 0, ro
    assert ro["frac"] is None or 0.0 < ro["frac"] <= 1.0, ro
    assert "HIP events" in ro["timing"]


def test_bench_cpu_baseline_and_timing_stride():
    """A small dense design with a short CPU baseline leg: cpu_baseline carries its value,
    unit, cores, kind and sample; --timing-stride 1 brackets every timed sweep."""
    d = _line(run_bench("--rows", "300", "--cols", "3000", "--steps", "6", "--warmup", "2",
                        "--cpu-sweeps", "2", "--no-fitted", "--timing-stride", "1"))
    cb = d["cpu_baseline"]
    for k in ("value", "unit", "cores", "kind", "sample"):
        assert k in cb, k
    assert cb["value"] > 0 and cb["kind"] in ("port", "reference")
    assert d["roofline"]["timing"].endswith("every timed launch")
