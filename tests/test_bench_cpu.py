"""bench.py dispatch, as the driver invokes it (no GPU needed).

`python bench.py --gpus N` without a torch.distributed launcher drives N GPUs from one
process (the .C entry points' RCCL shard group); with fewer than N visible GPUs it must exit
non-zero with a clear message instead of silently measuring one GPU.
"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run_bench(*args, env_extra=None):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.pop("RANK", None)
    env.pop("LOCAL_RANK", None)
    if env_extra:
        env.update(env_extra)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args],
                          capture_output=True, text=True, env=env, timeout=300, cwd=ROOT)


def _visible_gpus():
    import torch

    return torch.cuda.device_count()


@pytest.mark.skipif(_visible_gpus() >= 2, reason="needs a host with fewer than 2 GPUs")
def test_gpus_2_without_launcher_refuses_one_gpu():
    r = run_bench("--gpus", "2", "--steps", "2", "--warmup", "0", "--no-cpu-baseline",
                  "--rows", "64", "--cols", "300")
    assert r.returncode != 0
    assert "refusing to measure fewer GPUs than requested" in r.stderr, r.stderr[-2000:]
    assert not r.stdout.strip(), "no JSON line may be printed"


def test_world_size_mismatch_is_an_error():
    r = run_bench("--gpus", "4", "--steps", "2", "--warmup", "0",
                  env_extra={"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0
    assert "WORLD_SIZE=2 but --gpus=4" in r.stderr


@pytest.mark.parametrize("workload", ["c1", "c4"])
def test_unsharded_workloads_refuse_multi_gpu(workload):
    r = run_bench("--workload", workload, "--gpus", "2", "--steps", "2", "--warmup", "0")
    assert r.returncode != 0
    assert "does not shard" in r.stderr


def test_dominant_phase_roofline_formulas():
    """roofline_for: the Cholesky entry's flop rate and latency model follow DESIGN.md s8
    (m^3/3 flop per launch, m_pad/64 dependent block steps)."""
    sys.path.insert(0, ROOT)
    import bench

    class FakeBB:
        GRAM_OZAKI, GRAM_FP64 = 1, 0

    ctx = dict(bb=FakeBB, eng=None, kind="dense", n=1000, p=5000, p_loc=5000, gram_mode=1)
    r = bench.roofline_for("chol", 0.25, ctx, 1)
    assert r["bound"] == "mfma" and r["unit"] == "TFLOP/s"
    assert abs(r["achieved"] - 1000 ** 3 / 3 / 0.25e-3 / 1e12) < 1e-9
    assert r["latency_model"]["dependent_block_steps"] == 1024 // 64
    assert abs(r["frac"] - r["achieved"] / bench.FP64_MFMA_PEAK_TFLOPS) < 1e-15
    g = bench.roofline_for("gram", 0.05, ctx, 1)
    assert abs(g["achieved"] - 16.0 * 1000 * 1001 * 5000 / 0.05e-3 / 1e12) < 1e-6
    lg = dict(ctx, kind="logit", n=10000, p=1000, p_loc=1000)
    r = bench.roofline_for("chol", 0.25, lg, 1)
    assert r["latency_model"]["system"] == 1000
    assert r["latency_model"]["system_padded"] == 1024


@pytest.mark.parametrize("world", [1, 2])
@pytest.mark.parametrize("kind,n,p", [("dense", 2000, 50000), ("dense", 1000, 5000),
                                      ("sparse", 5000, 200000)])
def test_lambda_and_beta_roofline_entries(world, kind, n, p, monkeypatch):
    """The lambda entry (bound "valu": SIMD issue cycles per launch from a committed PMC
    profile of THIS tree over the live time; no profile -- another shape, a shard, another
    tree -- gives achieved = frac = None, never an error) and the dense beta entry."""
    sys.path.insert(0, ROOT)
    import bench

    class FakeBB:
        GRAM_OZAKI, GRAM_FP64 = 1, 0

        @staticmethod
        def set_tuning(key, value):
            return 1

    class FakeEng:
        @staticmethod
        def sparse_info():
            return dict(nnz=n * p // 100, pairs=0, col_mode=1, max_row=0)

    inst = "bb::k_lambda_xu<8, 8>"
    prof = {"source_sha": bench.tree_sha(), "configs": {"c3": {"n": 2000, "p": 50000, "kernels": {
        inst: {"SQ_INSTS_VALU": 5e7, "issue_cycles": 1.5e8, "issue_cycles_low": 1.2e8,
               "issue_cycles_high": 2.0e8}}}}}
    monkeypatch.setattr(bench, "_profiles", lambda pat: iter([(prof, "profiles/rXX_pmc_valu.json")]))
    p_loc = p // world
    ctx = dict(bb=FakeBB, eng=FakeEng, kind=kind, n=n, p=p, p_loc=p_loc, gram_mode=1,
               nid_cheb=True, instances={"lambda": inst})
    r = bench.roofline_for("lambda", 0.24, ctx, world)
    assert r["bound"] == "valu" and r["peak"] == bench.VALU_PEAK_GCYC
    assert abs(r["draws_per_s"] - p_loc / 0.24e-3) < 1e-6 * p_loc / 0.24e-3
    if kind == "dense" and world == 1 and n == 2000:
        assert r["kernel"] == inst
        assert abs(r["achieved"] - 1.5e8 / 0.24e-3 / 1e9) < 1e-6
        assert abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-12
        assert r["frac_bounds"][0] < r["frac"] < r["frac_bounds"][1]
        assert abs(r["hbm"]["achieved_GBps"] - (8.0 * n * p + 32.0 * p) / 0.24e-3 / 1e9) < 1e-6
    else:
        assert r["achieved"] is None and r["frac"] is None
    b = bench.roofline_for("beta", 0.135, ctx, world)
    assert b["bound"] == "hbm" and b["frac"] is not None


def test_pmc_lookup_matches_exact_instance_of_this_tree(monkeypatch):
    """the traffic of the E-apply must come from the instance that ran
    (k_eapply<8, false>), not from the no-op right-hand-side instance that shares its prefix,
    and a profile of another tree (or one without a recorded source) is not used."""
    sys.path.insert(0, ROOT)
    import bench

    def prof(sha):
        return {"source_sha": sha, "workload": {"n": 2000, "p": 50000}, "kernels": {
            "bb::k_eapply<8, false>": {"hbm_bytes": 8.3e8},
            "bb::k_eapply<8, true>": {"hbm_bytes": 2.1e4}}}

    monkeypatch.setattr(bench, "_profiles", lambda pat: iter([(prof(bench.tree_sha()), "f")]))
    assert bench.pmc_traffic(2000, 50000, 1, "bb::k_eapply<8, false>")[0] == 8.3e8
    assert bench.pmc_traffic(2000, 50000, 1, "bb::k_eapply<8, true>")[0] == 2.1e4
    assert bench.pmc_traffic(2000, 50000, 1, "bb::k_eapply")[0] is None  # no prefix match
    assert bench.pmc_traffic(2000, 50000, 1, None)[0] is None
    for sha in ("0123456789abcdef", None):
        monkeypatch.setattr(bench, "_profiles", lambda pat, s=sha: iter([(prof(s), "f")]))
        b, src, note = bench.pmc_traffic(2000, 50000, 1, "bb::k_eapply<8, false>")
        assert b is None and "not used" in note
