"""The lane schedule of the wave-adaptive tilted-stable draw (bb_sampler.h stable_wave_draw)
reproduces the sequential double rejection loop (retstable.cpp:162-256): a Python model of
the schedule over random counter-keyed acceptance patterns (tools/wave_draw_model.py); the
GPU test test_nid_gpu.py::test_lambda_wave_draw_same_bits checks the kernel's bits."""
from tools import wave_draw_model as m


def test_schedule_accepts_the_sequential_loops_attempts():
    assert m.check(trials=300, seed=3) == 600


def test_schedule_needs_fewer_rounds_than_fixed_groups():
    r = m.rounds(trials=300, seed=4)
    fixed, adaptive = r[8]
    assert adaptive < 0.85 * fixed, r
