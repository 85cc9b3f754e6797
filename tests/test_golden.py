"""The committed golden vectors (tests/golden/oracle_vectors.npz, made by
tests/golden/make_golden.py) are reproduced bit for bit by the oracle."""
import os

import numpy as np

from tests.golden.make_golden import vectors

HERE = os.path.dirname(os.path.abspath(__file__))


def test_oracle_reproduces_golden_vectors():
    ref = np.load(os.path.join(HERE, "golden", "oracle_vectors.npz"))
    cur = vectors()
    assert set(ref.files) == set(cur)
    for k in ref.files:
        assert np.array_equal(ref[k], cur[k]), k
