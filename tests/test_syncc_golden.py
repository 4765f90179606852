"""weight_syncc on identical replicas (s_q_g_p_c.py:963-970) against real Gloo: the oracle's
sequential fold equals Gloo's all_reduce(SUM) * 1/N at N = 3, 5, 6, 8 (fixture made by
tests/golden/make_golden_syncc.py), and the package's identity shortcut holds at N = 1, 2, 4."""
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, "golden"), os.path.join(HERE, "..", "oracle")]
import gen_inputs as G  # noqa: E402
import oracle as O  # noqa: E402

FIX = np.load(os.path.join(HERE, "golden", "syncc_gloo.npz"))


def _inputs(tag):
    i = 0 if tag == "small" else 1
    x = G.replica_values(int(FIX["sizes"][i]), int(FIX["seeds"][i]))
    assert G.checksum(x) == str(FIX[f"x_{tag}_checksum"])
    return x


@pytest.mark.parametrize("N", [3, 5, 6, 8])
def test_oracle_replica_mean_is_gloo(N):
    x = _inputs("small")
    got = O.replica_mean(x, N)
    np.testing.assert_array_equal(got.view(np.uint32), FIX[f"small_n{N}"].view(np.uint32))
    assert int(np.sum(got.view(np.uint32) != x.view(np.uint32))) > 0  # N = 3..8 move elements
    xl = _inputs("large")
    assert G.checksum(O.replica_mean(xl, N)) == str(FIX[f"large_n{N}_checksum"])


@pytest.mark.parametrize("N", [1, 2, 4])
def test_replica_mean_identity_worlds(N):
    """_ring_mean_is_identity's claim: at N = 1, 2, 4 the fold times fl(1/N) is x itself
    (no overflow); the package then skips the pass."""
    x = _inputs("small")
    ok = np.abs(x) * N < 3.0e38
    np.testing.assert_array_equal(O.replica_mean(x, N)[ok].view(np.uint32), x[ok].view(np.uint32))
