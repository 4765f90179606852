"""CPU tests of host-side logic: batch packing, slicing, capacities."""
import numpy as np
import torch

import deep_quantized_recommendation_model_dqrm_amd as dq
from deep_quantized_recommendation_model_dqrm_amd.comm import get_my_slice


def test_lookup_batch_ragged():
    idx = [torch.tensor([1, 2, 3]), torch.tensor([4]), torch.tensor([], dtype=torch.int64)]
    off = [torch.tensor([0, 2]), torch.tensor([0, 1]), torch.tensor([0, 0])]
    b = dq.LookupBatch(idx, off, device="cpu")
    assert b.num_tables == 3 and b.num_bags == 2
    assert b.idx_base_host == [0, 3, 4, 4]
    assert b.max_lookups == 3
    assert b.idx.tolist() == [1, 2, 3, 4]
    assert b.off.shape == (3, 2)


def test_lookup_batch_pooling_one():
    P = torch.arange(12).view(3, 4)
    b = dq.LookupBatch.pooling_one(P)
    assert b.off.tolist() == [[0, 1, 2, 3]] * 3
    assert b.idx_base_host == [0, 4, 8, 12]


def test_get_my_slice_matches_reference_partition():
    # dlrm_s_pytorch_single_gpu.py:989-993: contiguous, sizes differ by at most one
    for n, N in [(512, 4), (2048, 8), (10, 3), (7, 8)]:
        sl = [get_my_slice(n, N, r) for r in range(N)]
        assert sl[0].start == 0 and sl[-1].stop == n
        assert all(sl[r].stop == sl[r + 1].start for r in range(N - 1))
        sizes = [s.stop - s.start for s in sl]
        assert max(sizes) - min(sizes) <= 1


def test_default_caps():
    assert dq.default_caps([3, 1000, 10**7], 2048) == [3, 1000, 2048]


def test_reference_scale_host_helper():
    assert dq.reference_scale(0.0, 4) == np.float32(np.float32(1e-8) / np.float32(7))
    assert dq.reference_scale(7.0, 4) == 1.0
