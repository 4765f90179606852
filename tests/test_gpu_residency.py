"""GPU: the one-launch local step (dqrm_emb_bwd_apply_local) only runs when its grid can be
resident at once. Its workgroups wait for each other's gradient maxima, so on a CU-masked
stream (hipExtStreamCreateWithCUMask) -- or a partitioned device -- the library must take the
two-launch path instead, with identical results and no DQRM_ERRF_STALL.
Reference step: sgd_quantized_gradients_parallel_comm.py:850-890 (quantize_emb_grad) +
:601-628 (weight_update_parallel_comm) at world size 1."""
import ctypes

import numpy as np
import pytest
import torch

import gen_inputs as G

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dq():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import deep_quantized_recommendation_model_dqrm_amd as d

    d.build(verbose=False)
    d._lib.load()
    return d


def _hip():
    for name in ("libamdhip64.so", "/opt/rocm/lib/libamdhip64.so"):
        try:
            return ctypes.CDLL(name)
        except OSError:
            continue
    pytest.skip("libamdhip64.so not found")


def _masked_stream(n_cus: int):
    """A HIP stream whose CU mask enables the first n_cus CUs, wrapped for torch."""
    hip = _hip()
    words = 8
    mask = (ctypes.c_uint32 * words)()
    for i in range(n_cus):
        mask[i // 32] |= 1 << (i % 32)
    s = ctypes.c_void_p()
    rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(s), ctypes.c_uint32(words), mask)
    assert rc == 0, f"hipExtStreamCreateWithCUMask failed ({rc})"
    return hip, s, torch.cuda.ExternalStream(s.value)


def test_cu_masked_stream_takes_two_launch_path(dq):
    """TB shape (the reference's 26 TB tables, D=64, B=2048): on the default stream the step is
    ONE launch; on a 32-CU masked stream the library falls back to coalesce + apply_local.
    Three SparseGradExchange steps on the masked stream and three two-launch steps on a copy
    of the tables end bit-identical (W, |W| hierarchy, s_avg), with no device error flag."""
    from deep_quantized_recommendation_model_dqrm_amd.comm import HipExchangeKernels
    from deep_quantized_recommendation_model_dqrm_amd.workloads import TERABYTE_ROWS

    rows, D, B = TERABYTE_ROWS, 64, 2048
    T = len(rows)
    torch.cuda.set_device(0)
    sets = [dq.EmbeddingTableSet(rows, D, device="cuda", init="uniform", seed=11) for _ in range(2)]
    ex = dq.SparseGradExchange(sets[0], B, grad_bits=8)
    ws = dq.CoalescedGrad.allocate(rows, B, D, "cuda")
    s_avg = torch.zeros(T, dtype=torch.float32, device="cuda")
    batches = [dq.LookupBatch.pooling_one(torch.from_numpy(G.pooling_one(rows, B, 700 + k, dist=d)).cuda())
               for k, d in enumerate(("uniform", "zipf", "uniform"))]
    assert sets[0].apply_local_is_one_launch(batches[0])  # the default stream: all 256 CUs
    hip, raw, stream = _masked_stream(32)
    try:
        torch.cuda.synchronize()
        with torch.cuda.stream(stream):
            assert not sets[0].apply_local_is_one_launch(batches[0])
            for k, b in enumerate(batches):
                dy = torch.from_numpy(G.upstream_grad(T, B, D, 710 + k) * 20).cuda()
                sets[0].forward(b)
                ex.step(b, dy, lr=0.3)
            stream.synchronize()
        for k, b in enumerate(batches):
            dy = torch.from_numpy(G.upstream_grad(T, B, D, 710 + k) * 20).cuda()
            sets[1].forward(b)
            sets[1].backward_coalesce(b, dy, ws)
            HipExchangeKernels(sets[1]).apply_local(ws, 8, s_avg, 0.3, False)
        torch.cuda.synchronize()
        assert sets[0].read_errors() == 0  # in particular no DQRM_ERRF_STALL
        assert sets[1].read_errors() == 0
        assert torch.equal(ex.s_avg, s_avg)
        for name in ("W", "rowmax", "blkmax", "sblkmax", "tmax"):
            assert torch.equal(getattr(sets[0], name), getattr(sets[1], name)), name
        assert bool((s_avg > 0).all())  # every table received gradients
    finally:
        torch.cuda.synchronize()
        hip.hipStreamDestroy(raw)
        del sets, ex
        torch.cuda.empty_cache()


def test_one_launch_query_rejects_bad_arguments(dq):
    L = dq._lib
    lib = L.load()
    assert lib.dqrm_bwd_apply_local_is_one_launch(None, None, None) == L.DQRM_E_INVALID
    ts = dq.EmbeddingTableSet([10, 20], 16, device="cuda", init="uniform", seed=1)
    b = dq.LookupBatch.pooling_one(torch.zeros(2, 64, dtype=torch.int64, device="cuda"))
    assert ts.apply_local_is_one_launch(b)
    bags = dq.LookupBatch([torch.zeros(4, dtype=torch.int64)] * 2, [torch.tensor([0, 2])] * 2, device="cuda")
    assert not ts.apply_local_is_one_launch(bags)  # not in the Criteo form: the two calls
    assert np.isfinite(ts.scale.cpu().numpy()).all()
