"""GPU: dqrm_emb_fwd_after_update == dqrm_rows_changed + dqrm_emb_fwd, bit for bit.

The per-table module (grad_mode "sparse") hands torch.optim.SGD the uncoalesced COO grad
(dlrm_s_pytorch_single_gpu.py:1943-1950); the optimizer rewrites the looked-up rows outside
libdqrm, and the next forward must take its scale from the full table again
(quant_utils.py:141-194, q_m_n_q_g.py:317-398). The module now does the sync and the forward
in one call: one single-workgroup launch for a one-table set and a small batch, the two calls
otherwise. Both must leave the same output, scale, |W| hierarchy and dirty flags."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dq():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import deep_quantized_recommendation_model_dqrm_amd as d

    d.build(verbose=False)
    d._lib.load()
    return d


def _state(ts):
    return [x.clone() for x in (ts.W, ts.rowmax, ts.blkmax, ts.sblkmax, ts.tmax, ts.scale, ts.bdirty, ts.sdirty)]


@pytest.mark.parametrize("n,D,B,nchg,shrink", [
    (5000, 16, 128, 128, False),      # Kaggle-like table, the fused launch
    (5000, 16, 128, 128, True),       # rows shrink: block / superblock / table maxima re-reduced
    (200, 16, 64, 40, True),          # narrow table (one block)
    (300000, 64, 256, 256, True),     # D = 64, several superblocks
    (70000, 16, 2048, 2048, True),    # batch too large for one workgroup: the two calls
    (3, 16, 128, 128, False),         # 3 rows, every row changed many times (duplicates)
])
def test_fwd_after_update_matches_two_calls(dq, n, D, B, nchg, shrink):
    g = torch.Generator(device="cuda").manual_seed(n + D + B)
    a = dq.EmbeddingTableSet([n], D, device="cuda", init="uniform", seed=11)
    b = dq.EmbeddingTableSet([n], D, device="cuda", init="uniform", seed=11)
    for step in range(3):
        rows = torch.randint(0, n, (nchg,), generator=g, device="cuda")
        if shrink and step == 1:  # scale the table's largest rows down: holders shrink
            big = a.rowmax.topk(min(8, n)).indices
            rows = torch.cat([rows, big])
        delta = torch.randn(rows.numel(), D, generator=g, device="cuda") * 0.01
        u = rows.unique()
        # rows rewritten outside libdqrm (as torch.optim.SGD's index_add_ on the COO; its atomic
        # order with duplicates is not deterministic, so b takes a's result)
        if shrink:
            a.W.index_copy_(0, u, a.W[u] * 0.5)
        a.W.index_add_(0, rows, delta)
        b.W.copy_(a.W)
        idx = torch.randint(0, n, (B,), generator=g, device="cuda")
        off = torch.arange(B, dtype=torch.int64, device="cuda")
        batch = dq.LookupBatch([idx], [off], pooling_one=True)
        a.rows_changed(rows)
        ya = a.forward(batch)
        yb = b.forward(batch, changed_rows=rows)
        torch.cuda.synchronize()
        assert torch.equal(ya, yb), f"step {step}: forward outputs differ"
        for k, (x, y) in enumerate(zip(_state(a), _state(b))):
            assert torch.equal(x, y), f"step {step}: state array {k} differs"
        assert a.read_errors() == 0 and b.read_errors() == 0
    # the exact full-table scale (quant_utils.py:141-194) after the last sync
    tm = float(b.W.abs().max())
    assert float(b.tmax[0]) == tm


def test_fwd_after_update_flags_bad_rows(dq):
    ts = dq.EmbeddingTableSet([1000], 16, device="cuda", init="uniform", seed=3)
    idx = torch.randint(0, 1000, (64,), device="cuda")
    batch = dq.LookupBatch([idx], [torch.arange(64, device="cuda")], pooling_one=True)
    ts.forward(batch, changed_rows=torch.tensor([5, 1000, -1], device="cuda"))
    assert ts.read_errors() & dq._lib.DQRM_ERRF_INDEX


@pytest.mark.parametrize("fused_step", [False, True])
def test_module_sparse_steps_keep_exact_hierarchy(dq, fused_step):
    """A list of modules, grad_mode "sparse" + torch.optim.SGD for 4 steps (the unchanged
    single-GPU driver): after every step's next forward each table's |W| hierarchy equals a
    full rebuild from its W, and the output equals a plain refreshing forward on that W.
    fused_step False: the optimizer adds the COO and the module syncs the changed rows in its
    next forward (dqrm_emb_fwd_after_update); True (default): the optimizer's step runs as the
    module's own SGD kernel, so no rows are left to sync."""
    from deep_quantized_recommendation_model_dqrm_amd import quant_modules_not_quantize_grad as Q

    Q.set_fused_optimizer_step(fused_step)
    try:
        _module_sparse_steps(dq, Q, fused_step)
    finally:
        Q.set_fused_optimizer_step(True)


def _module_sparse_steps(dq, Q, fused_step):
    rows, D, B = [3, 61, 1500, 20000], 16, 128
    g = torch.Generator(device="cuda").manual_seed(5)
    mods = torch.nn.ModuleList([Q.QuantEmbeddingBagTwo(n, D, 4, grad_mode="sparse", init="device", device="cuda")
                                for n in rows])
    opt = torch.optim.SGD(list(mods.parameters()), lr=0.5)
    off = torch.arange(B, dtype=torch.int64, device="cuda")
    for step in range(4):
        P = [torch.randint(0, n, (B,), generator=g, device="cuda") for n in rows]
        dys = [torch.randn(B, D, generator=g, device="cuda") * 0.1 for _ in rows]
        pending = [bool(m._ext_rows) for m in mods]
        assert all(pending) == (step > 0 and not fused_step) and (any(pending) == all(pending))
        ly = [mods[t](P[t], off) for t in range(len(rows))]
        for t, m in enumerate(mods):
            ts = m._tset
            got = [x.clone() for x in (ts.rowmax, ts.blkmax, ts.sblkmax, ts.tmax, ts.scale)]
            ts.refresh_absmax()
            ref = [ts.rowmax, ts.blkmax, ts.sblkmax, ts.tmax]
            for k in range(4):
                assert torch.equal(got[k], ref[k]), f"step {step} table {t}: hierarchy level {k}"
            y = ts.forward(dq.LookupBatch([P[t]], [off], pooling_one=True))
            assert torch.equal(ly[t], y[0]), f"step {step} table {t}: output"
            assert torch.equal(got[4], ts.scale)
            assert ts.read_errors() == 0
        torch.autograd.backward(ly, dys)
        opt.step()
        opt.zero_grad(set_to_none=True)
