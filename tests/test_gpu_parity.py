"""GPU parity: libdqrm (HIP, via the C ABI) against the CPU oracle and golden fixtures.

Bar: bit-exact on indices, packing, counts and quantized integers; forward outputs and
updated weights are compared exactly too (the kernels reproduce the reference's f32
rounding); the north-star tolerance (1e-5) is only used against torch-CPU-native fixtures.
"""
import os

import numpy as np
import pytest
import torch

import gen_inputs as G
import oracle as O

pytestmark = pytest.mark.gpu

f32 = np.float32


@pytest.fixture(scope="module")
def dq():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import deep_quantized_recommendation_model_dqrm_amd as d

    d.build(verbose=False)
    d._lib.load()
    return d


@pytest.fixture(params=["flat", "flat2", "flat4", "slot", "ranges", "merge"])
def apply_kernel(request, dq):
    """Run the test once per dqrm_apply_sparse_update kernel (the AUTO choice depends on N);
    flat2 / flat4: the flat kernel with two / four entries per lane group (k_apply_flat2, N > 1), forced."""
    L = dq._lib
    lib = L.load()
    kind = {"flat": L.DQRM_APPLY_FLAT, "flat2": L.DQRM_APPLY_FLAT, "flat4": L.DQRM_APPLY_FLAT, "slot": L.DQRM_APPLY_SLOT,
            "ranges": L.DQRM_APPLY_RANGES, "merge": L.DQRM_APPLY_MERGE}[request.param]
    prev = lib.dqrm_set_apply_kernel(kind)
    old = os.environ.get("DQRM_FLAT_DUAL")
    os.environ["DQRM_FLAT_DUAL"] = {"flat2": "2", "flat4": "4"}.get(request.param, "0")
    yield request.param
    if old is None:
        os.environ.pop("DQRM_FLAT_DUAL", None)
    else:
        os.environ["DQRM_FLAT_DUAL"] = old
    lib.dqrm_set_apply_kernel(prev)


def load(golden_dir, name):
    return dict(np.load(os.path.join(golden_dir, name)))


def make_set(dq, Ws, packed=False):
    return dq.EmbeddingTableSet([w.shape[0] for w in Ws], Ws[0].shape[1], device="cuda", packed=packed,
                                init=None, weights=[torch.from_numpy(w) for w in Ws])


def to_batch(dq, idxs, offs):
    return dq.LookupBatch([torch.from_numpy(np.ascontiguousarray(i)) for i in idxs],
                          [torch.from_numpy(np.ascontiguousarray(o)) for o in offs], device="cuda")


from test_oracle_golden import SINGLE, regen_single, dp_inputs  # noqa: E402


@pytest.mark.parametrize("name", SINGLE)
def test_single_gpu_qat_steps_bitexact(dq, golden_dir, name):
    fx = load(golden_dir, name)
    Ws, batches, dys = regen_single(fx)
    bits, lr = int(fx["bits"]), float(fx["lr"])
    ts = make_set(dq, Ws)
    for k, ((idxs, offs), dy) in enumerate(zip(batches, dys)):
        b = to_batch(dq, idxs, offs)
        y = ts.forward(b, bits=bits, refresh_scale=True)
        np.testing.assert_array_equal(ts.scale.cpu().numpy(), fx[f"s{k}"])
        np.testing.assert_array_equal(y.cpu().numpy(), fx[f"y{k}"])
        ts.backward_sgd(b, torch.from_numpy(dy).cuda(), lr=lr, ste=True)
    assert ts.read_errors() == 0
    for t in range(len(Ws)):
        rows = torch.from_numpy(fx[f"rows_t{t}"]).cuda()
        np.testing.assert_array_equal(ts.table_weight(t)[rows].cpu().numpy(), fx[f"w_t{t}"])
    # the incrementally maintained |W| hierarchy equals a full recompute
    tmax_inc = ts.tmax.clone()
    ts.refresh_absmax()
    torch.testing.assert_close(tmax_inc, ts.tmax, rtol=0, atol=0)


@pytest.mark.parametrize("bits", [2, 4, 8, 16])
@pytest.mark.parametrize("case", ["tie", "zero"])
def test_edge_cases_bitexact(dq, golden_dir, bits, case):
    fx = load(golden_dir, "edge.npz")
    ts = make_set(dq, [fx[f"W_{case}"]])
    b = to_batch(dq, [fx[f"idx_{case}"]], [fx[f"off_{case}"]])
    y = ts.forward(b, bits=bits)
    assert ts.scale.item() == fx[f"{case}_b{bits}_s"]
    np.testing.assert_array_equal(y[0].cpu().numpy(), fx[f"{case}_b{bits}_y"])
    ts.backward_sgd(b, torch.from_numpy(fx[f"{case}_b{bits}_dy"][None]).cuda(), lr=0.1)
    np.testing.assert_array_equal(ts.W.cpu().numpy(), fx[f"{case}_b{bits}_w"])


def test_full_precision_flag(dq, golden_dir):
    fx = load(golden_dir, "edge.npz")
    ts = make_set(dq, [fx["W_tie"]])
    b = to_batch(dq, [fx["idx_tie"]], [fx["off_tie"]])
    y = ts.forward(b, full_precision=True)
    np.testing.assert_array_equal(y[0].cpu().numpy(), fx["fp_y"])
    ts.backward_sgd(b, torch.from_numpy(fx["fp_dy"][None]).cuda(), lr=0.1, ste=False)
    np.testing.assert_array_equal(ts.W.cpu().numpy(), fx["fp_w"])


def test_bag_major_layout_matches(dq):
    rows = [1000, 7, 50000]
    Ws = G.table_weights(rows, 32, 5)
    P = G.pooling_one(rows, 96, 6)
    ts = make_set(dq, Ws)
    b = dq.LookupBatch.pooling_one(torch.from_numpy(P).cuda())
    y_tbd = ts.forward(b)
    y_btd = ts.forward(b, layout="btd")
    torch.testing.assert_close(y_tbd.permute(1, 0, 2), y_btd, rtol=0, atol=0)


def test_packed_int4_path_bitexact(dq, golden_dir):
    """Packed rows equal the oracle's packing; the INT4 gather equals the FP32 fake-quant
    path; touched rows are repacked with the frozen scale after SGD."""
    fx = load(golden_dir, "kaggle_pool1.npz")
    Ws, batches, dys = regen_single(fx)
    ts = make_set(dq, Ws, packed=True)
    ts.refresh_scale_and_pack(4)
    s = ts.scale.cpu().numpy()
    np.testing.assert_array_equal(s, fx["s0"])
    for t in range(len(Ws)):
        np.testing.assert_array_equal(ts.table_packed(t).cpu().numpy(), O.pack_int4(Ws[t], s[t]))
    (idxs, offs), dy = batches[0], dys[0]
    b = to_batch(dq, idxs, offs)
    y_packed = ts.forward(b, refresh_scale=False, use_packed=True)
    np.testing.assert_array_equal(y_packed.cpu().numpy(), fx["y0"])
    ts.backward_sgd(b, torch.from_numpy(dy).cuda(), lr=0.1, repack=True)
    W_host = ts.W.cpu().numpy()
    P_host = ts.packed.cpu().numpy()
    for t in range(len(Ws)):
        base, n = ts.row_base[t], ts.num_rows[t]
        np.testing.assert_array_equal(P_host[base:base + n], O.pack_int4(W_host[base:base + n], s[t]))
    # scale refresh: tables whose max moved are fully repacked, the rest keep their rows
    ts.refresh_scale_and_pack(4)
    s2 = ts.scale.cpu().numpy()
    P2 = ts.packed.cpu().numpy()
    for t in range(len(Ws)):
        base, n = ts.row_base[t], ts.num_rows[t]
        assert s2[t] == O.table_scale(W_host[base:base + n], 4)
        np.testing.assert_array_equal(P2[base:base + n], O.pack_int4(W_host[base:base + n], s2[t]))


def _emulate_ranks(dq, ts, rank_batches, rank_dys, grad_bits, lr, mode=None, repack=False):
    """Run the exchange's three device steps for N ranks on one GPU (the all-gathers become
    stacking), exactly as SparseGradExchange does on each rank."""
    from deep_quantized_recommendation_model_dqrm_amd import _lib as L
    from deep_quantized_recommendation_model_dqrm_amd.comm import HipExchangeKernels, payload_bytes

    N = len(rank_batches)
    k = HipExchangeKernels(ts)
    max_lookups = max(b.max_lookups for b in rank_batches)
    wss = []
    for r in range(N):
        ws = dq.CoalescedGrad.allocate(ts.num_rows, max_lookups, ts.D, "cuda")
        k.coalesce(rank_batches[r], rank_dys[r], ws, True, "tbd")
        wss.append(ws)
    absmax_all = torch.stack([ws.absmax for ws in wss])
    caps = dq.default_caps(ts.num_rows, max_lookups)
    cap_base = torch.tensor(np.concatenate([[0], np.cumsum(caps)]), dtype=torch.int64, device="cuda")
    cap_total = int(sum(caps))
    P = payload_bytes(ts.T, cap_total, ts.D, grad_bits)
    payloads = torch.zeros(N, P, dtype=torch.uint8, device="cuda")
    s_avg = torch.zeros(ts.T, dtype=torch.float32, device="cuda")
    for r in range(N):
        k.quant_pack(wss[r], absmax_all, N, grad_bits, cap_base, cap_total, s_avg, payloads[r])
    if mode is None:
        mode = L.DQRM_UPD_FP32 if grad_bits == 32 else L.DQRM_UPD_DP
    k.apply(cap_base, cap_total, payloads, P, N, grad_bits, s_avg, lr, mode, repack)
    return wss, payloads, s_avg, cap_base.cpu().numpy()


def _local_scale(ws, T, bits):
    a = ws.absmax.view(T, -1).max(dim=1).values.cpu().numpy()
    return np.array([O.sym_scale(x, bits) for x in a], dtype=f32)


def _decode_payload(p, T, cap_base, D, bits, t):
    p = p.cpu().numpy()
    a16 = lambda x: (x + 15) & ~15  # noqa: E731
    CAP = int(cap_base[-1])
    S = 8  # DQRM_TABLE_SPLIT: the header holds per-(table, slot) counts
    cnt = int(p[: 4 * T * S].view(np.int32)[t * S: (t + 1) * S].sum())
    rows_off = a16(4 * T * S)
    vals_off = rows_off + a16(4 * CAP)
    rows = p[rows_off: rows_off + 4 * CAP].view(np.int32)[cap_base[t]: cap_base[t] + cnt]
    dt = np.int8 if bits <= 8 else np.int16
    vals = p[vals_off: vals_off + CAP * D * np.dtype(dt).itemsize].view(dt).reshape(CAP, D)
    return rows, vals[cap_base[t]: cap_base[t] + cnt].astype(f32)


DP = ["dp_n2.npz", "dp_n4.npz", "dp_n4_zipf.npz", "dp_n2_fp32.npz", "dp_n2_b16.npz"]


@pytest.mark.parametrize("name", DP)
def test_data_parallel_exchange_bitexact(dq, golden_dir, name, apply_kernel):
    fx = load(golden_dir, name)
    num_rows = fx["num_rows"].tolist()
    D, seed, N, bits = int(fx["D"]), int(fx["seed"]), int(fx["N"]), int(fx["bits"])
    quantized = bool(fx["quantized"])
    gb = bits if quantized else 32
    Ws = G.table_weights(num_rows, D, seed)
    ts = make_set(dq, Ws)
    for k in range(int(fx["steps"])):
        b, dys = dp_inputs(fx, k)
        rank_batches = [to_batch(dq, [x[0] for x in b[r]], [x[1] for x in b[r]]) for r in range(N)]
        rank_dys = [torch.from_numpy(np.stack(dys[r])).cuda() for r in range(N)]
        for rb in rank_batches:  # each rank's forward refreshes the same scale
            ts.forward(rb, refresh_scale=True)
        wss, payloads, s_avg, cb = _emulate_ranks(dq, ts, rank_batches, rank_dys, gb, float(fx["lr"]))
        if quantized:
            for t in range(len(num_rows)):
                assert s_avg[t].item() == fx[f"k{k}_t{t}_s_avg"]
                for r in range(N):
                    assert _local_scale(wss[r], len(num_rows), bits)[t] == fx[f"k{k}_t{t}_r{r}_s_loc"]
                    rows, q = _decode_payload(payloads[r], len(num_rows), cb, D, bits, t)
                    np.testing.assert_array_equal(rows, fx[f"k{k}_t{t}_r{r}_rows"])
                    np.testing.assert_array_equal(q, fx[f"k{k}_t{t}_r{r}_q"])
    assert ts.read_errors() == 0
    for t in range(len(num_rows)):
        rows = torch.from_numpy(fx[f"rows_t{t}"]).cuda()
        np.testing.assert_array_equal(ts.table_weight(t)[rows].cpu().numpy(), fx[f"w_t{t}"])


def test_simulated_dp_bitexact(dq, golden_dir, apply_kernel):
    from deep_quantized_recommendation_model_dqrm_amd import _lib as L

    fx = load(golden_dir, "sim_dp.npz")
    num_rows = fx["num_rows"].tolist()
    D, B, seed, N = int(fx["D"]), int(fx["B"]), int(fx["seed"]), int(fx["N"])
    Ws = G.table_weights(num_rows, D, seed)
    ts = make_set(dq, Ws)
    batches, dys = [], []
    for k in range(N):
        P = G.pooling_one(num_rows, B, seed + 17 * (k + 1))
        batches.append(dq.LookupBatch.pooling_one(torch.from_numpy(P).cuda()))
        dys.append(torch.from_numpy(G.upstream_grad(len(num_rows), B, D, seed + 31 * (k + 1))).cuda())
    ts.forward(batches[0])
    # micro-step scales: the FIRST micro-step's local scale is used for every micro-step
    from deep_quantized_recommendation_model_dqrm_amd.comm import HipExchangeKernels, payload_bytes
    kern = HipExchangeKernels(ts)
    caps = dq.default_caps(num_rows, B)
    cap_base = torch.tensor(np.concatenate([[0], np.cumsum(caps)]), dtype=torch.int64, device="cuda")
    cap_total = int(sum(caps))
    wss = []
    for k in range(N):
        ws = dq.CoalescedGrad.allocate(num_rows, B, D, "cuda")
        kern.coalesce(batches[k], dys[k], ws, True, "tbd")
        wss.append(ws)
    first_absmax = wss[0].absmax.clone().view(1, -1)
    Pb = payload_bytes(len(num_rows), cap_total, D, 8)
    payloads = torch.zeros(N, Pb, dtype=torch.uint8, device="cuda")
    s_first = torch.zeros(len(num_rows), dtype=torch.float32, device="cuda")
    for k in range(N):
        kern.quant_pack(wss[k], first_absmax, 1, 8, cap_base, cap_total, s_first, payloads[k])
    kern.apply(cap_base, cap_total, payloads, Pb, N, 8, s_first, 0.1, L.DQRM_UPD_SIMULATED, False)
    for t in range(len(num_rows)):
        assert s_first[t].item() == fx[f"s_t{t}"]
        np.testing.assert_array_equal(ts.table_weight(t).cpu().numpy(), fx[f"w_t{t}"])


def test_invalid_indices_flag_not_fault(dq):
    Ws = G.table_weights([100, 10], 16, 3)
    ts = make_set(dq, Ws)
    idx = [np.array([5, 100, -1, 3], np.int64), np.array([0, 9, 12, 1], np.int64)]
    off = [np.arange(4, dtype=np.int64), np.array([0, 1, 1, 3], np.int64)]
    b = to_batch(dq, idx, off)
    y = ts.forward(b)
    from deep_quantized_recommendation_model_dqrm_amd import _lib as L
    assert ts.read_errors() & L.DQRM_ERRF_INDEX
    y0, _ = O.emb_fwd(Ws[0], idx[0], off[0], O.table_scale(Ws[0], 4))
    np.testing.assert_array_equal(y[0].cpu().numpy(), y0)
    ts.backward_sgd(b, torch.zeros(2, 4, 16, device="cuda"), lr=0.1)
    assert ts.read_errors() & L.DQRM_ERRF_INDEX


@pytest.mark.parametrize("D", [16, 64])
def test_large_batch_no_capacity_cliff(dq, D):
    """B = 65,536 Criteo-form lookups per table (8x the in-LDS sort, so the tables sort in
    the workspace) on 3-row and 971-row tables plus a wide one: coalesce, SGD and the local
    update are bit-exact against the oracle -- the reference has no per-batch limit."""
    rows, B = [3, 971, 200000], 65536
    T = len(rows)
    Ws = G.table_weights(rows, D, 81)
    P = G.pooling_one(rows, B, 82, dist="zipf")
    P[0, : B // 2] = 1  # one 3-row table row holding half the batch: a 33k-lookup chain
    dy = G.upstream_grad(T, B, D, 83)
    ar = np.arange(B, dtype=np.int64)
    ts = make_set(dq, Ws)
    b = dq.LookupBatch.pooling_one(torch.from_numpy(P).cuda())
    ts.forward(b)
    s = ts.scale.cpu().numpy()
    ws = dq.CoalescedGrad.allocate(rows, B, D, "cuda")
    ts.backward_coalesce(b, torch.from_numpy(dy).cuda(), ws)
    for t in range(T):
        r_o, v_o, err = O.emb_bwd_coalesce(rows[t], P[t], ar, dy[t], s[t])
        r_g, v_g = _table_slots(ws, t)
        np.testing.assert_array_equal(r_g, r_o)
        np.testing.assert_array_equal(v_g, v_o)
        am = ws.absmax.view(T, -1)[t].max().item()
        assert am == np.abs(v_o).max()
    ts.backward_sgd(b, torch.from_numpy(dy).cuda(), lr=0.1)
    mask = torch.tensor([1, 0, 1], dtype=torch.int32, device="cuda")
    ts.local_update(b, torch.from_numpy(dy).cuda(), 0.05, table_mask=mask)
    assert ts.read_errors() == 0
    for t in range(T):
        Wo = Ws[t].copy()
        O.emb_bwd_sgd(Wo, P[t], ar, dy[t], s[t], 0.1)
        if t != 1:
            O.emb_local_update(Wo, P[t], ar, dy[t], s[t], 0.05)
        np.testing.assert_array_equal(ts.table_weight(t).cpu().numpy(), Wo)
    inc = [x.clone() for x in (ts.rowmax, ts.blkmax, ts.sblkmax, ts.tmax)]
    ts.refresh_absmax()
    for x, y in zip(inc, (ts.rowmax, ts.blkmax, ts.sblkmax, ts.tmax)):
        assert torch.equal(x, y)


def test_apply_crowded_slot_bitexact(dq, apply_kernel):
    """Two ranks x 65,536 lookups: a 200k-row table's row-range slot merges > DQRM_SLOT_KEYS
    payload entries (the slot kernel then applies it by the flat method) -- W equals
    oracle.dp_step, and the |W| hierarchy equals a rebuild."""
    rows, D, B, N = [971, 200000], 16, 65536, 2
    T = len(rows)
    Ws = G.table_weights(rows, D, 91)
    ts = make_set(dq, Ws)
    Ps = [G.pooling_one(rows, B, 92 + r) for r in range(N)]
    dys = [G.upstream_grad(T, B, D, 94 + r) for r in range(N)]
    rank_batches = [dq.LookupBatch.pooling_one(torch.from_numpy(P).cuda()) for P in Ps]
    ts.forward(rank_batches[0])
    s_fwd = ts.scale.cpu().numpy()
    wss, _, _, _ = _emulate_ranks(dq, ts, rank_batches, [torch.from_numpy(d).cuda() for d in dys], 8, 0.1)
    assert max(int(ws.ucount.cpu().max()) for ws in wss) * N > dq._lib.DQRM_SLOT_KEYS
    ar = np.arange(B, dtype=np.int64)
    O.dp_step(Ws, [[(Ps[r][t], ar) for t in range(T)] for r in range(N)],
              [[dys[r][t] for t in range(T)] for r in range(N)], s_fwd, 0.1, grad_bits=8)
    assert ts.read_errors() == 0
    for t in range(T):
        np.testing.assert_array_equal(ts.table_weight(t).cpu().numpy(), Ws[t])
    inc = [x.clone() for x in (ts.rowmax, ts.blkmax, ts.sblkmax, ts.tmax)]
    ts.refresh_absmax()
    for x, y in zip(inc, (ts.rowmax, ts.blkmax, ts.sblkmax, ts.tmax)):
        assert torch.equal(x, y)


def test_max_lookups_understated_is_flagged(dq):
    """A batch whose tables hold more lookups than dqrm_batch.max_lookups promised (the
    workspace's size) is skipped and flagged, never written out of bounds."""
    ts = make_set(dq, G.table_weights([100], 16, 3))
    W0 = ts.W.clone()
    b = dq.LookupBatch.pooling_one(torch.zeros(1, 9000, dtype=torch.int64, device="cuda"))
    b.c.max_lookups = 100
    ts.backward_sgd(b, torch.ones(1, 9000, 16, device="cuda"), lr=0.1)
    assert ts.read_errors() & dq._lib.DQRM_ERRF_OVERFLOW
    assert torch.equal(ts.W, W0)


def test_sgd_next_forward_understated_max_lookups_still_forwards(dq):
    """k_sgd_small with the next batch's forward (dqrm_emb_bwd_sgd_fwd, one launch) on a batch
    whose tables hold more lookups than dqrm_batch.max_lookups promised: the update is skipped
    and flagged (DQRM_ERRF_OVERFLOW), and the next batch's forward is still written -- equal to
    dqrm_emb_fwd on the unchanged tables, never left as garbage."""
    rows, D, B = [3, 500, 70000], 16, 128
    ts = dq.EmbeddingTableSet(rows, D, device="cuda", init="uniform", seed=4)
    W0 = ts.W.clone()
    b = dq.LookupBatch.pooling_one(torch.from_numpy(G.pooling_one(rows, B, 7)).cuda())
    nb = dq.LookupBatch.pooling_one(torch.from_numpy(G.pooling_one(rows, B, 8)).cuda())
    b.c.max_lookups = B - 28
    assert ts.sgd_fwd_is_one_launch(b, nb)
    out = torch.full((len(rows), B, D), 7.0, device="cuda")
    ts.backward_sgd_forward(b, torch.ones(len(rows), B, D, device="cuda"), 0.1, nb, out=out)
    assert ts.read_errors() & dq._lib.DQRM_ERRF_OVERFLOW
    assert torch.equal(ts.W, W0)
    assert torch.equal(out, ts.forward(nb))
    assert ts.read_errors() == 0


def test_presum_understated_max_lookups_is_flagged(dq):
    """dqrm_emb_bwd_lookup_grad_presum trusts no host-side bound: a table with more lookups
    than its LDS lists hold (DQRM_PRESUM_MAX_LOOKUPS), under a batch whose max_lookups
    understates it, is flagged DQRM_ERRF_OVERFLOW with its entries written as zero rows (no
    out-of-bounds LDS writes); the other table's entries are the normal presummed ones."""
    import ctypes as C
    from deep_quantized_recommendation_model_dqrm_amd import tables as TB

    rows, D = [50, 400], 16
    lens = [3000, 40]
    rng = np.random.default_rng(3)
    idxs = [rng.integers(0, n, size=l).astype(np.int64) for n, l in zip(rows, lens)]
    offs = [np.arange(l, dtype=np.int64)[:: max(1, l // 8)][:8] for l in lens]  # 8 bags per table
    ts = dq.EmbeddingTableSet(rows, D, device="cuda", init="uniform", seed=5)
    ts.scale.fill_(0.03)  # the STE's forward scale (no forward ran)
    b = to_batch(dq, idxs, offs)
    b.c.max_lookups = 100  # understated: table 0 has 3000 lookups
    dy = torch.from_numpy(G.upstream_grad(2, 8, D, 9)).cuda()
    Lk = sum(lens)
    r = torch.full((Lk,), -5, dtype=torch.int64, device="cuda")
    v = torch.full((Lk, D), 9.0, dtype=torch.float32, device="cuda")
    rc = ts.lib.dqrm_emb_bwd_lookup_grad_presum(C.byref(ts._c), C.byref(b.c), TB._ptr(dy), 8 * D, D, 1, TB._ptr(r),
                                                TB._ptr(v), TB._stream_handle())
    assert rc == 0
    assert ts.read_errors() & dq._lib.DQRM_ERRF_OVERFLOW
    assert torch.equal(r[:3000], torch.zeros(3000, dtype=torch.int64, device="cuda") + ts.row_base[0])
    assert torch.equal(v[:3000], torch.zeros(3000, D, device="cuda"))
    b2 = to_batch(dq, idxs[1:], offs[1:])  # table 1 alone, through the normal path
    ts1 = ts.view(1)
    ts1.scale.fill_(0.03)
    r1, v1 = ts1.lookup_grad(b2, dy[1:].contiguous(), presum=True)
    assert torch.equal(r[3000:] - ts.row_base[1], r1 - ts1.row_base[0])
    assert torch.equal(v[3000:], v1)


def test_kaggle_full_size_forward_and_step(dq):
    """Full Criteo-Kaggle tables (33.8M rows, D=16): forward of every table equals the
    oracle; after 3 SGD steps the scales still equal a full-table oracle scan."""
    rows = G.KAGGLE_ROWS
    ts = dq.EmbeddingTableSet(rows, 16, device="cuda", init="uniform", seed=11)
    B = 2048
    for k in range(3):
        P = G.pooling_one(rows, B, 40 + k, dist="zipf" if k % 2 else "uniform")
        b = dq.LookupBatch.pooling_one(torch.from_numpy(P).cuda())
        y = ts.forward(b).cpu().numpy()
        W = ts.W.cpu().numpy()
        s = ts.scale.cpu().numpy()
        for t in range(len(rows)):
            Wt = W[ts.row_base[t]: ts.row_base[t] + rows[t]]
            assert s[t] == O.table_scale(Wt, 4)
            yo, _ = O.emb_fwd(Wt, P[t], np.arange(B), s[t])
            np.testing.assert_array_equal(y[t], yo)
        dy = torch.from_numpy(G.upstream_grad(len(rows), B, 16, 50 + k)).cuda()
        ts.backward_sgd(b, dy, lr=0.1)
    assert ts.read_errors() == 0


def test_determinism_bitwise(dq):
    rows = [3, 1000, 200000]
    P = G.pooling_one(rows, 4096, 8, dist="zipf")
    dy = torch.from_numpy(G.upstream_grad(3, 4096, 64, 9)).cuda()
    outs = []
    for _ in range(2):
        ts = dq.EmbeddingTableSet(rows, 64, device="cuda", seed=4)
        b = dq.LookupBatch.pooling_one(torch.from_numpy(P).cuda())
        for _ in range(3):
            ts.forward(b)
            ts.backward_sgd(b, dy, lr=0.1)
        outs.append(ts.W.clone())
    assert torch.equal(outs[0], outs[1])


SORT_ROWS = [3, 62, 971, 5000, 300000]


def _table_slots(ws, t):
    """Concatenate table t's row-range slots of a coalesced workspace (host copies)."""
    from deep_quantized_recommendation_model_dqrm_amd import _lib as L

    ucount = ws.ucount.cpu().numpy()
    rows_all, vals_all = ws.rows.cpu().numpy(), ws.vals.cpu().numpy()
    rows, vals = [], []
    for k in range(t * L.DQRM_TABLE_SPLIT, (t + 1) * L.DQRM_TABLE_SPLIT):
        b = ws.slot_base[k]
        rows.append(rows_all[b: b + ucount[k]])
        vals.append(vals_all[b: b + ucount[k]])
    return np.concatenate(rows), np.concatenate(vals)


@pytest.mark.parametrize("D", [16, 64, 128])
@pytest.mark.parametrize("dist", ["uniform", "zipf", "bags"])
def test_slot_sort_and_segment_paths_bitexact(dq, D, dist):
    """Every per-slot sort strategy (register wave sort for <= 512 keys, radix on narrow
    row spans, LDS bitonic on crowded wide slots) and long segments that cross the LDS
    stage's chunks, in both the fused-SGD and the coalesce kernels, against the oracle."""
    rows = SORT_ROWS
    T = len(rows)
    Ws = G.table_weights(rows, D, 21)
    if dist == "bags":
        idxs, offs = G.random_bags(rows, 1024, 22, num_indices_per_lookup=6)
    else:
        P = G.pooling_one(rows, 4096, 22, dist=dist)
        idxs = [P[t] for t in range(T)]
        offs = [np.arange(P.shape[1], dtype=np.int64) for _ in range(T)]
    nb = len(offs[0])
    dy = G.upstream_grad(T, nb, D, 23)
    ts = make_set(dq, Ws)
    b = to_batch(dq, idxs, offs)
    ts.forward(b)
    s = ts.scale.cpu().numpy()
    ws = dq.CoalescedGrad.allocate(rows, b.max_lookups, D, "cuda")
    ts.backward_coalesce(b, torch.from_numpy(dy).cuda(), ws)
    for t in range(T):
        r_o, v_o, err = O.emb_bwd_coalesce(rows[t], idxs[t], offs[t], dy[t], s[t])
        assert err == 0
        r_g, v_g = _table_slots(ws, t)
        np.testing.assert_array_equal(r_g, r_o)
        np.testing.assert_array_equal(v_g, v_o)
    ts.backward_sgd(b, torch.from_numpy(dy).cuda(), lr=0.1)
    assert ts.read_errors() == 0
    for t in range(T):
        Wo = Ws[t].copy()
        O.emb_bwd_sgd(Wo, idxs[t], offs[t], dy[t], s[t], 0.1)
        np.testing.assert_array_equal(ts.table_weight(t).cpu().numpy(), Wo)
    tmax_inc = ts.tmax.clone()
    ts.refresh_absmax()
    torch.testing.assert_close(tmax_inc, ts.tmax, rtol=0, atol=0)


@pytest.mark.parametrize("grad_bits", [8, 32])
def test_exchange_many_ranks_long_segments(dq, grad_bits, apply_kernel):
    """N=12 emulated ranks: a row present in every rank's payload is a 12-entry segment in
    the apply kernel (the block-cooperative long-segment path); against oracle.dp_step."""
    rows, D, B, N = [3, 50, 2000], 32, 256, 12
    Ws = G.table_weights(rows, D, 31)
    ts = make_set(dq, Ws)
    Ps = [G.pooling_one(rows, B, 100 + r, dist="zipf") for r in range(N)]
    dys = [G.upstream_grad(len(rows), B, D, 200 + r) for r in range(N)]
    rank_batches = [dq.LookupBatch.pooling_one(torch.from_numpy(P).cuda()) for P in Ps]
    ts.forward(rank_batches[0])
    s_fwd = ts.scale.cpu().numpy()
    _emulate_ranks(dq, ts, rank_batches, [torch.from_numpy(d).cuda() for d in dys], grad_bits, 0.1)
    ar = np.arange(B, dtype=np.int64)
    O.dp_step(Ws, [[(Ps[r][t], ar) for t in range(len(rows))] for r in range(N)],
              [[dys[r][t] for t in range(len(rows))] for r in range(N)], s_fwd, 0.1, grad_bits=grad_bits)
    assert ts.read_errors() == 0
    for t in range(len(rows)):
        np.testing.assert_array_equal(ts.table_weight(t).cpu().numpy(), Ws[t])


@pytest.mark.parametrize("N", [1, 3, 6])
def test_apply_keeps_absmax_hierarchy_exact(dq, N, apply_kernel):
    """After the DP apply (large steps, so block-max holders shrink and other rows grow), the
    incrementally kept rowmax / block / superblock / table maxima equal a full rebuild from W
    (the flat kernel's atomicMax growth + bdirty/sdirty rescans, the slot kernel's block pass)."""
    rows, D, B = [7, 300, 70000, 400000], 16, 2048
    T = len(rows)
    Ws = G.table_weights(rows, D, 41)
    ts = make_set(dq, Ws)
    Ps = [G.pooling_one(rows, B, 300 + r, dist="zipf" if r % 2 else "uniform") for r in range(N)]
    dys = [G.upstream_grad(T, B, D, 400 + r) * 20 for r in range(N)]
    rank_batches = [dq.LookupBatch.pooling_one(torch.from_numpy(P).cuda()) for P in Ps]
    for it in range(3):
        ts.forward(rank_batches[0])
        _emulate_ranks(dq, ts, rank_batches, [torch.from_numpy(d).cuda() for d in dys], 8, 2.0 + it)
        assert ts.read_errors() == 0
        inc = [x.clone() for x in (ts.rowmax, ts.blkmax, ts.sblkmax, ts.tmax)]
        ts.refresh_absmax()
        for a, b in zip(inc, (ts.rowmax, ts.blkmax, ts.sblkmax, ts.tmax)):
            torch.testing.assert_close(a, b, rtol=0, atol=0)


@pytest.mark.parametrize("D,bits,repack", [(16, 8, False), (64, 8, True), (32, 4, False), (64, 16, False)])
def test_fused_local_apply_matches_payload_path_and_oracle(dq, D, bits, repack):
    """dqrm_apply_local (world size 1: quant-pack + apply fused) against the payload round
    trip (coalesce -> quant_pack -> apply) on a copy of the same tables, bit for bit (W,
    packed rows, s_avg and the |W| hierarchy), and against oracle.dp_step with N = 1."""
    from deep_quantized_recommendation_model_dqrm_amd import _lib as L
    from deep_quantized_recommendation_model_dqrm_amd.comm import HipExchangeKernels, payload_bytes

    rows, B = [3, 200, 5000, 300000], 1024
    T = len(rows)
    Ws = G.table_weights(rows, D, 51)
    P = G.pooling_one(rows, B, 52, dist="zipf")
    dy = G.upstream_grad(T, B, D, 53) * 10
    b = dq.LookupBatch.pooling_one(torch.from_numpy(P).cuda())
    sets = [make_set(dq, Ws, packed=repack) for _ in range(2)]
    s_avg = [torch.zeros(T, dtype=torch.float32, device="cuda") for _ in range(2)]
    caps = dq.default_caps(rows, B)
    cap_base = torch.tensor(np.concatenate([[0], np.cumsum(caps)]), dtype=torch.int64, device="cuda")
    cap_total = int(sum(caps))
    Pb = payload_bytes(T, cap_total, D, bits)
    payload = torch.zeros(1, Pb, dtype=torch.uint8, device="cuda")
    for it in range(3):
        for j, ts in enumerate(sets):
            if repack:
                ts.refresh_scale_and_pack(4)
            ts.forward(b)
            k = HipExchangeKernels(ts)
            ws = dq.CoalescedGrad.allocate(rows, B, D, "cuda")
            k.coalesce(b, torch.from_numpy(dy).cuda(), ws, True, "tbd")
            if j == 0:
                k.apply_local(ws, bits, s_avg[0], 0.5, repack)
            else:
                k.quant_pack(ws, ws.absmax.view(1, -1), 1, bits, cap_base, cap_total, s_avg[1], payload[0])
                k.apply(cap_base, cap_total, payload, Pb, 1, bits, s_avg[1], 0.5, L.DQRM_UPD_DP, repack)
        assert torch.equal(s_avg[0], s_avg[1])
        for name in ("W", "rowmax", "blkmax", "sblkmax", "tmax") + (("packed",) if repack else ()):
            assert torch.equal(getattr(sets[0], name), getattr(sets[1], name)), name
    assert sets[0].read_errors() == 0
    # one more fused step against the oracle's DP update with N = 1
    ts = make_set(dq, Ws)
    ts.forward(b)
    s_fwd = ts.scale.cpu().numpy()
    ex = dq.SparseGradExchange(ts, B, grad_bits=bits)
    ex.step(b, torch.from_numpy(dy).cuda(), lr=0.5)
    ar = np.arange(B, dtype=np.int64)
    Wo = [w.copy() for w in Ws]
    O.dp_step(Wo, [[(P[t], ar) for t in range(T)]], [[dy[t] for t in range(T)]], s_fwd, 0.5, grad_bits=bits)
    assert ts.read_errors() == 0
    for t in range(T):
        np.testing.assert_array_equal(ts.table_weight(t).cpu().numpy(), Wo[t])


def test_pooling_one_flag_matches_offsets_path(dq):
    """DQRM_BATCH_POOLING_ONE (offsets not read) gives the same forward, SGD and coalesce as
    the general offsets path on the same Criteo-form batch."""
    rows, D = [5, 3000, 200000], 64
    Ws = G.table_weights(rows, D, 71)
    P = torch.from_numpy(G.pooling_one(rows, 2048, 72, dist="zipf")).cuda()
    dy = torch.from_numpy(G.upstream_grad(len(rows), 2048, D, 73)).cuda()
    off = torch.arange(2048, device="cuda").expand(len(rows), 2048).contiguous()
    outs = []
    for b in (dq.LookupBatch.pooling_one(P), dq.LookupBatch(P, off)):
        assert b.c.flags == (1 if b.pooling_one else 0)
        ts = make_set(dq, Ws)
        y = ts.forward(b)
        ws = dq.CoalescedGrad.allocate(rows, 2048, D, "cuda")
        ts.backward_coalesce(b, dy, ws)
        ts.backward_sgd(b, dy, lr=0.1)
        outs.append((y.clone(), ws.vals.clone(), ws.rows.clone(), ts.W.clone()))
    for x, z in zip(*outs):
        assert torch.equal(x, z)


def test_data_parallel_cpu_native_fixture_within_tolerance(dq, golden_dir):
    """dp_n4_cpu_native.npz keeps torch-CPU's own coalesce order (an unstable sort, a
    library artifact; the reference's CUDA runs sum in lookup order). The HIP exchange sums
    in ascending lookup position, so against this fixture it holds the tolerance the CPU
    oracle test states (test_oracle_golden.py): scales within 2 ulp, rows exact, quantized
    ints within +-1 on <= 1 % of entries, weights within 1e-5. Against oracle.dp_step
    (same order) it is bit-exact."""
    fx = load(golden_dir, "dp_n4_cpu_native.npz")
    num_rows = fx["num_rows"].tolist()
    D, seed, N = int(fx["D"]), int(fx["seed"]), int(fx["N"])
    T = len(num_rows)
    Ws = G.table_weights(num_rows, D, seed)
    Wo = [w.copy() for w in Ws]
    ts = make_set(dq, Ws)
    n_q = n_diff = 0
    for k in range(int(fx["steps"])):
        b, dys = dp_inputs(fx, k)
        rank_batches = [to_batch(dq, [x[0] for x in b[r]], [x[1] for x in b[r]]) for r in range(N)]
        rank_dys = [torch.from_numpy(np.stack(dys[r])).cuda() for r in range(N)]
        for rb in rank_batches:
            ts.forward(rb, refresh_scale=True)
        s_fwd = ts.scale.cpu().numpy()
        wss, payloads, s_avg, cb = _emulate_ranks(dq, ts, rank_batches, rank_dys, 8, float(fx["lr"]))
        res = O.dp_step(Wo, b, dys, list(s_fwd), float(fx["lr"]), grad_bits=8)
        for t in range(T):
            assert s_avg[t].item() == res[t][0]
            ref = fx[f"k{k}_t{t}_s_avg"]
            assert abs(s_avg[t].item() - float(ref)) <= 2 * np.spacing(np.float32(ref))
            for r in range(N):
                rows, q = _decode_payload(payloads[r], T, cb, D, 8, t)
                np.testing.assert_array_equal(rows, fx[f"k{k}_t{t}_r{r}_rows"])
                np.testing.assert_array_equal(q, res[t][2][r])
                d = np.abs(q - fx[f"k{k}_t{t}_r{r}_q"])
                assert d.max() <= 1
                n_q += d.size
                n_diff += int((d > 0).sum())
    assert n_diff <= max(1, n_q // 100)
    assert ts.read_errors() == 0
    for t in range(T):
        W = ts.table_weight(t).cpu().numpy()
        np.testing.assert_array_equal(W, Wo[t])
        np.testing.assert_allclose(W[fx[f"rows_t{t}"]], fx[f"w_t{t}"], rtol=0, atol=1e-5)


# BASELINE config 5 shape: the Terabyte profile (D=64) with the big tables capped so the
# oracle's host copies stay small; at least one >= 300k-row table
C5_ROWS = [min(n, 300_000) for n in G.TERABYTE_ROWS]


@pytest.mark.parametrize("grad_bits", [8, 32])
@pytest.mark.parametrize("dist", ["uniform", "zipf"])
def test_config5_exchange_n8_d64(dq, dist, grad_bits, apply_kernel):
    """Config 5's exchange: N=8 emulated ranks at D=64 on TB-shaped tables, global batch
    2048 strong-scaled (256 per rank), two steps with the forward scale
    refreshed in between; both apply kernels; against oracle.dp_step, then the |W|
    hierarchy equals a rebuild."""
    rows, D, N, Bg = C5_ROWS, 64, 8, 2048
    T = len(rows)
    Ws = G.table_weights(rows, D, 141)
    ts = make_set(dq, Ws)
    for k in range(2):
        P = G.pooling_one(rows, Bg, 142 + k, dist=dist)
        dy = G.upstream_grad(T, Bg, D, 150 + k)
        sls = [dq.get_my_slice(Bg, N, r) for r in range(N)]
        Ps = [np.ascontiguousarray(P[:, sl]) for sl in sls]
        dys = [np.ascontiguousarray(dy[:, sl]) for sl in sls]
        rank_batches = [dq.LookupBatch.pooling_one(torch.from_numpy(x).cuda()) for x in Ps]
        ts.forward(rank_batches[0])
        s_fwd = ts.scale.cpu().numpy()
        for t in range(T):
            assert s_fwd[t] == O.table_scale(Ws[t], 4)
        _, _, s_avg, _ = _emulate_ranks(dq, ts, rank_batches, [torch.from_numpy(d).cuda() for d in dys],
                                        grad_bits, 0.1)
        ar = np.arange(Bg // N, dtype=np.int64)
        res = O.dp_step(Ws, [[(Ps[r][t], ar) for t in range(T)] for r in range(N)],
                        [[dys[r][t] for t in range(T)] for r in range(N)], list(s_fwd), 0.1, grad_bits=grad_bits)
        if grad_bits != 32:
            np.testing.assert_array_equal(s_avg.cpu().numpy(), np.array([x[0] for x in res], np.float32))
    assert ts.read_errors() == 0
    for t in range(T):
        np.testing.assert_array_equal(ts.table_weight(t).cpu().numpy(), Ws[t])
    inc = [x.clone() for x in (ts.rowmax, ts.blkmax, ts.sblkmax, ts.tmax)]
    ts.refresh_absmax()
    for x, y in zip(inc, (ts.rowmax, ts.blkmax, ts.sblkmax, ts.tmax)):
        assert torch.equal(x, y)


@pytest.mark.parametrize("dist", ["uniform", "zipf"])
def test_config4_kaggle_full_tables_n4(dq, dist, apply_kernel):
    """BASELINE config 4 at its own shape (run_dlrm_kaggle_gpu_gtone.sh:1): the 26 full
    Kaggle tables (33.8 M rows, D=16, on-device init), 4 emulated ranks x 128 samples (global
    512), INT8 gradients, two steps, both apply kernels. Every touched row equals oracle.dp_step
    on the compacted rows, the averaged scales equal the oracle's, untouched rows keep their
    bits, and the incrementally kept |W| hierarchy equals a rebuild."""
    rows, D, N, Bg = list(G.KAGGLE_ROWS), 16, 4, 512
    T = len(rows)
    torch.cuda.empty_cache()
    ts = dq.EmbeddingTableSet(rows, D, device="cuda", init="uniform", seed=91)
    try:
        for k in range(2):
            P = G.pooling_one(rows, Bg, 190 + k, dist=dist)
            dy = G.upstream_grad(T, Bg, D, 195 + k)
            sls = [dq.get_my_slice(Bg, N, r) for r in range(N)]
            Ps = [np.ascontiguousarray(P[:, sl]) for sl in sls]
            dys = [np.ascontiguousarray(dy[:, sl]) for sl in sls]
            rank_batches = [dq.LookupBatch.pooling_one(torch.from_numpy(x).cuda()) for x in Ps]
            ts.forward(rank_batches[0])
            s_fwd = ts.scale.cpu().numpy()
            compact, before, probe = [], [], []
            for t in range(T):  # the rows the step may touch, compacted (host copies stay small)
                u, inv = np.unique(P[t], return_inverse=True)
                compact.append((u, inv.astype(np.int64).reshape(P[t].shape)))
                Wt = ts.table_weight(t)
                before.append(Wt[torch.from_numpy(u).cuda()].cpu().numpy())
                mn, mx = torch.aminmax(Wt)
                assert s_fwd[t] == O.sym_scale(max(-float(mn), float(mx)), 4)
                free = np.setdiff1d(np.arange(min(rows[t], 4096)), u)[:64]  # untouched rows
                probe.append((free, Wt[torch.from_numpy(free).cuda()].cpu().numpy()))
            _, _, s_avg, _ = _emulate_ranks(dq, ts, rank_batches, [torch.from_numpy(d).cuda() for d in dys], 8, 0.1)
            ar = np.arange(Bg // N, dtype=np.int64)
            res = O.dp_step(before, [[(compact[t][1][sl], ar) for t in range(T)] for sl in sls],
                            [[dys[r][t] for t in range(T)] for r in range(N)], list(s_fwd), 0.1, grad_bits=8)
            np.testing.assert_array_equal(s_avg.cpu().numpy(), np.array([x[0] for x in res], np.float32))
            for t in range(T):
                got = ts.table_weight(t)[torch.from_numpy(compact[t][0]).cuda()].cpu().numpy()
                np.testing.assert_array_equal(got, before[t])
                free, wf = probe[t]
                np.testing.assert_array_equal(ts.table_weight(t)[torch.from_numpy(free).cuda()].cpu().numpy(), wf)
        assert ts.read_errors() == 0
        inc = [x.clone() for x in (ts.rowmax, ts.blkmax, ts.sblkmax, ts.tmax)]
        ts.refresh_absmax()
        for x, y in zip(inc, (ts.rowmax, ts.blkmax, ts.sblkmax, ts.tmax)):
            assert torch.equal(x, y)
    finally:
        del ts
        torch.cuda.empty_cache()


def test_terabyte_full_size_773m_rows(dq):
    """The bench's N=1 workload at full size (26 tables, 773,280,534 rows x 64, 198 GB in
    HBM): forward of every table equals the oracle on the rows it reads, the per-step table
    scales equal a full-table max computed independently (torch.amax), two DP steps update
    exactly the oracle's rows, and the incrementally kept |W| hierarchy equals a rebuild."""
    from deep_quantized_recommendation_model_dqrm_amd.workloads import TERABYTE_X16_ROWS

    rows, D, B = TERABYTE_X16_ROWS, 64, 2048
    T = len(rows)
    torch.cuda.empty_cache()
    ts = dq.EmbeddingTableSet(rows, D, device="cuda", init="uniform", seed=77)
    ex = dq.SparseGradExchange(ts, B, grad_bits=8)
    try:
        for k in range(2):
            P = G.pooling_one(rows, B, 160 + k, dist="zipf" if k else "uniform")
            dy = G.upstream_grad(T, B, D, 170 + k)
            b = dq.LookupBatch.pooling_one(torch.from_numpy(P).cuda())
            y = ts.forward(b).cpu().numpy()
            s = ts.scale.cpu().numpy()
            compact, before = [], []
            for t in range(T):
                Wt = ts.table_weight(t)
                mn, mx = torch.aminmax(Wt)  # no table-sized temporary (the largest is 41 GB)
                assert s[t] == O.sym_scale(max(-float(mn), float(mx)), 4)
                u, inv = np.unique(P[t], return_inverse=True)
                Wu = Wt[torch.from_numpy(u).cuda()].cpu().numpy()
                yo, _ = O.emb_fwd(Wu, inv.astype(np.int64), np.arange(B), s[t])
                np.testing.assert_array_equal(y[t], yo)
                compact.append((u, inv.astype(np.int64)))
                before.append(Wu)
            ex.step(b, torch.from_numpy(dy).cuda(), lr=0.1)
            O.dp_step(before, [[(c[1], np.arange(B)) for c in compact]], [[dy[t] for t in range(T)]], list(s), 0.1)
            for t in range(T):
                got = ts.table_weight(t)[torch.from_numpy(compact[t][0]).cuda()].cpu().numpy()
                np.testing.assert_array_equal(got, before[t])
        assert ts.read_errors() == 0
        inc = [x.clone() for x in (ts.blkmax, ts.sblkmax, ts.tmax)]
        rm = ts.rowmax.clone()
        ts.refresh_absmax()
        assert torch.equal(rm, ts.rowmax)
        del rm
        for x, z in zip(inc, (ts.blkmax, ts.sblkmax, ts.tmax)):
            assert torch.equal(x, z)
    finally:
        del ts, ex
        torch.cuda.empty_cache()


def test_terabyte_full_size_step_boundary_773m_rows(dq):
    """The exact form bench.py times at N=1 (bench.py step(): backward_apply_forward_local,
    k_coalesce_p1<APPLY> with the next batch's forward inside the launch) on the full
    773,280,534-row TB slab, pinned to the oracle on EVERY table over two steps: the first
    forward, then per step the averaged gradient scale s_avg, every row any of the batches
    touches (updated rows = oracle.dp_step, the others unchanged), the next batch's forward
    scale (= a full-table max taken independently with torch.aminmax) and the next batch's
    fake-quantized output (= oracle.emb_fwd on the updated rows); at the end the incremental
    |W| hierarchy equals a rebuild. Reference: quant_modules_not_quantize_grad.py:317-398,
    sgd_quantized_gradients_parallel_comm.py:601-628,850-890 (world size 1)."""
    from deep_quantized_recommendation_model_dqrm_amd.workloads import TERABYTE_X16_ROWS

    rows, D, B = TERABYTE_X16_ROWS, 64, 2048
    T = len(rows)
    torch.cuda.empty_cache()
    ts = dq.EmbeddingTableSet(rows, D, device="cuda", init="uniform", seed=78)
    ex = dq.SparseGradExchange(ts, B, grad_bits=8)
    try:
        Ps = [G.pooling_one(rows, B, 180 + k, dist="zipf" if k == 1 else "uniform") for k in range(3)]
        bs = [dq.LookupBatch.pooling_one(torch.from_numpy(P).cuda()) for P in Ps]
        assert ts.apply_fwd_local_is_one_launch(bs[0], bs[1])
        # compact host copies of every row the three batches touch, per table
        uniq, inv, Wc = [], [], []
        for t in range(T):
            u, iv = np.unique(np.concatenate([P[t] for P in Ps]), return_inverse=True)
            uniq.append(torch.from_numpy(u).cuda())
            inv.append([iv[k * B:(k + 1) * B].astype(np.int64) for k in range(3)])
            Wc.append(ts.table_weight(t)[uniq[t]].cpu().numpy())

        def full_scales():
            out = []
            for t in range(T):
                mn, mx = torch.aminmax(ts.table_weight(t))  # no table-sized temporary (largest 41 GB)
                out.append(O.sym_scale(max(-float(mn), float(mx)), 4))
            return np.array(out, dtype=np.float32)

        ar = np.arange(B, dtype=np.int64)
        y = ts.forward(bs[0]).cpu().numpy()
        s = full_scales()
        np.testing.assert_array_equal(ts.scale.cpu().numpy(), s)
        for t in range(T):
            np.testing.assert_array_equal(y[t], O.emb_fwd(Wc[t], inv[t][0], ar, s[t])[0])
        for k in range(2):
            dy = G.upstream_grad(T, B, D, 190 + k)
            yn = ts.backward_apply_forward_local(bs[k], torch.from_numpy(dy).cuda(), ex.ws, 8, ex.s_avg, 0.1,
                                                 bs[k + 1]).cpu().numpy()
            res = O.dp_step(Wc, [[(inv[t][k], ar) for t in range(T)]], [[dy[t] for t in range(T)]], list(s), 0.1)
            np.testing.assert_array_equal(ex.s_avg.cpu().numpy(), np.array([r[0] for r in res], np.float32))
            for t in range(T):
                np.testing.assert_array_equal(ts.table_weight(t)[uniq[t]].cpu().numpy(), Wc[t], err_msg=f"W {k} {t}")
            s = full_scales()
            np.testing.assert_array_equal(ts.scale.cpu().numpy(), s)
            for t in range(T):
                np.testing.assert_array_equal(yn[t], O.emb_fwd(Wc[t], inv[t][k + 1], ar, s[t])[0],
                                              err_msg=f"forward {k} {t}")
        assert ts.read_errors() == 0
        inc = [x.clone() for x in (ts.blkmax, ts.sblkmax, ts.tmax)]
        rm = ts.rowmax.clone()
        ts.refresh_absmax()
        assert torch.equal(rm, ts.rowmax)
        del rm
        for x, z in zip(inc, (ts.blkmax, ts.sblkmax, ts.tmax)):
            assert torch.equal(x, z)
    finally:
        del ts, ex
        torch.cuda.empty_cache()


COAL_ROWS = [3, 62, 971, 1435, 1792, 1793, 2208, 7112, 32768, 300000, 20_000_000]


@pytest.fixture
def general_coalesce(dq):
    """Force dqrm_emb_bwd_coalesce onto the general kernel for the duration of a block."""
    L = dq._lib
    lib = L.load()

    class _Ctx:
        def __enter__(self):
            self.prev = lib.dqrm_set_coalesce_kernel(L.DQRM_COALESCE_GENERAL)

        def __exit__(self, *exc):
            lib.dqrm_set_coalesce_kernel(self.prev)

    return _Ctx()


@pytest.mark.parametrize("D,B,dist", [(64, 2048, "uniform"), (64, 2048, "zipf"), (16, 2048, "uniform"),
                                      (16, 4096, "zipf"), (128, 2048, "uniform"), (32, 128, "uniform"),
                                      (64, 1, "uniform"), (4, 3000, "zipf"), (256, 700, "zipf")])
def test_criteo_form_coalesce_bitexact(dq, general_coalesce, D, B, dist):
    """The Criteo-form coalesce kernel (dqrm_coalesce.hip: dimension-split tables of < 8
    row blocks incl. the 1792/1793-row boundary; row spans <= 256 by ballot-ranked row
    counting, spans up to 4096 rows (32768-row table: exactly 4096) by atomic row counting
    with the comparison sort as the crowded (Zipf) fallback, wider spans by the MSD sort;
    chunked stages for slots larger than LDS) writes exactly the oracle's
    coalesced rows and values, the same counts as the general kernel, and per-table maxima
    equal to max|vals|; out-of-range indices are flagged and left out."""
    rows = COAL_ROWS
    T = len(rows)
    rng = np.random.default_rng(B * 7 + D)
    P = G.pooling_one(rows, B, 61 + D, dist=dist)
    if B > 8:
        P[0, 5] = 3          # out of range on the 3-row table
        P[2, 7] = -1         # negative on the 971-row table
    dy = G.upstream_grad(T, B, D, 62 + D)
    ts = dq.EmbeddingTableSet(rows, D, device="cuda", init="uniform", seed=5)
    scale = torch.from_numpy(rng.uniform(0.01, 0.1, size=T).astype(f32)).cuda()
    ts.scale.copy_(scale)
    b = dq.LookupBatch.pooling_one(torch.from_numpy(P).cuda())
    dyt = torch.from_numpy(dy).cuda()
    ws = dq.CoalescedGrad.allocate(rows, B, D, "cuda")
    ts.backward_coalesce(b, dyt, ws)
    err = ts.read_errors()
    ws_g = dq.CoalescedGrad.allocate(rows, B, D, "cuda")
    with general_coalesce:
        ts.backward_coalesce(b, dyt, ws_g)
    assert ts.read_errors() == err
    if B > 8:
        assert err & dq._lib.DQRM_ERRF_INDEX
    s = scale.cpu().numpy()
    ar = np.arange(B, dtype=np.int64)
    assert torch.equal(ws.ucount, ws_g.ucount)
    for t in range(T):
        r_o, v_o, _ = O.emb_bwd_coalesce(rows[t], P[t], ar, dy[t], s[t])
        r_n, v_n = _table_slots(ws, t)
        np.testing.assert_array_equal(r_n, r_o)
        np.testing.assert_array_equal(v_n, v_o)
        am = ws.absmax.view(T, -1)[t].max().item()
        assert am == (np.abs(v_o).max() if v_o.size else 0.0)
        assert am == ws_g.absmax.view(T, -1)[t].max().item()


@pytest.mark.parametrize("D,B,dist,bits,repack", [(64, 2048, "uniform", 8, False), (64, 2048, "zipf", 8, True),
                                                  (16, 2048, "uniform", 8, False), (16, 4096, "zipf", 4, False),
                                                  (4, 3000, "zipf", 8, False), (8, 700, "uniform", 16, False),
                                                  (256, 700, "zipf", 8, False), (32, 1, "uniform", 8, False)])
def test_fused_coalesce_apply_matches_two_launches(dq, D, B, dist, bits, repack):
    """dqrm_emb_bwd_apply_local (coalesce + local update in one launch: the table's
    workgroups meet once for the gradient maxima, then update their row ranges) against
    dqrm_emb_bwd_coalesce + dqrm_apply_local on a copy of the same tables, bit for bit over
    three steps with large updates (block-max holders shrink, other rows grow): W, packed
    rows, s_avg, rowmax / block / superblock / table maxima and the workspace's rows, counts
    and maxima (its values are scratch in the one-launch call); the kept hierarchy equals a
    rebuild; out-of-range indices raise the same flags."""
    from deep_quantized_recommendation_model_dqrm_amd.comm import HipExchangeKernels

    rows = COAL_ROWS
    T = len(rows)
    sets = [dq.EmbeddingTableSet(rows, D, device="cuda", packed=repack, init="uniform", seed=91) for _ in range(2)]
    assert torch.equal(sets[0].W, sets[1].W)
    s_avg = [torch.zeros(T, dtype=torch.float32, device="cuda") for _ in range(2)]
    for it in range(3):
        P = G.pooling_one(rows, B, 93 + it, dist=dist)
        if B > 8 and it == 1:
            P[0, 5] = 3          # out of range on the 3-row table
            P[2, 7] = -1         # negative on the 971-row table
        dy = torch.from_numpy(G.upstream_grad(T, B, D, 95 + it) * 30).cuda()
        b = dq.LookupBatch.pooling_one(torch.from_numpy(P).cuda())
        wss = []
        for j, ts in enumerate(sets):
            if repack:
                ts.refresh_scale_and_pack(4)
            ts.forward(b)
            ws = dq.CoalescedGrad.allocate(rows, B, D, "cuda")
            if j == 0:
                ts.backward_apply_local(b, dy, ws, bits, s_avg[0], 0.5, repack=repack)
            else:
                ts.backward_coalesce(b, dy, ws)
                HipExchangeKernels(ts).apply_local(ws, bits, s_avg[1], 0.5, repack)
            wss.append(ws)
        errs = [ts.read_errors() for ts in sets]
        assert errs[0] == errs[1]
        assert (errs[0] != 0) == (B > 8 and it == 1)
        assert torch.equal(s_avg[0], s_avg[1])
        assert torch.equal(wss[0].ucount, wss[1].ucount)
        assert torch.equal(wss[0].absmax, wss[1].absmax)
        for t in range(T):  # the one-launch call leaves workspace values scratch (kept on chip), and
            r0, _ = _table_slots(wss[0], t)  # a slot of distinct rows in lookup order (no sort)
            r1, _ = _table_slots(wss[1], t)
            np.testing.assert_array_equal(np.sort(r0), r1)
        for name in ("W", "rowmax", "blkmax", "sblkmax", "tmax") + (("packed",) if repack else ()):
            assert torch.equal(getattr(sets[0], name), getattr(sets[1], name)), (it, name)
    inc = [x.clone() for x in (sets[0].rowmax, sets[0].blkmax, sets[0].sblkmax, sets[0].tmax)]
    sets[0].refresh_absmax()
    for x, y in zip(inc, (sets[0].rowmax, sets[0].blkmax, sets[0].sblkmax, sets[0].tmax)):
        assert torch.equal(x, y)


def test_fused_step_alternating_set_and_view(dq):
    """The one-launch step alternately on an 8-table set (no spare workgroups: no sub-slots)
    and on a one-table view of its 100 k-row table (the view's spare groups give that table a
    second workgroup per slot): the two plans share the table's granules, so the sub-slots
    must agree on the launch epoch whatever ran before. Every step equals the two-launch path
    on a copy, and no stall is flagged."""
    from deep_quantized_recommendation_model_dqrm_amd.comm import HipExchangeKernels

    rows = [3, 971, 100000, 2208, 40000, 7, 5000, 300]
    T, D, B, tv = len(rows), 32, 1024, 2
    sets = [dq.EmbeddingTableSet(rows, D, device="cuda", init="uniform", seed=17) for _ in range(2)]
    views = [s.view(tv) for s in sets]
    s_avg = [torch.zeros(T, dtype=torch.float32, device="cuda") for _ in range(2)]
    sv_avg = [torch.zeros(1, dtype=torch.float32, device="cuda") for _ in range(2)]
    for it in range(6):
        P = G.pooling_one(rows, B, 301 + it)
        dy = torch.from_numpy(G.upstream_grad(T, B, D, 311 + it) * 30).cuda()
        on_view = it % 2 == 1
        if on_view:
            b = dq.LookupBatch.pooling_one(torch.from_numpy(P[tv: tv + 1].copy()).cuda())
            d = dy[tv: tv + 1].contiguous()
            targets, avg, nr = views, sv_avg, [rows[tv]]
        else:
            b = dq.LookupBatch.pooling_one(torch.from_numpy(P).cuda())
            d = dy
            targets, avg, nr = sets, s_avg, rows
        assert targets[0].apply_local_is_one_launch(b)
        for j, ts in enumerate(targets):
            ts.forward(b)
            ws = dq.CoalescedGrad.allocate(nr, B, D, "cuda")
            if j == 0:
                ts.backward_apply_local(b, d, ws, 8, avg[0], 0.5)
            else:
                ts.backward_coalesce(b, d, ws)
                HipExchangeKernels(ts).apply_local(ws, 8, avg[1], 0.5, False)
        assert [s.read_errors() for s in sets] == [0, 0], it
        assert torch.equal(avg[0], avg[1]), it
        for name in ("W", "rowmax", "blkmax", "sblkmax", "tmax"):
            assert torch.equal(getattr(sets[0], name), getattr(sets[1], name)), (it, name)


@pytest.mark.parametrize("B,D,dist", [(128, 16, "uniform"), (128, 16, "zipf"), (256, 16, "zipf"), (64, 64, "uniform"),
                                      (100, 4, "zipf"), (500, 8, "uniform"), (1, 16, "uniform"),
                                      # D = 32 at B = 512 / 400: the row hash no longer fits LDS
                                      # beside the dy stage; the batch takes k_bwd_fused
                                      (512, 32, "uniform"), (400, 32, "zipf")])
def test_sgd_small_criteo_form_matches_oracle(dq, B, D, dist):
    """The one-workgroup-per-table SGD kernel on Criteo-form batches (config 3: its row hash
    of position masks replaces the duplicate scan): three steps on tables from 3 rows (~B/3
    lookups per row, walked in position order) to 2 M rows equal the oracle's per-lookup
    torch.optim.SGD order bit for bit, in W and in the kept |W| hierarchy."""
    rows = [3, 4, 10, 27, 305, 3194, 100000, 2_000_000]
    T = len(rows)
    Ws = G.table_weights(rows, D, 21 + B)
    ts = make_set(dq, Ws)
    for it in range(3):
        P = G.pooling_one(rows, B, 22 + it, dist=dist)
        dy = G.upstream_grad(T, B, D, 25 + it) * 5
        b = dq.LookupBatch.pooling_one(torch.from_numpy(P).cuda())
        ts.forward(b)
        ts.backward_sgd(b, torch.from_numpy(dy).cuda(), lr=0.1)
        for t in range(T):
            O.emb_bwd_sgd(Ws[t], P[t], np.arange(B, dtype=np.int64), dy[t], O.table_scale(Ws[t], 4), 0.1)
    assert ts.read_errors() == 0
    for t in range(T):
        np.testing.assert_array_equal(ts.table_weight(t).cpu().numpy(), Ws[t])
    inc = [x.clone() for x in (ts.rowmax, ts.blkmax, ts.sblkmax, ts.tmax)]
    ts.refresh_absmax()
    for x, y in zip(inc, (ts.rowmax, ts.blkmax, ts.sblkmax, ts.tmax)):
        assert torch.equal(x, y)


@pytest.mark.parametrize("D,B,dist,layout,refresh,full", [(64, 2048, "uniform", "tbd", True, False),
                                                          (64, 2048, "zipf", "btd", True, False),
                                                          (16, 2048, "uniform", "btd", True, False),
                                                          (16, 4096, "zipf", "tbd", False, False),
                                                          (32, 1000, "uniform", "tbd", True, True),
                                                          (256, 700, "zipf", "btd", True, False)])
def test_fused_next_forward_matches_separate_calls(dq, D, B, dist, layout, refresh, full):
    """dqrm_emb_bwd_apply_fwd_local -- the one-launch update of step i with the forward of
    batch i+1 inside the same launch (each table's workgroups gather its next rows once the
    table's update and |W| maxima are final) -- against dqrm_emb_bwd_apply_local followed by
    dqrm_emb_fwd on a copy of the tables, bit for bit over four steps: the forward outputs,
    the forward scale, W, s_avg and the |W| hierarchy. Tables: dimension-split (3 ... 1793
    rows), row-split with and without sub-slots (2208 ... 20 M rows); out-of-range indices in
    a next batch give zeros and the same flag. Reference: apply_emb (dlrm_s_pytorch_single_gpu.py
    :609-674) after weight_update_parallel_comm (s_q_g_p_c.py:601-628)."""
    rows = COAL_ROWS
    T = len(rows)
    sets = [dq.EmbeddingTableSet(rows, D, device="cuda", init="uniform", seed=131) for _ in range(2)]
    s_avg = [torch.zeros(T, dtype=torch.float32, device="cuda") for _ in range(2)]
    Ps = [G.pooling_one(rows, B, 141 + k, dist=dist) for k in range(5)]
    Ps[2][0, 11] = 3       # out of range on the 3-row table (the forward of step 1's next batch)
    Ps[2][5, 9] = -2       # negative on a row-split table
    bs = [dq.LookupBatch.pooling_one(torch.from_numpy(P).cuda()) for P in Ps]
    assert sets[0].apply_fwd_local_is_one_launch(bs[0], bs[1])
    kw = dict(refresh_scale=refresh, full_precision=full, layout=layout)
    ys = [ts.forward(bs[0], **kw) for ts in sets]
    assert torch.equal(ys[0], ys[1])
    for it in range(4):
        dy = torch.from_numpy(G.upstream_grad(T, B, D, 151 + it) * 30).cuda()
        ws = [dq.CoalescedGrad.allocate(rows, B, D, "cuda") for _ in range(2)]
        y0 = sets[0].backward_apply_forward_local(bs[it], dy, ws[0], 8, s_avg[0], 0.5, bs[it + 1], **kw)
        sets[1].backward_apply_local(bs[it], dy, ws[1], 8, s_avg[1], 0.5)
        y1 = sets[1].forward(bs[it + 1], **kw)
        errs = [ts.read_errors() for ts in sets]
        assert errs[0] == errs[1] and (errs[0] != 0) == (it in (1, 2)), (it, errs)  # forward, then backward
        assert torch.equal(y0, y1), it
        assert torch.equal(s_avg[0], s_avg[1]), it
        for name in ("W", "rowmax", "blkmax", "sblkmax", "tmax", "scale"):
            assert torch.equal(getattr(sets[0], name), getattr(sets[1], name)), (it, name)
    # and the last output is the oracle's forward of the updated tables (every table)
    for t in range(T):
        yt = (y0[t] if layout == "tbd" else y0[:, t]).cpu().numpy()
        Wt = sets[0].table_weight(t).cpu().numpy()
        st = np.float32(1.0) if full else np.float32(sets[0].scale[t].item())
        want, _ = O.emb_fwd(Wt, Ps[4][t], np.arange(B, dtype=np.int64), st, 4, full_precision=full)
        np.testing.assert_array_equal(yt, want)


def test_fused_next_forward_packed_falls_back(dq):
    """A next batch the fused forward does not take (a different batch size) runs as the two
    calls, with the same results."""
    rows, D = [3, 971, 40000, 2208], 32
    T = len(rows)
    sets = [dq.EmbeddingTableSet(rows, D, device="cuda", init="uniform", seed=5) for _ in range(2)]
    s_avg = [torch.zeros(T, dtype=torch.float32, device="cuda") for _ in range(2)]
    b = dq.LookupBatch.pooling_one(torch.from_numpy(G.pooling_one(rows, 512, 1)).cuda())
    nb = dq.LookupBatch.pooling_one(torch.from_numpy(G.pooling_one(rows, 256, 2)).cuda())
    assert not sets[0].apply_fwd_local_is_one_launch(b, nb)
    dy = torch.from_numpy(G.upstream_grad(T, 512, D, 3) * 30).cuda()
    ws = [dq.CoalescedGrad.allocate(rows, 512, D, "cuda") for _ in range(2)]
    for ts in sets:
        ts.forward(b)
    y0 = sets[0].backward_apply_forward_local(b, dy, ws[0], 8, s_avg[0], 0.5, nb)
    sets[1].backward_apply_local(b, dy, ws[1], 8, s_avg[1], 0.5)
    y1 = sets[1].forward(nb)
    assert torch.equal(y0, y1)
    assert torch.equal(sets[0].W, sets[1].W)


def test_fused_next_forward_empty_update_still_forwards(dq):
    """An empty batch to update (no bags) leaves the tables alone, and the next batch's
    forward still runs and equals dqrm_emb_fwd (called through the C ABI: the Python wrapper
    has no empty dy to pass)."""
    import ctypes as C
    from deep_quantized_recommendation_model_dqrm_amd import tables as TB

    rows, D, B = COAL_ROWS, 64, 2048
    T = len(rows)
    ts = dq.EmbeddingTableSet(rows, D, device="cuda", init="uniform", seed=9)
    nb = dq.LookupBatch.pooling_one(torch.from_numpy(G.pooling_one(rows, B, 4)).cuda())
    # zero bags over valid pointers (a Python batch of zero bags has none to give)
    empty = TB.L.Batch(TB._ptr(nb.idx), TB._ptr(nb.off), TB._ptr(nb.idx_base), 0, 0, TB.L.DQRM_BATCH_POOLING_ONE, 0)
    W0 = ts.W.clone()
    ws = dq.CoalescedGrad.allocate(rows, B, D, "cuda")
    s_avg = torch.zeros(T, dtype=torch.float32, device="cuda")
    dy = torch.zeros(64, dtype=torch.float32, device="cuda")  # any valid pointer: no bags read it
    out = torch.full((T, B, D), 7.0, dtype=torch.float32, device="cuda")
    rc = ts.lib.dqrm_emb_bwd_apply_fwd_local(
        C.byref(ts._c), C.byref(empty), TB._ptr(dy), 0, D, 1, TB._ptr(ws.slot_cap_base), ws.cap_total,
        TB._ptr(ws.rows), TB._ptr(ws.vals), TB._ptr(ws.ucount), TB._ptr(ws.absmax), 8, TB._ptr(s_avg), 0.5, 0,
        *ts._ws_args(nb), C.byref(nb.c), 4, ts._fwd_flags(True, False, False), TB._ptr(out), B * D, D,
        TB._stream_handle())
    assert rc == 0
    assert ts.read_errors() == 0
    assert torch.equal(ts.W, W0)
    assert torch.equal(out, ts.forward(nb))
    out.fill_(7.0)  # and the SGD form (dqrm_emb_bwd_sgd_fwd)
    rc = ts.lib.dqrm_emb_bwd_sgd_fwd(
        C.byref(ts._c), C.byref(empty), TB._ptr(dy), 0, D, 1, 0.5, 0, *ts._ws_args(nb), C.byref(nb.c), 4,
        ts._fwd_flags(True, False, False), TB._ptr(out), B * D, D, TB._stream_handle())
    assert rc == 0
    assert torch.equal(ts.W, W0)
    assert torch.equal(out, ts.forward(nb))


@pytest.mark.parametrize("D,B,dist,form,refresh,full,layout",
                         [(16, 128, "uniform", "criteo", True, False, "tbd"), (16, 128, "zipf", "criteo", False, False, "tbd"),
                          (32, 512, "zipf", "criteo", True, False, "btd"), (16, 200, "uniform", "bags", True, False, "tbd"),
                          (64, 64, "uniform", "criteo", True, True, "btd"), (4, 256, "zipf", "criteo", True, False, "tbd"),
                          (16, 2048, "uniform", "criteo", True, False, "tbd")])
def test_fused_sgd_next_forward_matches_separate_calls(dq, D, B, dist, form, refresh, full, layout):
    """dqrm_emb_bwd_sgd_fwd -- the single-GPU SGD step with the next batch's forward in the
    same launch (k_sgd_small's workgroup holds its whole table, so the table max is final at
    its end) -- against dqrm_emb_bwd_sgd + dqrm_emb_fwd on a copy, bit for bit over four steps:
    outputs, scale, W and the |W| hierarchy; Kaggle-shaped tables (3 ... 20 000 rows), the
    Criteo form and bags (the update) with Criteo-form next batches, an out-of-range index in a
    next batch; B = 2048 takes the general kernel and the two calls."""
    rows = [min(n, 20000) for n in G.KAGGLE_ROWS]
    T = len(rows)
    sets = [dq.EmbeddingTableSet(rows, D, device="cuda", init="uniform", seed=171) for _ in range(2)]
    Ps = [G.pooling_one(rows, B, 181 + k, dist=dist) for k in range(5)]
    Ps[2][3, 5] = rows[3]  # out of range in the forward of step 1's next batch
    nbs = [dq.LookupBatch.pooling_one(torch.from_numpy(P).cuda()) for P in Ps]
    if form == "bags":
        bags = [G.random_bags(rows, B, 190 + k, num_indices_per_lookup=3) for k in range(4)]
        ubs = [to_batch(dq, idx, off) for idx, off in bags]
    else:
        ubs = nbs[:4]
    kw = dict(refresh_scale=refresh, full_precision=full, layout=layout)
    ys = [ts.forward(nbs[0]) for ts in sets]  # (sets the scales a held-scale forward uses)
    for it in range(4):
        dy = torch.from_numpy(G.upstream_grad(T, B, D, 201 + it) * 30).cuda()
        y0 = sets[0].backward_sgd_forward(ubs[it], dy, 0.5, nbs[it + 1], ste=not full, **kw)
        sets[1].backward_sgd(ubs[it], dy, 0.5, ste=not full)
        y1 = sets[1].forward(nbs[it + 1], **kw)
        errs = [ts.read_errors() for ts in sets]
        assert errs[0] == errs[1], (it, errs)
        assert torch.equal(y0, y1), it
        for name in ("W", "rowmax", "blkmax", "sblkmax", "tmax", "scale"):
            assert torch.equal(getattr(sets[0], name), getattr(sets[1], name)), (it, name)


def _payloads_for_ranks(dq, ts, rank_batches, rank_dys, grad_bits):
    """Every rank's coalesce + quantize-pack on one GPU (the all-gathers become stacking), as
    each rank of SparseGradExchange produces them; returns (payloads [N, P], s_avg, cap_base, cap_total)."""
    from deep_quantized_recommendation_model_dqrm_amd.comm import HipExchangeKernels, payload_bytes

    N = len(rank_batches)
    k = HipExchangeKernels(ts)
    max_lookups = max(b.max_lookups for b in rank_batches)
    wss = []
    for r in range(N):
        ws = dq.CoalescedGrad.allocate(ts.num_rows, max_lookups, ts.D, "cuda")
        k.coalesce(rank_batches[r], rank_dys[r], ws, True, "tbd")
        wss.append(ws)
    absmax_all = torch.stack([ws.absmax for ws in wss])
    caps = dq.default_caps(ts.num_rows, max_lookups)
    cap_base = torch.tensor(np.concatenate([[0], np.cumsum(caps)]), dtype=torch.int64, device="cuda")
    cap_total = int(sum(caps))
    P = payload_bytes(ts.T, cap_total, ts.D, grad_bits)
    payloads = torch.zeros(N, P, dtype=torch.uint8, device="cuda")
    s_avg = torch.zeros(ts.T, dtype=torch.float32, device="cuda")
    for r in range(N):
        k.quant_pack(wss[r], absmax_all, N, grad_bits, cap_base, cap_total, s_avg, payloads[r])
    return payloads, s_avg, cap_base, cap_total


@pytest.mark.parametrize("N,D,B,dist,bits", [(1, 64, 2048, "uniform", 8), (2, 64, 1024, "zipf", 8),
                                             (4, 16, 512, "uniform", 8), (8, 64, 256, "uniform", 8),
                                             (8, 32, 300, "zipf", 16), (3, 64, 700, "uniform", 32)])
@pytest.mark.parametrize("fused", ["merge", "flat"])
def test_merge_apply_with_next_forward_matches_separate_calls(dq, N, D, B, dist, bits, fused):
    """dqrm_apply_sparse_update_fwd -- merge: the merge apply of N ranks' payloads
    (DQRM_APPLY_MERGE) with the NEXT batch's forward in the same launch (each table's forward
    workgroups wait at the table's gate until its update and |W| maxima are final); flat: the
    flat apply, then its finalize and the next forward in ONE launch (k_finalize_fwd: the
    forward workgroups wait at the gate their table's finalize workgroup opens) -- against the
    flat apply + k_table_finalize + dqrm_emb_fwd on a copy of the tables, bit for bit over 3
    steps: W, the |W| hierarchy, the forward scale and the next batch's output. Then the output
    of the last step equals the oracle's forward of the updated tables (every table), and W
    equals oracle.dp_step over the ranks. Reference: s_q_g_p_c.py:601-628,850-890 and apply_emb
    (dlrm_s_pytorch_single_gpu.py:609-674)."""
    from deep_quantized_recommendation_model_dqrm_amd import _lib as L
    from deep_quantized_recommendation_model_dqrm_amd.comm import HipExchangeKernels

    lib = L.load()
    rows = COAL_ROWS
    T = len(rows)
    Ws = G.table_weights(rows, D, 171 + N)
    Wo = [w.copy() for w in Ws]
    sets = [make_set(dq, Ws) for _ in range(2)]
    mode = L.DQRM_UPD_FP32 if bits == 32 else L.DQRM_UPD_DP
    ar = np.arange(B, dtype=np.int64)
    Pn = [[G.pooling_one(rows, B, 181 + 10 * k + r, dist=dist) for r in range(N)] for k in range(4)]
    rank0 = [dq.LookupBatch.pooling_one(torch.from_numpy(Pn[k][0]).cuda()) for k in range(4)]
    ys = [ts.forward(rank0[0]) for ts in sets]
    assert torch.equal(ys[0], ys[1])
    for k in range(3):
        dys = [G.upstream_grad(T, B, D, 191 + 10 * k + r) * 30 for r in range(N)]
        rb = [dq.LookupBatch.pooling_one(torch.from_numpy(Pn[k][r]).cuda()) for r in range(N)]
        s_fwd = sets[0].scale.cpu().numpy().copy()
        outs = []
        for j, ts in enumerate(sets):
            payloads, s_avg, cap_base, cap_total = _payloads_for_ranks(
                dq, ts, rb, [torch.from_numpy(d).cuda() for d in dys], bits)
            kern = HipExchangeKernels(ts)
            if j == 0:
                prev = lib.dqrm_set_apply_kernel(L.DQRM_APPLY_MERGE if fused == "merge" else L.DQRM_APPLY_FLAT)
                try:
                    ws = torch.zeros(max(16, int(lib.dqrm_apply_workspace_bytes(N, cap_total))), dtype=torch.uint8,
                                     device="cuda")
                    assert lib.dqrm_apply_fwd_is_one_launch(ts.c, N, cap_total, ws.numel(), rank0[k + 1].c,
                                                            ts._fwd_flags(True, False, False)) == (fused == "merge")
                    y = torch.empty(T, B, D, device="cuda")
                    kern.apply_fwd(cap_base, cap_total, payloads, payloads.shape[1], N, bits, s_avg, 0.5, mode, False,
                                   rank0[k + 1], y, workspace=ws)
                finally:
                    lib.dqrm_set_apply_kernel(prev)
            else:
                prev = lib.dqrm_set_apply_kernel(L.DQRM_APPLY_FLAT)
                try:
                    kern.apply(cap_base, cap_total, payloads, payloads.shape[1], N, bits, s_avg, 0.5, mode, False)
                finally:
                    lib.dqrm_set_apply_kernel(prev)
                y = ts.forward(rank0[k + 1])
            outs.append(y)
        assert [ts.read_errors() for ts in sets] == [0, 0], k
        assert torch.equal(outs[0], outs[1]), k
        for name in ("W", "rowmax", "blkmax", "sblkmax", "tmax", "scale"):
            assert torch.equal(getattr(sets[0], name), getattr(sets[1], name)), (k, name)
        O.dp_step(Wo, [[(Pn[k][r][t], ar) for t in range(T)] for r in range(N)], [[dys[r][t] for t in range(T)]
                                                                                   for r in range(N)],
                  list(s_fwd), 0.5, grad_bits=bits)
    y = outs[0].cpu().numpy()
    s = sets[0].scale.cpu().numpy()
    for t in range(T):
        np.testing.assert_array_equal(sets[0].table_weight(t).cpu().numpy(), Wo[t])
        assert s[t] == O.table_scale(Wo[t], 4)
        np.testing.assert_array_equal(y[t], O.emb_fwd(Wo[t], Pn[3][0][t], ar, s[t])[0])
    inc = [x.clone() for x in (sets[0].rowmax, sets[0].blkmax, sets[0].sblkmax, sets[0].tmax)]
    sets[0].refresh_absmax()
    for x, z in zip(inc, (sets[0].rowmax, sets[0].blkmax, sets[0].sblkmax, sets[0].tmax)):
        assert torch.equal(x, z)


@pytest.mark.parametrize("N", [3, 5, 6, 8])
def test_replica_mean_matches_gloo_fixture(dq, golden_dir, N):
    """dqrm_replica_mean (weight_syncc on identical replicas, s_q_g_p_c.py:963-970) = real
    Gloo's all_reduce(SUM) * 1/N at N = 3, 5, 6, 8 (syncc_gloo.npz: every mantissa, exponents
    up to 2^122, zeros, subnormals, overflow to inf), bit for bit, incl. a 1 Mi-element vector
    (its checksum) and a length that is not a multiple of the kernel's vector width."""
    lib = dq._lib.load()
    fx = load(golden_dir, "syncc_gloo.npz")
    inv = float(np.float32(1.0 / N))
    for i, tag in enumerate(("small", "large")):
        x = G.replica_values(int(fx["sizes"][i]), int(fx["seeds"][i]))
        t = torch.from_numpy(x).cuda()
        dq._lib.check(lib.dqrm_replica_mean(t.data_ptr(), t.numel(), N, inv, None), "dqrm_replica_mean")
        got = t.cpu().numpy()
        if tag == "small":
            np.testing.assert_array_equal(got.view(np.uint32), fx[f"small_n{N}"].view(np.uint32))
        else:
            assert G.checksum(got) == str(fx[f"large_n{N}_checksum"])


@pytest.mark.parametrize("refresh,full_precision,layout", [(True, False, "tbd"), (False, False, "tbd"),
                                                           (True, True, "btd"), (True, False, "btd")])
def test_flat_finalize_forward_bag_batches(dq, refresh, full_precision, layout):
    """k_finalize_fwd with a bag-form next batch (offsets, multi-lookup bags, an empty bag), a
    frozen scale, full precision and both output layouts: dqrm_apply_sparse_update_fwd on the
    flat apply = the flat apply + k_table_finalize + dqrm_emb_fwd on a copy, bit for bit (W, the
    |W| hierarchy, the scale, the output); the output = oracle.emb_fwd of the updated tables."""
    import ctypes as C
    from deep_quantized_recommendation_model_dqrm_amd import _lib as L
    from deep_quantized_recommendation_model_dqrm_amd.comm import HipExchangeKernels

    lib = L.load()
    rows, D, B, N, bits = COAL_ROWS, 32, 384, 2, 8
    T = len(rows)
    Ws = G.table_weights(rows, D, 977)
    sets = [make_set(dq, Ws) for _ in range(2)]
    for ts in sets:  # the frozen scale of the refresh=False case (a held periodic-refresh scale)
        ts.scale.copy_(torch.from_numpy(np.array([O.table_scale(w, 4) for w in Ws], np.float32)))
    for k in range(2):
        rb = [dq.LookupBatch.pooling_one(torch.from_numpy(G.pooling_one(rows, B, 983 + 10 * k + r)).cuda())
              for r in range(N)]
        dys = [torch.from_numpy(G.upstream_grad(T, B, D, 991 + 10 * k + r) * 30).cuda() for r in range(N)]
        idxs, offs = G.random_bags(rows, 200, 997 + 10 * k, num_indices_per_lookup=3)
        for o in offs:
            o[7] = o[8]  # an empty bag
        nb = to_batch(dq, idxs, offs)
        outs = []
        prev = lib.dqrm_set_apply_kernel(L.DQRM_APPLY_FLAT)
        try:
            for j, ts in enumerate(sets):
                payloads, s_avg, cap_base, cap_total = _payloads_for_ranks(dq, ts, rb, dys, bits)
                kern = HipExchangeKernels(ts)
                shape = (T, 200, D) if layout == "tbd" else (200, T, D)
                y = torch.full(shape, float("nan"), device="cuda")
                if j == 0:
                    kern.apply_fwd(cap_base, cap_total, payloads, payloads.shape[1], N, bits, s_avg, 0.5,
                                   L.DQRM_UPD_DP, False, nb, y, refresh_scale=refresh, full_precision=full_precision,
                                   layout=layout)
                else:
                    kern.apply(cap_base, cap_total, payloads, payloads.shape[1], N, bits, s_avg, 0.5, L.DQRM_UPD_DP,
                               False)
                    ost, osb = (200 * D, D) if layout == "tbd" else (D, T * D)
                    L.check(lib.dqrm_emb_fwd(C.byref(ts.c), C.byref(nb.c), 4,
                                             ts._fwd_flags(refresh, False, full_precision), y.data_ptr(), ost, osb,
                                             None), "dqrm_emb_fwd")
                outs.append(y)
        finally:
            lib.dqrm_set_apply_kernel(prev)
        torch.cuda.synchronize()
        assert [ts.read_errors() for ts in sets] == [0, 0], k
        assert torch.equal(outs[0], outs[1]), k
        for name in ("W", "rowmax", "blkmax", "sblkmax", "tmax", "scale"):
            assert torch.equal(getattr(sets[0], name), getattr(sets[1], name)), (k, name)
        y = outs[0].cpu().numpy()
        s = sets[0].scale.cpu().numpy()
        for t in range(T):
            Wt = sets[0].table_weight(t).cpu().numpy()
            if refresh and not full_precision:
                assert s[t] == O.table_scale(Wt, 4)
            ref = O.emb_fwd(Wt, idxs[t], offs[t], s[t], full_precision=full_precision)[0]
            yt = y[t] if layout == "tbd" else y[:, t]
            np.testing.assert_array_equal(yt, ref)
