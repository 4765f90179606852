"""Ranking-range mixed-precision gradients, CPU side: the oracle
(oracle.rr_*) against the torch + real-Gloo fixture of the reference's call sequence
(tests/golden/make_golden_ranking.py, N=2, 26 tables, 2 steps): bit widths, per-table
scales and every rank's final tables bit for bit (the 32-bit tables diverge across ranks,
as the reference's local update makes them)."""
import os

import numpy as np

import gen_inputs as G
import oracle as O


def regen(fx):
    return (fx["rows"].tolist(), int(fx["D"]), int(fx["B"]), int(fx["seed"]), int(fx["N"]), int(fx["steps"]))


def final_tables(fx, r, rows, D, seed):
    W = G.table_weights(rows, D, seed)
    for t in range(len(rows)):
        W[t][fx[f"r{r}_rows_t{t}"]] = fx[f"r{r}_vals_t{t}"]
    return W


def step_inputs(rows, D, B, seed, N, k):
    from make_golden import get_my_slice

    P = G.pooling_one(rows, B, seed + 17 * (k + 1), dist="zipf" if k % 2 else "uniform")
    dy = G.upstream_grad(len(rows), B, D, seed + 31 * (k + 1))
    sls = [get_my_slice(B, N, r) for r in range(N)]
    batches = [[(np.ascontiguousarray(P[t, sl]), np.arange(sl.stop - sl.start, dtype=np.int64))
                for t in range(len(rows))] for sl in sls]
    dys = [[np.ascontiguousarray(dy[t, sl]) for t in range(len(rows))] for sl in sls]
    return batches, dys


def run_oracle(rows, D, B, seed, N, steps, rng_seed):
    Ws = [G.table_weights(rows, D, seed) for _ in range(N)]
    rng = np.random.RandomState(rng_seed)
    hist = []
    for k in range(steps):
        batches, dys = step_inputs(rows, D, B, seed, N, k)
        s_fwd = [[O.table_scale(w, 4) for w in Ws[r]] for r in range(N)]
        hist.append(O.rr_dp_step(Ws, batches, dys, s_fwd, 0.1, rng) + (s_fwd,))
    return Ws, hist


def test_ranking_oracle_matches_fixture(golden_dir):
    fx = dict(np.load(os.path.join(golden_dir, "ranking_n2.npz")))
    rows, D, B, seed, N, steps = regen(fx)
    Ws, hist = run_oracle(rows, D, B, seed, N, steps, int(fx["rng_seed"]))
    for k, (bits, scales, ranges, s_fwd) in enumerate(hist):
        for r in range(N):
            np.testing.assert_array_equal(bits, fx[f"r{r}_k{k}_bits"])
            np.testing.assert_array_equal(scales, fx[f"r{r}_k{k}_scale"])
            np.testing.assert_array_equal(np.asarray(s_fwd[r], np.float32), fx[f"r{r}_k{k}_eb"])
    assert set(hist[0][0].tolist()) == {0, 8, 32}
    for r in range(N):
        W = final_tables(fx, r, rows, D, seed)
        for t in range(len(rows)):
            np.testing.assert_array_equal(Ws[r][t], W[t], err_msg=f"rank {r} table {t}")
    # the 32-bit tables' local updates make the replicas differ
    assert any(not np.array_equal(Ws[0][t], Ws[1][t]) for t in range(len(rows)))


def test_thresholds():
    assert O.rr_thresholds(26) == (8, 22)
    z, e = O.rr_thresholds(13)
    assert 0 <= z < e < 13


# ---------------------------------------------------------------- Gloo world 2, host side
import socket  # noqa: E402
import sys  # noqa: E402

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _rank_main(rank, world, port, fx_path, out_dir):
    """SparseGradExchange's ranking-range methods (coalesce_ranges, exchange_ranked,
    apply_ranked, local_update) over Gloo with the oracle as the device kernels, driven in
    grad_precision_and_scale's order (rank 0 draws, bits broadcast)."""
    sys.path[:0] = [HERE, os.path.join(HERE, "golden"), os.path.join(HERE, "..", "oracle"), os.path.join(HERE, "..")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import oracle as O
        from cpu_exchange import HostBatch, HostTables, OracleExchangeKernels
        from deep_quantized_recommendation_model_dqrm_amd import SparseGradExchange

        fx = dict(np.load(fx_path))
        rows, D, B, seed, N, steps = regen(fx)
        tables = HostTables(G.table_weights(rows, D, seed))
        ex = SparseGradExchange(tables, B // world, grad_bits=8, kernels=OracleExchangeKernels(tables), device="cpu")
        rng = np.random.RandomState(int(fx["rng_seed"]))
        for k in range(steps):
            batches, dys = step_inputs(rows, D, B, seed, world, k)
            s_fwd = [O.table_scale(w, 4) for w in tables.Ws]
            batch = HostBatch([b[0] for b in batches[rank]], [b[1] for b in batches[rank]], s_fwd)
            dy = torch.from_numpy(np.stack(dys[rank]))
            rg = ex.coalesce_ranges(batch, dy)
            rl = [float(x) for x in (rg / (np.asarray(s_fwd, np.float32) * np.float32(7))).astype(np.float32)]
            bits = torch.from_numpy(O.rr_assign_bits(rl, rng)) if rank == 0 else torch.zeros(len(rows), dtype=torch.int32)
            dist.broadcast(bits, 0)
            b = bits.numpy()
            scale = np.where(b == 8, (np.maximum(rg, np.float32(1e-8)) / np.float32(127)).astype(np.float32), rg)
            ts = torch.from_numpy(scale.astype(np.float32))
            ex.exchange_ranked(bits, ts)
            ex.apply_ranked(0.1, ts)
            ex.kernels.local_update(batch, dy, True, "tbd", 0.1, (bits == 32).to(torch.int32), False)
            np.testing.assert_array_equal(b, fx[f"r{rank}_k{k}_bits"])
            np.testing.assert_array_equal(scale, fx[f"r{rank}_k{k}_scale"])
        np.savez(os.path.join(out_dir, f"r{rank}.npz"), *tables.Ws)
    finally:
        dist.destroy_process_group()


def test_ranked_exchange_gloo_matches_fixture(golden_dir, tmp_path):
    path = os.path.join(golden_dir, "ranking_n2.npz")
    mp.spawn(_rank_main, args=(2, _free_port(), path, str(tmp_path)), nprocs=2, join=True)
    fx = dict(np.load(path))
    rows, D, B, seed, N, steps = regen(fx)
    for r in range(2):
        got = np.load(os.path.join(tmp_path, f"r{r}.npz"))
        W = final_tables(fx, r, rows, D, seed)
        for t in range(len(rows)):
            np.testing.assert_array_equal(got[f"arr_{t}"], W[t], err_msg=f"rank {r} table {t}")
