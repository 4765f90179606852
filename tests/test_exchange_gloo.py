"""World-size-2 (and 3) Gloo runs of SparseGradExchange on CPU: the exchange's host side
(payload sizing, the per-slot max|grad| all-gather, the payload all-gather, rank handling)
with the oracle standing in for the three device kernels (tests/cpu_exchange.py). Every
rank must end bit-identical to oracle.dp_step over the global batch."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _rank_main(rank, world, port, grad_bits, out_dir, multi=False):
    sys.path[:0] = [HERE, os.path.join(HERE, "golden"), os.path.join(HERE, "..", "oracle"), os.path.join(HERE, "..")]
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import gen_inputs as G
        import oracle as O
        from cpu_exchange import HostBatch, HostTables, OracleExchangeKernels
        from deep_quantized_recommendation_model_dqrm_amd import MultiSetExchange, SparseGradExchange, get_my_slice

        rows, D, B = [3, 97, 5000, 70000], 16, 96 * world
        Ws = G.table_weights(rows, D, 7)
        sl = get_my_slice(B, world, rank)
        if multi:  # one single-table set per table (a ModuleList of per-table modules)
            sets = [HostTables([w]) for w in Ws]
            ex = MultiSetExchange(sets, B // world, grad_bits=grad_bits,
                                  kernels=[OracleExchangeKernels(t) for t in sets], device="cpu")
            assert ex.world == world
        else:
            tables = HostTables(Ws)
            ex = SparseGradExchange(tables, B // world, grad_bits=grad_bits, kernels=OracleExchangeKernels(tables),
                                    device="cpu")
            assert ex.world == world and ex.rank == rank
        for k in range(2):
            P = G.pooling_one(rows, B, 60 + k, dist="zipf" if k else "uniform")
            dy = G.upstream_grad(len(rows), B, D, 70 + k)
            cur = [t.Ws[0] for t in sets] if multi else tables.Ws
            s_fwd = [O.table_scale(w, 4) for w in cur]
            idxs = [np.ascontiguousarray(P[t, sl]) for t in range(len(rows))]
            offs = [np.arange(len(idxs[0]), dtype=np.int64) for _ in rows]
            dyr = torch.from_numpy(np.ascontiguousarray(dy[:, sl]))
            if multi:
                items = [(HostBatch([idxs[t]], [offs[t]], [s_fwd[t]]), dyr[t:t + 1], True, "tbd")
                         for t in range(len(rows))]
                if k == 1:  # a set without a backward this step sends no rows
                    items[1] = None
                ex.exchange(items)
                ex.apply(0.1)
            else:
                ex.step(HostBatch(idxs, offs, s_fwd), dyr, lr=0.1)
        out = [t.Ws[0] for t in sets] if multi else tables.Ws
        np.savez(os.path.join(out_dir, f"r{rank}.npz"), *out)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,grad_bits,multi", [(2, 8, False), (2, 32, False), (3, 8, False), (2, 16, False),
                                                   (2, 8, True), (3, 32, True)])
def test_exchange_gloo_matches_oracle(tmp_path, world, grad_bits, multi):
    """multi: MultiSetExchange over one single-table set per table -- the same two
    collectives for all sets, per-set results equal to the one-set exchange."""
    sys.path[:0] = [os.path.join(HERE, "golden")]
    import gen_inputs as G
    import oracle as O
    from deep_quantized_recommendation_model_dqrm_amd import get_my_slice

    mp.spawn(_rank_main, args=(world, _free_port(), grad_bits, str(tmp_path), multi), nprocs=world, join=True)
    rows, D, B = [3, 97, 5000, 70000], 16, 96 * world
    Ws = G.table_weights(rows, D, 7)
    for k in range(2):
        P = G.pooling_one(rows, B, 60 + k, dist="zipf" if k else "uniform")
        dy = G.upstream_grad(len(rows), B, D, 70 + k)
        s_fwd = [O.table_scale(w, 4) for w in Ws]
        sls = [get_my_slice(B, world, r) for r in range(world)]
        live = [t for t in range(len(rows)) if not (multi and k == 1 and t == 1)]
        sub = [Ws[t] for t in live]
        O.dp_step(sub, [[(np.ascontiguousarray(P[t, sl]), np.arange(sl.stop - sl.start, dtype=np.int64))
                         for t in live] for sl in sls],
                  [[np.ascontiguousarray(dy[t, sl]) for t in live] for sl in sls], [s_fwd[t] for t in live], 0.1,
                  grad_bits=grad_bits)
    for r in range(world):
        got = np.load(os.path.join(tmp_path, f"r{r}.npz"))
        for t in range(len(rows)):
            np.testing.assert_array_equal(got[f"arr_{t}"], Ws[t])
