"""GPU, 2 processes: the real HIP kernels of every rank + the exchanges (embedding tables
and MLP layers) over a process
group (Gloo, host-staged all-gathers, both ranks on cuda:0 -- the pool's boxes have one GPU;
RCCL is exercised by bench.py on multi-GPU nodes). Every rank must end bit-identical to
oracle.dp_step over the global batch."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
ROWS, D, B_GLOBAL, STEPS = [3, 200, 5000, 300000], 32, 512, 2


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _rank(rank, world, port, grad_bits, out_dir, transport="torch", fused_fwd=False):
    sys.path[:0] = [HERE, os.path.join(HERE, "golden"), os.path.join(HERE, "..", "oracle"), os.path.join(HERE, "..")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import gen_inputs as G
        import deep_quantized_recommendation_model_dqrm_amd as dq

        torch.cuda.set_device(0)
        Ws = G.table_weights(ROWS, D, 41)
        ts = dq.EmbeddingTableSet(ROWS, D, device="cuda", init=None, weights=[torch.from_numpy(w) for w in Ws])
        sl = dq.get_my_slice(B_GLOBAL, world, rank)
        ex = dq.SparseGradExchange(ts, sl.stop - sl.start, grad_bits=grad_bits, transport=transport)
        # torch: libdqrm's N > 1 orchestration (dqrm_exchange_grad / _apply with num_ranks = 2,
        # the C path RCCL runs) with its two all-gathers served by Gloo through the callback
        assert ex.transport == transport and (ex._x is not None) == (transport == "torch")
        assert ex._x is None or ex._x.num_ranks == world
        from deep_quantized_recommendation_model_dqrm_amd.dense import DenseGradExchange

        layers = []
        for W, bb in G.mlp_params(G.MLP_SHAPES, 2024):
            l = torch.nn.Linear(W.shape[1], W.shape[0]).cuda()
            with torch.no_grad():
                l.weight.copy_(torch.from_numpy(W))
                l.bias.copy_(torch.from_numpy(bb))
            layers.append(l)
        dex = DenseGradExchange(layers, grad_bits=grad_bits if grad_bits == 32 else 8)
        for k in range(STEPS):
            for l, (gW, gb) in zip(layers, G.mlp_grads(G.MLP_SHAPES, 2024, rank, k)):
                l.weight.grad = torch.from_numpy(gW).cuda()
                l.bias.grad = torch.from_numpy(gb).cuda()
            with torch.no_grad():
                dex.exchange()
                dex.apply(0.1)
        batches = [dq.LookupBatch.pooling_one(torch.from_numpy(np.ascontiguousarray(
            G.pooling_one(ROWS, B_GLOBAL, 50 + k, dist="zipf" if k % 2 else "uniform")[:, sl])).cuda())
            for k in range(STEPS + 1)]
        y = None
        for k in range(STEPS):
            dy = G.upstream_grad(len(ROWS), B_GLOBAL, D, 60 + k)
            b = batches[k]
            dyt = torch.from_numpy(np.ascontiguousarray(dy[:, sl])).cuda()
            if not fused_fwd:
                ts.forward(b)
                ex.step(b, dyt, lr=0.1)
                continue
            if k == 0:
                ts.forward(b)
            # the update of step k with the forward of step k+1 (dqrm_exchange_apply_fwd)
            ex.exchange(b, dyt)
            y = ex.apply_forward(0.1, batches[k + 1])
        torch.cuda.synchronize()
        if fused_fwd:
            np.save(os.path.join(out_dir, f"y{rank}.npy"), y.cpu().numpy())
        assert ts.read_errors() == 0
        if transport == "torch":  # both all-gathers of every step went through the C orchestration
            assert ex.dcomm.calls == STEPS * (2 if grad_bits != 32 else 1)
        mlp = {f"W{j}": l.weight.detach().cpu().numpy() for j, l in enumerate(layers)}
        mlp.update({f"b{j}": l.bias.detach().cpu().numpy() for j, l in enumerate(layers)})
        np.savez(os.path.join(out_dir, f"r{rank}.npz"), *[ts.table_weight(t).cpu().numpy() for t in range(len(ROWS))],
                 **mlp)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("grad_bits", [8, 32])
@pytest.mark.parametrize("transport", ["torch", "python", "torch_fused_fwd"])
def test_two_ranks_hip_exchange_matches_oracle(tmp_path, grad_bits, transport):
    """Two processes, the global batch sliced: every rank's tables and MLP layers equal
    oracle.dp_step / dense_dp_step over the whole batch, bit for bit. transport "torch":
    the step runs through libdqrm's exchange calls with num_ranks = 2 (the orchestration,
    buffer checks, gathered-maxima pitch and gathered-payload apply RCCL uses), the
    all-gathers served by Gloo; "python": kernels and collectives issued one by one.
    Reference: s_q_g_p_c.py:863-885 (scale all_reduce, sparse all_reduce), :601-628."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import gen_inputs as G
    import oracle as O
    from deep_quantized_recommendation_model_dqrm_amd import get_my_slice

    world = 2
    fused = transport == "torch_fused_fwd"  # + the next batch's forward in the apply's launch (merge kernel)
    mp.spawn(_rank, args=(world, _free_port(), grad_bits, str(tmp_path), "torch" if fused else transport, fused),
             nprocs=world, join=True)
    Ws = G.table_weights(ROWS, D, 41)
    sls = [get_my_slice(B_GLOBAL, world, r) for r in range(world)]
    for k in range(STEPS):
        P = G.pooling_one(ROWS, B_GLOBAL, 50 + k, dist="zipf" if k % 2 else "uniform")
        dy = G.upstream_grad(len(ROWS), B_GLOBAL, D, 60 + k)
        s_fwd = [O.table_scale(w, 4) for w in Ws]
        O.dp_step(Ws, [[(np.ascontiguousarray(P[t, sl]), np.arange(sl.stop - sl.start, dtype=np.int64))
                        for t in range(len(ROWS))] for sl in sls],
                  [[np.ascontiguousarray(dy[t, sl]) for t in range(len(ROWS))] for sl in sls], s_fwd, 0.1,
                  grad_bits=grad_bits)
    params = [(W.copy(), b.copy()) for W, b in G.mlp_params(G.MLP_SHAPES, 2024)]
    for k in range(STEPS):  # MLP: quantize_linear_grad / quantize_bias_grad path (s_q_g_p_c.py:892-961)
        O.dense_dp_step(params, [G.mlp_grads(G.MLP_SHAPES, 2024, r, k) for r in range(world)], 0.1,
                        quantized=grad_bits != 32)
    for r in range(world):
        got = np.load(os.path.join(tmp_path, f"r{r}.npz"))
        for t in range(len(ROWS)):
            np.testing.assert_array_equal(got[f"arr_{t}"], Ws[t])
        if fused:  # the last fused forward: the next batch on the updated tables, with their scale
            y = np.load(os.path.join(tmp_path, f"y{r}.npy"))
            P = G.pooling_one(ROWS, B_GLOBAL, 50 + STEPS, dist="zipf" if STEPS % 2 else "uniform")[:, sls[r]]
            for t in range(len(ROWS)):
                yo, _ = O.emb_fwd(Ws[t], np.ascontiguousarray(P[t]), np.arange(P.shape[1], dtype=np.int64),
                                  O.table_scale(Ws[t], 4))
                np.testing.assert_array_equal(y[t], yo)
        for j, (W, b) in enumerate(params):
            np.testing.assert_array_equal(got[f"W{j}"], W)
            np.testing.assert_array_equal(got[f"b{j}"], b)


SYNC_ROWS, SYNC_D = [5, 300, 20000], 16


def _sync_rank(rank, world, port, out_dir, same=False):
    sys.path[:0] = [HERE, os.path.join(HERE, "golden"), os.path.join(HERE, "..", "oracle"), os.path.join(HERE, "..")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import gen_inputs as G
        from torch import nn
        from deep_quantized_recommendation_model_dqrm_amd import sgd_quantized_gradients_parallel_comm as H
        from deep_quantized_recommendation_model_dqrm_amd.quant_modules_not_quantize_grad import (
            QuantEmbeddingBagCollection)

        torch.cuda.set_device(0)
        seed = 0 if same else rank
        torch.manual_seed(seed)  # each rank starts from its own tables and MLP, as the
        # reference's ranks do before the first weight_syncc (dp_one_parallel_comm.py:1801)
        model = nn.Module()
        Ws = G.table_weights(SYNC_ROWS, SYNC_D, 300 + seed)
        model.emb_l = QuantEmbeddingBagCollection(SYNC_ROWS, SYNC_D, weights=[torch.from_numpy(w) for w in Ws],
                                                  grad_mode="dp", use_packed_int4=True)
        model.emb_l._tset.refresh_scale_and_pack(4)
        model.bot_l = nn.Sequential(nn.Linear(13, SYNC_D)).cuda()
        model.top_l = nn.Sequential(nn.Linear(SYNC_D, 1)).cuda()
        before = {n: p.detach().cpu().numpy().copy() for n, p in model.named_parameters()}
        real = {}
        for n, p in model.named_parameters():  # the reference's arithmetic, on host copies
            x = p.detach().cpu().clone()
            dist.all_reduce(x, dist.ReduceOp.SUM)
            real[n] = x.mul_(1.0 / world).numpy()
        H.weight_syncc(model, world)
        ts = model.emb_l._tset
        inc = [x.clone() for x in (ts.rowmax, ts.blkmax, ts.sblkmax, ts.tmax)]
        ts.refresh_absmax()
        hier_ok = all(torch.equal(a, b) for a, b in zip(inc, (ts.rowmax, ts.blkmax, ts.sblkmax, ts.tmax)))
        after = {n: p.detach().cpu().numpy() for n, p in model.named_parameters()}
        np.savez(os.path.join(out_dir, f"s{rank}.npz"), hier_ok=np.array(hier_ok), packed=ts.packed.cpu().numpy(),
                 scale=ts.scale.cpu().numpy(), **{"b_" + k: v for k, v in before.items()},
                 **{"a_" + k: v for k, v in after.items()}, **{"r_" + k: v for k, v in real.items()})
    finally:
        dist.destroy_process_group()


def test_weight_syncc_two_ranks_different_tables(tmp_path):
    """weight_syncc at N=2 with each rank starting from different tables and MLP weights
    (s_q_g_p_c.py:963-970): every parameter becomes the fp32 rank-ordered mean
    (all_reduce SUM, then * 1/N) on both ranks, the |W| hierarchy equals a rebuild, and the
    INT4 rows are repacked with the new table scales."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import oracle as O

    world = 2
    mp.spawn(_sync_rank, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    got = [dict(np.load(os.path.join(tmp_path, f"s{r}.npz"))) for r in range(world)]
    names = [k[2:] for k in got[0] if k.startswith("b_")]
    assert "emb_l.embedding_bag.weight" in names and len(names) >= 5
    for n in names:
        mean = ((got[0]["b_" + n] + got[1]["b_" + n]).astype(np.float32) * np.float32(1.0 / world)).astype(np.float32)
        assert not np.array_equal(got[0]["b_" + n], got[1]["b_" + n]), n  # the ranks really started apart
        for r in range(world):
            np.testing.assert_array_equal(got[r]["a_" + n], mean, err_msg=n)
    W = got[0]["a_emb_l.embedding_bag.weight"]
    base = np.concatenate([[0], np.cumsum(SYNC_ROWS)])
    for r in range(world):
        assert bool(got[r]["hier_ok"])
        for t in range(len(SYNC_ROWS)):
            Wt = W[base[t]: base[t + 1]]
            s = O.table_scale(Wt, 4)
            assert got[r]["scale"][t] == s
            np.testing.assert_array_equal(got[r]["packed"][base[t]: base[t + 1]], O.pack_int4(Wt, s))


@pytest.mark.parametrize("world", [2, 3])
def test_weight_syncc_identical_replicas_local(tmp_path, world):
    """weight_syncc on bit-identical replicas (what the DP step maintains): one checksum
    all-gather, then the all-reduce's result computed locally -- the identity at N = 2,
    fl(fl(x + x) + x) * fl(1/3) at N = 3 (dqrm_replica_mean). Every parameter must equal
    what Gloo's all_reduce(SUM) * 1/N gives on the same inputs, on every rank, and the |W|
    hierarchy must equal a rebuild."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    mp.spawn(_sync_rank, args=(world, _free_port(), str(tmp_path), True), nprocs=world, join=True)
    got = [dict(np.load(os.path.join(tmp_path, f"s{r}.npz"))) for r in range(world)]
    names = [k[2:] for k in got[0] if k.startswith("b_")]
    moved = 0
    for n in names:
        for r in range(world):
            np.testing.assert_array_equal(got[r]["b_" + n], got[0]["b_" + n], err_msg=n)  # identical start
            np.testing.assert_array_equal(got[r]["a_" + n], got[r]["r_" + n], err_msg=n)  # = the all-reduce
        moved += int(np.sum(got[0]["a_" + n].view(np.int32) != got[0]["b_" + n].view(np.int32)))
    if world == 2:
        assert moved == 0
    else:
        assert moved > 0  # N = 3 moves about half of the elements by an ulp
    for r in range(world):
        assert bool(got[r]["hier_ok"])


HOOK_ROWS, HOOK_D, HOOK_B = [7, 300, 5000, 40000], 16, 256


def _hook_rank(rank, world, port, out_dir, veto_rank):
    """The unchanged DP driver's pattern: a ModuleList of per-table QuantEmbeddingBagTwo
    (grad_mode "dp") stepped through clear_gradients / backward / grad_update_parallel_comm /
    weight_update_parallel_comm. veto_rank >= 0: that rank cannot consolidate its tables
    (e.g. too little free memory), so NO rank may (the payload layouts must agree)."""
    sys.path[:0] = [HERE, os.path.join(HERE, "golden"), os.path.join(HERE, "..", "oracle"), os.path.join(HERE, "..")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import gen_inputs as G
        from torch import nn
        from deep_quantized_recommendation_model_dqrm_amd import quant_modules_not_quantize_grad as Q
        from deep_quantized_recommendation_model_dqrm_amd import sgd_quantized_gradients_parallel_comm as H
        import deep_quantized_recommendation_model_dqrm_amd as dq

        torch.cuda.set_device(0)
        if rank == veto_rank:
            H.can_consolidate = lambda mods: False  # this rank's memory check fails
        Ws = G.table_weights(HOOK_ROWS, HOOK_D, 77)
        model = nn.Module()
        model.emb_l = nn.ModuleList([Q.QuantEmbeddingBagTwo(n, HOOK_D, 4, embedding_id=t, grad_mode="dp",
                                                            weight=torch.from_numpy(Ws[t]))
                                     for t, n in enumerate(HOOK_ROWS)])
        model.bot_l, model.top_l = nn.ModuleList(), nn.ModuleList()
        sl = dq.get_my_slice(HOOK_B, world, rank)
        Bl = sl.stop - sl.start
        off = torch.arange(Bl, dtype=torch.int64, device="cuda")
        for k in range(2):
            P = G.pooling_one(HOOK_ROWS, HOOK_B, 90 + k)
            dy = G.upstream_grad(len(HOOK_ROWS), HOOK_B, HOOK_D, 95 + k)
            H.clear_gradients(model)
            ys = [model.emb_l[t](torch.from_numpy(np.ascontiguousarray(P[t, sl])).cuda(), off)
                  for t in range(len(HOOK_ROWS))]
            torch.autograd.backward(ys, [torch.from_numpy(np.ascontiguousarray(dy[t, sl])).cuda()
                                         for t in range(len(HOOK_ROWS))])
            H.grad_update_parallel_comm(model, world, True, 8)
            H.weight_update_parallel_comm(model, 0.1, num_gpus=world)
        torch.cuda.synchronize()
        consolidated = model._dqrm_consolidated is not False
        np.savez(os.path.join(out_dir, f"h{rank}.npz"), consolidated=np.array(consolidated),
                 *[model.emb_l[t].embedding_bag.weight.detach().cpu().numpy() for t in range(len(HOOK_ROWS))])
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("veto_rank", [-1, 1])
def test_two_ranks_modulelist_hooks_consolidation_agreed(tmp_path, veto_rank):
    """The DP hooks on a ModuleList at N=2: the tables are consolidated into one set only
    when every rank can (an all-reduce MIN of each rank's check); either way both ranks end
    bit-identical to oracle.dp_step over the global batch."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import gen_inputs as G
    import oracle as O
    from deep_quantized_recommendation_model_dqrm_amd import get_my_slice

    world = 2
    mp.spawn(_hook_rank, args=(world, _free_port(), str(tmp_path), veto_rank), nprocs=world, join=True)
    Ws = G.table_weights(HOOK_ROWS, HOOK_D, 77)
    sls = [get_my_slice(HOOK_B, world, r) for r in range(world)]
    for k in range(2):
        P = G.pooling_one(HOOK_ROWS, HOOK_B, 90 + k)
        dy = G.upstream_grad(len(HOOK_ROWS), HOOK_B, HOOK_D, 95 + k)
        s_fwd = [O.table_scale(w, 4) for w in Ws]
        O.dp_step(Ws, [[(np.ascontiguousarray(P[t, sl]), np.arange(sl.stop - sl.start, dtype=np.int64))
                        for t in range(len(HOOK_ROWS))] for sl in sls],
                  [[np.ascontiguousarray(dy[t, sl]) for t in range(len(HOOK_ROWS))] for sl in sls], s_fwd, 0.1,
                  grad_bits=8)
    for r in range(world):
        got = np.load(os.path.join(tmp_path, f"h{r}.npz"))
        assert bool(got["consolidated"]) == (veto_rank < 0)
        for t in range(len(HOOK_ROWS)):
            np.testing.assert_array_equal(got[f"arr_{t}"], Ws[t])
