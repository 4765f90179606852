"""GPU: the RCCL leg of the data-parallel step, executed. torch.distributed's "nccl" backend
is RCCL on ROCm; a one-GPU box can only host a world of size 1 (RCCL refuses two ranks on one
device), so these runs force the N > 1 code path at world size 1: both all-gathers of the
embedding exchange (per-slot max|grad|, fixed-capacity payload) and the MLP exchange's scale
all-gather + wire all-reduce are issued to RCCL (dtype / size checks, stream ordering against
RCCL's internal stream), and the results must equal the oracle bit for bit.
Reference: sgd_quantized_gradients_parallel_comm.py:850-890 (two collectives per table,
:865,878), :892-961 (MLP), :601-668 (updates)."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
ROWS, D, B, STEPS = [3, 200, 5000, 300000], 32, 512, 3


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _rank(rank, port, grad_bits, out_dir, transport="rccl"):
    sys.path[:0] = [HERE, os.path.join(HERE, "golden"), os.path.join(ROOT, "oracle"), ROOT]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), DQRM_C_COMM=transport)
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        import gen_inputs as G
        import deep_quantized_recommendation_model_dqrm_amd as dq
        from deep_quantized_recommendation_model_dqrm_amd.dense import DenseGradExchange

        assert dist.get_backend() == "nccl"
        Ws = G.table_weights(ROWS, D, 41)
        ts = dq.EmbeddingTableSet(ROWS, D, device="cuda", init=None, weights=[torch.from_numpy(w) for w in Ws])
        ex = dq.SparseGradExchange(ts, B, grad_bits=grad_bits, force_collectives=True)
        assert ex.coll and ex.world == 1
        # rccl: the two all-gathers are issued by libdqrm on its own RCCL communicator
        # (dqrm_exchange_grad / _apply); torch: the same calls, c10d's RCCL all-gathers served
        # through the callback; python: kernels and all-gathers issued from Python
        assert ex.transport == transport and (ex._x is not None) == (transport != "python")
        s_avgs = []
        for k in range(STEPS):
            P = G.pooling_one(ROWS, B, 50 + k, dist="zipf" if k % 2 else "uniform")
            dy = G.upstream_grad(len(ROWS), B, D, 60 + k)
            b = dq.LookupBatch.pooling_one(torch.from_numpy(P).cuda())
            ts.forward(b)
            ex.step(b, torch.from_numpy(dy).cuda(), lr=0.1)  # exchange (2 RCCL all-gathers) + apply
            s_avgs.append(ex.s_avg.cpu().numpy().copy())
        torch.cuda.synchronize()
        assert ts.read_errors() == 0
        layers = []
        for W, bb in G.mlp_params(G.MLP_SHAPES, 2024):
            lin = torch.nn.Linear(W.shape[1], W.shape[0]).cuda()
            with torch.no_grad():
                lin.weight.copy_(torch.from_numpy(W))
                lin.bias.copy_(torch.from_numpy(bb))
            layers.append(lin)
        dex = DenseGradExchange(layers, grad_bits=grad_bits if grad_bits == 32 else 8, force_collectives=True)
        for k in range(STEPS):
            for lin, (gW, gb) in zip(layers, G.mlp_grads(G.MLP_SHAPES, 2024, 0, k)):
                lin.weight.grad = torch.from_numpy(gW).cuda()
                lin.bias.grad = torch.from_numpy(gb).cuda()
            with torch.no_grad():
                dex.exchange()  # RCCL all-gather of the scales + all-reduce of the wire
                dex.apply(0.1)
        torch.cuda.synchronize()
        mlp = {f"W{j}": lin.weight.detach().cpu().numpy() for j, lin in enumerate(layers)}
        mlp.update({f"b{j}": lin.bias.detach().cpu().numpy() for j, lin in enumerate(layers)})
        np.savez(os.path.join(out_dir, "r0.npz"), *[ts.table_weight(t).cpu().numpy() for t in range(len(ROWS))],
                 s_avg=np.stack(s_avgs), **mlp)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("grad_bits,transport", [(8, "rccl"), (32, "rccl"), (8, "torch"), (8, "python")])
def test_rccl_world1_exchange_matches_oracle(tmp_path, grad_bits, transport):
    """SparseGradExchange(force_collectives=True) and DenseGradExchange(force_collectives=True)
    over a real RCCL communicator: W of every table after 3 steps, the per-step averaged
    scales and the MLP parameters equal oracle.dp_step / dense_dp_step at N = 1. c_comm: the
    embedding exchange's all-gathers issued by libdqrm (dqrm_comm, the default at world size 1
    on nccl), served by torch.distributed through the callback, or issued from Python."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import gen_inputs as G
    import oracle as O

    mp.spawn(_rank, args=(_free_port(), grad_bits, str(tmp_path), transport), nprocs=1, join=True)
    got = np.load(os.path.join(tmp_path, "r0.npz"))
    Ws = G.table_weights(ROWS, D, 41)
    for k in range(STEPS):
        P = G.pooling_one(ROWS, B, 50 + k, dist="zipf" if k % 2 else "uniform")
        dy = G.upstream_grad(len(ROWS), B, D, 60 + k)
        s_fwd = [O.table_scale(w, 4) for w in Ws]
        res = O.dp_step(Ws, [[(P[t], np.arange(B, dtype=np.int64)) for t in range(len(ROWS))]],
                        [[dy[t] for t in range(len(ROWS))]], s_fwd, 0.1, grad_bits=grad_bits)
        if grad_bits != 32:
            np.testing.assert_array_equal(got["s_avg"][k], np.array([x[0] for x in res], np.float32))
    for t in range(len(ROWS)):
        np.testing.assert_array_equal(got[f"arr_{t}"], Ws[t])
    params = [(W.copy(), b.copy()) for W, b in G.mlp_params(G.MLP_SHAPES, 2024)]
    for k in range(STEPS):
        O.dense_dp_step(params, [G.mlp_grads(G.MLP_SHAPES, 2024, 0, k)], 0.1, quantized=grad_bits != 32)
    for j, (W, b) in enumerate(params):
        np.testing.assert_array_equal(got[f"W{j}"], W)
        np.testing.assert_array_equal(got[f"b{j}"], b)


def test_bench_launcher_rccl_world1():
    """bench.py under torch.distributed.run (the driver's N > 1 launcher) at one rank with
    --force-collectives: the DP step's two RCCL all-gathers run inside the timed region and
    the line reports them; no device error flag."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "1", "--force-collectives", "--config", "kaggle", "--steps", "20", "--warmup", "5",
           "--cpu-baseline", "0", "--gather-batch", "0", "--mlp-iters", "5"]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    assert line["value"] is not None and line["device_errors"] == 0
    assert line["collectives"]["backend"] == "nccl" and line["collectives"]["per_step"] == 2
    assert line["collectives"]["issued_by"].startswith("libdqrm")
    assert line["config"]["n1_update"] in ("coalesce + quant-pack + payload apply (RCCL at world size 1)",
                                           "coalesce + quant-pack + payload apply with the next forward "
                                           "(RCCL at world size 1)")
    assert line["kernels_ms"].get("apply_sparse_update_fwd") or line["kernels_ms"].get("apply_sparse_update")
    assert line["mlp_grad_exchange"]["collectives"] == 2


def test_bench_two_ranks_gloo_on_one_gpu():
    """bench.py's N > 1 step end to end: two ranks under torch.distributed.run sharing the GPU over
    Gloo (the functional rehearsal of the multi-GPU driver run): the exchange's all-gathers served
    by torch.distributed through the library's callback, the flat apply (two entries per lane
    group at this size) then the finalize + next forward launch; both ranks' tables and maxima
    end bit-identical (the line's replica check) with no device error."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--dist-backend", "gloo", "--config", "kaggle", "--steps", "10", "--warmup", "3",
           "--cpu-baseline", "0", "--gather-batch", "0", "--mlp-iters", "0"]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["value"] is not None and line["device_errors"] == 0
    assert line["replicas_bit_identical"] is True
    assert line["collectives"]["world_size"] == 2 and line["collectives"]["per_step"] == 2
    assert "apply_sparse_update_fwd" in line["kernels_ms"]
