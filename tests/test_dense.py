"""Dense (MLP) gradient path of the DP step, CPU side:
  * the oracle (oracle.dense_*) against the torch + real-Gloo fixtures
    (tests/golden/make_golden_dense.py): N=2 bit-exact, N=4 bit-exact except the per-row
    weight scales, which Gloo sums in a position-dependent order (<= N-1 ulp);
  * DenseGradExchange's host side under Gloo world sizes 2 and 3 with the oracle standing
    in for the device kernels (tests/cpu_dense.py): every rank bit-identical to
    oracle.dense_dp_step over all ranks' gradients;
  * the wire-type rule (fp16 only where integer sums stay exact).
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import gen_inputs as G
import oracle as O
from deep_quantized_recommendation_model_dqrm_amd import _lib as L
from deep_quantized_recommendation_model_dqrm_amd.dense import DenseChannels, _wire_type

HERE = os.path.dirname(os.path.abspath(__file__))
f32 = np.float32


def _oracle_run(N, steps, quantized, shapes=G.MLP_SHAPES, seed=2024):
    params = [(W.copy(), b.copy()) for W, b in G.mlp_params(shapes, seed)]
    hist = []
    for k in range(steps):
        grads = [G.mlp_grads(shapes, seed, r, k) for r in range(N)]
        hist.append(O.dense_dp_step(params, grads, 0.1, bits=8, quantized=quantized))
    return params, hist


@pytest.mark.parametrize("name", ["dense_n2.npz", "dense_n4.npz", "dense_n2_fp32.npz"])
def test_dense_oracle_matches_fixture(golden_dir, name):
    fx = dict(np.load(os.path.join(golden_dir, name)))
    N, steps, quantized = int(fx["N"]), int(fx["steps"]), bool(fx["quantized"])
    assert [tuple(s) for s in fx["shapes"].tolist()] == G.MLP_SHAPES
    params, hist = _oracle_run(N, steps, quantized)
    exact_scales = N <= 2
    for k, (gs, ss) in enumerate(hist):
        for j in range(len(G.MLP_SHAPES)):
            if quantized:
                sw = fx[f"k{k}_l{j}_sw"]
                if exact_scales or sw.size == 1:  # one-element all_reduce: Gloo's descending order
                    np.testing.assert_array_equal(ss[j][0], sw)
                else:
                    assert np.all(np.abs(ss[j][0].view(np.int32) - sw.view(np.int32)) <= N - 1)
                np.testing.assert_array_equal(ss[j][1], np.float32(fx[f"k{k}_l{j}_sb"]).reshape(1))
            if exact_scales or not quantized:
                np.testing.assert_array_equal(gs[j][0], fx[f"k{k}_l{j}_gw"])
            np.testing.assert_array_equal(gs[j][1], fx[f"k{k}_l{j}_gb"])
    for j, (W, b) in enumerate(params):
        if exact_scales:
            np.testing.assert_array_equal(W, fx[f"l{j}_W"])
        else:  # a last-bit scale difference moves W by at most ~1e-9 per step here
            np.testing.assert_allclose(W, fx[f"l{j}_W"], rtol=0, atol=1e-6)
        np.testing.assert_array_equal(b, fx[f"l{j}_b"])


def test_n4_scale_order_is_the_only_difference(golden_dir):
    """With the fixture's own (Gloo-ordered) weight scales, the oracle's quantize /
    integer sum / decode reproduce the N=4 fixture's averaged gradients bit for bit."""
    fx = dict(np.load(os.path.join(golden_dir, "dense_n4.npz")))
    for j in range(len(G.MLP_SHAPES)):
        s = fx[f"k0_l{j}_sw"]
        grads = [G.mlp_grads(G.MLP_SHAPES, 2024, r, 0)[j][0] for r in range(4)]
        acc = sum(O.dense_quantize(g, s, 8).astype(np.float64) for g in grads).astype(f32)
        g = (f32(0.0) + (acc * f32(0.25)).astype(f32)).astype(f32)
        np.testing.assert_array_equal(g, fx[f"k0_l{j}_gw"])


def test_wire_type_rule():
    lib = L.load()
    for bits in (2, 4, 8, 9, 12, 16, 32):
        for n in (1, 2, 4, 8, 16, 17, 64):
            assert lib.dqrm_dense_wire_type(bits, n) == _wire_type(bits, n), (bits, n)
    assert _wire_type(8, 16) == L.DQRM_WIRE_F16 and _wire_type(8, 17) == L.DQRM_WIRE_I32
    assert _wire_type(32, 3) == L.DQRM_WIRE_F32 and _wire_type(17, 2) < 0


def test_channel_table_layout():
    layers = [torch.nn.Linear(i, o) for o, i in G.MLP_SHAPES]
    ch = DenseChannels(layers)
    assert ch.num_channels == sum(o + 1 for o, _ in G.MLP_SHAPES)
    assert ch.total_elems == sum(o * i + o for o, i in G.MLP_SHAPES)
    assert ch.weight_slices[1] == slice(33, 49) and ch.bias_index[1] == 49
    assert ch.len[:32].tolist() == [13] * 32 and ch.len[32] == 32
    assert ch.wire_off[33] == 32 * 13 + 32


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _rank_main(rank, world, port, quantized, out_dir):
    sys.path[:0] = [HERE, os.path.join(HERE, "golden"), os.path.join(HERE, "..", "oracle"), os.path.join(HERE, "..")]
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import gen_inputs as G
        from cpu_dense import OracleDenseKernels
        from deep_quantized_recommendation_model_dqrm_amd.dense import DenseChannels, DenseGradExchange

        layers = []
        for W, b in G.mlp_params(G.MLP_SHAPES, 2024):
            l = torch.nn.Linear(W.shape[1], W.shape[0])
            with torch.no_grad():
                l.weight.copy_(torch.from_numpy(W))
                l.bias.copy_(torch.from_numpy(b))
            layers.append(l)
        bits = 8 if quantized else 32
        ex = DenseGradExchange(layers, grad_bits=bits, kernels=OracleDenseKernels(DenseChannels(layers)),
                               device="cpu")
        ex.kernels.ch = ex.channels
        assert ex.world == world
        for k in range(2):
            for l, (gW, gb) in zip(layers, G.mlp_grads(G.MLP_SHAPES, 2024, rank, k)):
                l.weight.grad = torch.from_numpy(gW.copy())
                l.bias.grad = torch.from_numpy(gb.copy())
            with torch.no_grad():
                ex.exchange()
                ex.apply(0.1)
        arrs = {}
        for j, l in enumerate(layers):
            arrs[f"W{j}"] = l.weight.data.numpy().copy()
            arrs[f"b{j}"] = l.bias.data.numpy().copy()
            if quantized:
                arrs[f"sw{j}"] = l.weight_scaling_factor.numpy().copy()
        np.savez(os.path.join(out_dir, f"r{rank}.npz"), **arrs)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,quantized", [(2, True), (3, True), (2, False)])
def test_dense_exchange_gloo_matches_oracle(tmp_path, world, quantized):
    mp.spawn(_rank_main, args=(world, _free_port(), quantized, str(tmp_path)), nprocs=world, join=True)
    params, hist = _oracle_run(world, 2, quantized)
    for r in range(world):
        got = np.load(os.path.join(tmp_path, f"r{r}.npz"))
        for j, (W, b) in enumerate(params):
            np.testing.assert_array_equal(got[f"W{j}"], W)
            np.testing.assert_array_equal(got[f"b{j}"], b)
            if quantized:
                np.testing.assert_array_equal(got[f"sw{j}"], hist[-1][1][j][0])
