"""GPU: dense (MLP) gradient path through libdqrm's C ABI against the
oracle and the torch + Gloo fixtures (tests/golden/dense_*.npz).

N ranks are emulated in one process where needed: every rank's local scales come from the
HIP scale kernel, the HIP quant kernel writes every rank's wire, the wires are summed
exactly on the host (integers; what the RCCL all-reduce computes), and the HIP decode and
update kernels finish the step. Everything is compared bit for bit."""
import os

import numpy as np
import pytest
import torch

import gen_inputs as G
import oracle as O

pytestmark = pytest.mark.gpu
f32 = np.float32
SEED = 2024


@pytest.fixture(scope="module")
def D():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import deep_quantized_recommendation_model_dqrm_amd as d

    d._lib.load()
    from deep_quantized_recommendation_model_dqrm_amd import dense

    return dense


def _layers(shapes, seed=SEED):
    out = []
    for W, b in G.mlp_params(shapes, seed):
        l = torch.nn.Linear(W.shape[1], W.shape[0]).cuda()
        with torch.no_grad():
            l.weight.copy_(torch.from_numpy(W))
            l.bias.copy_(torch.from_numpy(b))
        l.weight.grad = torch.zeros_like(l.weight)
        l.bias.grad = torch.zeros_like(l.bias)
        out.append(l)
    return out


def _set_grads(layers, grads):
    for l, (gW, gb) in zip(layers, grads):
        l.weight.grad.copy_(torch.from_numpy(gW))
        l.bias.grad.copy_(torch.from_numpy(gb))


def emulated_step(D, layers, grads_per_rank, lr, bits=8, wire_type=None):
    """One exchange + update of N emulated ranks with the HIP kernels."""
    from deep_quantized_recommendation_model_dqrm_amd import _lib as L

    N = len(grads_per_rank)
    ch = D.DenseChannels(layers)
    k = D.HipDenseKernels(ch, "cuda")
    k.prepare()
    wt = wire_type or L.load().dqrm_dense_wire_type(bits, N)
    wdt = D._WIRE_DTYPE[wt]
    C = ch.num_channels
    s_all = torch.zeros(N, C, device="cuda")
    if bits != 32:
        for r in range(N):
            _set_grads(layers, grads_per_rank[r])
            k.scale(bits, s_all[r])
    s_avg = torch.zeros(C, device="cuda")
    total = torch.zeros(ch.total_elems, dtype=torch.float64)
    for r in range(N):
        _set_grads(layers, grads_per_rank[r])
        wire = torch.zeros(ch.total_elems, dtype=wdt, device="cuda")
        k.quant(bits, s_all if bits != 32 else None, N, s_avg if bits != 32 else None, wt, wire)
        total += wire.cpu().to(torch.float64)
    if bits == 32:  # FP32 sums: rank order (N-1 .. 0), like the oracle
        acc = None
        for r in reversed(range(N)):
            _set_grads(layers, grads_per_rank[r])
            wire = torch.zeros(ch.total_elems, dtype=wdt, device="cuda")
            k.quant(bits, None, N, None, wt, wire)
            acc = wire.cpu() if acc is None else acc + wire.cpu()
        summed = acc.cuda()
    else:
        assert torch.all(total.abs() <= 2048) or wt != L.DQRM_WIRE_F16
        summed = total.to(wdt).cuda()
    k.decode(summed, wt, N)
    k.update(s_avg if bits != 32 else None, lr)
    torch.cuda.synchronize()
    return s_avg.cpu().numpy(), ch


def _check(layers, params, g_o, s_o, s_avg, ch, quantized):
    for j, (l, (W, b)) in enumerate(zip(layers, params)):
        np.testing.assert_array_equal(l.weight.grad.cpu().numpy(), g_o[j][0])
        np.testing.assert_array_equal(l.bias.grad.cpu().numpy(), g_o[j][1])
        np.testing.assert_array_equal(l.weight.detach().cpu().numpy(), W)
        np.testing.assert_array_equal(l.bias.detach().cpu().numpy(), b)
        if quantized:
            np.testing.assert_array_equal(s_avg[ch.weight_slices[j]], s_o[j][0])
            assert s_avg[ch.bias_index[j]] == s_o[j][1][0]


@pytest.mark.parametrize("N,bits,steps", [(1, 8, 2), (2, 8, 2), (3, 8, 1), (4, 8, 2), (8, 8, 1), (2, 4, 1),
                                          (2, 16, 1), (2, 32, 2), (4, 32, 1)])
def test_dense_kernels_match_oracle(D, N, bits, steps):
    shapes = G.MLP_SHAPES + [(64, 200), (300, 5)]  # a row longer than two wavefronts, short rows
    layers = _layers(shapes)
    params = [(W.copy(), b.copy()) for W, b in G.mlp_params(shapes, SEED)]
    for k in range(steps):
        grads = [G.mlp_grads(shapes, SEED, r, k) for r in range(N)]
        s_avg, ch = emulated_step(D, layers, grads, 0.1, bits=bits)
        if bits == 32:
            g_o, s_o = O.dense_dp_step(params, grads, 0.1, quantized=False)
        else:
            g_o, s_o = _oracle_bits(params, grads, bits)
        _check(layers, params, g_o, s_o, s_avg, ch, bits != 32)


def _oracle_bits(params, grads, bits):
    return O.dense_dp_step(params, grads, 0.1, bits=bits, quantized=True)


def test_int32_wire_matches_fp16_wire(D):
    from deep_quantized_recommendation_model_dqrm_amd import _lib as L

    grads = [G.mlp_grads(G.MLP_SHAPES, SEED, r, 0) for r in range(4)]
    a, b = _layers(G.MLP_SHAPES), _layers(G.MLP_SHAPES)
    emulated_step(D, a, grads, 0.1, wire_type=L.DQRM_WIRE_F16)
    emulated_step(D, b, grads, 0.1, wire_type=L.DQRM_WIRE_I32)
    for x, y in zip(a, b):
        assert torch.equal(x.weight, y.weight) and torch.equal(x.bias, y.bias)


@pytest.mark.parametrize("name", ["dense_n2.npz", "dense_n2_fp32.npz"])
def test_dense_kernels_match_gloo_fixture(D, golden_dir, name):
    fx = dict(np.load(os.path.join(golden_dir, name)))
    N, steps, quantized = int(fx["N"]), int(fx["steps"]), bool(fx["quantized"])
    layers = _layers(G.MLP_SHAPES)
    for k in range(steps):
        grads = [G.mlp_grads(G.MLP_SHAPES, SEED, r, k) for r in range(N)]
        s_avg, ch = emulated_step(D, layers, grads, 0.1, bits=8 if quantized else 32)
        for j, l in enumerate(layers):
            np.testing.assert_array_equal(l.weight.grad.cpu().numpy(), fx[f"k{k}_l{j}_gw"])
            np.testing.assert_array_equal(l.bias.grad.cpu().numpy(), fx[f"k{k}_l{j}_gb"])
            if quantized:
                np.testing.assert_array_equal(s_avg[ch.weight_slices[j]], fx[f"k{k}_l{j}_sw"])
    for j, l in enumerate(layers):
        np.testing.assert_array_equal(l.weight.detach().cpu().numpy(), fx[f"l{j}_W"])
        np.testing.assert_array_equal(l.bias.detach().cpu().numpy(), fx[f"l{j}_b"])


def test_exchange_single_rank_and_table_rebuild(D):
    """DenseGradExchange at world size 1 (no collective); a replaced .grad tensor (new
    storage) is picked up by the channel table."""
    layers = _layers(G.MLP_SHAPES)
    params = [(W.copy(), b.copy()) for W, b in G.mlp_params(G.MLP_SHAPES, SEED)]
    ex = D.DenseGradExchange(layers, grad_bits=8)
    for k in range(3):
        grads = G.mlp_grads(G.MLP_SHAPES, SEED, 0, k)
        if k == 1:
            for l in layers:
                l.weight.grad = torch.zeros_like(l.weight)
        _set_grads(layers, grads)
        ex.exchange()
        ex.apply(0.1)
        g_o, s_o = O.dense_dp_step(params, [grads], 0.1)
        torch.cuda.synchronize()
        _check(layers, params, g_o, s_o, ex.s_avg.cpu().numpy(), ex.channels, True)


def test_dense_rejects_cpu_layers(D):
    from deep_quantized_recommendation_model_dqrm_amd import _lib as L

    l = torch.nn.Linear(4, 3)
    l.weight.grad = torch.zeros_like(l.weight)
    l.bias.grad = torch.zeros_like(l.bias)
    with pytest.raises(L.DQRMError):
        D.DenseGradExchange([l], grad_bits=8)


def test_dense_kernels_n4_fixture_within_gloo_order_tolerance(D, golden_dir):
    """dense_n4.npz (torch + real Gloo, N=4): the HIP path equals the oracle bit for bit,
    and the Gloo fixture at the tolerance its CPU test states (test_dense.py): Gloo sums the
    per-row weight scales in a position-dependent order, so those differ by <= N-1 ulp and
    W by <= 1e-6; bias scales (one-element all_reduce, descending order) and biases match
    exactly."""
    fx = dict(np.load(os.path.join(golden_dir, "dense_n4.npz")))
    N, steps = int(fx["N"]), int(fx["steps"])
    assert N == 4 and bool(fx["quantized"])
    layers = _layers(G.MLP_SHAPES)
    params = [(W.copy(), b.copy()) for W, b in G.mlp_params(G.MLP_SHAPES, SEED)]
    for k in range(steps):
        grads = [G.mlp_grads(G.MLP_SHAPES, SEED, r, k) for r in range(N)]
        s_avg, ch = emulated_step(D, layers, grads, 0.1, bits=8)
        gs, ss = O.dense_dp_step(params, grads, 0.1, bits=8, quantized=True)
        s_host = s_avg
        for j, l in enumerate(layers):
            sw = s_host[ch.weight_slices[j]]
            np.testing.assert_array_equal(sw, ss[j][0])  # HIP == oracle
            np.testing.assert_array_equal(l.weight.grad.cpu().numpy(), gs[j][0])
            np.testing.assert_array_equal(l.bias.grad.cpu().numpy(), gs[j][1])
            assert np.all(np.abs(sw.view(np.int32) - fx[f"k{k}_l{j}_sw"].view(np.int32)) <= N - 1)
            assert float(s_host[ch.bias_index[j]]) == float(ss[j][1][0]) == float(fx[f"k{k}_l{j}_sb"])
    for j, l in enumerate(layers):
        np.testing.assert_array_equal(l.weight.detach().cpu().numpy(), params[j][0])
        np.testing.assert_array_equal(l.bias.detach().cpu().numpy(), params[j][1])
        np.testing.assert_allclose(l.weight.detach().cpu().numpy(), fx[f"l{j}_W"], rtol=0, atol=1e-6)
        np.testing.assert_array_equal(l.bias.detach().cpu().numpy(), fx[f"l{j}_b"])
