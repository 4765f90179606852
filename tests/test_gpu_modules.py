"""GPU: the drop-in modules and DP hooks (reference-named API) against the oracle.

QuantEmbeddingBagTwo mirrors quant_modules_not_quantize_grad.py:240-398; the hooks mirror
sgd_quantized_gradients_parallel_comm.py (grad_update / weight_update / clear / weight_syncc).
"""
import numpy as np
import pytest
import torch
from torch import nn

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


@pytest.fixture(autouse=True)
def plain_linear_mlp():
    """The tiny models below use plain nn.Linear MLP layers; opt them into the MLP exchange
    (the reference itself exchanges only QuantLinear layers)."""
    from deep_quantized_recommendation_model_dqrm_amd import sgd_quantized_gradients_parallel_comm as H

    H.set_mlp_plain_linear(True)
    yield
    H.set_mlp_plain_linear(False)


def _qebt(n, D, W, **kw):
    from deep_quantized_recommendation_model_dqrm_amd.quant_modules_not_quantize_grad import QuantEmbeddingBagTwo

    return QuantEmbeddingBagTwo(n, D, embedding_bit=4, embedding_id=0, weight=torch.from_numpy(W), **kw)


@pytest.fixture
def per_lookup_grads():
    from deep_quantized_recommendation_model_dqrm_amd import quant_modules_not_quantize_grad as Q

    Q.set_sparse_grad_form("per_lookup")
    yield
    Q.set_sparse_grad_form("presummed")


def test_quant_embedding_bag_two_forward_and_sparse_grad(dq, per_lookup_grads):
    n, D = 5000, 16
    W = G.table_weights([n], D, 3)[0]
    (idx,), (off,) = G.random_bags([n], 64, 4, num_indices_per_lookup=5)
    m = _qebt(n, D, W)
    x, o = torch.from_numpy(idx).cuda(), torch.from_numpy(off).cuda()
    y = m(x, o)
    s = O.table_scale(W, 4)
    assert m.eb_scaling_factor.item() == s
    y_o, _ = O.emb_fwd(W, idx, off, s)
    np.testing.assert_array_equal(y.detach().cpu().numpy(), y_o)
    dy = G.upstream_grad(1, len(off), D, 5)[0]
    y.backward(torch.from_numpy(dy).cuda())
    g = m.embedding_bag.weight.grad
    # nn.EmbeddingBag(sparse=True)'s form: one entry per lookup, in lookup order, the
    # STE'd gradient row of its bag (uncoalesced)
    assert g.is_sparse and not g.is_coalesced()
    bag = np.repeat(np.arange(len(off)), np.diff(np.append(off, len(idx))))
    np.testing.assert_array_equal(g._indices()[0].cpu().numpy(), idx)
    np.testing.assert_array_equal(g._values().cpu().numpy(), ((dy * f32(s)) / f32(s))[bag])
    r_o, v_o, _ = O.emb_bwd_coalesce(n, idx, off, dy, s)
    gc = g.coalesce()  # ATen's coalesce: same rows, sums in its own order
    np.testing.assert_array_equal(gc.indices()[0].cpu().numpy(), r_o)
    np.testing.assert_allclose(gc.values().cpu().numpy(), v_o, rtol=0, atol=1e-6)
    # test_mode reuses the training scale; full precision is the plain bag sum
    y_t = m(x, o, test_mode=True)
    np.testing.assert_array_equal(y_t.detach().cpu().numpy(), y_o)
    y_fp = m(x, o, full_precision_flag=True)
    y_fo, _ = O.emb_fwd(W, idx, off, s, full_precision=True)
    np.testing.assert_array_equal(y_fp.detach().cpu().numpy(), y_fo)
    # reference attribute surface
    for name in ("eb_scaling_factor", "emb_scaling_factor", "gradient_bit_width", "now_iteration",
                 "iteration_bound", "iteration_nt"):
        assert hasattr(m, name)
    assert m.embedding_bag.weight.shape == (n, D)


@pytest.mark.parametrize("fused_step", [True, False])
def test_sparse_grad_sgd_step_matches_kaggle_pool1(dq, golden_dir, fused_step):
    """The single-GPU driver unchanged (dlrm_s_pytorch_single_gpu.py:1943-1950): 26
    QuantEmbeddingBagTwo(grad_mode="sparse") + torch.optim.SGD(lr=0.1).step(), against
    kaggle_pool1.npz (the reference's modules + SGD in torch-CPU). fused_step (default): the
    SGD step runs as the modules' own per-lookup update (the optimizer pre-step hook), so every
    forward, scale and W is bit-exact with the fixture. Without it, ATen-ROCm adds the
    presummed COO: W and the later forwards (whose scale follows max|W|) are held to 1e-6
    absolute (row sums round differently from torch-CPU's per-lookup adds)."""
    import os
    from test_oracle_golden import regen_single
    from deep_quantized_recommendation_model_dqrm_amd import quant_modules_not_quantize_grad as Q

    fx = dict(np.load(os.path.join(golden_dir, "kaggle_pool1.npz")))
    Ws, batches, dys = regen_single(fx)
    Q.set_fused_optimizer_step(fused_step)
    try:
        mods = nn.ModuleList([_qebt(w.shape[0], w.shape[1], w, grad_mode="sparse") for w in Ws])
        opt = torch.optim.SGD([m.embedding_bag.weight for m in mods], lr=float(fx["lr"]))
        for k, ((idxs, offs), dy) in enumerate(zip(batches, dys)):
            opt.zero_grad()
            ys = [m(torch.from_numpy(i).cuda(), torch.from_numpy(o).cuda()) for m, i, o in zip(mods, idxs, offs)]
            for t, (m, y) in enumerate(zip(mods, ys)):
                if k == 0 or fused_step:  # bit-exact
                    np.testing.assert_array_equal(y.detach().cpu().numpy(), fx[f"y{k}"][t])
                    assert m.eb_scaling_factor.item() == fx[f"s{k}"][t]
                else:  # after ATen's update (see above): the table max, hence the scale, within 1e-6
                    np.testing.assert_allclose(y.detach().cpu().numpy(), fx[f"y{k}"][t], rtol=0, atol=1e-6)
                    np.testing.assert_allclose(m.eb_scaling_factor.item(), fx[f"s{k}"][t], rtol=1e-6)
            torch.autograd.backward(ys, [torch.from_numpy(dy[t]).cuda() for t in range(len(ys))])
            opt.step()
            if fused_step:  # the modules applied their own updates; the optimizer added nothing
                assert all(m.embedding_bag.weight.grad is None for m in mods)
        exact = total = 0
        for t, m in enumerate(mods):
            rows = fx[f"rows_t{t}"]
            got = m.embedding_bag.weight.detach().cpu().numpy()[rows]
            if fused_step:
                np.testing.assert_array_equal(got, fx[f"w_t{t}"])
            np.testing.assert_allclose(got, fx[f"w_t{t}"], rtol=0, atol=1e-6)
            exact += int((got == fx[f"w_t{t}"]).sum())
            total += got.size
        assert exact > total // 2  # most elements still agree to the bit
        assert all(m._tset.read_errors() == 0 for m in mods)
    finally:
        Q.set_fused_optimizer_step(True)


@pytest.mark.parametrize("form", ["bags", "criteo"])
def test_presummed_sparse_grad_is_the_coalesced_gradient(dq, form):
    """The default grad_mode="sparse" COO (dqrm_emb_bwd_lookup_grad_presum): the reference's
    shape -- one entry per lookup, indices = the lookups' rows, in lookup order -- with each
    row's whole STE'd gradient, summed in lookup order, on its FIRST lookup and +0.0 on the
    later ones: bit-exact against the oracle's ordered coalesce (s_q_g_p_c.py:859's
    grad.coalesce() of the per-lookup COO), on bags (C1-style, duplicates within and across
    bags) and on Criteo-form batches of a 3-row and a 40-row table (~700 / ~50 lookups per row)."""
    D = 16
    if form == "bags":
        n = 50
        W = G.table_weights([n], D, 3)[0]
        (idx,), (off,) = G.random_bags([n], 128, 4, num_indices_per_lookup=10)
    else:
        n = 3
        W = G.table_weights([n], D, 3)[0]
        idx = G.pooling_one([n], 2048, 7)[0]
        off = np.arange(2048, dtype=np.int64)
    m = _qebt(n, D, W)
    x, o = torch.from_numpy(idx).cuda(), torch.from_numpy(off).cuda()
    y = m(x, o)
    s = O.table_scale(W, 4)
    dy = G.upstream_grad(1, len(off), D, 5)[0]
    y.backward(torch.from_numpy(dy).cuda())
    g = m.embedding_bag.weight.grad
    assert g.is_sparse and not g.is_coalesced()
    gi, gv = g._indices()[0].cpu().numpy(), g._values().cpu().numpy()
    np.testing.assert_array_equal(gi, idx)
    r_o, v_o, _ = O.emb_bwd_coalesce(n, idx, off, dy, s)
    first = {}
    for j, r in enumerate(idx):
        first.setdefault(int(r), j)
    for r, v in zip(r_o, v_o):
        np.testing.assert_array_equal(gv[first[int(r)]], v)
    later = np.array([first[int(r)] != j for j, r in enumerate(idx)])
    assert later.any() and not gv[later].any()
    assert not np.signbit(gv[later]).any()  # +0.0: the optimizer adds -lr * +0 = -0.0 (identity)
    np.testing.assert_array_equal(g.coalesce().values().cpu().numpy(), v_o)
    assert m._tset.read_errors() == 0


def test_sparse_sgd_default_is_deterministic(dq):
    """The unchanged single-GPU driver (26-style per-table modules + torch.optim.SGD on their
    COO grads, dlrm_s_pytorch_single_gpu.py:1943-1950), 4 steps on tables of 3..100k rows
    with heavy duplicates (~700 lookups per row of the 3-row table, dy x 10). Default (the
    fused optimizer step): W equals the oracle's torch sparse SGD -- -lr * g of every lookup
    added in lookup order (oracle.emb_bwd_sgd) -- bit for bit, hence is deterministic. With the
    fused step off, ATen adds the presummed COO: two runs are bit-identical and W is within
    1e-5 relative of the oracle (row sums round differently); the per-lookup COO is the reference's
    own (ATen's atomic scatter-add orders its duplicates run to run)."""
    from deep_quantized_recommendation_model_dqrm_amd import quant_modules_not_quantize_grad as Q

    rows, D, B = [3, 10, 27, 5000, 100000], 16, 2048
    Ws = G.table_weights(rows, D, 41)
    P = [G.pooling_one(rows, B, 50 + k, dist="zipf") for k in range(4)]
    dys = [G.upstream_grad(len(rows), B, D, 60 + k) * 10 for k in range(4)]

    def run(form, fused):
        Q.set_sparse_grad_form(form)
        Q.set_fused_optimizer_step(fused)
        try:
            mods = nn.ModuleList([_qebt(n, D, w, grad_mode="sparse") for n, w in zip(rows, Ws)])
            opt = torch.optim.SGD([m.embedding_bag.weight for m in mods], lr=0.1)
            off = torch.arange(B, device="cuda")
            for k in range(4):
                opt.zero_grad()
                ys = [m(torch.from_numpy(P[k][t]).cuda(), off) for t, m in enumerate(mods)]
                torch.autograd.backward(ys, [torch.from_numpy(dys[k][t]).cuda() for t in range(len(rows))])
                opt.step()
            assert all(m._tset.read_errors() == 0 for m in mods)
            return [m.embedding_bag.weight.detach().cpu().numpy().copy() for m in mods]
        finally:
            Q.set_sparse_grad_form("presummed")
            Q.set_fused_optimizer_step(True)

    Wo = [w.copy() for w in Ws]
    ar = np.arange(B, dtype=np.int64)
    for k in range(4):
        for t in range(len(rows)):
            O.emb_bwd_sgd(Wo[t], P[k][t], ar, dys[k][t], O.table_scale(Wo[t], 4), 0.1)
    fused = run("presummed", True)
    for x, z in zip(fused, Wo):
        np.testing.assert_array_equal(x, z)
    a, b = run("presummed", False), run("presummed", False)
    for x, y, z in zip(a, b, Wo):
        np.testing.assert_array_equal(x, y)
        np.testing.assert_allclose(x, z, rtol=1e-5, atol=1e-6)  # |W| reaches ~2 here (dy x 10)


def test_fused_optimizer_step_falls_back_when_grad_changes(dq):
    """The fused optimizer step applies only the COO the last backward produced, as is: a
    gradient accumulated over two backwards, a grad edited in place, or an optimizer with
    another optimizer (Adagrad) get the optimizer's own step on the COO (the module then syncs
    its |W| maxima)."""
    from deep_quantized_recommendation_model_dqrm_amd import quant_modules_not_quantize_grad as Q

    n, D, B = 300, 16, 256
    W = G.table_weights([n], D, 3)[0]
    P = [G.pooling_one([n], B, 70 + k)[0] for k in range(2)]
    dy = [G.upstream_grad(1, B, D, 80 + k)[0] for k in range(2)]
    off = torch.arange(B, device="cuda")

    def step(kind):
        m = _qebt(n, D, W, grad_mode="sparse")
        opt = (torch.optim.Adagrad([m.embedding_bag.weight], lr=0.1) if kind == "adagrad"
               else torch.optim.SGD([m.embedding_bag.weight], lr=0.1))
        opt.zero_grad()
        for k in range(2 if kind == "accumulate" else 1):
            m(torch.from_numpy(P[k]).cuda(), off).backward(torch.from_numpy(dy[k]).cuda())
        g = m.embedding_bag.weight.grad
        if kind == "scaled":
            g.mul_(0.5)
        expect = m.embedding_bag.weight.detach().clone()
        if kind != "adagrad":  # what SGD's add of the (accumulated / scaled) COO gives
            expect.add_(g.coalesce(), alpha=-0.1)
        opt.step()
        got = m.embedding_bag.weight.detach().clone()
        return m, got, expect

    for kind in ("accumulate", "scaled"):
        m, got, expect = step(kind)
        torch.testing.assert_close(got, expect, rtol=0, atol=1e-6)
        assert m._sgd_pend is None
        y = m(torch.from_numpy(P[0]).cuda(), off)  # the next forward's scale follows the changed rows
        assert m.eb_scaling_factor.item() == O.table_scale(got.cpu().numpy(), 4)
    m, got, _ = step("adagrad")  # not SGD: the optimizer's own step ran (grad kept)
    assert m.embedding_bag.weight.grad is not None
    assert not torch.equal(got, torch.from_numpy(W).cuda())


def test_quant_embedding_bag_two_fused_sgd(dq):
    n, D = 3000, 32
    W = G.table_weights([n], D, 8)[0]
    P = G.pooling_one([n], 512, 9, dist="zipf")[0]
    m = _qebt(n, D, W, grad_mode="fused_sgd", lr=0.1)
    x = torch.from_numpy(P).cuda()
    off = torch.arange(512, device="cuda")
    Wo = W.copy()
    for k in range(3):
        s = O.table_scale(Wo, 4)
        y = m(x, off)
        dy = G.upstream_grad(1, 512, D, 10 + k)[0]
        y.backward(torch.from_numpy(dy).cuda())
        O.emb_bwd_sgd(Wo, P, np.arange(512), dy, s, 0.1)
    np.testing.assert_array_equal(m.embedding_bag.weight.detach().cpu().numpy(), Wo)


class TinyDLRM(nn.Module):
    """emb_l / bot_l / top_l as DLRM_Net exposes them (dlrm_s_pytorch_single_gpu.py)."""

    def __init__(self, dq, rows, D, Ws):
        super().__init__()
        from deep_quantized_recommendation_model_dqrm_amd.quant_modules_not_quantize_grad import (
            QuantEmbeddingBagCollection,
        )

        self.emb_l = QuantEmbeddingBagCollection(rows, D, weights=[torch.from_numpy(w) for w in Ws],
                                                 grad_mode="dp")
        self.bot_l = nn.Sequential(nn.Linear(13, D), nn.ReLU()).cuda()
        self.top_l = nn.Sequential(nn.Linear(D * (len(rows) + 1), 1)).cuda()

    def forward(self, dense, lS_o, lS_i):
        x = self.bot_l(dense)
        ly = self.emb_l(lS_o, lS_i, layout="btd")
        z = torch.cat([x.unsqueeze(1), ly], dim=1).flatten(1)
        return self.top_l(z)


@pytest.mark.parametrize("emb_q,mlp_q", [(True, True), (False, False)])
def test_dp_hooks_single_rank_match_oracle(dq, emb_q, mlp_q):
    from deep_quantized_recommendation_model_dqrm_amd import sgd_quantized_gradients_parallel_comm as H

    rows, D, B = [4, 300, 20000], 16, 128
    Ws = G.table_weights(rows, D, 12)
    torch.manual_seed(0)
    model = TinyDLRM(dq, rows, D, Ws)
    Wo = [w.copy() for w in Ws]
    for k in range(2):
        P = G.pooling_one(rows, B, 20 + k)
        lS_i = torch.from_numpy(P).cuda()
        lS_o = torch.arange(B, device="cuda").repeat(len(rows), 1)
        dense = torch.rand(B, 13, device="cuda")
        H.clear_gradients(model)
        s_fwd = [O.table_scale(w, 4) for w in Wo]
        out = model(dense, lS_o, lS_i)
        loss = out.pow(2).mean()
        loss.backward()
        # the tables' upstream gradient, kept on device by grad_mode="dp", drives the oracle
        batch, dy, ste, layout = model.emb_l._pending
        assert layout == "btd"
        dy_np = dy.detach().permute(1, 0, 2).contiguous().cpu().numpy()
        mlp = [model.bot_l[0], model.top_l[0]]
        mlp_p = [(l.weight.detach().cpu().numpy().copy(), l.bias.detach().cpu().numpy().copy()) for l in mlp]
        mlp_g = [(l.weight.grad.cpu().numpy().copy(), l.bias.grad.cpu().numpy().copy()) for l in mlp]
        H.grad_update_parallel_comm(model, 1, emb_grad_quantized=emb_q, num_bits=8, mlp_layer_quantized=mlp_q)
        H.weight_update_parallel_comm(model, 0.1, emb_grad_quantized=emb_q, num_gpus=1,
                                      mlp_layer_quantized=mlp_q)
        O.dp_step(Wo, [[(P[t], np.arange(B)) for t in range(len(rows))]], [[dy_np[t] for t in range(len(rows))]],
                  s_fwd, 0.1, grad_bits=8 if emb_q else 32)
        # MLP branch through libdqrm's dense kernels (s_q_g_p_c.py:337-409, 630-668)
        g_o, s_o = O.dense_dp_step(mlp_p, [mlp_g], 0.1, bits=8, quantized=mlp_q)
        for l, (W, b), (gw, gb), (sw, sb) in zip(mlp, mlp_p, g_o, s_o):
            np.testing.assert_array_equal(l.weight.detach().cpu().numpy(), W)
            np.testing.assert_array_equal(l.bias.detach().cpu().numpy(), b)
            np.testing.assert_array_equal(l.weight.grad.cpu().numpy(), gw)
            np.testing.assert_array_equal(l.bias.grad.cpu().numpy(), gb)
            if mlp_q:
                np.testing.assert_array_equal(l.weight_scaling_factor.cpu().numpy(), sw)
                assert float(l.bias_scaling_factor) == float(sb[0])
        if emb_q:
            s_avg = model.emb_l.emb_scaling_factor.cpu().numpy()
            for t in range(len(rows)):
                r_o, v_o, _ = O.emb_bwd_coalesce(rows[t], P[t], np.arange(B), dy_np[t], s_fwd[t])
                assert s_avg[t] == O.grad_scale(v_o, 8)
    for t in range(len(rows)):
        np.testing.assert_array_equal(model.emb_l.table_weight(t).detach().cpu().numpy(), Wo[t])
    assert model.emb_l._tset.read_errors() == 0


class ListDLRM(nn.Module):
    """The unchanged DP driver's model: emb_l = nn.ModuleList of one QuantEmbeddingBagTwo
    per table (dlrm_s_pytorch_tb_dp_one_parallel_comm.py:380), apply_emb's per-table loop."""

    def __init__(self, rows, D, Ws, **kw):
        super().__init__()
        self.emb_l = nn.ModuleList([_qebt(n, D, W, grad_mode="dp", **kw) for n, W in zip(rows, Ws)])
        self.bot_l = nn.Sequential(nn.Linear(13, D), nn.ReLU()).cuda()
        self.top_l = nn.Sequential(nn.Linear(D * (len(rows) + 1), 1)).cuda()

    def forward(self, dense, lS_o, lS_i):
        x = self.bot_l(dense)
        ly = [e(lS_i[t], lS_o[t]) for t, e in enumerate(self.emb_l)]
        return self.top_l(torch.cat([x] + ly, dim=1))


@pytest.mark.parametrize("consolidate", [True, False])
@pytest.mark.parametrize("emb_q", [True, False])
def test_dp_hooks_over_module_list_of_26_tables(dq, emb_q, consolidate):
    """grad_update / weight_update_parallel_comm over a ModuleList of 26 single-table
    modules run ONE exchange for all of them and match oracle.dp_step table by table;
    emb_scaling_factor per module. consolidate: the hooks move the 26 tables into one table
    set on first use (one coalesce / quantize-pack / apply launch per step for all tables,
    the modules running on one-table views of it); otherwise one MultiSetExchange over the
    modules' own sets (launches per module, still 2 collectives per step at N>1)."""
    from deep_quantized_recommendation_model_dqrm_amd import sgd_quantized_gradients_parallel_comm as H
    from deep_quantized_recommendation_model_dqrm_amd.comm import ConsolidatedExchange, MultiSetExchange

    rows, D, B = [min(n, 20000) for n in G.KAGGLE_ROWS], 16, 128
    Ws = G.table_weights(rows, D, 61)
    torch.manual_seed(0)
    H.set_consolidate_tables(consolidate)
    model = ListDLRM(rows, D, Ws)
    Wo = [w.copy() for w in Ws]
    for k in range(2):
        P = G.pooling_one(rows, B, 62 + k, dist="zipf" if k else "uniform")
        lS_i = torch.from_numpy(P).cuda()
        lS_o = torch.arange(B, device="cuda").repeat(len(rows), 1)
        H.clear_gradients(model)
        s_fwd = [O.table_scale(w, 4) for w in Wo]
        model(torch.rand(B, 13, device="cuda"), lS_o, lS_i).pow(2).mean().backward()
        dy_np = [m._pending[1].detach().cpu().numpy()[0] for m in model.emb_l]
        H.grad_update_parallel_comm(model, 1, emb_grad_quantized=emb_q, num_bits=8)
        H.weight_update_parallel_comm(model, 0.1, emb_grad_quantized=emb_q, num_gpus=1)
        res = O.dp_step(Wo, [[(P[t], np.arange(B)) for t in range(len(rows))]], [dy_np], s_fwd, 0.1,
                        grad_bits=8 if emb_q else 32)
        if emb_q:
            for t, m in enumerate(model.emb_l):
                assert m.emb_scaling_factor.item() == res[t][0]
    H.set_consolidate_tables(True)
    ex = model._dqrm_emb_exchange[1]
    if consolidate:  # one exchange over one set, the modules on views of it
        assert isinstance(ex, ConsolidatedExchange) and ex.tables.T == len(rows)
        assert all(m._tset.parent is ex.tables and m._tset.parent_index == t for t, m in enumerate(model.emb_l))
        assert all(m.embedding_bag.weight.data_ptr() == ex.tables.table_weight(t).data_ptr()
                   for t, m in enumerate(model.emb_l))
    else:
        assert isinstance(ex, MultiSetExchange) and len(ex.parts) == len(rows)
    assert len({m._tset.err.data_ptr() for m in model.emb_l}) == 1  # one error word, one read per step
    for t, m in enumerate(model.emb_l):
        np.testing.assert_array_equal(m.embedding_bag.weight.detach().cpu().numpy(), Wo[t])
        inc = m._tset.tmax.clone()
        m._tset.refresh_absmax()
        assert torch.equal(inc, m._tset.tmax)


def test_hooks_and_modules_raise_on_device_errors(dq):
    """An out-of-range index is flagged by the kernels and surfaces as DQRMError: from
    weight_update_parallel_comm for grad_mode="dp", from a following training call for the
    single-GPU modes (ATen raises on such input; nothing trains on silently). The checks
    poll an asynchronous snapshot of the flag word (no host sync), so the error surfaces
    once that snapshot has landed: within two calls here."""
    from deep_quantized_recommendation_model_dqrm_amd import _lib as L
    from deep_quantized_recommendation_model_dqrm_amd import quant_modules_not_quantize_grad as Q
    from deep_quantized_recommendation_model_dqrm_amd import sgd_quantized_gradients_parallel_comm as H

    Q.set_error_check_interval(1)  # poll on every call (default: every 8th)
    try:
        _raise_on_device_errors(dq, L, H)
    finally:
        Q.set_error_check_interval(8)


def _raise_on_device_errors(dq, L, H):
    rows, D, B = [10, 300], 16, 64
    Ws = G.table_weights(rows, D, 71)
    model = ListDLRM(rows, D, Ws)
    P = G.pooling_one(rows, B, 72)
    P[1, 5] = 300  # one past the end of table 1
    lS_o = torch.arange(B, device="cuda").repeat(len(rows), 1)
    model(torch.rand(B, 13, device="cuda"), lS_o, torch.from_numpy(P).cuda()).sum().backward()
    H.grad_update_parallel_comm(model, 1, num_bits=8)
    with pytest.raises(L.DQRMError, match="0x1"):
        for _ in range(2):
            H.weight_update_parallel_comm(model, 0.1, num_gpus=1)
            torch.cuda.synchronize()
    m = _qebt(rows[1], D, Ws[1], grad_mode="fused_sgd", lr=0.1)
    x, off = torch.from_numpy(P[1]).cuda(), torch.arange(B, device="cuda")
    m(x, off).sum().backward()
    with pytest.raises(L.DQRMError):
        for _ in range(2):
            m(x, off)
            torch.cuda.synchronize()


def test_weight_syncc_single_rank_is_identity(dq):
    from deep_quantized_recommendation_model_dqrm_amd import sgd_quantized_gradients_parallel_comm as H

    rows, D = [10, 500], 16
    Ws = G.table_weights(rows, D, 13)
    model = TinyDLRM(dq, rows, D, Ws)
    before = [p.detach().clone() for p in model.parameters()]
    H.weight_syncc(model, 1)
    for a, p in zip(before, model.parameters()):
        assert torch.equal(a, p.detach())
    assert float(model.emb_l._tset.tmax.max()) == max(float(np.abs(w).max()) for w in Ws)


def test_simulated_dp_module_api(dq):
    """sgd_quantized_gradients.py's buffer API over 4 micro-steps on one GPU."""
    from deep_quantized_recommendation_model_dqrm_amd import sgd_quantized_gradients as S

    rows, D, B, N = [6, 700, 40000], 16, 128, 4
    Ws = G.table_weights(rows, D, 14)
    model = TinyDLRM(dq, rows, D, Ws)
    Wo = [w.copy() for w in Ws]
    s_fwd = [O.table_scale(w, 4) for w in Wo]
    per_table = [([], []) for _ in rows]
    S.grad_buffer_zeroing(model)
    for k in range(N):
        P = G.pooling_one(rows, B, 30 + k, dist="zipf")
        out = model(torch.rand(B, 13, device="cuda"), torch.arange(B, device="cuda").repeat(len(rows), 1),
                    torch.from_numpy(P).cuda())
        out.pow(2).mean().backward()
        dy_np = model.emb_l._pending[1].detach().permute(1, 0, 2).contiguous().cpu().numpy()
        S.grad_buffer_update_added_quantization(model, N)
        for t in range(len(rows)):
            r, v, _ = O.emb_bwd_coalesce(rows[t], P[t], np.arange(B), dy_np[t], s_fwd[t])
            per_table[t][0].append(r)
            per_table[t][1].append(v)
    S.weights_update_added_quantization(model, 0.1, N)
    s_got = model.emb_l.emb_scaling_factor.cpu().numpy()
    for t in range(len(rows)):
        s = O.grad_scale(per_table[t][1][0], 8)  # the first micro-step's scale is kept
        assert s_got[t] == s
        buf = {}  # the reference's coalesced integer buffer (exact sums)
        for r_k, v_k in zip(*per_table[t]):
            for row, q in zip(r_k.tolist(), O.quantize(v_k, s, 8)):
                buf[row] = buf[row] + q if row in buf else q.copy()
        b_rows = np.array(sorted(buf), dtype=np.int64)
        O.simulated_dp_apply(Wo[t], b_rows, np.stack([buf[r] for r in b_rows.tolist()]), s, N, 0.1)
        np.testing.assert_array_equal(model.emb_l.table_weight(t).detach().cpu().numpy(), Wo[t])


def test_simulated_dp_unquantized_module_api(dq):
    """sgd_quantized_gradients.py:88-91 + :374-377 (emb_grad_quantized=False): the buffer
    sums grad / N per lookup in micro-step order; W += -lr * buffer. Bit-exact vs the oracle."""
    from deep_quantized_recommendation_model_dqrm_amd import sgd_quantized_gradients as S

    rows, D, B, N = [6, 700, 40000], 16, 128, 3
    Ws = G.table_weights(rows, D, 15)
    model = TinyDLRM(dq, rows, D, Ws)
    Wo = [w.copy() for w in Ws]
    s_fwd = [O.table_scale(w, 4) for w in Wo]
    batches, dys = [[] for _ in rows], [[] for _ in rows]
    S.grad_buffer_zeroing(model)
    for k in range(N):
        P = G.pooling_one(rows, B, 60 + k, dist="zipf")
        out = model(torch.rand(B, 13, device="cuda"), torch.arange(B, device="cuda").repeat(len(rows), 1),
                    torch.from_numpy(P).cuda())
        out.pow(2).mean().backward()
        dy_np = model.emb_l._pending[1].detach().permute(1, 0, 2).contiguous().cpu().numpy()
        S.grad_buffer_update_added_quantization(model, N, emb_grad_quantized=False)
        for t in range(len(rows)):
            batches[t].append((P[t], np.arange(B)))
            dys[t].append(dy_np[t])
    S.weights_update_added_quantization(model, 0.1, N, emb_grad_quantized=False)
    for t in range(len(rows)):
        O.simulated_dp_fp32(Wo[t], batches[t], dys[t], s_fwd[t], N, 0.1)
        np.testing.assert_array_equal(model.emb_l.table_weight(t).detach().cpu().numpy(), Wo[t])
    S.grad_buffer_zeroing(model)
    assert model.emb_l._sim_fp32 == []


@pytest.mark.parametrize("packed", [False, True])
def test_periodic_scale_refresh(dq, packed):
    """The period counters of q_m_n_q_g.py:303-315,354-363 (bound = P after the first
    refresh): the scale is recomputed at training calls 1, P+2, 2P+3, ... and frozen in
    between, while fused SGD keeps moving W (and, on the packed-INT4 path, repacks touched
    rows with the frozen scale). Pooling one, so the packed and FP32 forwards agree."""
    n, D, B, P, steps = 2000, 16, 256, 3, 9
    W = G.table_weights([n], D, 51)[0]
    m = _qebt(n, D, W, grad_mode="fused_sgd", lr=0.2, scale_period=P, use_packed_int4=packed)
    Wo = W.copy()
    s = None
    now = bound = nt = 0
    off = torch.arange(B, device="cuda")
    for k in range(steps):
        due = now == bound  # reference counter update
        if due:
            nt, now = nt + 1, 0
            if nt == 1 and bound == 0:
                bound += P
        else:
            nt, now = nt + 1, now + 1
        if due:
            s = O.table_scale(Wo, 4)
        Pk = G.pooling_one([n], B, 60 + k, dist="zipf")[0]
        y = m(torch.from_numpy(Pk).cuda(), off)
        y_o, _ = O.emb_fwd(Wo, Pk, np.arange(B), s)
        np.testing.assert_array_equal(y.detach().cpu().numpy(), y_o, err_msg=f"step {k}")
        assert m.eb_scaling_factor.item() == s
        assert (m.now_iteration.item(), m.iteration_bound.item(), m.iteration_nt.item()) == (now, bound, nt)
        dy = G.upstream_grad(1, B, D, 70 + k)[0] * f32(40.0)  # large enough to move the table max
        y.backward(torch.from_numpy(dy).cuda())
        O.emb_bwd_sgd(Wo, Pk, np.arange(B), dy, s, 0.2)
    np.testing.assert_array_equal(m.embedding_bag.weight.detach().cpu().numpy(), Wo)
    assert O.table_scale(Wo, 4) != s, "the table max should have moved while the scale was frozen"
