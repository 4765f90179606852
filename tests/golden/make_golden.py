"""Generate the golden fixtures under tests/golden/ with PyTorch (CPU) + Gloo.

The reference repository cannot be imported here (environment denial), and
its own tests hold no golden vectors. The arithmetic of the reference's hot path lives in
PyTorch, which IS available (2.10.0 CPU). This script therefore re-states the reference's
call sequence and executes it with the real torch ops (file:line of each call below):

  forward   QuantEmbeddingBagTwo.forward   quant_modules_not_quantize_grad.py:317-398
              scale  = symmetric_linear_quantization_param_two(bits, W)   quant_utils.py:141-194
              out    = nn.EmbeddingBag(mode="sum", sparse=True)(idx, off)  :288,367
              q      = SymmetricQuantFunction.apply(out, bits, scale)      quant_utils.py:322-346
              y      = q * scale                                           :393
  backward  SymmetricQuantFunction.backward: grad / scale                  quant_utils.py:349-363
  SGD       torch.optim.SGD(lr).step() on the sparse grad                 dlrm_s_pytorch_single_gpu.py:1736,1946
  DP        quantize_emb_grad + grad_update/weight_update_parallel_comm    s_q_g_p_c.py:257-317,601-628,850-890
            executed over N real Gloo processes (dist.all_reduce dense + sparse). grad.coalesce()
            is evaluated with CUDA's semantics (stable order, see stable_coalesce) because the
            reference's DP runs coalesce CUDA tensors; dp_n4_cpu_native.npz keeps torch CPU's
            own coalesce (unstable-sort order) and is compared within tolerance.
  sim-DP    grad_buffer_update_added_quantization / weights_update_added_quantization
                                                                           sgd_quantized_gradients.py:56-94,349-379

Run:  python tests/golden/make_golden.py        (writes tests/golden/*.npz; ~1 min)
"""
from __future__ import annotations

import os
import sys
import tempfile

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import gen_inputs as G  # noqa: E402

torch.set_num_threads(1)


# ----------------------------------------------------------------------------- restatement
class RefSymmetricQuant(torch.autograd.Function):
    """Same ops as SymmetricQuantFunction (quant_utils.py:316-363) with a CPU zero point."""

    @staticmethod
    def forward(ctx, x, k, scale):
        n = 2 ** (k - 1) - 1
        zero_point = torch.tensor(0.0)
        # linear_quantize (quant_utils.py:75-101)
        if len(x.shape) == 2:
            s = scale.view(-1, 1) if (len(scale.shape) != 1 or scale.shape[0] != 1) else scale
            zp = zero_point.view(-1, 1)
        else:
            s, zp = scale.view(-1), zero_point.view(-1)
        q = torch.round(1.0 / s * x + zp)
        q = torch.clamp(q, -n - 1, n)
        ctx.scale = scale
        return q

    @staticmethod
    def backward(ctx, g):
        scale = ctx.scale
        scale = scale.view(-1, 1) if len(g.shape) == 2 else scale.view(-1)
        return g / scale, None, None


def stable_coalesce(sp: torch.Tensor) -> torch.Tensor:
    """Tensor.coalesce() with CUDA semantics: stable sort of the indices, then each
    duplicate segment summed sequentially from 0 in ascending lookup position
    (the reference's DP runs coalesce CUDA tensors; torch CPU's coalesce instead sums in
    the order of an unstable std::sort permutation, a library artifact)."""
    idx = sp._indices()[0]
    vals = sp._values()
    order = torch.sort(idx, stable=True).indices.tolist()
    rows, sums = [], []
    for p in order:
        r = int(idx[p])
        if rows and rows[-1] == r:
            sums[-1] = sums[-1] + vals[p]
        else:
            rows.append(r)
            sums.append(torch.zeros_like(vals[p]) + vals[p])
    out = torch.sparse_coo_tensor(torch.tensor([rows], dtype=torch.int64), torch.stack(sums), sp.size())
    return out._coalesced_(True)


def ref_scale(values: torch.Tensor, bits: int) -> torch.Tensor:
    """symmetric_linear_quantization_param_two (quant_utils.py:141-194)."""
    with torch.no_grad():
        w_min, _ = torch.min(torch.min(values, dim=0).values, dim=0)
        w_max, _ = torch.max(torch.max(values, dim=0).values, dim=0)
        n = 2 ** (bits - 1) - 1
        scale = max(w_min.abs(), w_max.abs())
        return torch.clamp(scale, min=1e-8) / n


class RefQuantEmbeddingBag(torch.nn.Module):
    """QuantEmbeddingBagTwo's forward path (training mode, scale recomputed every call)."""

    def __init__(self, W: np.ndarray, bits: int = 4):
        super().__init__()
        n, d = W.shape
        self.bits = bits
        self.embedding_bag = torch.nn.EmbeddingBag(n, d, mode="sum", sparse=True)
        self.embedding_bag.weight.data = torch.tensor(W, requires_grad=True)
        self.eb_scaling_factor = None

    def forward(self, idx, off, full_precision_flag=False):
        if not full_precision_flag:
            self.eb_scaling_factor = ref_scale(self.embedding_bag.weight.data, self.bits)
        out = self.embedding_bag(idx, off, per_sample_weights=None)
        if full_precision_flag:
            return out
        q = RefSymmetricQuant.apply(out, self.bits, self.eb_scaling_factor)
        return q * self.eb_scaling_factor


def single_gpu_steps(Ws, batches, dys, lr=0.1, bits=4, full_precision=False):
    """Run len(batches) single-GPU QAT steps (forward, backward, torch.optim.SGD.step)."""
    mods = [RefQuantEmbeddingBag(W, bits) for W in Ws]
    opt = torch.optim.SGD([m.embedding_bag.weight for m in mods], lr=lr)
    rec = []
    for (idxs, offs), dy in zip(batches, dys):
        opt.zero_grad()
        ys, ss = [], []
        loss = 0
        for t, m in enumerate(mods):
            y = m(torch.from_numpy(idxs[t]), torch.from_numpy(offs[t]), full_precision_flag=full_precision)
            ys.append(y.detach().numpy().copy())
            ss.append(np.float32(0) if full_precision else m.eb_scaling_factor.numpy().copy())
            loss = loss + (y * torch.from_numpy(dy[t])).sum()
        loss.backward()
        opt.step()
        rec.append((ys, ss))
    return mods, rec


def touched(batches, t):
    return np.unique(np.concatenate([b[0][t] for b in batches])).astype(np.int64)


def save(name, **arrs):
    path = os.path.join(HERE, name)
    np.savez_compressed(path, **arrs)
    print("wrote", path, sum(np.asarray(v).nbytes for v in arrs.values()), "bytes raw")


# ----------------------------------------------------------------------------- cases
def case_single(name, num_rows, D, B, seed, bags="random", steps=2, bits=4, full_precision=False):
    Ws = G.table_weights(num_rows, D, seed)
    W0 = [w.copy() for w in Ws]
    batches, dys = [], []
    T = len(num_rows)
    for k in range(steps):
        if bags == "random":
            idxs, offs = G.random_bags(num_rows, B, seed + 17 * (k + 1))
        else:
            P = G.pooling_one(num_rows, B, seed + 17 * (k + 1), dist=bags)
            idxs = [P[t] for t in range(T)]
            offs = [np.arange(B, dtype=np.int64) for _ in range(T)]
        batches.append((idxs, offs))
        dys.append(G.upstream_grad(T, B, D, seed + 31 * (k + 1)))
    mods, rec = single_gpu_steps(Ws, batches, dys, bits=bits, full_precision=full_precision)
    out = dict(
        num_rows=np.asarray(num_rows, np.int64), D=np.int64(D), B=np.int64(B), seed=np.int64(seed),
        steps=np.int64(steps), bits=np.int64(bits), full_precision=np.int64(full_precision),
        bags=np.array(bags), lr=np.float32(0.1),
        input_checksum=np.array(G.checksum(W0, [b[0] for b in batches], [b[1] for b in batches], dys)),
    )
    for k, (ys, ss) in enumerate(rec):
        out[f"y{k}"] = np.stack(ys)
        out[f"s{k}"] = np.asarray(ss, np.float32)
    for t in range(T):
        rows = touched(batches, t)
        out[f"rows_t{t}"] = rows
        out[f"w_t{t}"] = mods[t].embedding_bag.weight.data.numpy()[rows]
    save(name, **out)


def case_edge():
    """Hand-built tables: .5 ties, clamp saturation, empty bags, duplicate rows in a bag,
    an all-zero table (scale floor 1e-8), bits 2/8/16, full precision."""
    D = 4
    W_tie = np.array([[7.0, 0.0, 0.0, 0.0],
                      [2.5, 3.5, -2.5, -0.5],
                      [0.5, 1.5, -1.5, 4.5],
                      [6.5, -6.5, 5.5, -7.0],
                      [-3.0, 3.0, 2.25, -2.75],
                      [1e-3, -1e-3, 0.0, -0.0]], dtype=np.float32)
    W_zero = np.zeros((4, D), dtype=np.float32)
    idx_tie = np.array([0, 1, 1, 2, 2, 3, 4, 3, 3, 5, 5], dtype=np.int64)
    off_tie = np.array([0, 1, 2, 4, 7, 7, 9, 9], dtype=np.int64)  # bags: [0] [1] [1,2] [2,3,4] [3,3] [] [5,5] []
    idx_zero = np.array([0, 1, 3, 3], dtype=np.int64)
    off_zero = np.array([0, 2, 2], dtype=np.int64)
    rs = np.random.RandomState(7)
    out = {}
    for bits in (2, 4, 8, 16):
        for name, W, idx, off in (("tie", W_tie, idx_tie, off_tie), ("zero", W_zero, idx_zero, off_zero)):
            dy = (rs.standard_normal((1, off.size, D)) * 0.5).astype(np.float32)
            mods, rec = single_gpu_steps([W.copy()], [([idx], [off])], [dy], bits=bits)
            out[f"{name}_b{bits}_y"] = rec[0][0][0]
            out[f"{name}_b{bits}_s"] = np.float32(rec[0][1][0])
            out[f"{name}_b{bits}_dy"] = dy[0]
            out[f"{name}_b{bits}_w"] = mods[0].embedding_bag.weight.data.numpy().copy()
    dy = (rs.standard_normal((1, off_tie.size, D)) * 0.5).astype(np.float32)
    mods, rec = single_gpu_steps([W_tie.copy()], [([idx_tie], [off_tie])], [dy], full_precision=True)
    out["fp_y"] = rec[0][0][0]
    out["fp_dy"] = dy[0]
    out["fp_w"] = mods[0].embedding_bag.weight.data.numpy().copy()
    out.update(W_tie=W_tie, W_zero=W_zero, idx_tie=idx_tie, off_tie=off_tie, idx_zero=idx_zero, off_zero=off_zero)
    save("edge.npz", **out)


def get_my_slice(n, my_size, my_rank):  # dlrm_s_pytorch_single_gpu.py:989-993
    k, m = divmod(n, my_size)
    return slice(my_rank * k + min(my_rank, m), (my_rank + 1) * k + min(my_rank + 1, m), 1)


def _dp_worker(rank, N, init_file, cfg, result_path):
    dist.init_process_group("gloo", init_method="file://" + init_file, rank=rank, world_size=N)
    torch.set_num_threads(1)
    num_rows, D, Bg, seed, bits, quantized, steps = (cfg[k] for k in
                                                     ("num_rows", "D", "B", "seed", "bits", "quantized", "steps"))
    T = len(num_rows)
    Ws = G.table_weights(num_rows, D, seed)
    mods = [RefQuantEmbeddingBag(W, 4) for W in Ws]
    lr = 0.1
    recs = {}
    for k in range(steps):
        P = G.pooling_one(num_rows, Bg, seed + 17 * (k + 1), dist=cfg.get("dist", "uniform"))
        dy_g = G.upstream_grad(T, Bg, D, seed + 31 * (k + 1))
        sl = get_my_slice(Bg, N, rank)
        # clear_gradients (s_q_g_p_c.py:714-734)
        for m in mods:
            if m.embedding_bag.weight.grad is not None:
                m.embedding_bag.weight.grad.zero_()
        loss = 0
        for t, m in enumerate(mods):
            idx = torch.from_numpy(P[t, sl].copy())
            off = torch.arange(idx.numel(), dtype=torch.int64)
            y = m(idx, off)
            loss = loss + (y * torch.from_numpy(dy_g[t, sl].copy())).sum()
        loss.backward()
        with torch.no_grad():
            for t, m in enumerate(mods):
                grad = m.embedding_bag.weight.grad
                coalesce = (lambda x: x.coalesce()) if cfg.get("native_coalesce") else stable_coalesce
                if quantized:  # quantize_emb_grad (s_q_g_p_c.py:850-890)
                    g = coalesce(grad)
                    scale = ref_scale(g.values(), bits)
                    s_loc = scale.clone()
                    dist.all_reduce(scale, dist.ReduceOp.SUM)
                    scale.mul_(1.0 / N)
                    scale = scale.view(-1)
                    q = RefSymmetricQuant.apply(g.values(), bits, scale)
                    upd = torch.sparse_coo_tensor(g.indices(), q, size=g.size())
                    rec_rows, rec_q = g.indices()[0].numpy().copy(), q.numpy().copy()
                    dist.all_reduce(upd, dist.ReduceOp.SUM)
                    upd.mul_(1.0 / N)
                    grad.zero_()
                    grad.add_(upd)
                    # weight_update_parallel_comm (:618-622)
                    grad_update_n = grad * scale.item()
                    m.embedding_bag.weight.data.add_(-lr * grad_update_n)
                    gl = [None] * N
                    dist.all_gather_object(gl, (float(s_loc), rec_rows, rec_q))
                    recs[f"k{k}_t{t}_s_avg"] = np.float32(scale.item())
                    for r in range(N):
                        recs[f"k{k}_t{t}_r{r}_s_loc"] = np.float32(gl[r][0])
                        recs[f"k{k}_t{t}_r{r}_rows"] = gl[r][1]
                        recs[f"k{k}_t{t}_r{r}_q"] = gl[r][2]
                else:  # emb_grad_quantized=False branch (:319-327) + update (:626)
                    g = coalesce(grad)
                    dist.all_reduce(g, dist.ReduceOp.SUM)
                    g.mul_(1.0 / N)
                    m.embedding_bag.weight.data.add_(-lr * g)
    if rank == 0:
        for t in range(T):
            recs[f"w_t{t}"] = mods[t].embedding_bag.weight.data.numpy().copy()
        np.savez_compressed(result_path, **recs)
    dist.barrier()
    dist.destroy_process_group()


def case_dp(name, N, quantized=True, bits=8, steps=2, dist_kind="uniform", native_coalesce=False):
    cfg = dict(num_rows=[3, 50, 1000, 20000], D=16, B=64, seed=321, bits=bits, quantized=quantized, steps=steps,
               dist=dist_kind, native_coalesce=native_coalesce)
    with tempfile.TemporaryDirectory() as tmp:
        init_file = os.path.join(tmp, "init")
        res = os.path.join(tmp, "res.npz")
        mp.spawn(_dp_worker, args=(N, init_file, cfg, res), nprocs=N, join=True)
        recs = dict(np.load(res))
    T = len(cfg["num_rows"])
    # final tables are dense and small except the 20000-row one: keep touched rows only
    out = {k: v for k, v in recs.items() if not k.startswith("w_t")}
    Ws0 = G.table_weights(cfg["num_rows"], cfg["D"], cfg["seed"])
    for t in range(T):
        changed = np.nonzero(np.any(recs[f"w_t{t}"] != Ws0[t], axis=1))[0]
        rows = np.union1d(changed, G.pooling_one(cfg["num_rows"], cfg["B"], cfg["seed"] + 17)[t])
        out[f"rows_t{t}"] = rows.astype(np.int64)
        out[f"w_t{t}"] = recs[f"w_t{t}"][rows]
    out.update(num_rows=np.asarray(cfg["num_rows"], np.int64), D=np.int64(cfg["D"]), B=np.int64(cfg["B"]),
               seed=np.int64(cfg["seed"]), N=np.int64(N), bits=np.int64(bits), quantized=np.int64(quantized),
               steps=np.int64(steps), dist=np.array(dist_kind), lr=np.float32(0.1),
               native_coalesce=np.int64(native_coalesce))
    save(name, **out)


def case_simulated_dp():
    """Simulated DP (sgd_quantized_gradients.py:56-94,349-379) over N=2 micro-steps with the
    first micro-step's scale; buffer of integer grads; W -= lr * buffer * (s/N)."""
    num_rows, D, B, seed, N = [5, 400], 8, 16, 99, 2
    Ws = G.table_weights(num_rows, D, seed)
    mods = [RefQuantEmbeddingBag(W, 4) for W in Ws]
    out = {}
    buffers = [None] * len(mods)
    scales = [None] * len(mods)
    for k in range(N):
        P = G.pooling_one(num_rows, B, seed + 17 * (k + 1))
        dy = G.upstream_grad(len(num_rows), B, D, seed + 31 * (k + 1))
        for m in mods:
            if m.embedding_bag.weight.grad is not None:
                m.embedding_bag.weight.grad.zero_()
        loss = 0
        for t, m in enumerate(mods):
            y = m(torch.from_numpy(P[t]), torch.arange(B, dtype=torch.int64))
            loss = loss + (y * torch.from_numpy(dy[t])).sum()
        loss.backward()
        with torch.no_grad():
            for t, m in enumerate(mods):
                g = stable_coalesce(m.embedding_bag.weight.grad)
                if scales[t] is None:
                    scales[t] = ref_scale(g.values(), 8).view(-1)
                q = RefSymmetricQuant.apply(g.values(), 8, scales[t])
                upd = torch.sparse_coo_tensor(g.indices(), q, size=g.size())
                buffers[t] = upd if buffers[t] is None else (buffers[t] + upd)
                buffers[t] = buffers[t].coalesce()
    with torch.no_grad():
        for t, m in enumerate(mods):
            weight_update = buffers[t] * (scales[t].item() / N)
            m.embedding_bag.weight.data.add_(-0.1 * weight_update)
            out[f"s_t{t}"] = np.float32(scales[t].item())
            out[f"buf_rows_t{t}"] = buffers[t].indices()[0].numpy().copy()
            out[f"buf_q_t{t}"] = buffers[t].values().numpy().copy()
            out[f"w_t{t}"] = m.embedding_bag.weight.data.numpy().copy()
    out.update(num_rows=np.asarray(num_rows, np.int64), D=np.int64(D), B=np.int64(B), seed=np.int64(seed),
               N=np.int64(N), lr=np.float32(0.1))
    save("sim_dp.npz", **out)


if __name__ == "__main__":
    case_edge()
    case_single("c1_random_bags.npz", [10000] * 8, 16, 128, 123, bags="random", steps=2)
    case_single("kaggle_pool1.npz", [min(n, 20000) for n in G.KAGGLE_ROWS], 16, 128, 123, bags="uniform", steps=2)
    case_single("kaggle_pool1_zipf.npz", [min(n, 20000) for n in G.KAGGLE_ROWS], 16, 128, 124, bags="zipf", steps=2)
    case_single("tb_pool1_d64.npz", [min(n, 4096) for n in G.TERABYTE_ROWS], 64, 64, 125, bags="uniform", steps=2)
    case_single("c1_bits8.npz", [2000] * 3, 16, 64, 126, bags="random", steps=1, bits=8)
    case_dp("dp_n2.npz", 2)
    case_dp("dp_n4.npz", 4)
    case_dp("dp_n4_zipf.npz", 4, dist_kind="zipf")
    case_dp("dp_n2_fp32.npz", 2, quantized=False)
    case_dp("dp_n2_b16.npz", 2, bits=16, steps=1)
    case_dp("dp_n4_cpu_native.npz", 4, native_coalesce=True)
    case_simulated_dp()
