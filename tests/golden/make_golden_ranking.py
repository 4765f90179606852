"""Golden fixtures of the ranking-range mixed-precision gradient path (§8(f) #3), made with
PyTorch (CPU) + real Gloo process groups running the reference's call sequence
(sgd_quantized_gradients_parallel_comm.py @ 2024-10-24, call site
dlrm_s_pytorch_tb_dp_one_parallel_comm.py:1897-1899):

  grad_precision_and_scale(dlrm, N, rank)                       :158-255
      range = finding_range_for_gradient(grad.coalesce().values()); all_reduce; * 1/N
      emb_scaling_factor = range; range_list += (range / (eb_scaling_factor * 7)).item()
      rank 0: list_id = np.random.choice(26, 26, replace=False, p=range_list/sum)[::-1]
              j <= 8 -> 0 bits, j <= 22 -> 8 bits, else 32; broadcast(gradient_bit_width, 0)
      8-bit tables: emb_scaling_factor = clamp(range, 1e-8) / 127
  grad_update_parallel_comm(..., ranking_range=True)           :280-309 (0/32 skipped)
      quantize_emb_grad_two: q = SymmetricQuantFunction(values, bits, scale); all_reduce; * 1/N
  weight_update_parallel_comm(..., ranking_range=True)         :610-622
      0: no update; 32: W.add_(-lr * grad) (local grad); 8: W.add_(-lr * (grad * s.item()))

numpy's global RNG is seeded identically on every rank (only rank 0 draws). coalesce is
evaluated with CUDA's stable order (make_golden.stable_coalesce), as for the other DP
fixtures. The reference itself cannot be imported here.
Run:  python tests/golden/make_golden_ranking.py   (writes tests/golden/ranking_n2.npz)
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
from make_golden import RefQuantEmbeddingBag, RefSymmetricQuant, get_my_slice, stable_coalesce  # noqa: E402

torch.set_num_threads(1)
ROWS = [3, 4, 10, 14, 36, 62, 102, 122, 300, 500, 700, 900, 1200, 1500, 2000, 2500, 3000, 3500, 4000,
        4500, 5000, 6000, 7000, 8000, 9000, 10000]
D, B_GLOBAL, SEED, RNG_SEED, STEPS = 16, 64, 555, 77, 2


def finding_range_for_gradient(values):  # quant_utils.py, tensor branch
    w_min, _ = torch.min(torch.min(values, dim=0, out=None).values, dim=0, out=None)
    w_max, _ = torch.max(torch.max(values, dim=0, out=None).values, dim=0, out=None)
    return max(w_min.abs(), w_max.abs())


def _worker(rank, N, init_file, result_path):
    dist.init_process_group("gloo", init_method="file://" + init_file, rank=rank, world_size=N)
    torch.set_num_threads(1)
    np.random.seed(RNG_SEED)
    mods = [RefQuantEmbeddingBag(W, 4) for W in G.table_weights(ROWS, D, SEED)]
    for m in mods:
        m.gradient_bit_width = torch.zeros(1)
    lr, recs = 0.1, {}
    for k in range(STEPS):
        P = G.pooling_one(ROWS, B_GLOBAL, SEED + 17 * (k + 1), dist="zipf" if k % 2 else "uniform")
        dy_g = G.upstream_grad(len(ROWS), B_GLOBAL, D, SEED + 31 * (k + 1))
        sl = get_my_slice(B_GLOBAL, N, rank)
        for m in mods:  # clear_gradients
            if m.embedding_bag.weight.grad is not None:
                m.embedding_bag.weight.grad.zero_()
        loss = 0
        for t, m in enumerate(mods):
            idx = torch.from_numpy(P[t, sl].copy())
            y = m(idx, torch.arange(idx.numel(), dtype=torch.int64))
            loss = loss + (y * torch.from_numpy(dy_g[t, sl].copy())).sum()
        loss.backward()
        with torch.no_grad():
            # grad_precision_and_scale (:176-255)
            range_list = []
            for t, m in enumerate(mods):
                r = finding_range_for_gradient(stable_coalesce(m.embedding_bag.weight.grad).values())
                dist.all_reduce(r, op=dist.ReduceOp.SUM)
                r.mul_(1.0 / N)
                m.emb_scaling_factor = r
                range_list.append((r / (m.eb_scaling_factor * 7)).item())
            if rank == 0:
                prob_l = range_list / (np.sum(range_list))
                list_id = np.random.choice(26, 26, replace=False, p=prob_l)
                list_id = list_id[::-1]
                for j, t in enumerate(list_id):
                    if j <= 8:
                        mods[t].gradient_bit_width.zero_()
                    elif j <= 22:
                        mods[t].gradient_bit_width.zero_().add_(8)
                    else:
                        mods[t].gradient_bit_width.zero_().add_(32)
            dist.barrier()
            for t, m in enumerate(mods):
                dist.broadcast(m.gradient_bit_width, 0)
                if m.gradient_bit_width == 0 or m.gradient_bit_width == 32:
                    continue
                n = 2 ** (m.gradient_bit_width - 1) - 1
                m.emb_scaling_factor = torch.clamp(m.emb_scaling_factor, min=1e-8) / n
            # grad_update_parallel_comm, ranking_range=True (:278-309)
            for t, m in enumerate(mods):
                bw = m.gradient_bit_width.item()
                if bw == 0 or bw == 32:
                    continue
                g = stable_coalesce(m.embedding_bag.weight.grad)
                upd = torch.sparse_coo_tensor(g.indices(), RefSymmetricQuant.apply(g.values(), m.gradient_bit_width,
                                                                                   m.emb_scaling_factor),
                                              size=g.size())
                dist.all_reduce(upd, dist.ReduceOp.SUM)
                upd.mul_(1.0 / N)
                m.embedding_bag.weight.grad.zero_()
                m.embedding_bag.weight.grad.add_(upd)
            # weight_update_parallel_comm, ranking_range=True (:605-622)
            for t, m in enumerate(mods):
                bw = m.gradient_bit_width.item()
                if bw == 0:
                    continue
                if bw == 32:
                    m.embedding_bag.weight.data.add_(-lr * m.embedding_bag.weight.grad)
                else:
                    grad_update_n = m.embedding_bag.weight.grad * m.emb_scaling_factor.item()
                    m.embedding_bag.weight.data.add_(-lr * grad_update_n)
            recs[f"k{k}_bits"] = np.array([int(m.gradient_bit_width.item()) for m in mods], np.int32)
            recs[f"k{k}_scale"] = np.array([float(m.emb_scaling_factor) for m in mods], np.float32)
            recs[f"k{k}_eb"] = np.array([float(m.eb_scaling_factor) for m in mods], np.float32)
    for t, m in enumerate(mods):
        recs[f"w_t{t}"] = m.embedding_bag.weight.data.numpy().copy()
    np.savez_compressed(result_path + f".r{rank}.npz", **recs)
    dist.barrier()
    dist.destroy_process_group()


def main(N=2, name="ranking_n2.npz"):
    with tempfile.TemporaryDirectory() as tmp:
        res = os.path.join(tmp, "res")
        mp.spawn(_worker, args=(N, os.path.join(tmp, "init"), res), nprocs=N, join=True)
        out = {}
        W0 = G.table_weights(ROWS, D, SEED)
        for r in range(N):
            for k, v in np.load(res + f".r{r}.npz").items():
                if k.startswith("w_t"):  # final tables as a patch over the initial ones
                    t = int(k[3:])
                    ch = np.nonzero(np.any(v != W0[t], axis=1))[0]
                    out[f"r{r}_rows_t{t}"] = ch.astype(np.int64)
                    out[f"r{r}_vals_t{t}"] = v[ch]
                else:
                    out[f"r{r}_{k}"] = v
    out.update(rows=np.asarray(ROWS, np.int64), D=np.int64(D), B=np.int64(B_GLOBAL), seed=np.int64(SEED),
               rng_seed=np.int64(RNG_SEED), N=np.int64(N), steps=np.int64(STEPS), lr=np.float32(0.1))
    np.savez_compressed(os.path.join(HERE, name), **out)
    print("wrote", name, {k: out[k].tolist() for k in out if k.endswith("_bits")})


if __name__ == "__main__":
    main()
