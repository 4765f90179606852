"""Golden fixtures of the dense (MLP) gradient path of the data-parallel step, made with
PyTorch (CPU) + real Gloo process groups running the reference's call sequence
(sgd_quantized_gradients_parallel_comm.py @ 2024-10-24):

  quantize_linear_grad(layer, 8, parallel=True, num_gpus=N)    :892-929
      w_min/w_max = torch.min/max(grad, dim=1); scale = symmetric_linear_quantization_params(
      8, w_min, w_max, per_channel=True) (quant_utils.py:196-220); all_reduce(scale); *1/N;
      grad_up = SymmetricQuantFunction.apply(grad, 8, scale); all_reduce(grad_up); *1/N
  quantize_bias_grad(layer, 8, parallel=True, num_gpus=N)      :931-961
  grad_update_parallel_comm MLP branch                          :337-409
      layer.weight.grad.zero_(); layer.weight.grad.add_(buffer_changes)
  weight_update_parallel_comm MLP branch                        :630-668
      layer.weight.data.add_(-lr * layer.weight.grad * layer.weight_scaling_factor.view(-1, 1))
      layer.bias.data.add_(-lr * layer.bias.grad * layer.bias_scaling_factor)
  mlp_layer_quantized=False: all_reduce(grad); grad.mul_(1/N); W.add_(-lr * grad)

The reference itself cannot be imported here (environment denial); the ops
are PyTorch's. Gloo sums a one-element tensor in descending rank order but a vector in a
position-dependent order (ring chunks; measured), so for N >= 3 the per-row weight scales
of the fixture may differ from the build's fixed order in the last bit: the tests compare
those within 1 ulp and everything else exactly.

Run:  python tests/golden/make_golden_dense.py    (writes tests/golden/dense_*.npz)
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
from make_golden import RefSymmetricQuant  # noqa: E402

torch.set_num_threads(1)
SEED = 2024


def sym_params(num_bits, smin, smax, per_channel=False):  # quant_utils.py:196-220
    n = 2 ** (num_bits - 1) - 1
    if per_channel:
        scale, _ = torch.max(torch.stack([smin.abs(), smax.abs()], dim=1), dim=1)
        return torch.clamp(scale, min=1e-8) / n
    scale = max(smin.abs(), smax.abs())
    return torch.clamp(scale, min=1e-8) / n


def _worker(rank, N, init_file, cfg, result_path):
    dist.init_process_group("gloo", init_method="file://" + init_file, rank=rank, world_size=N)
    torch.set_num_threads(1)
    shapes, steps, quantized, lr = cfg["shapes"], cfg["steps"], cfg["quantized"], 0.1
    layers = []
    for W, b in G.mlp_params(shapes, SEED):
        l = torch.nn.Linear(W.shape[1], W.shape[0])
        with torch.no_grad():
            l.weight.copy_(torch.from_numpy(W))
            l.bias.copy_(torch.from_numpy(b))
        layers.append(l)
    recs = {}
    for k in range(steps):
        for l, (gW, gb) in zip(layers, G.mlp_grads(shapes, SEED, rank, k)):
            l.weight.grad = torch.from_numpy(gW.copy())
            l.bias.grad = torch.from_numpy(gb.copy())
        with torch.no_grad():
            for j, l in enumerate(layers):
                if quantized:
                    # quantize_linear_grad (:892-929)
                    w = l.weight.grad
                    w_min, _ = torch.min(w, dim=1, out=None)
                    w_max, _ = torch.max(w, dim=1, out=None)
                    s = sym_params(8, w_min, w_max, True)
                    dist.all_reduce(s, dist.ReduceOp.SUM)
                    s.mul_(1.0 / N)
                    q = RefSymmetricQuant.apply(w, 8, s)
                    dist.all_reduce(q, dist.ReduceOp.SUM)
                    q.mul_(1.0 / N)
                    l.weight_scaling_factor = s
                    l.weight.grad.zero_()
                    l.weight.grad.add_(q)
                    # quantize_bias_grad (:931-961)
                    b = l.bias.grad
                    b_min, _ = torch.min(b, dim=0, out=None)
                    b_max, _ = torch.max(b, dim=0, out=None)
                    sb = sym_params(8, b_min, b_max)
                    dist.all_reduce(sb, dist.ReduceOp.SUM)
                    sb.mul_(1.0 / N)
                    qb = RefSymmetricQuant.apply(b, 8, sb)
                    dist.all_reduce(qb, dist.ReduceOp.SUM)
                    qb.mul_(1.0 / N)
                    l.bias_scaling_factor = sb
                    l.bias.grad.zero_()
                    l.bias.grad.add_(qb)
                    recs[f"k{k}_l{j}_sw"] = s.numpy().copy()
                    recs[f"k{k}_l{j}_sb"] = np.float32(sb.item())
                else:
                    dist.all_reduce(l.weight.grad, dist.ReduceOp.SUM)
                    l.weight.grad.mul_(1.0 / N)
                    dist.all_reduce(l.bias.grad, dist.ReduceOp.SUM)
                    l.bias.grad.mul_(1.0 / N)
                recs[f"k{k}_l{j}_gw"] = l.weight.grad.numpy().copy()
                recs[f"k{k}_l{j}_gb"] = l.bias.grad.numpy().copy()
            # weight_update_parallel_comm (:630-668)
            for l in layers:
                if quantized:
                    l.weight.data.add_(-lr * l.weight.grad * l.weight_scaling_factor.view(-1, 1))
                    l.bias.data.add_(-lr * l.bias.grad * l.bias_scaling_factor)
                else:
                    l.weight.data.add_(-lr * l.weight.grad)
                    l.bias.data.add_(-lr * l.bias.grad)
    for j, l in enumerate(layers):
        recs[f"l{j}_W"] = l.weight.data.numpy().copy()
        recs[f"l{j}_b"] = l.bias.data.numpy().copy()
    np.savez_compressed(result_path + f".r{rank}.npz", **recs)
    dist.barrier()
    dist.destroy_process_group()


def case(name, N, quantized=True, steps=2):
    cfg = dict(shapes=G.MLP_SHAPES, steps=steps, quantized=quantized)
    with tempfile.TemporaryDirectory() as tmp:
        init_file = os.path.join(tmp, "init")
        res = os.path.join(tmp, "res")
        mp.spawn(_worker, args=(N, init_file, cfg, res), nprocs=N, join=True)
        r0 = dict(np.load(res + ".r0.npz"))
        for r in range(1, N):  # every rank must hold the same model (Gloo results are replicated)
            rr = np.load(res + f".r{r}.npz")
            for k in r0:
                assert np.array_equal(r0[k], rr[k]), (name, r, k)
    r0.update(N=np.int64(N), quantized=np.int64(quantized), steps=np.int64(steps), seed=np.int64(SEED),
              lr=np.float32(0.1), shapes=np.asarray(G.MLP_SHAPES, np.int64))
    np.savez_compressed(os.path.join(HERE, name), **r0)
    print("wrote", name)


if __name__ == "__main__":
    case("dense_n2.npz", 2)
    case("dense_n4.npz", 4)
    case("dense_n2_fp32.npz", 2, quantized=False)
