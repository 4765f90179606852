"""Golden fixtures for weight_syncc on identical replicas, made with real Gloo process groups
(PyTorch CPU) running the reference's arithmetic (sgd_quantized_gradients_parallel_comm.py
@ 2024-10-24, :963-970; the DP driver initialises Gloo, dlrm_s_pytorch_tb_dp_one_parallel_comm.py:1408-1413):

    dist.all_reduce(param, dist.ReduceOp.SUM); param.mul_(1. / num_gpus)

Every rank holds the same values (what the DP step maintains between syncs), so the result
depends only on the order in which Gloo adds the N copies. The fixture pins that order for
N = 3, 5, 6, 8 at two sizes: a short vector (stored whole) and a 1 Mi-element one (spread
over many ring chunks; stored as a checksum of the result and of every rank's agreement).
The package computes the same result locally (dqrm_replica_mean: a sequential fold
fl(...fl(x + x) + x ...) * fl(1/N)); tests/test_syncc_golden.py and
tests/test_gpu_parity.py::test_replica_mean_matches_gloo_fixture check it against this file.

The reference itself cannot be imported here (environment denial); the
collective is torch's Gloo backend, the one the reference's driver runs.

Run:  python tests/golden/make_golden_syncc.py    (writes tests/golden/syncc_gloo.npz)
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

WORLDS = (3, 5, 6, 8)
SMALL, LARGE = 4099, 1 << 20
SEED_SMALL, SEED_LARGE = 963, 970


def _worker(rank, N, init_file, out_dir):
    dist.init_process_group("gloo", init_method="file://" + init_file, rank=rank, world_size=N)
    torch.set_num_threads(1)
    try:
        res = {}
        for tag, n, seed in (("small", SMALL, SEED_SMALL), ("large", LARGE, SEED_LARGE)):
            p = torch.from_numpy(G.replica_values(n, seed))
            with torch.no_grad():
                dist.all_reduce(p, dist.ReduceOp.SUM)
                p.mul_(1. / N)
            res[tag] = p.numpy().copy()
        np.savez(os.path.join(out_dir, f"r{rank}.npz"), **res)
    finally:
        dist.destroy_process_group()


def run(N):
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(N, os.path.join(d, "init"), d), nprocs=N, join=True)
        got = [dict(np.load(os.path.join(d, f"r{r}.npz"))) for r in range(N)]
    for r in range(1, N):
        for k in got[0]:
            assert np.array_equal(got[r][k].view(np.uint32), got[0][k].view(np.uint32)), (N, r, k)
    return got[0]


def main():
    out = {"worlds": np.array(WORLDS, np.int32), "sizes": np.array([SMALL, LARGE], np.int64),
           "seeds": np.array([SEED_SMALL, SEED_LARGE], np.int64),
           "x_small_checksum": np.array(G.checksum(G.replica_values(SMALL, SEED_SMALL))),
           "x_large_checksum": np.array(G.checksum(G.replica_values(LARGE, SEED_LARGE)))}
    for N in WORLDS:
        r = run(N)
        out[f"small_n{N}"] = r["small"]
        out[f"large_n{N}_checksum"] = np.array(G.checksum(r["large"]))
        print(N, "moved", int(np.sum(r["small"].view(np.uint32) != G.replica_values(SMALL, SEED_SMALL).view(np.uint32))))
    np.savez_compressed(os.path.join(HERE, "syncc_gloo.npz"), **out)


if __name__ == "__main__":
    main()
