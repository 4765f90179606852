#!/usr/bin/env python3
"""Bandwidth of the row-wise PTQ gather (dqrm_rowwise_bag) and prepack (dqrm_rowwise_prepack).

The reference serves a PTQ model with one ops.quantized.embedding_bag_{4bit,byte}_rowwise_offsets
call per table (dlrm_s_pytorch_single_gpu_documentingp.py:653-663); this times exactly that,
one launch per table, at the C5 table shapes (D=64, the TB row counts of SURVEY.md 8(d)) or the
Kaggle shapes (D=16), pooling one, B samples per launch. Packed tables are synthesised as
random payload bytes with valid scale/bias fields (content does not change the access pattern).

Algorithmic bytes per launch (SURVEY.md 8(d), K3 with the row-wise row size):
    B * (row_bytes + 8 idx + 8 offset + 4 D out)       row_bytes = D/2 + 4 (4-bit), D + 8 (8-bit)
Prepack: n * (4 D read + row_bytes write).

usage: python tools/bench_rowwise.py [--shape tb|kaggle] [--batch 65536] [--iters 50]
(kernel-only durations: run under rocprofv3 --kernel-trace --stats, tools/prof_rowwise.sh)
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import CONFIGS  # noqa: E402
import deep_quantized_recommendation_model_dqrm_amd as dq  # noqa: E402
from deep_quantized_recommendation_model_dqrm_amd import quantized_ops as Q  # noqa: E402


def synth_packed(n, D, bits, dev):
    rb = D // 2 + 4 if bits == 4 else D + 8
    p = torch.randint(0, 256, (n, rb), dtype=torch.uint8, device=dev)
    if bits == 4:
        sb = torch.tensor([0.01, -0.05], dtype=torch.float16).view(torch.uint8)
        p[:, D // 2:] = sb.to(dev)
    else:
        sb = torch.tensor([0.001, -0.1], dtype=torch.float32).view(torch.uint8)
        p[:, D:] = sb.to(dev)
    return p


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="tb", choices=["tb", "kaggle"])
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--iters", type=int, default=50)
    args = ap.parse_args()
    dq.build(verbose=False)
    dev = torch.device("cuda")
    cfg = CONFIGS["terabyte" if args.shape == "tb" else "kaggle"]
    rows, D = cfg["rows"], cfg["dim"]
    B = args.batch
    out = []
    for bits in (4, 8):
        rb = D // 2 + 4 if bits == 4 else D + 8
        tables = [synth_packed(n, D, bits, dev) for n in rows]
        idx = [torch.randint(0, n, (B,), device=dev) for n in rows]
        off = torch.arange(B, device=dev)
        bag = Q.embedding_bag_4bit_rowwise_offsets if bits == 4 else Q.embedding_bag_byte_rowwise_offsets
        for _ in range(3):
            for t in range(len(rows)):
                bag(tables[t], idx[t], off, check=False)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.iters):
            for t in range(len(rows)):
                bag(tables[t], idx[t], off, check=False)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / (args.iters * len(rows))
        algo = B * (rb + 8 + 8 + 4 * D)
        out.append({"op": f"rowwise{bits}_bag", "shape": args.shape, "D": D, "B": B, "tables": len(rows),
                    "us_per_launch_incl_host": round(us, 2), "algo_bytes_per_launch": algo,
                    "GBps_incl_host": round(algo / us / 1e3, 1)})
        del tables
        torch.cuda.empty_cache()
        # prepack of one large table
        n = 50_000_000 if args.shape == "tb" else 10_000_000
        W = torch.rand(n, D, device=dev) - 0.5
        pre = Q.embedding_bag_4bit_prepack if bits == 4 else Q.embedding_bag_byte_prepack
        pre(W)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(5):
            pre(W)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / 5
        algo = n * (4 * D + rb)
        out.append({"op": f"rowwise{bits}_prepack", "rows": n, "D": D, "us": round(us, 1),
                    "algo_bytes": algo, "GBps": round(algo / us / 1e3, 1)})
        del W
        torch.cuda.empty_cache()
    for o in out:
        print(json.dumps(o))


if __name__ == "__main__":
    main()
