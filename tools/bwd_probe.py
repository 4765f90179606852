"""Time the backward's kernels (K4a sort, K4b segments) per table mix under rocprofv3.

usage: rocprofv3 --kernel-trace --stats -d gpurun_out/probe -o p --output-format csv -- \
           python3 tools/bwd_probe.py <mix> [B] [mode]
mix: tb (reference TB rows, D=64), narrow / mid / wide (the TB tables of <=256, 257..100k,
>100k rows), kaggle (D=16); mode: coalesce (default) | sgd
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import deep_quantized_recommendation_model_dqrm_amd as dq  # noqa: E402
from deep_quantized_recommendation_model_dqrm_amd.workloads import KAGGLE_ROWS, TERABYTE_ROWS  # noqa: E402

mix = sys.argv[1] if len(sys.argv) > 1 else "tb"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 2048
mode = sys.argv[3] if len(sys.argv) > 3 else "coalesce"
D = 16 if mix == "kaggle" else 64
rows = {
    "tb": TERABYTE_ROWS,
    "kaggle": KAGGLE_ROWS,
    "narrow": [n for n in TERABYTE_ROWS if n <= 256],
    "mid": [n for n in TERABYTE_ROWS if 256 < n <= 100_000],
    "wide": [n for n in TERABYTE_ROWS if n > 100_000],
}[mix]
T = len(rows)
ts = dq.EmbeddingTableSet(rows, D, device="cuda", init="uniform", seed=1)
g = torch.Generator(device="cuda").manual_seed(5)
P = torch.stack([torch.randint(0, n, (B,), generator=g, device="cuda") for n in rows])
b = dq.LookupBatch.pooling_one(P)
dy = torch.randn(T, B, D, device="cuda", generator=g) * 0.05
ts.forward(b)
ws = dq.CoalescedGrad.allocate(rows, B, D, "cuda")
for _ in range(60):
    if mode == "sgd":
        ts.backward_sgd(b, dy, lr=1e-4)
    else:
        ts.backward_coalesce(b, dy, ws)
torch.cuda.synchronize()
print(f"{mix} T={T} B={B} D={D} mode={mode} errors={ts.read_errors()}")
