"""Time the DP update kernel (dqrm_apply_sparse_update: k_apply_flat and the per-slot
k_table_apply, each + k_table_finalize) for N emulated ranks on
one GPU: N different ranks' payloads (coalesce + quant-pack of N different batch slices)
gathered into one buffer, exactly what the RCCL all-gather delivers at N GPUs.
usage: python tools/bench_apply_ranks.py [terabyte|tbsmall|kaggle] [flat,slot,ranges,merge] [B per rank] [N list, e.g. 1,2,4,8] -> one JSON line per N"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests", "golden")]
import deep_quantized_recommendation_model_dqrm_amd as dq  # noqa: E402
from deep_quantized_recommendation_model_dqrm_amd import _lib as L  # noqa: E402
import gen_inputs as G  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "terabyte"
D = 64 if cfg.startswith("tb") or cfg == "terabyte" else 16
rows = [n * 16 if n >= 1_000_000 else n for n in G.TERABYTE_ROWS] if D == 64 else G.KAGGLE_ROWS
if cfg == "tbsmall":  # the TB shape with every table capped at 2 M rows (~2 GB of W): the same entries, few TLB misses
    rows = [min(n, 2_000_000) for n in rows]
B = 2048
T = len(rows)
ts = dq.EmbeddingTableSet(rows, D, device="cuda", init="uniform", seed=3)
lib = L.load()
KINDS = {"flat": L.DQRM_APPLY_FLAT, "slot": L.DQRM_APPLY_SLOT, "ranges": L.DQRM_APPLY_RANGES,
         "merge": L.DQRM_APPLY_MERGE}
modes = sys.argv[2].split(",") if len(sys.argv) > 2 else ["flat", "slot", "merge"]
B = int(sys.argv[3]) if len(sys.argv) > 3 else B
ex = dq.SparseGradExchange(ts, B, grad_bits=8)
NS = [int(x) for x in sys.argv[4].split(",")] if len(sys.argv) > 4 else [1, 2, 4, 8]
for mode, N in [(m, n) for m in modes for n in NS]:
    lib.dqrm_set_apply_kernel(KINDS[mode])
    gathered = torch.zeros(N, ex.payload_bytes, dtype=torch.uint8, device="cuda")
    for r in range(N):
        P = torch.stack([torch.randint(0, n, (B,), device="cuda") for n in rows])
        b = dq.LookupBatch.pooling_one(P)
        dy = torch.randn(T, B, D, device="cuda") * 0.05
        ts.forward(b)
        ex.kernels.coalesce(b, dy, ex.ws, True, "tbd")
        ex.kernels.quant_pack(ex.ws, ex.ws.absmax.view(1, -1), 1, 8, ex.cap_base, ex.cap_total, ex.s_avg, ex.payload)
        gathered[r].copy_(ex.payload)

    aws = torch.zeros(max(16, int(lib.dqrm_apply_workspace_bytes(N, ex.cap_total))), dtype=torch.uint8, device="cuda")

    def run():
        ex.kernels.apply(ex.cap_base, ex.cap_total, gathered, ex.payload_bytes, N, 8, ex.s_avg, 1e-3,
                         L.DQRM_UPD_DP, False, workspace=aws)

    for _ in range(5):
        run()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(30)]
    for a, c in ev:
        a.record()
        run()
        c.record()
    torch.cuda.synchronize()
    ms = float(np.median([a.elapsed_time(c) for a, c in ev]))
    assert ts.read_errors() == 0
    print(json.dumps({"kernel": f"apply_sparse_update ({mode})" + (" + finalize" if mode in ("flat", "slot") else
                                                                   " (k_merge_pos + k_apply_pos)" if N > 1 else ""),
                      "config": cfg, "emulated_ranks": N, "batch_per_rank": B,
                      "ms": round(ms, 4)}), flush=True)
