"""Table-size profiles of the reference's benchmark configurations and device-side synthetic
Criteo-form batches (BASELINE.json configs).

The reference's datasets cannot be fetched here, so benchmarks run on synthetic indices of
the same shape: one index per (table, sample), offsets = arange(B)
(collate_wrapper_criteo_offset, dlrm_data_pytorch.py:328-345).
"""
from __future__ import annotations

import math

import torch

# Criteo-Kaggle table sizes (bash_scripts/Kaggle/emb_bit_4.txt:16-41)
KAGGLE_ROWS = [1460, 583, 10131227, 2202608, 305, 24, 12517, 633, 3, 93145, 5683, 8351593, 3194, 27,
               14992, 5461306, 10, 5652, 2173, 4, 7046547, 18, 15, 286181, 105, 142572]
# reference TB profile at --max-ind-range=10M (python_profiling_script/finding_kaggle_compression_ratio.py:5)
TERABYTE_ROWS = [9980200, 26095, 17224, 7383, 20152, 3, 7112, 1435, 62, 9756762, 1332128, 314263, 10, 2208,
                 11168, 122, 4, 971, 14, 9994101, 7267918, 9946670, 415284, 12422, 102, 36]
# BASELINE config 5 (~800 M rows): the TB profile with its six >= 1 M-row tables x16 (773,280,534 rows)
TERABYTE_X16_ROWS = [n * 16 if n >= 1_000_000 else n for n in TERABYTE_ROWS]

# A diagnostic profile, not a BASELINE config: the TB profile with its >= 1 M-row tables cut to
# 500 k rows (3.8 M rows, 0.98 GB): the same lookups and (uniform) distinct rows per step as
# "terabyte", on a slab whose pages a TLB can cover -- separates address translation from the
# rest of the step's cost.
TERABYTE_1G_ROWS = [500_000 if n >= 1_000_000 else n for n in TERABYTE_ROWS]

# name -> (rows, embedding dim); the bench's --config
CONFIGS = {
    "terabyte": (TERABYTE_X16_ROWS, 64),   # BASELINE configs[4]
    "terabyte_ref": (TERABYTE_ROWS, 64),   # the reference's own TB run (49.1 M rows)
    "terabyte_1g": (TERABYTE_1G_ROWS, 64),  # diagnostic (translation A/B), see above
    "kaggle": (KAGGLE_ROWS, 16),           # BASELINE configs[1-3]
}

# the reference scripts' MLPs (bash_scripts/): Kaggle --arch-mlp-bot=13-512-256-64-16
# --arch-mlp-top=512-256-1; Terabyte 13-512-256-64 / 512-512-256-1; the top MLP's input is
# D + T(T+1)/2 (dot interaction of T+1 vectors, dlrm_s_pytorch_single_gpu.py create_mlp)
MLPS = {
    "terabyte": ([13, 512, 256, 64], [64 + 351, 512, 512, 256, 1]),
    "terabyte_ref": ([13, 512, 256, 64], [64 + 351, 512, 512, 256, 1]),
    "terabyte_1g": ([13, 512, 256, 64], [64 + 351, 512, 512, 256, 1]),
    "kaggle": ([13, 512, 256, 64, 16], [16 + 351, 512, 256, 1]),
}


def synthetic_indices(rows, B: int, seed: int, dist: str = "uniform", device="cuda") -> torch.Tensor:
    """[T, B] int64 Criteo-form indices generated on the device. "uniform": U[0, n_t);
    "zipf": a power law over the row id via an inverse transform on a log scale
    (row = floor(n^u) - 1, u ~ U[0, 1)), the hot rows at the low ids."""
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    cols = []
    for n in rows:
        if dist == "uniform":
            cols.append(torch.randint(0, n, (B,), generator=g, device=device, dtype=torch.int64))
        elif dist == "zipf":
            u = torch.rand(B, generator=g, device=device, dtype=torch.float64)
            z = torch.floor(torch.exp(u * math.log(float(n)))) - 1
            cols.append(z.clamp_(0, n - 1).to(torch.int64))
        else:
            raise ValueError(dist)
    return torch.stack(cols)


__all__ = ["KAGGLE_ROWS", "TERABYTE_ROWS", "TERABYTE_X16_ROWS", "TERABYTE_1G_ROWS", "CONFIGS", "MLPS", "synthetic_indices"]
