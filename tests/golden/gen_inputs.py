"""Deterministic input generators shared by make_golden.py and the tests.

Inputs are regenerated from seeds (numpy's legacy RandomState / MT19937, whose stream is
stable across numpy versions); fixtures store the expected outputs plus a checksum of the
generated inputs so drift in a generator is caught.

Distributions follow the reference:
  table init   U(-sqrt(1/n), +sqrt(1/n))     quant_modules_not_quantize_grad.py:273-275
  random bags  generate_dist_input_batch     dlrm_data_pytorch.py:1099-1157 ("uniform")
  Criteo form  one index per (table, sample), offsets = arange(B)   dlrm_data_pytorch.py:328-345
"""
from __future__ import annotations

import hashlib

import numpy as np

# table-size profiles live in the package (bench.py uses them too)
import os as _os  # noqa: E402
import sys as _sys  # noqa: E402

_ROOT = _os.path.dirname(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))))
if _ROOT not in _sys.path:
    _sys.path.insert(0, _ROOT)
from deep_quantized_recommendation_model_dqrm_amd.workloads import KAGGLE_ROWS, TERABYTE_ROWS  # noqa: E402,F401


def table_weights(num_rows, dim, seed):
    out = []
    for t, n in enumerate(num_rows):
        rs = np.random.RandomState(seed + 1000 * t)
        b = np.sqrt(1.0 / n)
        out.append(rs.uniform(low=-b, high=b, size=(n, dim)).astype(np.float32))
    return out


def random_bags(num_rows, B, seed, num_indices_per_lookup=10, fixed=False):
    """Per table: (idx int64 [L_t], off int64 [B]) with unique sorted indices per bag."""
    rs = np.random.RandomState(seed)
    idxs, offs = [], []
    for size in num_rows:
        off, ind, o = [], [], 0
        for _ in range(B):
            if fixed:
                g = np.int64(num_indices_per_lookup)
            else:
                r = rs.random_sample(1)
                g = np.int64(np.round(max(1.0, float(r[0]) * min(size, num_indices_per_lookup))))
            r = rs.random_sample(int(g))
            grp = np.unique(np.round(r * (size - 1)).astype(np.int64))
            off.append(o)
            ind.extend(grp.tolist())
            o += grp.size
        idxs.append(np.asarray(ind, dtype=np.int64))
        offs.append(np.asarray(off, dtype=np.int64))
    return idxs, offs


def pooling_one(num_rows, B, seed, dist="uniform", alpha=1.05):
    """[T, B] int64 Criteo-form indices (one lookup per sample and table)."""
    rs = np.random.RandomState(seed)
    out = np.empty((len(num_rows), B), dtype=np.int64)
    for t, n in enumerate(num_rows):
        if dist == "uniform":
            out[t] = rs.randint(0, n, size=B)
        elif dist == "zipf":
            z = rs.zipf(alpha, size=B) - 1
            out[t] = np.minimum(z, n - 1)
        else:
            raise ValueError(dist)
    return out


def upstream_grad(T, B, D, seed, scale=0.05):
    rs = np.random.RandomState(seed)
    return (rs.standard_normal((T, B, D)) * scale).astype(np.float32)


def checksum(*arrays) -> str:
    h = hashlib.sha256()

    def feed(a):
        if isinstance(a, (list, tuple)):
            for x in a:
                feed(x)
        else:
            h.update(np.ascontiguousarray(a).tobytes())

    feed(arrays)
    return h.hexdigest()[:16]


# ---------------------------------------------------------------- dense (MLP) layers
# Small DLRM-shaped MLPs for the dense-gradient fixtures: bot_l 13-32-16, top_l 24-16-1
# (the reference's ln_bot / ln_top structure, dlrm_s_pytorch_single_gpu.py create_mlp).
MLP_SHAPES = [(32, 13), (16, 32), (16, 24), (1, 16)]


def mlp_params(shapes, seed):
    """[(W [out, in], b [out])] with nn.Linear-like U(+-1/sqrt(in)) init."""
    rs = np.random.RandomState(seed)
    out = []
    for o, i in shapes:
        b = 1.0 / np.sqrt(i)
        out.append((rs.uniform(-b, b, (o, i)).astype(np.float32), rs.uniform(-b, b, o).astype(np.float32)))
    return out


def mlp_grads(shapes, seed, rank, step):
    """Per-rank synthetic dense gradients [(gW, gb)]: per-row magnitudes spread over three
    decades (so per-channel scales differ), one all-zero weight row (the 1e-8 clamp)."""
    rs = np.random.RandomState(seed + 7919 * rank + 104729 * step)
    out = []
    for k, (o, i) in enumerate(shapes):
        mag = (10.0 ** rs.uniform(-4, -1, (o, 1))).astype(np.float32)
        gW = (rs.standard_normal((o, i)) * mag).astype(np.float32)
        if k == 1:
            gW[3] = 0.0
        gb = (rs.standard_normal(o) * 10.0 ** rs.uniform(-3, -1)).astype(np.float32)
        out.append((gW, gb))
    return out


# ---------------------------------------------------------------- weight_syncc replicas
def replica_values(n, seed):
    """f32 parameter values for the identical-replica weight_syncc fixtures: significands
    uniform over all 2^23 mantissas, exponents over the f32 normal range a world of 8 can
    sum without overflow, plus zeros, subnormals and values that overflow at 3..8 ranks."""
    rs = np.random.RandomState(seed)
    mant = rs.randint(0, 1 << 23, n).astype(np.uint32)
    expo = rs.randint(1, 250, n).astype(np.uint32)  # up to 2^122
    sign = rs.randint(0, 2, n).astype(np.uint32) << 31
    x = (sign | (expo << 23) | mant).view(np.float32).copy()
    x[:8] = np.array([0.0, -0.0, 1e-45, -3e-39, 1.0, 1.5, 3.0e38, -1.2e38], np.float32)
    return x
