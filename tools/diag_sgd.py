"""Per-phase wall-clock breakdown of the small-batch SGD kernel k_sgd_small (BASELINE
config 3: Kaggle, B = 128) on the diagnostic build (tools/build_diag.sh). Stamps: 0 start,
1 indices landed, 2 dy staged (barrier), 3 duplicate scan done, 4 rows updated (barrier),
6 shrunk blocks re-reduced, 5 end.
usage: python tools/diag_sgd.py [B]"""
import ctypes as C
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("DQRM_LIB_PATH", os.path.join(ROOT, "tools", "diag_build", "libdqrm_clock.so"))
import deep_quantized_recommendation_model_dqrm_amd as dq  # noqa: E402
from deep_quantized_recommendation_model_dqrm_amd import _lib as L  # noqa: E402
from deep_quantized_recommendation_model_dqrm_amd.workloads import CONFIGS, synthetic_indices  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 128
rows, D = CONFIGS["kaggle"]
T = len(rows)
lib = L.load()
lib.dqrm_diag_clock_read.argtypes = [C.c_void_p, C.c_int]
ts = dq.EmbeddingTableSet(rows, D, device="cuda", init="uniform", seed=3)
batches = [dq.LookupBatch.pooling_one(synthetic_indices(rows, B, 11 + k)) for k in range(8)]
dy = torch.randn(T, B, D, device="cuda", generator=torch.Generator(device="cuda").manual_seed(5)) * 0.05
for i in range(40):
    ts.forward(batches[i % 8])
    ts.backward_sgd(batches[i % 8], dy, 0.1)
torch.cuda.synchronize()
acc = []
for i in range(16):
    ts.forward(batches[i % 8])
    ts.backward_sgd(batches[i % 8], dy, 0.1)
    torch.cuda.synchronize()
    buf = np.zeros(T * 16, dtype=np.uint64)
    lib.dqrm_diag_clock_read(buf.ctypes.data, buf.size)
    acc.append(buf.reshape(T, 16).astype(np.int64).copy())
c = np.stack(acc)  # [it, T, 16]
k0 = c[:, :, 0].min(axis=1, keepdims=True)
end = (c[:, :, 5] - k0) / 100
print(f"kaggle B={B}: span per launch (us) median {np.median(end.max(axis=1)):.1f}, max {end.max():.1f}")
print("per table, median over launches (us): start | idx | staged | scan | updated | rereduce | end || end")
for t in np.argsort(-np.median(end, axis=0)):
    p = c[:, t] - k0[:, 0:1]
    ph = [np.median(p[:, 0])] + [np.median(p[:, j] - p[:, i]) for i, j in ((0, 1), (1, 2), (2, 3), (3, 4))]
    v6 = (p[:, 6] > p[:, 4]) & (p[:, 6] <= p[:, 5])  # stamped in this launch (a block re-reduced)
    rr = np.median(np.where(v6, p[:, 6] - p[:, 4], 0))
    tail = np.median(p[:, 5] - np.where(v6, p[:, 6], p[:, 4]))
    print(f"t{t:2d} n={rows[t]:>9d}: " + " ".join(f"{x / 100:5.1f}" for x in ph) + f" {rr / 100:5.1f} {tail / 100:5.1f}"
          f" || {np.median(end[:, t]):5.1f}")
v6all = (c[:, :, 6] > c[:, :, 4]) & (c[:, :, 6] <= c[:, :, 5])
print(f"launches x tables with a shrunk block re-reduced: {v6all.mean():.2f}")
print("errors", ts.read_errors())
