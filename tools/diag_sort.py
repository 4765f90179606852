"""Per-phase wall-clock breakdown of the fused backward kernel (k_bwd_fused) on the
diagnostic build (tools/build_diag.sh -> tools/diag_build/libdqrm_clock.so): for every
table, its slowest slot's stamps in microseconds from the kernel's first stamp: start,
keys gathered, sorted, heads (+ prefetched rows in LDS), segments written, end.
usage: python tools/diag_sort.py [terabyte_ref|kaggle|terabyte] [B]"""
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
from deep_quantized_recommendation_model_dqrm_amd.workloads import CONFIGS  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "terabyte_ref"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 2048
mode = sys.argv[3] if len(sys.argv) > 3 else "coalesce"
rows, D = CONFIGS[cfg]
T, S = len(rows), L.DQRM_TABLE_SPLIT
lib = L.load()
lib.dqrm_diag_clock_read.argtypes = [C.c_void_p, C.c_int]
lib.dqrm_diag_clock_read.restype = C.c_int
ts = dq.EmbeddingTableSet(rows, D, device="cuda", init="uniform", seed=1)
g = torch.Generator(device="cuda").manual_seed(5)  # the batch tools/bwd_probe.py times
P = torch.stack([torch.randint(0, n, (B,), generator=g, device="cuda") for n in rows])
b = dq.LookupBatch.pooling_one(P)
dy = torch.randn(T, B, D, device="cuda", generator=g) * 0.05
ws = dq.CoalescedGrad.allocate(rows, B, D, "cuda")
for _ in range(5):
    if mode == "sgd":
        ts.backward_sgd(b, dy, lr=1e-4)
    else:
        ts.backward_coalesce(b, dy, ws)
torch.cuda.synchronize()
buf = np.zeros(T * S * 16, dtype=np.uint64)
lib.dqrm_diag_clock_read(buf.ctypes.data, buf.size)
c = buf.reshape(T, S, 16).astype(np.int64)
k0 = c[:, :, 0][c[:, :, 0] > 0].min()
end = c[:, :, 5]
print(f"{cfg} B={B} {mode}: kernel span {(end.max() - k0) / 100:.1f} us; per table, slowest slot (us from kernel start)")
names = ["start", "keys", "presort", "sorted", "heads", "segments", "end"]
order = [0, 1, 6, 2, 3, 4, 5]
print(f"{mode}:  t       rows slot " + " ".join(f"{n:>8s}" for n in names))
for t in np.argsort(-end.max(axis=1)):
    s = int(np.argmax(end[t]))
    print(f"{t:3d} {rows[t]:>10d}   {s}  " + " ".join(
        f"{(c[t, s, q] - k0) / 100:8.1f}" if c[t, s, q] > 0 else "       -" for q in order))

# thread 0's segment batches (stamps 7..14) of the slowest slot
t = int(np.argmax(end.max(axis=1)))
sl = int(np.argmax(end[t]))
print(f"t{t} slot{sl} staged chunk stamps (fetched, walked)...:", " ".join(f"{(c[t, sl, q] - k0) / 100:.1f}" for q in range(7, 16) if c[t, sl, q] > 0))
