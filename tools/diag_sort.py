"""Per-phase wall-clock breakdown of K4a (k_sort_slots) on the diagnostic build
(tools/build_diag.sh -> tools/diag_build/libdqrm_clock.so): for every table, its slowest
slot's stamps in microseconds from the kernel's first stamp: start, keys gathered, sorted,
heads + record run reserved, records written, end.
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
rows, D = CONFIGS[cfg]
T, S = len(rows), L.DQRM_TABLE_SPLIT
lib = L.load()
lib.dqrm_diag_clock_read.argtypes = [C.c_void_p, C.c_int]
lib.dqrm_diag_clock_read.restype = C.c_int
ts = dq.EmbeddingTableSet(rows, D, device="cuda", init="uniform", seed=3)
P = torch.stack([torch.randint(0, n, (B,), device="cuda") for n in rows])
b = dq.LookupBatch.pooling_one(P)
dy = torch.randn(T, B, D, device="cuda") * 0.05
ws = dq.CoalescedGrad.allocate(rows, B, D, "cuda")
for _ in range(5):
    ts.backward_coalesce(b, dy, ws)
torch.cuda.synchronize()
buf = np.zeros(T * S * 16, dtype=np.uint64)
lib.dqrm_diag_clock_read(buf.ctypes.data, buf.size)
c = buf.reshape(T, S, 16).astype(np.int64)
k0 = c[:, :, 0][c[:, :, 0] > 0].min()
end = c[:, :, 5]
print(f"{cfg} B={B}: K4a span {(end.max() - k0) / 100:.1f} us; per table, slowest slot (us from kernel start)")
names = ["start", "keys", "sorted", "heads", "records", "end"]
print("  t       rows slot " + " ".join(f"{n:>8s}" for n in names))
for t in np.argsort(-end.max(axis=1)):
    s = int(np.argmax(end[t]))
    print(f"{t:3d} {rows[t]:>10d}   {s}  " + " ".join(
        f"{(c[t, s, q] - k0) / 100:8.1f}" if c[t, s, q] > 0 else "       -" for q in range(6)))
