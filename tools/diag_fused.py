"""Per-phase wall-clock breakdown of the fused backward kernel (k_bwd_fused) on the
diagnostic build (tools/build_diag.sh -> tools/diag_build/libdqrm_clock.so).

Stamps (thread 0 of every (table, slot) workgroup, 100 MHz wall clock): 0 start, 1 keys
gathered, 6 dy prefetch issued + keys rewritten, 2 sorted, 3 heads, 4 segments done (all
stores landed), 5 end. usage: python tools/diag_fused.py [terabyte|terabyte_ref|kaggle] [B] [coalesce|sgd]
"""
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

cfg = sys.argv[1] if len(sys.argv) > 1 else "terabyte"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 2048
mode = sys.argv[3] if len(sys.argv) > 3 else "coalesce"
rows, D = CONFIGS[cfg]
T = len(rows)
lib = L.load()
lib.dqrm_diag_clock_read.argtypes = [C.c_void_p, C.c_int]
ts = dq.EmbeddingTableSet(rows, D, device="cuda", init="uniform", seed=3)
g = torch.Generator(device="cuda").manual_seed(5)
P = torch.stack([torch.randint(0, n, (B,), generator=g, device="cuda") for n in rows])
b = dq.LookupBatch.pooling_one(P)
dy = torch.randn(T, B, D, device="cuda", generator=g) * 0.05
ws = dq.CoalescedGrad.allocate(rows, B, D, "cuda")
ts.forward(b)


def run():
    if mode == "sgd":
        ts.backward_sgd(b, dy, lr=1e-4)
    else:
        ts.backward_coalesce(b, dy, ws)


for _ in range(5):
    run()
torch.cuda.synchronize()
buf = np.zeros(8192 * 16, dtype=np.uint64)
spans = []
for it in range(5):
    run()
    torch.cuda.synchronize()
    buf[:] = 0
    lib.dqrm_diag_clock_read(buf.ctypes.data, buf.size)
    c = buf[: T * 8 * 16].reshape(T, 8, 16).astype(np.int64)
    k0 = c[:, :, 0][c[:, :, 0] > 0].min()
    spans.append((c[:, :, 5].max() - k0) / 100)
print(f"{cfg} B={B} D={D} mode={mode}: kernel span (stamps) us per run: {' '.join(f'{s:.1f}' for s in spans)}")
print("per table, slowest slot (us): start | gather | prefetch+rewrite | sort | heads | segments | tail || end")
order = np.argsort(-c[:, :, 5].max(axis=1))
for t in order:
    s = int(np.argmax(c[t, :, 5]))
    p = c[t, s]
    if p[1] == 0:
        print(f"t{t:2d} n={rows[t]:>10d} slot{s}: inactive/empty  end {(p[5] - k0) / 100:6.1f}")
        continue
    marks = [p[0], p[1], p[6], p[2], p[3], p[4], p[5]]
    ph = [(marks[0] - k0)] + [marks[i + 1] - marks[i] for i in range(6)]
    print(f"t{t:2d} n={rows[t]:>10d} slot{s}: " + " ".join(f"{x / 100:6.1f}" for x in ph) +
          f" || {(p[5] - k0) / 100:6.1f}")
fr = []
for t in range(T):
    for s in range(8):
        p = c[t, s]
        if p[1] > 0 and p[5] > p[0] and p[15] > p[7]:
            fr.append((p[15] - p[7]) / ((p[5] - p[0]) / 100.0) / 1e3)
print(f"in-kernel clock (s_memtime / wall): median {np.median(fr):.2f} GHz, min {min(fr):.2f}, max {max(fr):.2f}")
idx_land = [(c[t, s, 8] - c[t, s, 0]) / 100 for t in range(T) for s in range(8) if c[t, s, 8] > 0]
print(f"idx loads landed after (us): median {np.median(idx_land):.2f} max {max(idx_land):.2f}")
print("errors", ts.read_errors())
