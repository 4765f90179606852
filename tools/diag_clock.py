"""Per-phase wall-clock breakdown of the slot kernels (diagnostic build with
-DDQRM_DIAG_CLOCK: tools/diag_build/libdqrm_clock.so). For every table, the slowest slot's
phases in microseconds: start offset, gather/keys, sort, short segments, long segments,
tail (maintenance / workspace writes), end."""
import ctypes as C
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests", "golden")]
os.environ.setdefault("DQRM_LIB_PATH", os.path.join(ROOT, "tools", "diag_build", "libdqrm_clock.so"))
import deep_quantized_recommendation_model_dqrm_amd as dq  # noqa: E402
from deep_quantized_recommendation_model_dqrm_amd import _lib as L  # noqa: E402
import gen_inputs as G  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "terabyte"
D = 64 if cfg.startswith("terabyte") else 16
rows = [n * 16 if n >= 1_000_000 else n for n in G.TERABYTE_ROWS] if cfg == "terabyte" else \
    (G.TERABYTE_ROWS if cfg == "terabyte_ref" else G.KAGGLE_ROWS)
B = int(sys.argv[2]) if len(sys.argv) > 2 else 2048
T = len(rows)
lib = L.load()
lib.dqrm_diag_clock_read.argtypes = [C.c_void_p, C.c_int]
ts = dq.EmbeddingTableSet(rows, D, device="cuda", init="uniform", seed=3)
P = torch.stack([torch.randint(0, n, (B,), device="cuda") for n in rows])
b = dq.LookupBatch.pooling_one(P)
dy = torch.randn(T, B, D, device="cuda") * 0.05
ex = dq.SparseGradExchange(ts, B, grad_bits=8)
buf = np.zeros(T * 8 * 16, dtype=np.uint64)


def report(name):
    buf[:] = 0
    lib.dqrm_diag_clock_read(buf.ctypes.data, buf.size)
    c = buf.reshape(T, 8, 16).astype(np.int64)
    k0 = c[:, :, 0].min()
    print(f"== {name}: kernel span {(c[:, :, 5].max() - k0) / 100:.1f} us "
          "(per table, slowest slot: start gather sort short long tail | end)")
    order = np.argsort(-c[:, :, 5].max(axis=1))
    for t in order[:12]:
        s = int(np.argmax(c[t, :, 5]))
        p = c[t, s]
        ph = [(p[0] - k0)] + [p[i + 1] - p[i] for i in range(5)]
        print(f"t{t:2d} n={rows[t]:>10d} slot{s}: " + " ".join(f"{x / 100:6.1f}" for x in ph) +
              f" | {(p[5] - k0) / 100:6.1f}   (sort {(p[6] - p[1]) / 100:4.1f} heads {(p[2] - p[6]) / 100:4.1f})" +
              (f" long: prefix {(p[8] - p[3]) / 100:4.1f} fetch+stage {(p[9] - p[8]) / 100:4.1f} "
               f"reduce0 {(p[10] - p[9]) / 100:4.1f} rest {(p[4] - p[10]) / 100:4.1f}" if p[4] - p[3] > 200 else "") +
              (f" short: issue {(p[11] - p[2]) / 100:4.1f} land {(p[12] - p[11]) / 100:4.1f} "
               f"store {(p[13] - p[12]) / 100:4.1f} loop {(p[14] - p[13]) / 100:4.1f} drain {(p[15] - p[14]) / 100:4.1f}"
               if p[11] > p[2] > 0 else ""))


for _ in range(3):
    ts.forward(b)
    ex.step(b, dy, lr=0.1)
torch.cuda.synchronize()
ex.kernels.coalesce(b, dy, ex.ws, True, "tbd")
report("coalesce (k_table_bwd MODE 1)")
ex.kernels.quant_pack(ex.ws, ex.ws.absmax.view(1, -1), 1, 8, ex.cap_base, ex.cap_total, ex.s_avg, ex.payload)
ex.kernels.apply(ex.cap_base, ex.cap_total, ex.payload.view(1, -1), ex.payload_bytes, 1, 8, ex.s_avg, 0.1,
                 L.DQRM_UPD_DP, False)
report("apply (k_table_apply, N=1)")
ts.backward_sgd(b, dy, lr=0.1)
report("fused SGD (k_table_bwd MODE 0)")
