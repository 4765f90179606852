"""Diagnostic: per-kernel time of the backward/exchange kernels on subsets of the tables."""
import sys, os, json
import numpy as np, torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests", "golden")]
import deep_quantized_recommendation_model_dqrm_amd as dq
import gen_inputs as G

def timeit(fn, reps=20):
    for _ in range(3): fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps): fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3  # us

D = int(sys.argv[1]) if len(sys.argv) > 1 else 64
B = int(sys.argv[2]) if len(sys.argv) > 2 else 2048
tb = G.TERABYTE_ROWS
subsets = {"all": tb, "big(>=1e4)": [n for n in tb if n >= 10000], "mid(1e3..1e4)": [n for n in tb if 1000 <= n < 10000],
           "small(<1e3)": [n for n in tb if n < 1000], "n=3": [3], "n=62": [62], "n=971": [971], "n=9.9M": [9980200]}
res = {}
for name, rows in subsets.items():
    ts = dq.EmbeddingTableSet(rows, D, device="cuda", seed=1)
    P = torch.from_numpy(G.pooling_one(rows, B, 5)).cuda()
    b = dq.LookupBatch.pooling_one(P)
    dy = torch.randn(len(rows), B, D, device="cuda") * 0.05
    ex = dq.SparseGradExchange(ts, B, grad_bits=8)
    ts.forward(b)
    r = {}
    r["fwd"] = timeit(lambda: ts.forward(b))
    r["coalesce"] = timeit(lambda: ex.kernels.coalesce(b, dy, ex.ws, True, "tbd"))
    r["step"] = timeit(lambda: ex.step(b, dy, 0.1))
    r["sgd"] = timeit(lambda: ts.backward_sgd(b, dy, 0.1))
    res[name] = {k: round(v, 1) for k, v in r.items()}
    print(name, len(rows), res[name], flush=True)
