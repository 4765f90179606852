"""Time the coalesce kernel of diagnostic builds (DQRM_LIB_PATH) on table subsets."""
import sys, os
import torch
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
    return e0.elapsed_time(e1) / reps * 1e3
D, B = 64, 2048
for name, rows in {"n=3": [3], "n=62": [62], "n=9.9M": [9980200]}.items():
    ts = dq.EmbeddingTableSet(rows, D, device="cuda", seed=1)
    b = dq.LookupBatch.pooling_one(torch.from_numpy(G.pooling_one(rows, B, 5)).cuda())
    dy = torch.randn(len(rows), B, D, device="cuda") * 0.05
    ex = dq.SparseGradExchange(ts, B, grad_bits=8)
    print(os.environ.get("DQRM_LIB_PATH", "full"), name, round(timeit(lambda: ex.kernels.coalesce(b, dy, ex.ws, True, "tbd")), 1), flush=True)
