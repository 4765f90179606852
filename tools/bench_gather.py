"""Sweep the fused forward (INT4 packed and FP32 fake-quant paths): GB/s on algorithmic bytes."""
import sys, os, json
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests", "golden")]
import deep_quantized_recommendation_model_dqrm_amd as dq
import gen_inputs as G

def timeit(fn, reps=30):
    for _ in range(5): fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps): fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3

cfg = sys.argv[1] if len(sys.argv) > 1 else "tbref"
rows = {"tbref": G.TERABYTE_ROWS, "tb16": [n * 16 if n >= 10**6 else n for n in G.TERABYTE_ROWS], "kaggle": G.KAGGLE_ROWS}[cfg]
D = 16 if cfg == "kaggle" else 64
ts = dq.EmbeddingTableSet(rows, D, device="cuda", packed=True, seed=3)
ts.refresh_scale_and_pack(4)
T = len(rows)
for dist_kind in ("uniform", "zipf"):
    for B in (2048, 16384, 65536, 262144):
        g = torch.Generator(device="cuda").manual_seed(B)
        if dist_kind == "uniform":
            P = torch.stack([torch.randint(0, n, (B,), generator=g, device="cuda") for n in rows])
        else:
            P = torch.stack([(torch.floor(torch.exp(torch.rand(B, generator=g, device="cuda", dtype=torch.float64)
                                                     * torch.log(torch.tensor(float(n))))) - 1).clamp_(0, n - 1).long()
                             for n in rows])
        b = dq.LookupBatch.pooling_one(P)
        y = torch.empty(T, B, D, device="cuda")
        tp = timeit(lambda: ts.forward(b, refresh_scale=False, use_packed=True, out=y))
        tpn = timeit(lambda: ts.forward(b, refresh_scale=False, use_packed=True, out=y, nt_store=True))
        tf = timeit(lambda: ts.forward(b, refresh_scale=True, out=y))
        bp = T * B * (D // 2 + 16 + D * 4)
        bf = T * B * (D * 4 + 16 + D * 4)
        print(json.dumps({"cfg": cfg, "dist": dist_kind, "B": B, "int4_us": round(tp, 1), "int4_GBps": round(bp / tp / 1e3, 1),
                          "int4_frac": round(bp / tp / 1e3 / 8000, 3), "int4nt_GBps": round(bp / tpn / 1e3, 1), "fp32_us": round(tf, 1),
                          "fp32_GBps": round(bf / tf / 1e3, 1)}), flush=True)
