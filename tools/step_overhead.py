"""Host-overhead check: the bench step timed (a) plain, (b) with per-kernel events, (c) as one
captured HIP graph replay. TB config, N=1."""
import os, sys, time
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests", "golden")]
import deep_quantized_recommendation_model_dqrm_amd as dq
from deep_quantized_recommendation_model_dqrm_amd import _lib as L
import gen_inputs as G

rows = [n * 16 if n >= 1_000_000 else n for n in G.TERABYTE_ROWS]
D, B, T = 64, 2048, len(rows)
ts = dq.EmbeddingTableSet(rows, D, device="cuda", init="uniform", seed=1)
P = torch.stack([torch.randint(0, n, (B,), device="cuda") for n in rows])
b = dq.LookupBatch.pooling_one(P)
dy = torch.randn(T, B, D, device="cuda") * 0.05
y = torch.empty(T, B, D, device="cuda")
ex = dq.SparseGradExchange(ts, B, grad_bits=8)
k = ex.kernels

def step():
    ts.forward(b, bits=4, refresh_scale=True, out=y)
    k.coalesce(b, dy, ex.ws, True, "tbd")
    k.quant_pack(ex.ws, ex.ws.absmax.view(1, -1), 1, 8, ex.cap_base, ex.cap_total, ex.s_avg, ex.payload)
    k.apply(ex.cap_base, ex.cap_total, ex.payload.view(1, -1), ex.payload_bytes, 1, 8, ex.s_avg, 0.1, L.DQRM_UPD_DP, False)

def timed(fn, n=200):
    for _ in range(20): fn()
    torch.cuda.synchronize(); t = time.perf_counter()
    for _ in range(n): fn()
    torch.cuda.synchronize(); return (time.perf_counter() - t) / n * 1e6

t_plain = timed(step)
ev = [torch.cuda.Event(enable_timing=True) for _ in range(8)]
def step_ev():
    ev[0].record(); ts.forward(b, bits=4, refresh_scale=True, out=y); ev[1].record()
    ev[2].record(); k.coalesce(b, dy, ex.ws, True, "tbd"); ev[3].record()
    ev[4].record(); k.quant_pack(ex.ws, ex.ws.absmax.view(1, -1), 1, 8, ex.cap_base, ex.cap_total, ex.s_avg, ex.payload); ev[5].record()
    ev[6].record(); k.apply(ex.cap_base, ex.cap_total, ex.payload.view(1, -1), ex.payload_bytes, 1, 8, ex.s_avg, 0.1, L.DQRM_UPD_DP, False); ev[7].record()
t_ev = timed(step_ev)
# host-only cost of issuing one step (no GPU wait)
torch.cuda.synchronize(); t = time.perf_counter()
for _ in range(50): step()
t_issue = (time.perf_counter() - t) / 50 * 1e6
torch.cuda.synchronize()
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    for _ in range(3): step()
torch.cuda.current_stream().wait_stream(s)
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    step()
t_graph = timed(g.replay)
print(f"plain {t_plain:.1f} us/step | with 8 events {t_ev:.1f} | host issue {t_issue:.1f} | graph replay {t_graph:.1f}")
print("errors", ts.read_errors())
