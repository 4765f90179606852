"""Host-side cost of the N > 1 exchange step (bench.py --force-collectives) at world size 1:
per call of the step (forward, coalesce, scale all-gather, quantize-pack, payload all-gather,
apply) the host time it takes to issue it (perf_counter, no device sync inside the step), the
whole step issued back to back (host issue rate), and the device-synchronised step time.
If the host issue time per step is close to the synchronised step time the step is host-bound.
usage: python tools/prof_exchange.py [config] [batch_per_gpu] [steps]"""
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import deep_quantized_recommendation_model_dqrm_amd as dq  # noqa: E402
from deep_quantized_recommendation_model_dqrm_amd import _lib as L  # noqa: E402
from deep_quantized_recommendation_model_dqrm_amd.workloads import CONFIGS, synthetic_indices  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "terabyte_ref"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 2048
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 200
for k, v in (("RANK", "0"), ("WORLD_SIZE", "1"), ("MASTER_ADDR", "127.0.0.1"), ("MASTER_PORT", "29517")):
    os.environ.setdefault(k, v)
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", device_id=dev)
rows, D = CONFIGS[cfg]
T = len(rows)
ts = dq.EmbeddingTableSet(rows, D, device=dev, init="uniform", seed=5)
batches = [dq.LookupBatch.pooling_one(synthetic_indices(rows, B, 11 + k, device=dev)) for k in range(8)]
dy = torch.randn(T, B, D, device=dev) * 0.05
y = torch.empty(T, B, D, device=dev)
ex = dq.SparseGradExchange(ts, B, grad_bits=8, force_collectives=True)
kern = ex.kernels
names = ["forward", "coalesce", "allgather_scales", "quant_pack", "allgather_payload", "apply"]


LIB = ex._x is not None and os.environ.get("PROF_SPLIT", "0") != "1"
if LIB:
    names = ["forward", "exchange_grad", "exchange_apply"]


def step(i, clk=None):
    b = batches[i % 8]
    t = [time.perf_counter()]
    if LIB:  # the library-issued exchange: two host calls
        ts.forward(b, bits=4, refresh_scale=True, out=y)
        t.append(time.perf_counter())
        ex.exchange(b, dy)
        t.append(time.perf_counter())
        ex.apply(0.1, mode=L.DQRM_UPD_DP)
        t.append(time.perf_counter())
        if clk is not None:
            clk.append(np.diff(t))
        return
    ts.forward(b, bits=4, refresh_scale=True, out=y)
    t.append(time.perf_counter())
    kern.coalesce(b, dy, ex.ws, True, "tbd")
    t.append(time.perf_counter())
    ex._all_gather(ex.absmax_all, ex.ws.absmax)
    t.append(time.perf_counter())
    kern.quant_pack(ex.ws, ex.absmax_all, ex.world, 8, ex.cap_base, ex.cap_total, ex.s_avg, ex.payload)
    t.append(time.perf_counter())
    ex._all_gather(ex.gathered, ex.payload)
    t.append(time.perf_counter())
    kern.apply(ex.cap_base, ex.cap_total, ex.gathered, ex.payload_bytes, ex.world, 8, ex.s_avg, 0.1, L.DQRM_UPD_DP,
               False)
    t.append(time.perf_counter())
    if clk is not None:
        clk.append(np.diff(t))


for i in range(30):
    step(i)
torch.cuda.synchronize()
# host issue cost per call: the device may fall behind, so issue in short bursts and sync
clk = []
for i in range(steps):
    step(i, clk)
    if i % 4 == 3:
        torch.cuda.synchronize()
torch.cuda.synchronize()
c = np.array(clk) * 1e6
# synchronised step time
torch.cuda.synchronize()
t0 = time.perf_counter()
for i in range(steps):
    step(i)
torch.cuda.synchronize()
wall = (time.perf_counter() - t0) / steps * 1e6
# host issue rate with the device never waited on (bounded by the device when it is slower)
per = {n: (round(float(np.median(c[:, j])), 2), round(float(np.mean(c[:, j])), 2)) for j, n in enumerate(names)}
print({"config": cfg, "batch_per_gpu": B, "library_exchange": LIB, "host_us_median_mean": per,
       "host_issue_us_per_step_median": round(float(np.median(c.sum(1))), 2),
       "synced_us_per_step": round(wall, 2)})
dist.destroy_process_group()
