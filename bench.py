#!/usr/bin/env python3
"""Benchmark: DQRM data-parallel QAT embedding step on MI355X (1..8 GPUs, one process each).

A step = one pass of the hot path over one synthetic batch per rank:
  forward   26-table fake-quant EmbeddingBag (exact per-step table scale, FP32-row gather)
  backward  STE + sparse backward + coalesce + local INT8 grad scale        (K4)
  comm      RCCL all-gather of the [T] scales, quantize-pack to INT8       (K5)
            RCCL all-gather of the fixed-capacity {rows, int8} payloads
  update    decode all ranks' payloads, integer union-sum, dequant, SGD    (K6)
At N=1 there is nothing to exchange: K5 + K6 run as one fused kernel (dqrm_apply_local:
the same quantize, dequantize and SGD arithmetic, bit-identical W; --unfused-local runs the
payload round trip instead).
The MLP/interaction layers are outside the north-star path and are not run;
the upstream gradient dL/dy is a fixed synthetic tensor.

Prints ONE JSON line (rank 0). N=1 by default; N>1 is launched by torch.distributed.run.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))

import deep_quantized_recommendation_model_dqrm_amd as dq  # noqa: E402
from deep_quantized_recommendation_model_dqrm_amd import _lib as L  # noqa: E402
import gen_inputs as G  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)

CONFIGS = {
    # BASELINE.json configs[4]: Criteo-Terabyte shape, D=64, ~773M rows: the reference TB
    # profile (--max-ind-range=10M) with its six >=1M-row tables scaled x16
    "terabyte": dict(rows=[n * 16 if n >= 1_000_000 else n for n in G.TERABYTE_ROWS], dim=64),
    # the reference's actual TB run (49.1M rows)
    "terabyte_ref": dict(rows=G.TERABYTE_ROWS, dim=64),
    # BASELINE.json configs[2-3]: Criteo-Kaggle, D=16
    "kaggle": dict(rows=G.KAGGLE_ROWS, dim=16),
}
# the reference scripts' MLPs (bash_scripts/): Kaggle --arch-mlp-bot=13-512-256-64-16
# --arch-mlp-top=512-256-1; Terabyte 13-512-256-64 / 512-512-256-1; the top MLP's input is
# D + T(T+1)/2 (dot interaction of T+1 vectors, dlrm_s_pytorch_single_gpu.py create_mlp)
MLPS = {
    "terabyte": ([13, 512, 256, 64], [64 + 351, 512, 512, 256, 1]),
    "terabyte_ref": ([13, 512, 256, 64], [64 + 351, 512, 512, 256, 1]),
    "kaggle": ([13, 512, 256, 64, 16], [16 + 351, 512, 256, 1]),
}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=100)
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--config", default="terabyte", choices=sorted(CONFIGS))
    p.add_argument("--batch-per-gpu", type=int, default=2048,
                   help="samples per rank per step (reference TB mini-batch 2048)")
    p.add_argument("--grad-bits", type=int, default=8)
    p.add_argument("--lr", type=float, default=0.1)
    p.add_argument("--index-dist", default="uniform", choices=["uniform", "zipf"])
    p.add_argument("--num-batches", type=int, default=8, help="distinct resident batches cycled")
    p.add_argument("--gather-batch", type=int, default=65536,
                   help="bags per table for the INT4 packed-gather bandwidth phase (0 = skip)")
    p.add_argument("--gather-iters", type=int, default=50)
    p.add_argument("--mlp-iters", type=int, default=50,
                   help="iterations of the MLP INT8 gradient exchange phase (0 = skip)")
    p.add_argument("--cpu-baseline", type=int, default=1)
    p.add_argument("--seed", type=int, default=123)
    p.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                   help="nccl (= RCCL on ROCm) for measurements; gloo only to rehearse N>1 on one GPU")
    p.add_argument("--unfused-local", action="store_true",
                   help="N=1: run quant-pack + payload apply instead of the fused dqrm_apply_local")
    p.add_argument("--sample-every", type=int, default=8,
                   help="bracket the dominant kernel with HIP events on every k-th timed step")
    p.add_argument("--traffic-profile", default=None,
                   help="rocprofv3 PMC summary (tools/prof_summary.py) for roofline.traffic; "
                        "default profiles/r1_<config>_summary.json when present")
    return p.parse_args()


PROFILE_TAG = {"terabyte": "tb", "terabyte_ref": "tbref", "kaggle": "kaggle"}
KERNEL_SYMBOL = {  # bench phase -> libdqrm kernel (as named in the rocprofv3 summary)
    "emb_fwd": "k_emb_fwd<{lpr},",
    "bwd_coalesce": "k_table_bwd<{lpr}, 1>",
    "grad_quant_pack": "k_quant_pack<{lpr}>",
    "apply_sparse_update": "k_apply_flat<{lpr}>",
    "apply_local": "k_apply_local<{lpr}>",
}


def pmc_traffic(path, phase, D):
    """HBM bytes per launch of the phase's kernel from a committed rocprofv3 PMC summary
    (2 x FETCH_SIZE + WRITE_SIZE, MI355X_MICROARCH.md HBM section), or None."""
    if not path or not os.path.exists(path):
        return None
    prefix = KERNEL_SYMBOL[phase].format(lpr=D // 4)
    for name, v in json.load(open(path))["kernels"].items():
        if name.startswith(prefix) and v.get("hbm_bytes_per_launch") is not None:
            return {"bytes": round(v["hbm_bytes_per_launch"]), "profiled_avg_us": round(v["avg_us"], 2),
                    "source": os.path.relpath(path, ROOT)}
    return None


def make_batches(rows, B_global, rank, world, count, seed, dist_kind, device):
    """Global Criteo-form batches [T, B_global] generated identically on every rank, each
    rank keeping its contiguous slice (get_my_slice, dlrm_s_pytorch_single_gpu.py:989-993)."""
    g = torch.Generator(device=device)
    out = []
    sl = dq.get_my_slice(B_global, world, rank)
    for k in range(count):
        g.manual_seed(seed * 1000 + k)
        cols = []
        for n in rows:
            if dist_kind == "uniform":
                cols.append(torch.randint(0, n, (B_global,), generator=g, device=device, dtype=torch.int64))
            else:  # Zipf(1.05)-like power law via inverse transform on a log scale
                u = torch.rand(B_global, generator=g, device=device, dtype=torch.float64)
                z = torch.floor(torch.exp(u * np.log(float(n)))) - 1
                cols.append(z.clamp_(0, n - 1).to(torch.int64))
        P = torch.stack(cols)[:, sl].contiguous()
        out.append(dq.LookupBatch.pooling_one(P))
    return out


def timed_events(n):
    return [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        if world == 1 and a.gpus > 1:
            print("N>1 must be launched with torch.distributed.run", file=sys.stderr)
            sys.exit(2)
    ndev = torch.cuda.device_count()
    local = local % max(ndev, 1)  # gloo rehearsal: ranks may share a GPU
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if a.dist_backend == "nccl":  # RCCL over xGMI, one process per GPU
            dist.init_process_group("nccl", device_id=dev)
        else:  # gloo: functional rehearsal of the N>1 path (e.g. several ranks on one GPU)
            dist.init_process_group("gloo")
    cfg = CONFIGS[a.config]
    rows, D, B = cfg["rows"], cfg["dim"], a.batch_per_gpu
    T = len(rows)

    t0 = time.time()
    ts = dq.EmbeddingTableSet(rows, D, device=dev, packed=a.gather_batch > 0, init="uniform", seed=a.seed)
    batches = make_batches(rows, B * world, rank, world, a.num_batches, a.seed, a.index_dist, dev)
    dy = torch.randn(T, B, D, device=dev, generator=torch.Generator(device=dev).manual_seed(a.seed + rank)) * 0.05
    y = torch.empty(T, B, D, device=dev)
    ex = dq.SparseGradExchange(ts, B, grad_bits=a.grad_bits)
    kern = ex.kernels
    torch.cuda.synchronize()
    setup_s = time.time() - t0

    # N=1: quantize-pack + apply fused (dqrm_apply_local; same quantize/dequantize/SGD
    # arithmetic, bit-identical W, no payload since nothing is exchanged)
    fused = world == 1 and not a.unfused_local
    names = (["emb_fwd", "bwd_coalesce", "apply_local"] if fused
             else ["emb_fwd", "bwd_coalesce", "grad_quant_pack", "apply_sparse_update"])

    def step(i, ev=None, only=None):
        """One QAT step. ev: per-phase (start, end) events; only: bracket just that phase."""
        b = batches[i % len(batches)]

        def mark(j, k):
            if ev is not None and (only is None or only == j):
                ev[j][k].record()

        mark(0, 0)
        ts.forward(b, bits=4, refresh_scale=True, out=y)
        mark(0, 1)
        mark(1, 0)
        kern.coalesce(b, dy, ex.ws, True, "tbd")
        mark(1, 1)
        if fused:
            mark(2, 0)
            kern.apply_local(ex.ws, a.grad_bits, ex.s_avg, a.lr, False)
            mark(2, 1)
            return
        if ex.world == 1:
            absmax_all = ex.ws.absmax.view(1, -1)
        else:
            ex._all_gather(ex.absmax_all, ex.ws.absmax)
            absmax_all = ex.absmax_all
        mark(2, 0)
        kern.quant_pack(ex.ws, absmax_all, ex.world, a.grad_bits, ex.cap_base, ex.cap_total, ex.s_avg, ex.payload)
        mark(2, 1)
        if ex.world == 1:
            gathered = ex.payload.view(1, -1)
        else:
            ex._all_gather(ex.gathered, ex.payload)
            gathered = ex.gathered
        mark(3, 0)
        kern.apply(ex.cap_base, ex.cap_total, gathered, ex.payload_bytes, ex.world, a.grad_bits, ex.s_avg, a.lr,
                   L.DQRM_UPD_DP, False)
        mark(3, 1)

    for i in range(a.warmup):
        step(i)
    # per-phase breakdown (untimed): every kernel bracketed by events; picks the dominant one
    nb = max(10, min(50, a.steps))
    bev = [timed_events(len(names)) for _ in range(nb)]
    for i in range(nb):
        step(i, bev[i])
    torch.cuda.synchronize()
    kms = {n: float(np.mean([bev[i][j][0].elapsed_time(bev[i][j][1]) for i in range(nb)])) for j, n in enumerate(names)}
    dom = max(kms, key=kms.get)
    dj = names.index(dom)
    # timed region: plain steps; the dominant kernel is bracketed by HIP events (on the stream
    # it runs on) on every sample_every-th step, so the events barely perturb the timing
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    evs = [timed_events(len(names)) for _ in range(a.steps)]
    sampled = [i for i in range(a.steps) if i % a.sample_every == 0]
    t_start = time.perf_counter()
    for i in range(a.steps):
        step(a.warmup + i, evs[i] if i % a.sample_every == 0 else None, only=dj)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t_start
    if world > 1:
        e = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())
    dom_ms = float(np.mean([evs[i][dj][0].elapsed_time(evs[i][dj][1]) for i in sampled]))

    # algorithmic bytes per launch; unique counts from the last step
    U = int(ex.ws.ucount.sum().item())
    L_tot = T * B
    alg = {
        "emb_fwd": L_tot * (D * 4 + 8) + T * B * 8 + T * B * D * 4 + T * 4,
        "bwd_coalesce": L_tot * 8 + T * B * 8 + L_tot * D * 4 + U * (D * 4 + 4),
        "grad_quant_pack": U * (D * 4 + 4) + U * (D + 4),
        "apply_sparse_update": world * U * (D + 4) + U * D * 8 + U * 4,
        "apply_local": U * (D * 4 + 4) + U * D * 8 + U * 4,
    }
    achieved = alg[dom] / (dom_ms * 1e-3) / 1e9
    err = ts.read_errors()

    # INT4 packed-gather bandwidth phase (north-star gather metric), outside the timed step
    gather = None
    if a.gather_batch > 0:
        ts.refresh_scale_and_pack(4)
        Bg = a.gather_batch
        gb = make_batches(rows, Bg, 0, 1, 2, a.seed + 7, a.index_dist, dev)
        yg = torch.empty(T, Bg, D, device=dev)
        for i in range(5):
            ts.forward(gb[i % 2], refresh_scale=False, use_packed=True, out=yg)
        gev = timed_events(a.gather_iters)
        for i in range(a.gather_iters):
            gev[i][0].record()
            ts.forward(gb[i % 2], refresh_scale=False, use_packed=True, out=yg)
            gev[i][1].record()
        torch.cuda.synchronize()
        g_ms = float(np.mean([e0.elapsed_time(e1) for e0, e1 in gev]))
        g_bytes = T * Bg * (D // 2 + 8 + 8 + D * 4) + T * 4
        g_gbs = g_bytes / (g_ms * 1e-3) / 1e9
        gather = {"kernel": "k_emb_fwd (INT4 packed, pooling 1)", "bags_per_table": Bg, "ms": round(g_ms, 4),
                  "alg_bytes": g_bytes, "GBps": round(g_gbs, 1), "frac_of_peak": round(g_gbs / HBM_PEAK_GBS, 4),
                  "bytes_per_lookup": D // 2 + 8 + 8 + D * 4}
        del yg, gb

    mlp = dense_phase(a, dev, world, rank) if a.mlp_iters > 0 else None

    cpu = None  # the CPU baseline is an N=1 figure: rank 0 of a single-rank run only
    if world == 1 and a.cpu_baseline:
        cpu = cpu_baseline(rows, D, min(B, 2048), a.seed)

    # replicas must stay bit-identical (deterministic kernels, same exchanged data): compare a
    # checksum of every rank's W bit patterns and table maxima (outside the timed region)
    wbits = ts.W.view(-1).view(torch.int32)
    wsum = sum(c.sum(dtype=torch.int64) for c in wbits.split(1 << 26))  # 512 MB int64 temporaries
    cs = torch.stack([wsum, ts.tmax.view(torch.int32).sum(dtype=torch.int64)])
    if world > 1:
        allcs = [torch.zeros_like(cs) for _ in range(world)]
        dist.all_gather(allcs, cs)
        replicas_match = all(torch.equal(allcs[0], c) for c in allcs)
    else:
        replicas_match = True
    prof = a.traffic_profile or os.path.join(ROOT, "profiles", f"r1_{PROFILE_TAG[a.config]}_summary.json")
    traffic = pmc_traffic(prof, dom, D)
    if rank == 0:
        value = world * B * a.steps / elapsed
        line = {
            "metric": "QAT-step samples/sec (DP embedding QAT step: INT4 fake-quant gather + sparse SGD + INT8 sparse-grad all-reduce)",
            "value": round(value, 1),
            "unit": "samples/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(elapsed / a.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32 (int4 fake-quant activations, int8 gradients)",
            "data": "synthetic (uniform-random Criteo-form indices, U(+-sqrt(1/n)) tables, N(0,0.05) dL/dy)"
            if a.index_dist == "uniform" else "synthetic (power-law indices)",
            "config": {
                "workload": f"criteo-{a.config} embedding QAT step",
                "tables": T, "total_rows": sum(rows), "emb_dim": D,
                "batch_per_gpu": B, "global_batch": B * world, "pooling": 1,
                "grad_bits": a.grad_bits, "scale_period": 1, "parallelism": f"dp{world} (tables replicated)",
            },
            "roofline": {"kernel": dom, "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic["bytes"] if traffic else None, "traffic_unit": "bytes/launch",
                         "traffic_src": traffic,
                         "alg_bytes_per_launch": alg[dom], "avg_launch_ms": round(dom_ms, 5),
                         "timed_launches": len(sampled)},
            "kernels_ms": {k: round(v, 5) for k, v in kms.items()},
            "kernels_ms_note": "untimed breakdown pass, every kernel bracketed by events",
            "int4_gather": gather,
            "mlp_grad_exchange": mlp,
            "cpu_baseline": cpu,
            "device_errors": err,
            "replicas_bit_identical": replicas_match,
            "setup_s": round(setup_s, 1),
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def dense_phase(a, dev, world, rank):
    """MLP half of the DP step, outside the timed embedding step:
    per-channel INT8 quantize of every bot_l/top_l gradient, scale all-gather, fp16-wire
    all-reduce (RCCL at N>1), decode, SGD update -- DenseGradExchange.exchange + apply.
    Algorithmic bytes per step (P params, w wire bytes/elem): 4P (scale) + 4P + wP (quant)
    + wP + 4P (decode) + 12P (update)."""
    from deep_quantized_recommendation_model_dqrm_amd.dense import DenseGradExchange

    bot, top = MLPS[a.config]
    g = torch.Generator(device=dev).manual_seed(a.seed + 101 * rank)
    layers = []
    for dims in (bot, top):
        for i, o in zip(dims[:-1], dims[1:]):
            l = torch.nn.Linear(i, o).to(dev)
            l.weight.grad = torch.randn(o, i, device=dev, generator=g) * 1e-3
            l.bias.grad = torch.randn(o, device=dev, generator=g) * 1e-3
            layers.append(l)
    ex = DenseGradExchange(layers, grad_bits=8)
    P = ex.channels.total_elems
    wire_b = ex.wire.element_size()
    with torch.no_grad():
        for _ in range(5):
            ex.exchange()
            ex.apply(1e-6)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        ev = timed_events(a.mlp_iters)
        for i in range(a.mlp_iters):
            ev[i][0].record()
            ex.exchange()
            ex.apply(1e-6)
            ev[i][1].record()
        torch.cuda.synchronize()
    ms = float(np.median([e0.elapsed_time(e1) for e0, e1 in ev]))
    # scale: read g; quant: read g, write wire; decode: read wire, write g; update: read g, p, write p
    alg = P * 4 + (P * 4 + P * wire_b) + (P * wire_b + P * 4) + 3 * P * 4
    return {"layers": f"bot {'-'.join(map(str, bot))}, top {'-'.join(map(str, top))}", "params": P,
            "channels": ex.channels.num_channels, "wire": str(ex.wire.dtype).replace("torch.", ""),
            "wire_bytes_per_rank": P * wire_b, "ms": round(ms, 4), "alg_bytes": alg,
            "GBps": round(alg / (ms * 1e-3) / 1e9, 1), "launches": 4, "collectives": 2 if world > 1 else 0,
            "note": "median of per-iteration HIP events; exchange+apply of all layers"}


def cpu_baseline(rows, D, B, seed):
    """The oracle (C restatement of the reference path, single thread) on a bounded sample:
    tables capped at 1M rows (host RAM), a few full QAT steps incl. the reference's per-step
    full-table |W| scan. kind = "port" (the reference itself cannot run here)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O

    O.build()
    cap_rows = [min(n, 1_000_000) for n in rows]
    rs = np.random.RandomState(seed)
    Ws = [rs.uniform(-np.sqrt(1 / n), np.sqrt(1 / n), (n, D)).astype(np.float32) for n in cap_rows]
    T = len(rows)
    t0 = time.perf_counter()
    steps = 0
    while True:
        P = np.stack([rs.randint(0, n, B) for n in cap_rows]).astype(np.int64)
        dyc = (rs.standard_normal((T, B, D)) * 0.05).astype(np.float32)
        s_fwd = []
        for t in range(T):
            s = O.table_scale(Ws[t], 4)
            O.emb_fwd(Ws[t], P[t], np.arange(B), s)
            s_fwd.append(s)
        O.dp_step(Ws, [[(P[t], np.arange(B)) for t in range(T)]], [[dyc[t] for t in range(T)]], s_fwd, 0.1, 8)
        steps += 1
        el = time.perf_counter() - t0
        if el > 10.0 or steps >= 50:
            break
    return {"value": round(steps * B / el, 1), "unit": "samples/s", "cores": 1, "kind": "port",
            "sample": f"{steps} QAT steps, B={B}, {T} tables capped at 1M rows (D={D}), oracle C restatement, 1 thread"}


if __name__ == "__main__":
    main()
