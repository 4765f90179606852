#!/usr/bin/env python3
"""Benchmark: DQRM's QAT embedding step on MI355X (1..8 GPUs, one process each).

--mode dp  (default; BASELINE configs 4-5) one data-parallel QAT step per rank:
  forward   26-table fake-quant EmbeddingBag (exact per-step table scale, FP32-row gather;
            with --scale-period P --use-packed: INT4 rows between the periodic scale refreshes)
  backward  STE + sparse backward + coalesce + local INT8 grad scale        (k_bwd_fused)
  comm      RCCL all-gather of the per-slot max|grad|, quantize-pack to INT8, RCCL
            all-gather of the fixed-capacity {rows, int8} payloads
  update    decode all ranks' payloads, integer union-sum, dequant, SGD (+ INT4 repack)
  At N=1 there is nothing to exchange: backward + quantize + update run as ONE launch
  (dqrm_emb_bwd_apply_local; bit-identical W): --two-launch-local times the coalesce +
  dqrm_apply_local pair, --unfused-local the payload round trip.
--mode fwd (BASELINE config 2) the forward alone.
--mode sgd (BASELINE config 3) forward + fused STE/sparse-backward/SGD (dqrm_emb_bwd_sgd).
--graph captures one step per resident batch in a HIP graph (torch.cuda.CUDAGraph) and
replays it, taking the host launch path out of the timed region (the B=128 configs are
launch-bound).

The MLP/interaction layers are outside the north-star path and are not run;
the upstream gradient dL/dy is a fixed synthetic tensor. The MLP's INT8 gradient exchange
(8(f) #1) is timed in its own phase, outside the step.

Prints ONE JSON line (rank 0). N=1 by default; N>1 is launched by torch.distributed.run.
A run whose kernels raised device error flags prints value null and exits with status 3.
"""
from __future__ import annotations

import argparse
import json
import os
import re
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import deep_quantized_recommendation_model_dqrm_amd as dq  # noqa: E402
from deep_quantized_recommendation_model_dqrm_amd import _lib as L  # noqa: E402
from deep_quantized_recommendation_model_dqrm_amd.workloads import (  # noqa: E402
    CONFIGS as _CONFIGS, MLPS, synthetic_indices)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
CONFIGS = {k: dict(rows=r, dim=d) for k, (r, d) in _CONFIGS.items()}
# host tables of the PyTorch-CPU baseline: the reference's own TB run stands in for the
# 773 M-row profile (its 198 GB of FP32 rows exceed one bench run's host-memory budget)
CPU_TABLES = {"terabyte": "terabyte_ref", "terabyte_ref": "terabyte_ref", "terabyte_1g": "terabyte_1g",
              "kaggle": "kaggle"}


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=100)
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--config", default="terabyte", choices=sorted(CONFIGS))
    p.add_argument("--mode", default="dp", choices=["dp", "fwd", "sgd", "dropin-sgd", "dropin-dp", "dlrm"],
                   help="dp: data-parallel QAT step; fwd: forward only; sgd: forward + fused sparse SGD; "
                        "dropin-sgd / dropin-dp: the reference drivers' call pattern through the drop-in "
                        "modules and hooks (see dropin_main); dlrm: the whole single-GPU DLRM QAT step "
                        "(MLPs, interaction, BCE, backward, SGD; see dlrm_main)")
    p.add_argument("--dropin-form", default="list", choices=["list", "collection"],
                   help="drop-in / dlrm modes: the unchanged drivers' ModuleList of per-table "
                        "QuantEmbeddingBagTwo, or one QuantEmbeddingBagCollection replacing apply_emb's loop")
    p.add_argument("--grad-mode", default="sparse", choices=["sparse", "fused_sgd"],
                   help="dropin-sgd: module grad_mode (sparse = torch.optim.SGD on the per-lookup COO)")
    p.add_argument("--sync-every", type=int, default=0,
                   help="dp mode: weight_syncc every K steps inside the timed region (the DP driver's "
                        "replica averaging, every 200 iterations, dlrm_s_pytorch_tb_dp_one_parallel_comm.py:1924-1936)")
    p.add_argument("--batch-per-gpu", type=int, default=2048,
                   help="samples per rank per step (weak scaling; reference TB mini-batch 2048)")
    p.add_argument("--global-batch", type=int, default=0,
                   help="strong scaling: samples per step over all ranks, each rank taking its "
                        "get_my_slice share (SURVEY 8(d) C5: 2048 over 8 GPUs)")
    p.add_argument("--scaling", default="weak", choices=["weak", "strong"],
                   help="weak: --batch-per-gpu samples per rank; strong: --batch-per-gpu is the GLOBAL "
                        "batch split over the ranks (config 5 as SURVEY 8(d) writes it: "
                        "--scaling strong = 2048 over N GPUs); --global-batch overrides both")
    p.add_argument("--grad-bits", type=int, default=8)
    p.add_argument("--lr", type=float, default=0.1)
    p.add_argument("--scale-period", type=int, default=0,
                   help="refresh the table scales every P steps (q_m_n_q_g.py:303-315); 0 = every step")
    p.add_argument("--use-packed", action="store_true",
                   help="with --scale-period: gather INT4 rows between refreshes, repack touched rows")
    p.add_argument("--graph", action="store_true", help="replay the steps from captured HIP graphs (N=1)")
    p.add_argument("--graph-steps", type=int, default=8,
                   help="consecutive steps (one per resident batch) captured in each HIP graph: one "
                        "graph launch per that many steps (must divide --steps, else 1)")
    p.add_argument("--index-dist", default="uniform", choices=["uniform", "zipf"])
    p.add_argument("--num-batches", type=int, default=8, help="distinct resident batches cycled")
    p.add_argument("--gather-batch", type=int, default=65536,
                   help="bags per table for the INT4 packed-gather bandwidth phase (0 = skip)")
    p.add_argument("--gather-iters", type=int, default=50)
    p.add_argument("--mlp-iters", type=int, default=50,
                   help="iterations of the MLP INT8 gradient exchange phase (0 = skip)")
    p.add_argument("--cpu-baseline", type=int, default=1)
    p.add_argument("--cpu-seconds", type=float, default=12.0, help="time budget of the CPU baseline sample")
    p.add_argument("--seed", type=int, default=123)
    p.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                   help="nccl (= RCCL on ROCm) for measurements; gloo only to rehearse N>1 on one GPU")
    p.add_argument("--unfused-local", action="store_true",
                   help="N=1: run quant-pack + payload apply instead of the fused dqrm_apply_local")
    p.add_argument("--force-collectives", action="store_true",
                   help="run the N>1 exchange (two all-gathers, quantize-pack, payload apply; the MLP "
                        "exchange's collectives) through the process group at world size 1 too: the RCCL leg "
                        "on a one-GPU box")
    p.add_argument("--comm", default="rccl", choices=["rccl", "torch", "python"],
                   help="N > 1 (or forced) exchange transport: rccl = libdqrm issues both all-gathers on its own "
                        "RCCL communicator between the kernels (falls back to torch if RCCL cannot be set up); "
                        "torch = the same C step with torch.distributed serving the all-gathers; python = the "
                        "kernels and collectives issued one by one from Python (A/B)")
    p.add_argument("--emulate-ranks", type=int, default=1,
                   help="N > 1 on ONE GPU: time rank 0's step of an N-rank run (its slice: --batch-per-gpu "
                        "per rank, or --global-batch / --scaling strong split N ways) with the other ranks' "
                        "maxima and payloads precomputed from their own slices; the two all-gathers are replaced "
                        "by those resident buffers (rank 0's parts written in place), so the line is the per-rank "
                        "kernel time at N without xGMI time (a projection input, not a measurement of N GPUs)")
    p.add_argument("--separate-forward", action="store_true",
                   help="N=1 one-launch step: the forward as its own launch (dqrm_emb_fwd) instead of inside "
                        "the previous step's update launch (dqrm_emb_bwd_apply_fwd_local)")
    p.add_argument("--two-launch-local", action="store_true",
                   help="N=1: coalesce + dqrm_apply_local as two launches (not dqrm_emb_bwd_apply_local)")
    p.add_argument("--sample-every", type=int, default=0,
                   help="also bracket the dominant kernel with HIP events on every k-th TIMED step "
                        "(0 = never: the roofline is timed on the untimed breakdown pass's >= 16 "
                        "bracketed launches, so no event work sits inside the timed region)")
    p.add_argument("--traffic-profile", default=None,
                   help="rocprofv3 PMC summary (tools/prof_summary.py) for roofline.traffic; "
                        "default profiles/r2_<config>_summary.json when present")
    return p.parse_args(argv)


PROFILE_TAG = {"terabyte": "tb", "terabyte_ref": "tbref", "terabyte_1g": "tb1g", "kaggle": "kaggle"}
KERNEL_SYMBOL = {  # bench phase -> libdqrm kernel (as named in the rocprofv3 summary)
    "emb_fwd": "k_emb_fwd<{lpr},",
    "emb_fwd_packed": "k_emb_fwd_packed<{lpr},",
    # Criteo form (<APPLY, row-major stage>; round-3 summaries: <APPLY>) / general
    "bwd_coalesce": ("k_coalesce_p1<false,", "k_coalesce_p1<false>", "k_coalesce_p1", "k_bwd_fused<{lpr}, 1>"),
    "bwd_apply_local": ("k_coalesce_p1<true,", "k_coalesce_p1<true>"),  # N=1: coalesce + update in one launch
    # N=1 at the step boundary: the same kernel, with the next batch's forward inside
    "bwd_apply_fwd_local": ("k_coalesce_p1<true,", "k_coalesce_p1<true>"),
    "bwd_sgd": ("k_sgd_small<{lpr}, false>", "k_sgd_small<{lpr}>", "k_bwd_fused<{lpr}, 0>"),  # small batches / general
    "bwd_sgd_fwd": ("k_sgd_small<{lpr}, true>",),  # ... with the next batch's forward in the launch
    "grad_quant_pack": ("k_qpack<{lpr}>", "k_quant_pack<{lpr}>"),
    "apply_sparse_update": ("k_apply_flat2<{lpr},", "k_apply_flat<{lpr},", "k_apply_pos<{lpr}, false>",
                            "k_apply_ranges<{lpr}>"),
    # N > 1 at the step boundary: the apply of step i + the forward of step i+1 in one launch (merge)
    "apply_sparse_update_fwd": ("k_apply_pos<{lpr}, true>",),
    # ... or the flat apply, then its finalize + the forward in one launch: a list = both kernels' sum
    "apply_sparse_update_fwd_fin": [("k_apply_flat2<{lpr},", "k_apply_flat<{lpr},"), "k_finalize_fwd<{lpr},"],
    "apply_local": "k_apply_local<{lpr},",
}


def pmc_traffic(path, phase, D, workload=None):
    """HBM bytes per launch of the phase's kernel from a committed rocprofv3 PMC summary
    (reads by L2 request size + WRITE_SIZE when the summary has the request-size pass, else
    2 x FETCH_SIZE + WRITE_SIZE; tools/prof_summary.py), or None. The summary must
    have been profiled on the same workload (tools/prof_summary.py records the profiled bench
    line's config, batch per GPU, mode and N=1 update form): a summary of another batch
    size or mode is refused, not rescaled."""
    if not path or not os.path.exists(path) or phase not in KERNEL_SYMBOL:
        return None
    summ = json.load(open(path))
    if workload is not None and summ.get("workload") != workload:
        return None
    sym = KERNEL_SYMBOL[phase]
    kernels = summ["kernels"]

    def one(alts):  # the first kernel matching one of the alternative prefixes
        prefixes = tuple(p.format(lpr=D // 4) for p in alts)
        for name, v in sorted(kernels.items(), key=lambda kv: [kv[0].startswith(p) for p in prefixes], reverse=True):
            if name.startswith(prefixes) and v.get("hbm_bytes_per_launch") is not None:
                return v
        return None

    # a list: the phase is several launches, their bytes and times summed; a tuple: alternatives
    parts = ([one(p if isinstance(p, tuple) else (p,)) for p in sym] if isinstance(sym, list)
             else [one(sym if isinstance(sym, tuple) else (sym,))])
    if any(v is None for v in parts):
        return None
    med = [v.get("median_us") for v in parts]
    return {"bytes": round(sum(v["hbm_bytes_per_launch"] for v in parts)), "correction": summ.get("correction"),
            "profiled_avg_us": round(sum(v["avg_us"] for v in parts), 2),
            "profiled_median_us": round(sum(med), 2) if all(med) else None,
            "source": os.path.relpath(path, ROOT)}


def latest_profile(tag):
    """The newest round's committed rocprofv3 summary for a config (profiles/rN_<tag>_summary.json)."""
    import glob

    cands = sorted(glob.glob(os.path.join(ROOT, "profiles", f"r*_{tag}_summary.json")),
                   key=lambda p: int(re.match(r"r(\d+)_", os.path.basename(p)).group(1)))
    return cands[-1] if cands else None


def alg_bytes(phase, T, B, D, U, world=1, pool1=True, repack=False):
    """Algorithmic bytes per launch: what the algorithm must move, no more.
    L = T*B lookups, U = distinct (table, row) pairs. Criteo-form batches
    (DQRM_BATCH_POOLING_ONE) never read the offsets."""
    L = T * B
    offs = 0 if pool1 else T * B * 8
    pk = U * (D // 2) if repack else 0
    return {
        # index + FP32 row per lookup, FP32 output row per bag, the [T] scales
        "emb_fwd": L * (D * 4 + 8) + offs + L * D * 4 + T * 4,
        "emb_fwd_packed": L * (D // 2 + 8) + offs + L * D * 4 + T * 4,
        # index + dy row per lookup; one coalesced {row, D x f32} record per distinct row
        "bwd_coalesce": L * 8 + offs + L * D * 4 + U * (D * 4 + 4),
        # index + dy row per lookup; W row read+write and |W| row max per distinct row
        "bwd_sgd": L * 8 + offs + L * D * 4 + U * D * 8 + U * 4 + pk,
        "bwd_sgd_fwd": L * 8 + offs + L * D * 4 + U * D * 8 + U * 4 + pk + L * (D * 4 + 8) + offs + L * D * 4 + T * 4,
        # N=1 backward + update in one launch: as bwd_sgd (the coalesced rows never need HBM)
        "bwd_apply_local": L * 8 + offs + L * D * 4 + U * D * 8 + U * 4 + pk,
        # ... and the next batch's forward in the same launch: + emb_fwd's bytes
        "bwd_apply_fwd_local": L * 8 + offs + L * D * 4 + U * D * 8 + U * 4 + pk
                               + L * (D * 4 + 8) + offs + L * D * 4 + T * 4,
        "grad_quant_pack": U * (D * 4 + 4) + U * (D + 4),
        "apply_sparse_update": world * U * (D + 4) + U * D * 8 + U * 4 + pk,
        "apply_sparse_update_fwd": world * U * (D + 4) + U * D * 8 + U * 4 + pk + L * (D * 4 + 8) + offs
                                   + L * D * 4 + T * 4,
        "apply_local": U * (D * 4 + 4) + U * D * 8 + U * 4 + pk,
    }[phase]


def make_batches(rows, B_global, rank, world, count, seed, dist_kind, device):
    """Global Criteo-form batches [T, B_global] generated identically on every rank, each
    rank keeping its contiguous slice (get_my_slice, dlrm_s_pytorch_single_gpu.py:989-993)."""
    sl = dq.get_my_slice(B_global, world, rank)
    return [dq.LookupBatch.pooling_one(
        synthetic_indices(rows, B_global, seed * 1000 + k, dist_kind, device)[:, sl].contiguous())
        for k in range(count)]


def timed_events(n):
    return [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]


def phase_names(mode, use_packed, fused, one_launch=False, next_fwd=False, coll_fwd=False):
    fwd = "emb_fwd_packed" if use_packed else "emb_fwd"
    if mode == "fwd":
        return [fwd]
    if coll_fwd:  # N > 1: the apply of step i and the forward of step i+1 in one launch
        return ["bwd_coalesce", "grad_quant_pack", "apply_sparse_update_fwd"]
    if mode == "sgd":
        return ["bwd_sgd_fwd"] if next_fwd else [fwd, "bwd_sgd"]
    if fused and one_launch and next_fwd:
        return ["bwd_apply_fwd_local"]
    if fused and one_launch:
        return [fwd, "bwd_apply_local"]
    return [fwd, "bwd_coalesce"] + (["apply_local"] if fused else ["grad_quant_pack", "apply_sparse_update"])


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world == 1 and a.gpus > 1:
        print("N>1 must be launched with torch.distributed.run", file=sys.stderr)
        sys.exit(2)
    if a.use_packed and a.scale_period <= 0:
        print("--use-packed needs --scale-period P > 0", file=sys.stderr)
        sys.exit(2)
    if a.graph and world > 1:
        print("--graph runs at N=1 only (the collectives stay eager)", file=sys.stderr)
        sys.exit(2)
    if a.scaling == "strong" and a.global_batch <= 0:
        a.global_batch = a.batch_per_gpu  # the batch is the global one, split over the ranks
    strong = a.global_batch > 0
    if strong and a.global_batch % world:  # the reference skips such batches (parallel_comm.py:1855-1856)
        print(f"--global-batch {a.global_batch} is not divisible by {world} ranks", file=sys.stderr)
        sys.exit(2)
    ndev = torch.cuda.device_count()
    local = local % max(ndev, 1)  # gloo rehearsal: ranks may share a GPU
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    coll = world > 1 or a.force_collectives  # the exchange runs through the process group
    if coll:
        if world == 1:  # a lone rank outside torch.distributed.run
            for k, v in (("RANK", "0"), ("WORLD_SIZE", "1"), ("MASTER_ADDR", "127.0.0.1"), ("MASTER_PORT", "29511")):
                os.environ.setdefault(k, v)
        if a.dist_backend == "nccl":  # RCCL over xGMI, one process per GPU
            dist.init_process_group("nccl", device_id=dev)
        else:  # gloo: functional rehearsal of the N>1 path (e.g. several ranks on one GPU)
            dist.init_process_group("gloo")
    if a.emulate_ranks > 1:
        if world > 1 or a.mode != "dp":
            print("--emulate-ranks runs the dp step at world size 1", file=sys.stderr)
            sys.exit(2)
        emulate_main(a, dev)
        return
    if a.mode.startswith("dropin"):
        dropin_main(a, world, rank, dev)
        return
    if a.mode == "dlrm":
        dlrm_main(a, world, rank, dev)
        return
    cfg = CONFIGS[a.config]
    rows, D = cfg["rows"], cfg["dim"]
    T = len(rows)
    B_global = a.global_batch if strong else a.batch_per_gpu * world
    B = B_global // world

    t0 = time.time()
    ts = dq.EmbeddingTableSet(rows, D, device=dev, packed=a.gather_batch > 0 or a.use_packed, init="uniform",
                              seed=a.seed)
    batches = make_batches(rows, B_global, rank, world, a.num_batches, a.seed, a.index_dist, dev)
    dy = torch.randn(T, B, D, device=dev, generator=torch.Generator(device=dev).manual_seed(a.seed + rank)) * 0.05
    y = torch.empty(T, B, D, device=dev)
    comm = a.comm if a.dist_backend == "nccl" or a.comm != "rccl" else "torch"
    ex = (dq.SparseGradExchange(ts, B, grad_bits=a.grad_bits, force_collectives=a.force_collectives,
                                transport=comm if coll else None)
          if a.mode == "dp" else None)
    if a.use_packed:
        ts.refresh_scale_and_pack(4)
    torch.cuda.synchronize()
    setup_s = time.time() - t0

    # N=1: quantize-pack + apply fused (dqrm_apply_local; same quantize/dequantize/SGD
    # arithmetic, bit-identical W, no payload since nothing is exchanged)
    fused = not coll and not a.unfused_local
    # one launch (dqrm_emb_bwd_apply_local) for Criteo-form batches of <= 4096 lookups, <= 32 tables
    # whose grid the device can hold at once (the library decides; asked here for the line)
    one_launch = fused and not a.two_launch_local and ts.apply_local_is_one_launch(batches[0])
    repack = a.use_packed
    # ... and at the step boundary the NEXT batch's forward inside that launch (the update of
    # step i and apply_emb of step i+1 are adjacent in the training loop; dqrm_emb_bwd_apply_fwd_local):
    # each timed step still runs one forward and one backward + update
    next_fwd = (one_launch and a.mode == "dp" and not a.use_packed and not a.separate_forward
                and len(batches) > 1 and ts.apply_fwd_local_is_one_launch(batches[0], batches[1]))
    # the same for the single-GPU SGD step (dqrm_emb_bwd_sgd_fwd: one launch when the small-batch
    # kernel takes the update, config 3)
    if a.mode == "sgd" and not a.use_packed and not a.separate_forward and len(batches) > 1:
        next_fwd = ts.sgd_fwd_is_one_launch(batches[0], batches[1])  # else the forward as its own phase
    # N > 1 (or forced): the apply of step i and the forward of step i+1 through one call
    # (dqrm_exchange_apply_fwd / dqrm_apply_sparse_update_fwd) when it saves a launch: the merge
    # kernel runs both in one launch, the flat kernel's finalize shares a launch with the forward
    coll_form = (ex.apply_fwd_form(batches[1]) if coll and a.mode == "dp" and not a.use_packed
                 and not a.separate_forward and len(batches) > 1 else "separate")
    coll_fwd = coll_form != "separate"
    names = phase_names(a.mode, a.use_packed, fused, one_launch, next_fwd, coll_fwd)

    # N > 1 (or forced) over RCCL: the exchange is issued by libdqrm in two calls per step
    # (dqrm_exchange_grad: coalesce + both all-gathers + quantize-pack; dqrm_exchange_apply);
    # the untimed breakdown pass issues the kernels one by one to time each
    lib_exchange = ex is not None and ex._x is not None

    def step(i, ev=None, only=None, refresh=None, split=False):
        """One step of the selected mode. ev: per-phase (start, end) events; only: bracket
        just that phase; refresh: refresh the table scales (default: by --scale-period);
        split: the library-issued exchange as its separate calls (breakdown pass)."""
        b = batches[i % len(batches)]
        if refresh is None:
            refresh = a.scale_period <= 0 or i % a.scale_period == 0

        def mark(j, k):
            if ev is not None and (only is None or only == j):
                ev[j][k].record()

        if coll_fwd:  # this batch's forward ran in the previous step's apply launch; this one runs the next's
            nxt = batches[(i + 1) % len(batches)]
            rf = a.scale_period <= 0 or (i + 1) % a.scale_period == 0
            if lib_exchange and not split:
                ex.exchange(b, dy)
                ex.apply_forward(a.lr, nxt, out=y, bits=4, refresh_scale=rf, mode=L.DQRM_UPD_DP)
                return
            kern = ex.kernels
            mark(0, 0)
            kern.coalesce(b, dy, ex.ws, True, "tbd")
            mark(0, 1)
            ex._all_gather(ex.absmax_all, ex.ws.absmax)
            mark(1, 0)
            kern.quant_pack(ex.ws, ex.absmax_all, ex.world, a.grad_bits, ex.cap_base, ex.cap_total, ex.s_avg,
                            ex.payload)
            mark(1, 1)
            ex._all_gather(ex.gathered, ex.payload)
            mark(2, 0)
            kern.apply_fwd(ex.cap_base, ex.cap_total, ex.gathered, ex.payload_bytes, ex.world, a.grad_bits, ex.s_avg,
                           a.lr, L.DQRM_UPD_DP, False, nxt, y, bits=4, refresh_scale=rf, workspace=ex.apply_ws)
            mark(2, 1)
            return
        if next_fwd:  # this batch's forward ran in the previous step's launch; this one runs the next's
            nxt = batches[(i + 1) % len(batches)]
            rf = a.scale_period <= 0 or (i + 1) % a.scale_period == 0
            mark(0, 0)
            if a.mode == "sgd":
                ts.backward_sgd_forward(b, dy, a.lr, nxt, bits=4, refresh_scale=rf, out=y, repack=repack)
            else:
                ts.backward_apply_forward_local(b, dy, ex.ws, a.grad_bits, ex.s_avg, a.lr, nxt, bits=4,
                                                refresh_scale=rf, out=y)
            mark(0, 1)
            return
        mark(0, 0)
        if a.use_packed:
            if refresh:  # periodic refresh: new scales, tables whose scale moved are repacked
                ts.refresh_scale_and_pack(4)
            ts.forward(b, bits=4, refresh_scale=False, use_packed=True, out=y)
        else:
            ts.forward(b, bits=4, refresh_scale=refresh, out=y)
        mark(0, 1)
        if a.mode == "fwd":
            return
        mark(1, 0)
        if a.mode == "sgd":
            ts.backward_sgd(b, dy, a.lr, repack=repack)
            mark(1, 1)
            return
        kern = ex.kernels
        if lib_exchange and not split:
            ex.exchange(b, dy)
            ex.apply(a.lr, mode=L.DQRM_UPD_DP, repack=repack)
            return
        if one_launch:
            kern.coalesce_apply_local(b, dy, ex.ws, True, "tbd", a.grad_bits, ex.s_avg, a.lr, repack)
            mark(1, 1)
            return
        kern.coalesce(b, dy, ex.ws, True, "tbd")
        mark(1, 1)
        if fused:
            mark(2, 0)
            kern.apply_local(ex.ws, a.grad_bits, ex.s_avg, a.lr, repack)
            mark(2, 1)
            return
        if not ex.coll:
            absmax_all = ex.ws.absmax.view(1, -1)
        else:
            ex._all_gather(ex.absmax_all, ex.ws.absmax)
            absmax_all = ex.absmax_all
        mark(2, 0)
        kern.quant_pack(ex.ws, absmax_all, ex.world, a.grad_bits, ex.cap_base, ex.cap_total, ex.s_avg, ex.payload)
        mark(2, 1)
        if not ex.coll:
            gathered = ex.payload.view(1, -1)
        else:
            ex._all_gather(ex.gathered, ex.payload)
            gathered = ex.gathered
        mark(3, 0)
        kern.apply(ex.cap_base, ex.cap_total, gathered, ex.payload_bytes, ex.world, a.grad_bits, ex.s_avg, a.lr,
                   L.DQRM_UPD_DP, repack)
        mark(3, 1)

    if next_fwd or coll_fwd:  # the first batch's forward (every later one runs inside the previous step's launch)
        ts.forward(batches[0], bits=4, out=y)
    for i in range(a.warmup):
        step(i)
    torch.cuda.synchronize()
    # per-phase breakdown (untimed, eager): every phase bracketed by events; picks the dominant.
    # Periodic mode: steady-state steps only; the refresh (every P steps) is timed apart.
    nb = max(16, min(50, a.steps))  # >= 16 bracketed launches of every phase
    bev = [timed_events(len(names)) for _ in range(nb)]
    for i in range(nb):
        step(i, bev[i], refresh=a.scale_period <= 0, split=True)
    torch.cuda.synchronize()
    refresh_ms = None
    if a.use_packed:  # new scales from the |W| hierarchy + INT4 repack of every table whose scale moved
        rev = timed_events(3)
        for e0, e1 in rev:
            ts.pscale.fill_(float("nan"))
            e0.record()
            ts.refresh_scale_and_pack(4)
            e1.record()
        torch.cuda.synchronize()
        refresh_ms = float(np.mean([e0.elapsed_time(e1) for e0, e1 in rev]))
    kms = {n: float(np.mean([bev[i][j][0].elapsed_time(bev[i][j][1]) for i in range(nb)]))
           for j, n in enumerate(names)}
    dom = max(kms, key=kms.get)
    dj = names.index(dom)

    graphs = None
    gs = 1
    if a.graph:
        # gs consecutive steps (batches k .. k+gs-1) per captured graph, one graph per window of
        # the resident batches; a graph launch costs more than a B=128 step, so it is paid once
        # per gs steps. Periodic-refresh runs keep one step per graph (refresh steps run eager).
        gs = a.graph_steps if (a.scale_period <= 1 and a.graph_steps > 1 and a.steps % a.graph_steps == 0
                               and (a.warmup + a.steps) % a.graph_steps == 0) else 1
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        graphs = []
        with torch.cuda.stream(s):
            for k in range(0, max(len(batches), gs), gs):
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=s):
                    for j in range(gs):
                        step(k + j, refresh=a.scale_period <= 0)
                graphs.append(g)
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()

    sync_every = a.sync_every if a.mode == "dp" else 0
    if sync_every and a.graph:
        print("--sync-every runs eager (no --graph)", file=sys.stderr)
        sys.exit(2)
    from deep_quantized_recommendation_model_dqrm_amd.sgd_quantized_gradients_parallel_comm import sync_table_set

    def run(i, ev=None):
        if graphs is None or (a.scale_period > 1 and i % a.scale_period == 0):
            step(i, ev, only=dj)
        elif i % gs == 0:  # steps i .. i+gs-1 (batches (i+j) % len(batches), as the eager run)
            graphs[(i % max(len(batches), gs)) // gs].replay()
        if sync_every and (i + 1) % sync_every == 0:  # weight_syncc (checksum gate + local ring mean)
            sync_table_set(ts, world)

    sync_ms = None
    if sync_every:  # the sync alone, outside the timed region (a few calls)
        torch.cuda.synchronize()
        t0s = time.perf_counter()
        for _ in range(3):
            sync_table_set(ts, world)
        torch.cuda.synchronize()
        sync_ms = (time.perf_counter() - t0s) / 3 * 1e3

    # timed region: plain steps. The dominant kernel's roofline time comes from the breakdown
    # pass above (>= 16 event-bracketed launches); --sample-every k also brackets every k-th
    # timed step (events on the stream the kernel runs on; not with graphs or the library exchange)
    if coll:
        dist.barrier()
    torch.cuda.synchronize()
    every = a.sample_every
    sampled = ([] if graphs is not None or lib_exchange or every <= 0 else
               [i for i in range(a.steps) if i % every == 0])
    evs = {i: timed_events(len(names)) for i in sampled}
    t_start = time.perf_counter()
    for i in range(a.steps):
        run(a.warmup + i, evs.get(i))
    if coll:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t_start
    if world > 1:
        e = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())
    dom_ms = (float(np.mean([evs[i][dj][0].elapsed_time(evs[i][dj][1]) for i in sampled])) if sampled
              else kms[dom])  # the breakdown pass's average over its nb >= 16 bracketed launches

    # algorithmic bytes per launch; distinct rows of the last step's batch
    if ex is not None:
        U = int(ex.ws.ucount.sum().item())
    else:
        P = batches[(a.warmup + a.steps - 1) % len(batches)].idx.view(T, -1)
        U = int(sum(torch.unique(P[t]).numel() for t in range(T)))
    alg = alg_bytes(dom, T, B, D, U, world, pool1=True, repack=repack)
    step_alg = sum(alg_bytes(n, T, B, D, U, world, pool1=True, repack=repack) for n in names)
    achieved = alg / (dom_ms * 1e-3) / 1e9
    err = ts.read_errors()

    gather = gather_phase(a, ts, rows, T, D, dev) if a.gather_batch > 0 else None
    mlp = dense_phase(a, dev, world, rank, coll) if a.mlp_iters > 0 else None

    cpu = cpu_c = None  # the CPU baselines are N=1 figures: a single-rank run only
    if world == 1 and a.cpu_baseline:
        cpu = cpu_baseline_torch(a, B)
        cpu_c = cpu_baseline_oracle(a, min(B, 2048))

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
    n1_update = ("SGD of step i + forward of step i+1 (dqrm_emb_bwd_sgd_fwd)" if a.mode == "sgd" and next_fwd else
                 None if a.mode != "dp" or world > 1 else
                 "coalesce + quant-pack + payload apply with the next forward (RCCL at world size 1)"
                 if coll and coll_fwd else
                 "coalesce + quant-pack + payload apply (RCCL at world size 1)" if coll else
                 "one launch: update of step i + forward of step i+1 (dqrm_emb_bwd_apply_fwd_local)" if next_fwd else
                 "one launch (dqrm_emb_bwd_apply_local)" if one_launch else
                 "coalesce + dqrm_apply_local" if fused else "coalesce + quant-pack + payload apply")
    workload = {"config": a.config, "mode": a.mode, "batch_per_gpu": B, "n1_update": n1_update,
                "index_dist": a.index_dist}
    # (the forced-collectives N > 1 form is profiled under its own tag, e.g. r5_tbforced)
    prof = a.traffic_profile or latest_profile(PROFILE_TAG[a.config] + ("forced" if coll and world == 1 else ""))
    traffic = pmc_traffic(prof, dom + ("_fin" if dom == "apply_sparse_update_fwd" and coll_form == "fin_fwd" else ""),
                          D, workload)
    med_us = traffic["profiled_median_us"] if traffic else None
    if rank == 0:
        value = B_global * a.steps / elapsed
        metric = {
            "dp": "QAT-step samples/sec (DP embedding QAT step: INT4 fake-quant gather + sparse SGD + "
                  "INT8 sparse-grad all-reduce)",
            "fwd": "forward samples/sec (INT4 fake-quant EmbeddingBag forward, 26 tables)",
            "sgd": "QAT-step samples/sec (1-GPU embedding QAT step: INT4 fake-quant gather + fused sparse SGD)",
        }[a.mode]
        colls = None
        if a.mode == "dp":
            colls = {"world_size": world, "backend": a.dist_backend if coll else None,
                     "issued_by": ({"rccl": "libdqrm (dqrm_comm: RCCL ncclAllGather between the step's kernels)",
                                    "torch": "libdqrm's exchange, all-gathers served by torch.distributed",
                                    "python": "torch.distributed"}.get(ex.transport) if coll else None),
                    "per_step": 2 if coll else 0,
                    "scale_allgather_bytes_per_rank": ex.ws.absmax.numel() * 4,
                    "payload_allgather_bytes_per_rank": int(ex.payload_bytes)}
        line = {
            "metric": metric,
            "value": round(value, 1) if err == 0 else None,
            "unit": "samples/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(elapsed / a.steps * 1e3, 4),
            "us_per_step": round(elapsed / a.steps * 1e6, 2),
            "higher_is_better": True,
            "scaling": "strong" if strong else "weak",
            "vs_baseline": None,
            "dtype": "f32 (int4 fake-quant activations, int8 gradients)",
            "data": ("synthetic (uniform-random Criteo-form indices, U(+-sqrt(1/n)) tables, N(0,0.05) dL/dy)"
                     if a.index_dist == "uniform" else "synthetic (power-law indices)"),
            "config": {
                "workload": f"criteo-{a.config} embedding " + {"dp": "QAT step", "fwd": "forward",
                                                               "sgd": "QAT step (fused SGD)"}[a.mode],
                "mode": a.mode, "tables": T, "total_rows": sum(rows), "emb_dim": D,
                "batch_per_gpu": B, "global_batch": B_global, "pooling": 1,
                "grad_bits": a.grad_bits if a.mode == "dp" else None,
                "scale_period": max(a.scale_period, 1), "packed_int4_forward": a.use_packed,
                "hip_graph": a.graph, "graph_steps": gs if a.graph else None,
                "n1_update": n1_update,
                "parallelism": f"dp{world} (tables replicated)",
            },
            "roofline": {"kernel": dom, "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic["bytes"] if traffic else None, "traffic_unit": "bytes/launch",
                         "traffic_src": traffic,
                         "alg_bytes_per_launch": alg, "avg_launch_ms": round(dom_ms, 5),
                         "timed_launches": len(sampled) if sampled else nb,
                         # the same bytes over rocprofv3's median kernel time of this workload
                         # (events bracket the launch and read a few us above the kernel)
                         "frac_rocprof_median": (round(alg / (med_us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4)
                                                 if med_us else None),
                         "workload_profiled": workload},
            # the whole step against the same peak: every phase's algorithmic bytes / step time
            "step_roofline": {"alg_bytes_per_step": step_alg,
                              "achieved": round(step_alg / (elapsed / a.steps) / 1e9, 1),
                              "frac": round(step_alg / (elapsed / a.steps) / 1e9 / HBM_PEAK_GBS, 4),
                              "phases": names},
            "kernels_ms": {k: round(v, 5) for k, v in kms.items()},
            "kernels_ms_note": "untimed eager breakdown pass, every phase bracketed by events; " + (
                "bwd_sgd_fwd = the SGD of this step's batch, then the next batch's forward, one workgroup per "
                "table (one launch when the small-batch kernel runs)" if a.mode == "sgd" and next_fwd
                else "bwd_apply_fwd_local is ONE launch per step: coalesce, quantize, update and the |W| hierarchy of "
                "this step's batch, then the next batch's fake-quant forward, table by table" if next_fwd
                else "bwd_apply_local is ONE launch (coalesce, quantize, update and the |W| hierarchy)" if one_launch
                else "apply_local = the fused quantize + update kernel + a short k_table_finalize launch" if fused
                else "sgd = one launch (|W| hierarchy inside)" if a.mode == "sgd"
                else "apply_sparse_update_fwd = the payload merge + update of this step and the next batch's forward, "
                "one launch (k_apply_pos<LPR, true>: each table's forward once its update and |W| maxima are final)"
                if coll_form == "one_launch"
                else "apply_sparse_update_fwd = the payload decode + update (k_apply_flat), then the |W| finalize and "
                "the next batch's forward in one launch (k_finalize_fwd: each table's scale once its finalize "
                "workgroup opened the table's gate)"
                if coll_form == "fin_fwd"
                else "apply_sparse_update = " + L.apply_update_form(world) if a.mode == "dp" else "forward only"),
            "weight_syncc": ({"every": sync_every, "ms_per_call": round(sync_ms, 3),
                              "amortized_us_per_step": round(sync_ms * 1e3 / sync_every, 2),
                              "in_timed_region": True} if sync_every else None),
            "scale_refresh_ms": round(refresh_ms, 4) if refresh_ms is not None else None,
            "scale_refresh_note": ("full INT4 repack of all tables (worst case: every scale moved), once per "
                                   f"{a.scale_period} steps" if refresh_ms is not None else None),
            "launch_share": (round(max(0.0, 1.0 - sum(kms.values()) / (elapsed / a.steps * 1e3)), 4)
                             if not a.graph else None),
            "collectives": colls,
            "int4_gather": gather,
            "mlp_grad_exchange": mlp,
            "cpu_baseline": cpu,
            "cpu_baseline_oracle_c": cpu_c,
            "device_errors": err,
            "replicas_bit_identical": replicas_match,
            "setup_s": round(setup_s, 1),
        }
        print(json.dumps(line), flush=True)
    if coll:
        dist.barrier()
        dist.destroy_process_group()
    if err:  # a step that dropped or mis-indexed lookups is not a measurement
        print(f"device error flags 0x{err:x}", file=sys.stderr)
        sys.exit(3)


def emulate_main(a, dev):
    """rank 0 of an N-rank data-parallel step on one GPU (--emulate-ranks N): the kernels rank 0
    runs at N GPUs -- forward, coalesce of its slice, quantize-pack against all N ranks' maxima
    (the rank-averaged scale), the apply over all N payloads (+ the finalize launch) -- with
    the two all-gathers replaced by resident buffers: every other rank's per-slot maxima and
    INT8 payload of each resident batch are computed beforehand from that rank's own slice
    (untimed), and rank 0's coalesce / quantize-pack write their maxima / payload straight into
    row 0 of the gathered buffers (what the all-gather leaves there). What the line adds to a
    real N-GPU step is the xGMI time of the two all-gathers, estimated in DESIGN.md 6."""
    N = a.emulate_ranks
    cfg = CONFIGS[a.config]
    rows, D = cfg["rows"], cfg["dim"]
    T = len(rows)
    strong = a.scaling == "strong" or a.global_batch > 0
    B_global = (a.global_batch or a.batch_per_gpu) if strong else a.batch_per_gpu * N
    if B_global % N:
        print(f"global batch {B_global} is not divisible by {N} ranks", file=sys.stderr)
        sys.exit(2)
    B = B_global // N
    nb = a.num_batches
    gb = a.grad_bits
    S = L.DQRM_TABLE_SPLIT
    t0 = time.time()
    ts = dq.EmbeddingTableSet(rows, D, device=dev, init="uniform", seed=a.seed)
    ex = dq.SparseGradExchange(ts, B, grad_bits=gb)
    kern = ex.kernels
    per_rank = [make_batches(rows, B_global, r, N, nb, a.seed, a.index_dist, dev) for r in range(N)]
    dys = [torch.randn(T, B, D, device=dev, generator=torch.Generator(device=dev).manual_seed(a.seed + r)) * 0.05
           for r in range(N)]
    am_all = [torch.zeros(N, T * S, dtype=torch.float32, device=dev) for _ in range(nb)]
    gathered = [torch.zeros(N, ex.payload_bytes, dtype=torch.uint8, device=dev) for _ in range(nb)]
    wss = [dq.CoalescedGrad.allocate(rows, B, D, dev, absmax=am_all[k][0]) for k in range(nb)]
    tmp = dq.CoalescedGrad.allocate(rows, B, D, dev)
    s_tmp = torch.zeros(T, dtype=torch.float32, device=dev)
    for k in range(nb):  # the other ranks' maxima, then their payloads (against every rank's maxima)
        ts.forward(per_rank[0][k], bits=4)
        for r in range(1, N):
            kern.coalesce(per_rank[r][k], dys[r], tmp, True, "tbd")
            am_all[k][r].copy_(tmp.absmax)
        kern.coalesce(per_rank[0][k], dys[0], wss[k], True, "tbd")
        for r in range(1, N):
            kern.coalesce(per_rank[r][k], dys[r], tmp, True, "tbd")
            kern.quant_pack(tmp, am_all[k], N, gb, ex.cap_base, ex.cap_total, s_tmp, gathered[k][r])
    del tmp
    y = torch.empty(T, B, D, device=dev)
    torch.cuda.synchronize()
    setup_s = time.time() - t0
    # the apply of step i with the forward of step i+1 in one launch (dqrm_apply_sparse_update_fwd),
    # as bench.py's N > 1 step runs it; --separate-forward: the forward as its own launch
    import ctypes as C

    aws = torch.zeros(max(16, int(ts.lib.dqrm_apply_workspace_bytes(N, ex.cap_total))), dtype=torch.uint8, device=dev)
    form = ts.lib.dqrm_apply_fwd_form(C.byref(ts.c), N, ex.cap_total, aws.numel(), C.byref(per_rank[0][1 % nb].c),
                                      ts._fwd_flags(True, False, False))
    fused = not a.separate_forward and form in (L.DQRM_APPLY_FWD_ONE_LAUNCH, L.DQRM_APPLY_FWD_FIN_FWD)
    names = (["bwd_coalesce", "grad_quant_pack", "apply_sparse_update_fwd"] if fused
             else ["emb_fwd", "bwd_coalesce", "grad_quant_pack", "apply_sparse_update"])

    def step(i, ev=None):
        k = i % nb
        b = per_rank[0][k]

        def mark(j, e):
            if ev is not None:
                ev[j][e].record()

        j0 = 0
        if not fused:
            mark(0, 0)
            ts.forward(b, bits=4, out=y)
            mark(0, 1)
            j0 = 1
        mark(j0, 0)
        kern.coalesce(b, dys[0], wss[k], True, "tbd")  # maxima -> row 0 of the "gathered" maxima
        mark(j0, 1)
        mark(j0 + 1, 0)
        kern.quant_pack(wss[k], am_all[k], N, gb, ex.cap_base, ex.cap_total, ex.s_avg, gathered[k][0])
        mark(j0 + 1, 1)
        mark(j0 + 2, 0)
        if fused:  # this step's update + the next step's forward
            kern.apply_fwd(ex.cap_base, ex.cap_total, gathered[k], ex.payload_bytes, N, gb, ex.s_avg, a.lr,
                           L.DQRM_UPD_DP, False, per_rank[0][(i + 1) % nb], y, workspace=aws)
        else:  # the apply alone (with the merge workspace: the AUTO choice at N > 1)
            kern.apply_fwd(ex.cap_base, ex.cap_total, gathered[k], ex.payload_bytes, N, gb, ex.s_avg, a.lr,
                           L.DQRM_UPD_DP, False, None, y, workspace=aws)
        mark(j0 + 2, 1)

    if fused:
        ts.forward(per_rank[0][0], bits=4, out=y)
    for i in range(a.warmup):
        step(i)
    torch.cuda.synchronize()
    nbk = max(16, min(50, a.steps))
    bev = [timed_events(len(names)) for _ in range(nbk)]
    for i in range(nbk):
        step(a.warmup + i, bev[i])
    torch.cuda.synchronize()
    kms = {n: float(np.median([bev[i][j][0].elapsed_time(bev[i][j][1]) for i in range(nbk)]))
           for j, n in enumerate(names)}
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    for i in range(a.steps):
        step(a.warmup + nbk + i)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t_start
    err = ts.read_errors()
    us = elapsed / a.steps * 1e6
    U = int(wss[(a.warmup + nbk + a.steps - 1) % nb].ucount.sum().item())
    line = {
        "metric": "emulated per-rank DP QAT step (rank 0 of N; all-gathers replaced by resident buffers)",
        "value": None, "unit": "samples/s", "n_gpus": 1, "emulated_ranks": N, "steps": a.steps, "warmup": a.warmup,
        "us_per_step": round(us, 2), "higher_is_better": True, "scaling": "strong" if strong else "weak",
        "projected_samples_per_s_without_collectives": round(B_global / (us * 1e-6), 1),
        "config": {"workload": f"criteo-{a.config} embedding QAT step", "tables": T, "total_rows": sum(rows),
                   "emb_dim": D, "batch_per_rank": B, "global_batch": B_global, "grad_bits": gb,
                   "index_dist": a.index_dist},
        "kernels_ms_median": {k: round(v, 5) for k, v in kms.items()},
        "alg_bytes": {n: alg_bytes(n, T, B, D, U, N, pool1=True) for n in names},
        "distinct_rows_rank0": U,
        "payload_bytes_per_rank": int(ex.payload_bytes), "maxima_bytes_per_rank": T * S * 4,
        "apply_update_form": L.apply_update_form(N),
        # coalesce, quantize-pack, then: merge (k_merge_pos at N > 1 + k_apply_pos with the forward) /
        # flat (k_apply_flat + k_finalize_fwd) / separate (forward + k_apply_flat + k_table_finalize)
        "step_launches": (4 if form == L.DQRM_APPLY_FWD_FIN_FWD or N > 1 else 3) if fused else 5,
        "forward_in_apply_launch": fused and form == L.DQRM_APPLY_FWD_ONE_LAUNCH,
        "forward_in_finalize_launch": fused and form == L.DQRM_APPLY_FWD_FIN_FWD,
        "device_errors": err, "setup_s": round(setup_s, 1),
    }
    print(json.dumps(line), flush=True)
    if err:
        sys.exit(3)


def count_launches(fn, steps=3):
    """Device kernels launched per call of fn (torch.profiler over `steps` calls; None when the
    profiler cannot trace the device here)."""
    try:
        from torch.profiler import ProfilerActivity, profile

        torch.cuda.synchronize()
        with profile(activities=[ProfilerActivity.CUDA]) as prof:
            for _ in range(steps):
                fn()
            torch.cuda.synchronize()
        n = sum(1 for e in prof.events() if e.device_type == torch.autograd.DeviceType.CUDA)
        return round(n / steps, 1) if n else None
    except Exception:  # noqa: BLE001 -- a measurement aid only
        return None


def dropin_main(a, world, rank, dev):
    """The reference drivers' own call pattern through the drop-in (BASELINE configs 3-4),
    timed as a whole step with its host work (module calls, autograd, optimizer, hooks):

    dropin-sgd  dlrm_s_pytorch_single_gpu.py:609-674,1943-1950 -- apply_emb's per-table loop
                over 26 QuantEmbeddingBagTwo (--dropin-form list) or one
                QuantEmbeddingBagCollection (collection), backward from a fixed dL/dy, then
                torch.optim.SGD.step() (grad_mode sparse: the per-lookup COO) or nothing
                (fused_sgd: the update ran in the backward kernel);
    dropin-dp   dlrm_s_pytorch_tb_dp_one_parallel_comm.py:1888-1904 -- clear_gradients,
                forward, backward, grad_update_parallel_comm(..., 8 bits),
                weight_update_parallel_comm; a ModuleList is consolidated into one table set
                by the hooks on first use.
    The line also carries the direct-API step (EmbeddingTableSet / SparseGradExchange) at
    the same shape, and the device launches per step."""
    from torch import nn

    from deep_quantized_recommendation_model_dqrm_amd import quant_modules_not_quantize_grad as Q
    from deep_quantized_recommendation_model_dqrm_amd import sgd_quantized_gradients_parallel_comm as H

    cfg = CONFIGS[a.config]
    rows, D = cfg["rows"], cfg["dim"]
    T = len(rows)
    B_global = a.global_batch if a.global_batch > 0 else a.batch_per_gpu * world
    B = B_global // world
    dp = a.mode == "dropin-dp"
    gm = "dp" if dp else a.grad_mode
    Q.set_pooling_one_inputs(True)  # Criteo-form inputs (offsets = arange), as the drivers feed
    t0 = time.time()
    if a.dropin_form == "list":
        emb = nn.ModuleList([Q.QuantEmbeddingBagTwo(n, D, 4, embedding_id=i, init="device", grad_mode=gm, lr=a.lr,
                                                    device=dev) for i, n in enumerate(rows)])
    else:
        emb = Q.QuantEmbeddingBagCollection(rows, D, 4, init="device", grad_mode=gm, lr=a.lr, device=dev)
    model = nn.Module()
    model.emb_l, model.bot_l, model.top_l = emb, nn.ModuleList(), nn.ModuleList()
    params = [p for p in model.parameters()]
    opt = torch.optim.SGD(params, lr=a.lr) if (not dp and gm == "sparse") else None
    batches = make_batches(rows, B_global, rank, world, a.num_batches, a.seed, a.index_dist, dev)
    lS_o = torch.arange(B, dtype=torch.int64, device=dev)
    g = torch.Generator(device=dev).manual_seed(a.seed + rank)
    dys = [torch.randn(B, D, device=dev, generator=g) * 0.05 for _ in range(T)]
    setup_s = time.time() - t0

    def step(i):
        P = batches[i % len(batches)].idx.view(T, B)
        if dp:
            H.clear_gradients(model)
        if a.dropin_form == "list":
            ly = [emb[t](P[t], lS_o) for t in range(T)]
        else:
            ly = emb(lS_o.expand(T, B), P)
        torch.autograd.backward(ly, dys)
        if dp:
            H.grad_update_parallel_comm(model, world, True, a.grad_bits)
            H.weight_update_parallel_comm(model, a.lr, num_gpus=world)
        elif opt is not None:
            opt.step()
            opt.zero_grad(set_to_none=True)

    for i in range(a.warmup):
        step(i)
    launches = count_launches(lambda: step(0))
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    tst = time.perf_counter()
    for i in range(a.steps):
        step(a.warmup + i)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - tst
    if world > 1:
        e = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())
    errs = (emb[0]._tset if a.dropin_form == "list" else emb._tset).read_errors()
    del model, emb, opt
    torch.cuda.empty_cache()

    # the direct-API step at the same shape, for comparison (same process, fresh tables)
    ts = dq.EmbeddingTableSet(rows, D, device=dev, init="uniform", seed=a.seed)
    ex = dq.SparseGradExchange(ts, B, grad_bits=a.grad_bits) if dp else None
    dyt = torch.stack(dys)

    def direct(i):
        b = batches[i % len(batches)]
        ts.forward(b, bits=4)
        if dp:
            ex.step(b, dyt, a.lr)
        else:
            ts.backward_sgd(b, dyt, a.lr)

    for i in range(a.warmup):
        direct(i)
    direct_launches = count_launches(lambda: direct(0))
    torch.cuda.synchronize()
    tdt = time.perf_counter()
    for i in range(a.steps):
        direct(a.warmup + i)
    torch.cuda.synchronize()
    direct_s = time.perf_counter() - tdt
    del ts, ex
    torch.cuda.empty_cache()
    ref_us = torch_reference_gpu(a, rows, D, B, dev, batches, dys, dp) if world == 1 else None
    if rank == 0:
        us = elapsed / a.steps * 1e6
        dus = direct_s / a.steps * 1e6
        line = {
            "metric": ("drop-in DP QAT-step samples/sec (ModuleList/collection + the four grad-comm hooks)" if dp else
                       "drop-in single-GPU QAT-step samples/sec (modules + " +
                       ("torch.optim.SGD)" if gm == "sparse" else "fused SGD in the backward)")),
            "value": round(B_global * a.steps / elapsed, 1) if errs == 0 else None,
            "unit": "samples/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": round(us / 1e3, 4), "us_per_step": round(us, 2), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32 (int4 fake-quant activations)",
            "data": "synthetic (uniform-random Criteo-form indices, device-initialised U(+-sqrt(1/n)) tables)",
            "config": {"workload": f"criteo-{a.config} embedding {a.mode} ({a.dropin_form})", "tables": T,
                       "total_rows": sum(rows), "emb_dim": D, "batch_per_gpu": B, "global_batch": B_global,
                       "grad_mode": gm, "grad_bits": a.grad_bits if dp else None, "pooling": 1,
                       "parallelism": f"dp{world} (tables replicated)"},
            "launches_per_step": launches,
            "direct_api": {"us_per_step": round(dus, 2), "launches_per_step": direct_launches,
                           "dropin_over_direct": round(us / dus, 2)},
            "torch_gpu_reference": ({"us_per_step": round(ref_us, 2), "dropin_speedup": round(ref_us / us, 2),
                                     "what": "the reference's modules as PyTorch ops on this GPU, same shape "
                                             "(nn.EmbeddingBag sparse + per-step full-table aminmax scale + "
                                             "fake-quant STE, autograd, " +
                                             ("quantize_emb_grad + weight update at one rank)" if dp else
                                              "torch.optim.SGD)")} if ref_us else None),
            "device_errors": errs, "setup_s": round(setup_s, 1),
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


class DLRMNet(torch.nn.Module):
    """DLRM_Net of the single-GPU driver (dlrm_s_pytorch_single_gpu.py:271-962) at the
    reference scripts' Kaggle shape: bottom MLP 13-512-256-64-16 (ReLU after every layer),
    26 embedding tables, dot interaction without self-interaction (:696-801: the 351 pairs
    j < i of the 27 vectors, concatenated after the bottom output -> 367), top MLP
    367-512-256-1 (ReLU, ReLU, sigmoid), create_mlp's init (N(0, sqrt(2/(m+n))) weights,
    N(0, sqrt(1/m)) biases, :293-336). `emb(P)` returns the 26 pooled vectors as [B, T, D]."""

    def __init__(self, bot, top, emb, seed):
        super().__init__()
        rs = np.random.RandomState(seed)

        def mlp(dims, sigmoid_last):
            layers = []
            for k, (n, m) in enumerate(zip(dims[:-1], dims[1:])):
                lin = torch.nn.Linear(n, m)
                with torch.no_grad():
                    lin.weight.copy_(torch.from_numpy(rs.normal(0.0, np.sqrt(2 / (m + n)), (m, n)).astype(np.float32)))
                    lin.bias.copy_(torch.from_numpy(rs.normal(0.0, np.sqrt(1 / m), m).astype(np.float32)))
                layers += [lin, torch.nn.Sigmoid() if sigmoid_last and k == len(dims) - 2 else torch.nn.ReLU()]
            return torch.nn.Sequential(*layers)

        self.bot_l = mlp(bot, False)
        self.top_l = mlp(top, True)
        self.emb = emb
        self._li = self._lj = None

    def forward(self, X, P):
        x = self.bot_l(X)
        ly = self.emb(P)                                           # [B, T, D]
        Tm = torch.cat([x.unsqueeze(1), ly], dim=1)                # [B, T+1, D]
        Z = torch.bmm(Tm, Tm.transpose(1, 2))
        if self._li is None:
            n = Tm.shape[1]
            self._li = torch.tensor([i for i in range(n) for j in range(i)], device=X.device)
            self._lj = torch.tensor([j for i in range(n) for j in range(i)], device=X.device)
        R = torch.cat([x, Z[:, self._li, self._lj]], dim=1)
        return self.top_l(R)


class _RefEmb(torch.nn.Module):
    """The reference's embedding layer as PyTorch ops (QuantEmbeddingBagTwo on ATen): per table
    nn.EmbeddingBag(mode="sum", sparse=True), the full-table aminmax scale every training
    forward, fake quant + dequant with the STE backward."""

    def __init__(self, rows, D, dev):
        super().__init__()
        self.bags = torch.nn.ModuleList()
        for n in rows:
            w = torch.empty(n, D, device=dev).uniform_(-float(np.sqrt(1 / n)), float(np.sqrt(1 / n)))
            self.bags.append(torch.nn.EmbeddingBag(n, D, mode="sum", sparse=True, _weight=w))
        self.register_buffer("off", torch.zeros(0, dtype=torch.int64, device=dev))

    def forward(self, P):
        B = P.shape[1]
        if self.off.numel() != B:
            self.off = torch.arange(B, dtype=torch.int64, device=P.device)
        ys = []
        for t, e in enumerate(self.bags):
            with torch.no_grad():
                mn, mx = torch.aminmax(e.weight)
                s = torch.clamp(torch.maximum(mn.abs(), mx.abs()), min=1e-8) / 7.0
            ys.append(_FakeQuantSTE.apply(e(P[t], self.off), s, 4))
        return torch.stack(ys, dim=1)


def dlrm_main(a, world, rank, dev):
    """BASELINE config 3 as SURVEY 8(d) C3 writes it: the single-GPU driver's whole QAT step
    (dlrm_s_pytorch_single_gpu.py:804-890 forward, :1936-1950 loss / backward / SGD) at the
    Kaggle shape -- bottom MLP, 26 INT4 fake-quant EmbeddingBag tables, dot interaction, top
    MLP, BCE, backward, SGD lr 0.1 -- with the embeddings from
      --dropin-form collection: one QuantEmbeddingBagCollection, grad_mode fused_sgd (the
                                 sparse SGD runs inside the backward kernel),
      --dropin-form list:       26 QuantEmbeddingBagTwo modules + torch.optim.SGD on their
                                 per-lookup COO grads (--grad-mode sparse) or fused_sgd,
    next to the same model with the reference's modules as PyTorch ops on the same GPU. The
    MLPs, interaction and loss are PyTorch (hipBLASLt GEMMs): outside the north-star path,
    inside this measurement. --graph replays whole steps from HIP graphs (one per resident
    batch); the loss is not copied to the host per step (the driver's E.detach().cpu() is a
    logging sync)."""
    from deep_quantized_recommendation_model_dqrm_amd import quant_modules_not_quantize_grad as Q

    if world > 1:
        print("--mode dlrm is the single-GPU step (config 3)", file=sys.stderr)
        sys.exit(2)
    rows, D = CONFIGS[a.config]["rows"], CONFIGS[a.config]["dim"]
    T = len(rows)
    B = a.batch_per_gpu
    bot, top = MLPS[a.config]
    Q.set_pooling_one_inputs(True)
    gm = "fused_sgd" if a.dropin_form == "collection" else a.grad_mode
    g = torch.Generator(device=dev).manual_seed(a.seed)
    batches = make_batches(rows, B, 0, 1, a.num_batches, a.seed, a.index_dist, dev)
    Ps = [b.idx.view(T, B) for b in batches]
    Xs = [torch.rand(B, bot[0], device=dev, generator=g) for _ in range(a.num_batches)]
    Ys = [torch.round(torch.rand(B, 1, device=dev, generator=g)) for _ in range(a.num_batches)]
    lS_o = torch.arange(B, dtype=torch.int64, device=dev)

    def build(kind):
        if kind == "collection":
            coll = Q.QuantEmbeddingBagCollection(rows, D, 4, init="device", grad_mode="fused_sgd", lr=a.lr, device=dev)
            emb = lambda P: coll(lS_o.expand(T, B), P, layout="btd")  # noqa: E731
            holder, emb_params = coll, []
        elif kind == "list":
            mods = torch.nn.ModuleList([Q.QuantEmbeddingBagTwo(n, D, 4, embedding_id=i, init="device", grad_mode=gm,
                                                               lr=a.lr, device=dev) for i, n in enumerate(rows)])
            emb = lambda P: torch.stack([mods[t](P[t], lS_o) for t in range(T)], dim=1)  # noqa: E731
            holder = mods
            emb_params = [] if gm == "fused_sgd" else [m.embedding_bag.weight for m in mods]
        else:
            holder = _RefEmb(rows, D, dev)
            emb, emb_params = holder, list(holder.parameters())

        class _E(torch.nn.Module):
            def __init__(self):
                super().__init__()
                self.h = holder

            def forward(self, P):
                return emb(P)

        net = DLRMNet(bot, top, _E(), a.seed).to(dev)
        params = list(net.bot_l.parameters()) + list(net.top_l.parameters()) + emb_params
        opt = torch.optim.SGD(params, lr=a.lr)
        return net, opt, holder

    loss_fn = torch.nn.BCELoss(reduction="mean")

    def timed(kind, graph):
        net, opt, holder = build(kind)

        def step(i):
            k = i % a.num_batches
            opt.zero_grad(set_to_none=True)
            E = loss_fn(net(Xs[k], Ps[k]), Ys[k])
            E.backward()
            opt.step()
            return E

        for i in range(a.warmup):
            step(i)
        torch.cuda.synchronize()
        launches = count_launches(lambda: step(0))
        graphs = None
        if graph:
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                for i in range(3):
                    step(i)
            torch.cuda.current_stream().wait_stream(s)
            torch.cuda.synchronize()
            graphs = []
            for k in range(a.num_batches):
                gr = torch.cuda.CUDAGraph()
                opt.zero_grad(set_to_none=True)
                with torch.cuda.graph(gr):
                    E = loss_fn(net(Xs[k], Ps[k]), Ys[k])
                    E.backward()
                    opt.step()
                graphs.append(gr)
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(a.steps):
            if graphs is not None:
                graphs[i % a.num_batches].replay()
            else:
                step(a.warmup + i)
        torch.cuda.synchronize()
        us = (time.perf_counter() - t0) / a.steps * 1e6
        errs = None
        if kind == "collection":
            errs = holder._tset.read_errors()
        elif kind == "list":
            errs = 0
            for m in holder:
                errs |= m._tset.read_errors()
        del net, opt, holder, graphs
        torch.cuda.empty_cache()
        return us, launches, errs

    us, launches, errs = timed(a.dropin_form, a.graph)
    ref_us, ref_launches, _ = timed("torch", False)
    line = {
        "metric": "DLRM QAT-step samples/sec, 1 GPU (config 3: bottom/top MLP, dot interaction, 26 INT4 "
                  "fake-quant EmbeddingBag tables, BCE, backward, SGD lr %g)" % a.lr,
        "value": round(B * a.steps / (us * 1e-6 * a.steps), 1) if not errs else None,
        "unit": "samples/s", "n_gpus": 1, "steps": a.steps, "warmup": a.warmup,
        "ms_per_step": round(us / 1e3, 4), "us_per_step": round(us, 2), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f32 (int4 fake-quant embeddings, fp32 MLP)",
        "data": "synthetic (uniform-random Criteo-form indices, U[0,1) dense features, Bernoulli labels)",
        "config": {"workload": f"criteo-{a.config} DLRM QAT step ({a.dropin_form}, {gm})", "tables": T,
                   "total_rows": sum(rows), "emb_dim": D, "batch_per_gpu": B, "mlp_bot": bot, "mlp_top": top,
                   "interaction": "dot", "loss": "BCE", "optimizer": "SGD lr %g" % a.lr,
                   "hip_graph": a.graph, "parallelism": "dp1"},
        "launches_per_step": launches,
        "torch_gpu_reference": {"us_per_step": round(ref_us, 2), "launches_per_step": ref_launches,
                                "speedup": round(ref_us / us, 2),
                                "what": "the same model and step with the reference's embedding modules as "
                                        "PyTorch ops on this GPU (nn.EmbeddingBag sparse + per-step full-table "
                                        "aminmax scale + fake-quant STE, torch.optim.SGD), eager"},
        "reference_published": "27.6 ms/it on 1x A5000 (bash_scripts/Kaggle/emb_bit_4.txt:49-50; other "
                               "hardware, loss copied to host every step: context only)",
        "device_errors": errs,
    }
    print(json.dumps(line), flush=True)


def torch_reference_gpu(a, rows, D, B, dev, batches, dys, dp, steps=30):
    """The reference's own step as PyTorch ops on this GPU at the drop-in's shape (what a user
    of the reference runs on MI355X without this package): per table nn.EmbeddingBag(mode="sum",
    sparse=True), the full-table aminmax scale every forward (quant_utils.py:141-194), fake
    quant + dequant with the STE backward (_FakeQuantSTE); autograd; then torch.optim.SGD's
    sparse step (single GPU) or quantize_emb_grad at one rank + W.add_ (s_q_g_p_c.py:850-890,
    601-628). Returns us per step (host work included, as the drop-in line)."""
    T = len(rows)
    embs = []
    for n in rows:
        w = torch.empty(n, D, device=dev).uniform_(-float(np.sqrt(1 / n)), float(np.sqrt(1 / n)))
        embs.append(torch.nn.EmbeddingBag(n, D, mode="sum", sparse=True, _weight=w))
    off = torch.arange(B, dtype=torch.int64, device=dev)
    opt = None if dp else torch.optim.SGD([e.weight for e in embs], lr=a.lr)

    def step(i):
        P = batches[i % len(batches)].idx.view(T, B)
        ys = []
        for t, e in enumerate(embs):
            with torch.no_grad():
                mn, mx = torch.aminmax(e.weight)
                s = torch.clamp(torch.maximum(mn.abs(), mx.abs()), min=1e-8) / 7.0
            ys.append(_FakeQuantSTE.apply(e(P[t], off), s, 4))
        torch.autograd.backward(ys, dys)
        if opt is not None:
            opt.step()
            opt.zero_grad(set_to_none=True)
            return
        with torch.no_grad():
            for e in embs:
                gc = e.weight.grad.coalesce()
                v = gc.values()
                sg = torch.clamp(v.abs().max(), min=1e-8) / 127.0
                q = torch.clamp(torch.round(1.0 / sg * v), -128, 127)
                e.weight.add_(torch.sparse_coo_tensor(gc.indices(), q * sg, gc.shape), alpha=-a.lr)
                e.weight.grad = None

    for i in range(5):
        step(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        step(5 + i)
    torch.cuda.synchronize()
    us = (time.perf_counter() - t0) / steps * 1e6
    del embs, opt
    torch.cuda.empty_cache()
    return us


def gather_phase(a, ts, rows, T, D, dev):
    """INT4 packed-gather bandwidth phase (north-star gather metric), outside the timed step."""
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
    per = D // 2 + 8 + D * 4  # packed row + int64 index + f32 output row (offsets unread, pooling 1)
    g_bytes = T * Bg * per + T * 4
    g_gbs = g_bytes / (g_ms * 1e-3) / 1e9
    return {"kernel": "k_emb_fwd_packed (INT4 rows, pooling 1)", "bags_per_table": Bg, "ms": round(g_ms, 4),
            "alg_bytes": g_bytes, "GBps": round(g_gbs, 1), "frac_of_peak": round(g_gbs / HBM_PEAK_GBS, 4),
            "bytes_per_lookup": per}


def dense_phase(a, dev, world, rank, coll=False):
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
            lin = torch.nn.Linear(i, o).to(dev)
            lin.weight.grad = torch.randn(o, i, device=dev, generator=g) * 1e-3
            lin.bias.grad = torch.randn(o, device=dev, generator=g) * 1e-3
            layers.append(lin)
    ex = DenseGradExchange(layers, grad_bits=8, force_collectives=coll)
    P = ex.channels.total_elems
    wire_b = ex.wire.element_size()
    with torch.no_grad():
        for _ in range(5):
            ex.exchange()
            ex.apply(1e-6)
        if coll:
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
            "GBps": round(alg / (ms * 1e-3) / 1e9, 1), "launches": 4, "collectives": 2 if ex.coll else 0,
            "note": "median of per-iteration HIP events; exchange+apply of all layers"}


class _FakeQuantSTE(torch.autograd.Function):
    """SymmetricQuantFunction (quant_utils.py:316-363) followed by the dequant
    (q_m_n_q_g.py:393): q = clamp(round(1/s * x + 0)), y = q * s; backward (g * s) / s."""

    @staticmethod
    def forward(ctx, x, s, bits):
        ctx.s = s
        n = 2 ** (bits - 1) - 1
        return torch.clamp(torch.round(1.0 / s * x + 0), -n - 1, n) * s

    @staticmethod
    def backward(ctx, g):
        return (g * ctx.s) / ctx.s, None, None


def cpu_threads() -> int:
    """Host threads this process may use: OMP_NUM_THREADS (16 on the GPU box, its CPU
    share) when set, else every CPU."""
    return int(os.environ.get("OMP_NUM_THREADS") or os.cpu_count() or 1)


def cpu_baseline_torch(a, B, rows_override=None):
    """The reference's step in PyTorch on the host CPU, on a bounded sample: per step and
    table, the full-table min/max scale (quant_utils.py:141-194), nn.EmbeddingBag(mode="sum",
    sparse=True) forward, fake quant + dequant with the STE backward, autograd to the sparse
    COO grad; then --mode dp: quantize_emb_grad at one rank (coalesce, max|g|/127 scale,
    round/clamp, s_q_g_p_c.py:850-890) and W.add_(-lr * grad * scale) (:601-628); --mode
    sgd: torch.optim.SGD's sparse step; --mode fwd: the forward alone. kind "port": the
    reference itself may not be run here."""
    torch.set_num_threads(cpu_threads())
    cores = torch.get_num_threads()
    tables = CPU_TABLES[a.config]
    rows, D = (rows_override, _CONFIGS[tables][1]) if rows_override else _CONFIGS[tables]
    T = len(rows)
    g = torch.Generator().manual_seed(a.seed)
    t_init = time.perf_counter()
    embs = []
    tile = torch.empty(1 << 18, D).uniform_(-1.0, 1.0, generator=g)  # CPU RNG is one thread: tile it
    for n in rows:
        w = torch.empty(n, D)
        for r0 in range(0, n, tile.shape[0]):
            k = min(tile.shape[0], n - r0)
            torch.mul(tile[:k], float(np.sqrt(1 / n)), out=w[r0:r0 + k])
        embs.append(torch.nn.EmbeddingBag(n, D, mode="sum", sparse=True, _weight=w))
    init_s = time.perf_counter() - t_init
    off = torch.arange(B, dtype=torch.int64)
    opt = torch.optim.SGD([e.weight for e in embs], lr=a.lr) if a.mode == "sgd" else None
    steps, t0 = 0, time.perf_counter()
    while True:
        idx = [torch.randint(0, n, (B,), generator=g) for n in rows]
        ys = []
        for t, e in enumerate(embs):
            with torch.no_grad():
                mn, mx = torch.aminmax(e.weight)
                s = torch.clamp(torch.maximum(mn.abs(), mx.abs()), min=1e-8) / 7.0
            ys.append(_FakeQuantSTE.apply(e(idx[t], off), s, 4))
        if a.mode != "fwd":
            torch.autograd.backward(ys, [torch.full_like(y, 1e-3) for y in ys])
            if opt is not None:
                opt.step()
                opt.zero_grad(set_to_none=True)
            else:
                with torch.no_grad():
                    for e in embs:
                        gc = e.weight.grad.coalesce()
                        v = gc.values()
                        sg = torch.clamp(v.abs().max(), min=1e-8) / 127.0
                        q = torch.clamp(torch.round(1.0 / sg * v), -128, 127)
                        e.weight.add_(torch.sparse_coo_tensor(gc.indices(), q * sg, gc.shape), alpha=-a.lr)
                        e.weight.grad = None
        steps += 1
        el = time.perf_counter() - t0
        if el > a.cpu_seconds or steps >= 500:
            break
    gb = sum(rows) * D * 4 / 1e9
    return {"value": round(steps * B / el, 1), "unit": "samples/s", "cores": cores, "kind": "port",
            "sample": f"{steps} {a.mode} steps of B={B}: the reference's op sequence in PyTorch-CPU "
                      f"({cores} threads) on the '{tables}' tables ({sum(rows):,} rows x {D}, {gb:.1f} GB"
                      + (", standing in for the 773 M-row GPU workload" if a.config == "terabyte" else "")
                      + f"); table init {init_s:.1f} s untimed"}


def cpu_baseline_oracle(a, B):
    """Secondary figure: the oracle's C restatement (test infrastructure, one thread) on
    tables capped at 1 M rows, a few seconds of dp steps."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O

    O.build()
    rows, D = _CONFIGS[CPU_TABLES[a.config]]
    cap_rows = [min(n, 1_000_000) for n in rows]
    rs = np.random.RandomState(a.seed)
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
        if el > a.cpu_seconds / 3 or steps >= 50:
            break
    return {"value": round(steps * B / el, 1), "unit": "samples/s", "cores": 1, "kind": "port",
            "sample": f"{steps} dp steps, B={B}, {T} tables capped at 1M rows (D={D}), oracle C restatement, "
                      "1 thread"}


if __name__ == "__main__":
    main()
