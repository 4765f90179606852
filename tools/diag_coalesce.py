"""Per-phase wall-clock breakdown of the Criteo-form coalesce kernel (k_coalesce_p1) on the
diagnostic build (tools/build_diag_coal.sh). Stamps: 0 start, 1 indices landed, 2 slot
compacted, 3 sorted, 4 heads, 5 stage landed, 6 segments done (stores issued), 7 end (a
table's slowest workgroup over its slots and, in the one-launch step, sub-slots); with
"apply" (the one-launch local step, dqrm_emb_bwd_apply_local): 11 the table's workgroups
met, 16 every load landed (the W prefetch), 14 prefetched rows updated, 15 all rows
updated, 12 owned blocks re-reduced, 13 end (after the table's last-workgroup finalize);
with "applyfwd" (dqrm_emb_bwd_apply_fwd_local: the next batch's forward in the same launch)
also 18, the workgroup's forward share done.
usage: python tools/diag_coalesce.py [terabyte|terabyte_ref|kaggle] [B] [apply|applyfwd]"""
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
APPLY = len(sys.argv) > 3 and sys.argv[3] in ("apply", "applyfwd")
FWD = len(sys.argv) > 3 and sys.argv[3] == "applyfwd"
rows, D = CONFIGS[cfg]
T = len(rows)
lib = L.load()
lib.dqrm_diag_coal_read.argtypes = [C.c_void_p, C.c_int]
ts = dq.EmbeddingTableSet(rows, D, device="cuda", init="uniform", seed=3)
g = torch.Generator(device="cuda").manual_seed(5)
NS = 32  # stamp slots per workgroup (dqrm_coalesce.hip g_coal_clk)
STE = os.environ.get("DIAG_STE", "1") != "0"  # DIAG_STE=0: without the STE division (a what-if, not the path)
NB = 8  # distinct resident batches cycled, as bench.py (cold rows and translations every launch)
bs = [dq.LookupBatch.pooling_one(torch.stack([torch.randint(0, n, (B,), generator=g, device="cuda") for n in rows]))
      for _ in range(NB)]
dy = torch.randn(T, B, D, device="cuda", generator=g) * 0.05
ws = dq.CoalescedGrad.allocate(rows, B, D, "cuda")
s_avg = torch.zeros(T, device="cuda")
y = torch.empty(T, B, D, device="cuda")


def run(i):
    b = bs[i % NB]
    if FWD:  # this batch's forward ran in the previous launch
        ts.backward_apply_forward_local(b, dy, ws, 8, s_avg, 0.01, bs[(i + 1) % NB], ste=STE, out=y)
    elif APPLY:
        ts.forward(b)
        ts.backward_apply_local(b, dy, ws, 8, s_avg, 0.01, ste=STE)
    else:
        ts.backward_coalesce(b, dy, ws)


ts.forward(bs[0])
for i in range(3 * NB):
    run(i)
torch.cuda.synchronize()
cs = []
for i in range(NB):  # one launch per batch, read after each
    buf = np.zeros(2 * T * 8 * NS, dtype=np.uint64)
    run(i)
    lib.dqrm_diag_coal_read(buf.ctypes.data, buf.size)
    # rows: sub-slot 0 of every (table, slot), then sub-slot 1 (the spare groups of the
    # one-launch step); per table 16 "slots": 0-7 sub-slot 0, 8-15 sub-slot 1
    c = buf.reshape(2, T, 8, NS).transpose(1, 0, 2, 3).reshape(T, 16, NS).astype(np.int64)
    k0 = c[:, :, 0][c[:, :, 0] > 0].min()
    c = np.where(c >= k0, c - k0, -1)  # -1: not stamped in this launch
    cs.append(c)
end = 18 if FWD else 13 if APPLY else 7
spans = [c[:, :, end].max() / 100 for c in cs]
print(f"{cfg} B={B} D={D}: span median {np.median(spans):.1f} us over {NB} launches (min {min(spans):.1f}, "
      f"max {max(spans):.1f}), each on a batch not used in the previous {NB - 1}")
print("per table, slowest slot, median over launches (us): start | idx | compact | sort | heads | land | segs | tail || end")


def slow(c, t, k):
    return c[t, int(np.argmax(c[t, :, k]))]


order = np.argsort(-np.median([c[:, :, 7].max(axis=1) for c in cs], axis=0))
for t in order:
    ps = [slow(c, t, 7) for c in cs]
    if ps[0][2] < 0:
        print(f"t{t:2d} n={rows[t]:>10d}: inactive")
        continue
    ph = np.median([[p[0]] + [p[i + 1] - p[i] for i in range(7)] for p in ps], axis=0)
    print(f"t{t:2d} n={rows[t]:>10d}: " + " ".join(f"{x / 100:5.1f}" for x in ph)
          + f" || {np.median([p[7] for p in ps]) / 100:5.1f}")
sub = [(c[t, s, 8] - c[t, s, 1], c[t, s, 9] - c[t, s, 8], c[t, s, 10] - c[t, s, 9], c[t, s, 2] - c[t, s, 10])
       for c in cs for t in range(T) for s in range(16) if c[t, s, 2] >= 0 and c[t, s, 10] >= 0]
sub = np.array(sub) / 100
print("compact split (median us): idx-wait %.2f  compaction %.2f  report+barrier %.2f  prefetch-issue %.2f" %
      tuple(np.median(sub, axis=0)))
lw = [(c[t, s, 17] - c[t, s, 4], c[t, s, 5] - c[t, s, 17]) for c in cs for t in range(T) for s in range(16)
      if c[t, s, 17] >= 0 and c[t, s, 4] >= 0 and c[t, s, 5] >= 0]
if lw:
    lw = np.array(lw) / 100
    print("land split (median us): dy prefetch still in flight after the heads %.2f  landing + W issue %.2f" %
          tuple(np.median(lw, axis=0)))
if APPLY:
    print("apply phases per table, slowest slot, median (us): segments done->met (incl. the wait) | "
          "met->updated | updated->end || end")
    for t in np.argsort(-np.median([c[:, :, 13].max(axis=1) for c in cs], axis=0)):
        ps = [slow(c, t, 13) for c in cs]
        if ps[0][11] < 0:
            continue
        ph = np.median([[p[11] - p[6], p[12] - p[11], p[13] - p[12], p[13], p[16] - p[11], p[14] - p[16],
                         p[15] - p[14], p[12] - p[15]] for p in ps], axis=0) / 100
        print(f"t{t:2d} n={rows[t]:>10d}: {ph[0]:5.1f} {ph[1]:5.1f} {ph[2]:5.1f} || {ph[3]:5.1f}   "
              f"(updated = W landed {ph[4]:4.1f} | prefetched rows {ph[5]:4.1f} | rest+barrier {ph[6]:4.1f} | "
              f"re-reduce {ph[7]:4.1f})")
if FWD:
    print("next-batch forward per table, slowest workgroup, median (us): finalize end -> forward done "
          "(= lists | final max seen | first rows landed (wave 0) | rest + stores) || end")
    for t in np.argsort(-np.median([c[:, :, 18].max(axis=1) for c in cs], axis=0)):
        ps = [slow(c, t, 18) for c in cs]
        ph = np.median([[p[18] - max(p[13], 0), p[20] - p[13], p[19] - p[20], p[21] - p[19], p[18] - p[21], p[18]]
                        for p in ps], axis=0) / 100
        print(f"t{t:2d} n={rows[t]:>10d}: {ph[0]:5.1f} (= {ph[1]:4.1f} | {ph[2]:4.1f} | {ph[3]:4.1f} | {ph[4]:4.1f}) "
              f"|| {ph[5]:5.1f}")
    w13 = [c[t, s, 13] for c in cs for t in range(T) for s in range(16) if c[t, s, 13] >= 0]
    print("table last-arrival spread: see 'apply phases' ends above; workgroups stamped:", len(w13))
print("errors", ts.read_errors())
