import json, os, sys
import numpy as np
import torch
ROOT = os.environ["GRAFT_REPO_ROOT"] if "GRAFT_REPO_ROOT" in os.environ else "/root/repo"
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "tests", "golden"), ROOT]
import gen_inputs as G
import deep_quantized_recommendation_model_dqrm_amd as dq
from deep_quantized_recommendation_model_dqrm_amd import _lib as L
from deep_quantized_recommendation_model_dqrm_amd.comm import HipExchangeKernels
D, B, dist = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
rows = [3, 200, 1435, 500, 2_000_000, 800_000, 40_000, 7112, 9_000_000, 100]
T = len(rows)
sets = [dq.EmbeddingTableSet(rows, D, device="cuda", init="uniform", seed=7) for _ in range(2)]
s_avg = [torch.zeros(T, dtype=torch.float32, device="cuda") for _ in range(2)]
P = G.pooling_one(rows, B, 70, dist=dist)
dy = torch.from_numpy(G.upstream_grad(T, B, D, 80) * 30).cuda()
b = dq.LookupBatch.pooling_one(torch.from_numpy(P).cuda())
for j, ts in enumerate(sets):
    ts.forward(b)
    ws = dq.CoalescedGrad.allocate(rows, B, D, "cuda")
    if j == 0:
        ts.backward_apply_local(b, dy, ws, 8, s_avg[0], 0.5)
    else:
        ts.backward_coalesce(b, dy, ws)
        HipExchangeKernels(ts).apply_local(ws, 8, s_avg[1], 0.5, False)
e0 = sets[0].read_errors()
out = {"D": D, "dist": dist, "err": e0, "savg_eq": bool(torch.equal(s_avg[0], s_avg[1]))}
bad = {}
for t in range(T):
    a, c = sets[0].table_weight(t), sets[1].table_weight(t)
    d = (a != c).any(dim=1).nonzero().flatten().cpu().numpy()
    if d.size:
        nblk = (rows[t] + 255) // 256
        slots = sorted(set(int(np.searchsorted([nblk * s // 8 * 256 for s in range(1, 9)], r, side="right")) for r in d))
        bad[t] = {"nrows_bad": int(d.size), "slots": slots, "first": d[:5].tolist()}
out["bad"] = bad
print(json.dumps(out))
