"""GPU: the one-launch local step (dqrm_emb_bwd_apply_local) when its workgroups do NOT all
meet at the rendezvous. Its table's workgroups wait for each other's gradient maxima; if one
gives up (DQRM_ERRF_STALL: another stream held CUs, so not every workgroup was resident) its
rows must still be applied -- by the table's last-arriving workgroup, which has every slot's
maximum -- so a table is updated completely, never half.

The stall is forced: DQRM_STALL_SPIN=0 (read once per process, hence a child process) makes a
workgroup give up after its second poll, so most tables see stalls in every step. W, the |W|
hierarchy and the averaged scales must equal the two-launch path (dqrm_emb_bwd_coalesce +
dqrm_apply_local) bit for bit, and the flag must be raised.
Reference step: sgd_quantized_gradients_parallel_comm.py:601-628 (with :850-890 at N = 1)."""
import json
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)

CHILD = r"""
import json, sys
import numpy as np
import torch
sys.path[:0] = [{here!r}, {golden!r}, {root!r}]
import gen_inputs as G
import deep_quantized_recommendation_model_dqrm_amd as dq
from deep_quantized_recommendation_model_dqrm_amd import _lib as L
from deep_quantized_recommendation_model_dqrm_amd.comm import HipExchangeKernels
rows, D, B, steps = {rows!r}, {D}, {B}, 3
T = len(rows)
sets = [dq.EmbeddingTableSet(rows, D, device="cuda", init="uniform", seed=7) for _ in range(2)]
s_avg = [torch.zeros(T, dtype=torch.float32, device="cuda") for _ in range(2)]
flags = 0
for it in range(steps):
    P = G.pooling_one(rows, B, 70 + it, dist={dist!r})
    dy = torch.from_numpy(G.upstream_grad(T, B, D, 80 + it) * 30).cuda()
    b = dq.LookupBatch.pooling_one(torch.from_numpy(P).cuda())
    assert sets[0].apply_local_is_one_launch(b)
    for j, ts in enumerate(sets):
        ts.forward(b)
        ws = dq.CoalescedGrad.allocate(rows, B, D, "cuda")
        if j == 0:
            ts.backward_apply_local(b, dy, ws, 8, s_avg[0], 0.5)
        else:
            ts.backward_coalesce(b, dy, ws)
            HipExchangeKernels(ts).apply_local(ws, 8, s_avg[1], 0.5, False)
    e0, e1 = sets[0].read_errors(), sets[1].read_errors()
    assert e1 == 0 and (e0 & ~L.DQRM_ERRF_STALL) == 0, (e0, e1)
    flags += 1 if e0 & L.DQRM_ERRF_STALL else 0
    assert torch.equal(s_avg[0], s_avg[1]), it
    for name in ("W", "rowmax", "blkmax", "sblkmax", "tmax"):
        assert torch.equal(getattr(sets[0], name), getattr(sets[1], name)), (it, name)
inc = [x.clone() for x in (sets[0].rowmax, sets[0].blkmax, sets[0].sblkmax, sets[0].tmax)]
sets[0].refresh_absmax()
for x, y in zip(inc, (sets[0].rowmax, sets[0].blkmax, sets[0].sblkmax, sets[0].tmax)):
    assert torch.equal(x, y)
print(json.dumps({{"stalled_steps": flags}}))
"""


CHILD_FWD = r"""
import json, sys
import numpy as np
import torch
sys.path[:0] = [{here!r}, {golden!r}, {root!r}]
import gen_inputs as G
import deep_quantized_recommendation_model_dqrm_amd as dq
from deep_quantized_recommendation_model_dqrm_amd import _lib as L
from deep_quantized_recommendation_model_dqrm_amd.comm import HipExchangeKernels
rows, D, B, steps = {rows!r}, {D}, {B}, 3
T = len(rows)
sets = [dq.EmbeddingTableSet(rows, D, device="cuda", init="uniform", seed=7) for _ in range(2)]
s_avg = [torch.zeros(T, dtype=torch.float32, device="cuda") for _ in range(2)]
bs = [dq.LookupBatch.pooling_one(torch.from_numpy(G.pooling_one(rows, B, 70 + k, dist={dist!r})).cuda())
      for k in range(steps + 1)]
assert sets[0].apply_fwd_local_is_one_launch(bs[0], bs[1])
for ts in sets:
    ts.forward(bs[0])
flags = 0
for it in range(steps):
    dy = torch.from_numpy(G.upstream_grad(T, B, D, 80 + it) * 30).cuda()
    ws = [dq.CoalescedGrad.allocate(rows, B, D, "cuda") for _ in range(2)]
    y0 = sets[0].backward_apply_forward_local(bs[it], dy, ws[0], 8, s_avg[0], 0.5, bs[it + 1])
    sets[1].backward_coalesce(bs[it], dy, ws[1])  # the two-launch path (no rendezvous to stall)
    HipExchangeKernels(sets[1]).apply_local(ws[1], 8, s_avg[1], 0.5, False)
    y1 = sets[1].forward(bs[it + 1])
    e0, e1 = sets[0].read_errors(), sets[1].read_errors()
    assert e1 == 0 and (e0 & ~L.DQRM_ERRF_STALL) == 0, (e0, e1)
    flags += 1 if e0 & L.DQRM_ERRF_STALL else 0
    assert torch.equal(y0, y1), it
    assert torch.equal(s_avg[0], s_avg[1]), it
    for name in ("W", "rowmax", "blkmax", "sblkmax", "tmax", "scale"):
        assert torch.equal(getattr(sets[0], name), getattr(sets[1], name)), (it, name)
print(json.dumps({{"stalled_steps": flags}}))
"""


@pytest.mark.parametrize("D,B,dist", [(64, 2048, "uniform"), (16, 2048, "zipf")])
def test_forced_stalls_fused_next_forward(D, B, dist):
    """The same forced stalls with the next batch's forward inside the launch
    (dqrm_emb_bwd_apply_fwd_local): a stalled workgroup's forward share is the last
    arriver's, which applied its rows; the outputs equal the separate forward's bit for bit."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    rows = [3, 200, 1435, 500, 2_000_000, 800_000, 40_000, 7112, 9_000_000, 100]
    code = CHILD_FWD.format(here=HERE, golden=os.path.join(HERE, "golden"), root=ROOT, rows=rows, D=D, B=B,
                            dist=dist)
    env = dict(os.environ, DQRM_STALL_SPIN="0")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["stalled_steps"] >= 1


@pytest.mark.parametrize("D,B,dist", [(64, 2048, "uniform"), (16, 2048, "zipf"), (32, 1000, "uniform")])
def test_forced_stalls_apply_every_row(D, B, dist):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    # row-split tables with and without sub-slots (T = 10: 54 spare workgroups), dimension-split
    # tables (3 / 200 / 1435 rows), a 2-block table
    rows = [3, 200, 1435, 500, 2_000_000, 800_000, 40_000, 7112, 9_000_000, 100]
    code = CHILD.format(here=HERE, golden=os.path.join(HERE, "golden"), root=ROOT, rows=rows, D=D, B=B, dist=dist)
    env = dict(os.environ, DQRM_STALL_SPIN="0")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["stalled_steps"] >= 1  # the recovery path ran (and the results above are exact)
