"""Host-side checks of bench.py's contract (no GPU): workload shapes, the PMC traffic lookup
that feeds roofline.traffic, and the N>1 launch guard (N>1 only under torch.distributed.run)."""
import importlib.util
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def bench():
    spec = importlib.util.spec_from_file_location("dqrm_bench", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_workload_shapes(bench):
    tb, ref, kg = (bench.CONFIGS[k] for k in ("terabyte", "terabyte_ref", "kaggle"))
    assert len(tb["rows"]) == len(ref["rows"]) == len(kg["rows"]) == 26
    assert tb["dim"] == ref["dim"] == 64 and kg["dim"] == 16
    assert sum(tb["rows"]) == 773_280_534  # the N=1 workload named in DESIGN.md §7
    # the scaled profile multiplies exactly the >=1M-row tables of the reference TB run
    for a, b in zip(tb["rows"], ref["rows"]):
        assert a == (b * 16 if b >= 1_000_000 else b)
    for name, (bot, top) in bench.MLPS.items():
        D, T = bench.CONFIGS[name]["dim"], 26
        assert bot[0] == 13 and bot[-1] == D and top[-1] == 1
        assert top[0] == D + T * (T + 1) // 2


def test_pmc_traffic_lookup(bench, tmp_path):
    """roofline.traffic comes from a tools/prof_summary.py summary: the phase's kernel is
    matched by its template prefix (LPR = D/4), absent files or kernels give None."""
    summ = {"kernels": {
        "k_bwd_fused<16, 1>(FArgs)": {"avg_us": 25.5, "hbm_bytes_per_launch": 4.5e7},
        "k_bwd_fused<16, 0>(FArgs)": {"avg_us": 50.0, "hbm_bytes_per_launch": 9.0e7},
        "k_emb_fwd<4, 2>(FwdArgs)": {"avg_us": 9.0, "hbm_bytes_per_launch": None},
    }}
    path = tmp_path / "s.json"
    path.write_text(json.dumps(summ))
    t = bench.pmc_traffic(str(path), "bwd_coalesce", 64)
    assert t["bytes"] == 45_000_000 and t["profiled_avg_us"] == 25.5
    assert bench.pmc_traffic(str(path), "bwd_sgd", 64)["bytes"] == 90_000_000
    assert bench.pmc_traffic(str(path), "bwd_coalesce", 16) is None  # LPR 4 not profiled
    assert bench.pmc_traffic(str(path), "emb_fwd", 16) is None  # no PMC pass for it
    assert bench.pmc_traffic(str(tmp_path / "missing.json"), "bwd_coalesce", 64) is None
    assert bench.pmc_traffic(None, "bwd_coalesce", 64) is None
    summ["kernels"]["k_coalesce_p1(CoalesceArgs)"] = {"avg_us": 23.6, "hbm_bytes_per_launch": 2.3e7}
    path.write_text(json.dumps(summ))  # the Criteo-form coalesce kernel is found first
    assert bench.pmc_traffic(str(path), "bwd_coalesce", 64)["bytes"] == 23_000_000
    wl = {"config": "terabyte", "mode": "dp", "batch_per_gpu": 2048, "n1_update": "x", "index_dist": "uniform"}
    assert bench.pmc_traffic(str(path), "bwd_coalesce", 64, wl) is None  # no workload recorded: refused
    summ["workload"] = dict(wl)
    path.write_text(json.dumps(summ))
    assert bench.pmc_traffic(str(path), "bwd_coalesce", 64, wl)["bytes"] == 23_000_000
    assert bench.pmc_traffic(str(path), "bwd_coalesce", 64, dict(wl, batch_per_gpu=128)) is None  # other batch
    for name in sorted(os.listdir(os.path.join(ROOT, "profiles"))):  # committed summaries parse
        if name.startswith("r2_") and name.endswith("_summary.json"):
            for ph in bench.KERNEL_SYMBOL:
                bench.pmc_traffic(os.path.join(ROOT, "profiles", name), ph, 64)


def test_alg_bytes_pooling_one_reads_no_offsets(bench):
    T, B, D, U = 26, 2048, 64, 40000
    L = T * B
    assert bench.alg_bytes("bwd_coalesce", T, B, D, U) == L * 8 + L * D * 4 + U * (D * 4 + 4)
    assert bench.alg_bytes("bwd_coalesce", T, B, D, U, pool1=False) - bench.alg_bytes(
        "bwd_coalesce", T, B, D, U) == T * B * 8
    assert bench.alg_bytes("emb_fwd_packed", T, B, D, U) == L * (D // 2 + 8) + L * D * 4 + T * 4
    assert bench.alg_bytes("apply_local", T, B, D, U, repack=True) - bench.alg_bytes(
        "apply_local", T, B, D, U) == U * D // 2
    assert bench.alg_bytes("apply_sparse_update", T, B, D, U, world=8) > bench.alg_bytes(
        "apply_sparse_update", T, B, D, U, world=1)
    assert set(bench.KERNEL_SYMBOL) >= {n for m in ("dp", "fwd", "sgd") for f in (True, False)
                                        for n in bench.phase_names(m, f, f)}


def test_phase_names(bench):
    assert bench.phase_names("fwd", False, True) == ["emb_fwd"]
    assert bench.phase_names("sgd", True, True) == ["emb_fwd_packed", "bwd_sgd"]
    assert bench.phase_names("dp", False, True) == ["emb_fwd", "bwd_coalesce", "apply_local"]
    assert bench.phase_names("dp", False, False) == ["emb_fwd", "bwd_coalesce", "grad_quant_pack",
                                                     "apply_sparse_update"]
    assert bench.phase_names("dp", False, True, True) == ["emb_fwd", "bwd_apply_local"]
    # the step boundary in one launch: the update of step i and the forward of step i+1
    assert bench.phase_names("dp", False, True, True, True) == ["bwd_apply_fwd_local"]
    T, B, D, U = 26, 2048, 64, 40000
    assert bench.alg_bytes("bwd_apply_fwd_local", T, B, D, U) == (bench.alg_bytes("bwd_apply_local", T, B, D, U)
                                                                  + bench.alg_bytes("emb_fwd", T, B, D, U))
    assert "bwd_apply_fwd_local" in bench.KERNEL_SYMBOL
    assert bench.phase_names("sgd", False, True, False, True) == ["bwd_sgd_fwd"]
    assert bench.alg_bytes("bwd_sgd_fwd", T, B, D, U) == (bench.alg_bytes("bwd_sgd", T, B, D, U)
                                                          + bench.alg_bytes("emb_fwd", T, B, D, U))


@pytest.mark.parametrize("mode", ["dp", "sgd", "fwd"])
def test_cpu_baseline_torch_runs(bench, mode):
    """The PyTorch-CPU restatement of the reference step runs on small tables and reports
    the threads it used."""
    a = bench.parse(["--mode", mode, "--cpu-seconds", "0.2", "--config", "kaggle"])
    r = bench.cpu_baseline_torch(a, 64, rows_override=[100, 7, 3000])
    assert r["value"] > 0 and r["cores"] == bench.cpu_threads() and r["kind"] == "port"
    assert r["unit"] == "samples/s" and mode in r["sample"]


def test_fake_quant_ste_matches_reference_form(bench):
    import torch

    x = torch.tensor([0.0, 0.05, -0.3, 1.0, -1.0, 0.149], requires_grad=True)
    s = torch.tensor(0.1)
    y = bench._FakeQuantSTE.apply(x, s, 4)
    assert torch.equal(y, torch.clamp(torch.round(1.0 / s * x.detach()), -8, 7) * s)
    y.backward(torch.full_like(y, 0.3))
    assert torch.equal(x.grad, (torch.full_like(y, 0.3) * s) / s)


def test_committed_bench_line_fields():
    path = os.path.join(ROOT, "profiles", "r1_bench_tb_v6.json")
    if not os.path.exists(path):
        pytest.skip("no committed bench line")
    line = json.loads(open(path).read().strip().splitlines()[-1])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in line, k
    r = line["roofline"]
    assert r["bound"] == "hbm" and r["unit"] == "GB/s" and r["peak"] == 8000.0
    assert abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-3
    assert line["cpu_baseline"]["kind"] in ("port", "reference") and line["cpu_baseline"]["cores"] >= 1
    assert line["n_gpus"] == 1 and line["config"]["workload"]


def test_multi_gpu_needs_distributed_launcher():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 2 and "torch.distributed.run" in p.stderr


def test_bench_rejects_inconsistent_flags():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--use-packed"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 2 and "--scale-period" in p.stderr


def test_dlrm_net_shapes_cpu(bench):
    """config 3's model (mode dlrm): the Kaggle MLPs, 26 pooled vectors and the dot
    interaction's 351 pairs give the top MLP its 367 inputs; BCE backward reaches every
    MLP parameter and the embedding tables' sparse grads."""
    import torch

    bot, top = bench.MLPS["kaggle"]
    rows = [50 + 3 * t for t in range(26)]
    emb = bench._RefEmb(rows, 16, torch.device("cpu"))
    net = bench.DLRMNet(bot, top, emb, 0)
    B = 8
    X = torch.rand(B, 13)
    P = torch.stack([torch.randint(0, n, (B,)) for n in rows])
    p = net(X, P)
    assert p.shape == (B, 1) and bool(((p > 0) & (p < 1)).all())
    assert net.top_l[0].in_features == 367
    torch.nn.BCELoss()(p, torch.ones(B, 1)).backward()
    assert all(q.grad is not None for q in net.bot_l.parameters())
    assert all(b.weight.grad is not None and b.weight.grad.is_sparse for b in emb.bags)
