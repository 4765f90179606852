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


def test_pmc_traffic_reads_committed_summary(bench):
    path = os.path.join(ROOT, "profiles", "r1_tb_summary.json")
    if not os.path.exists(path):
        pytest.skip("no committed TB PMC summary")
    t = bench.pmc_traffic(path, "bwd_coalesce", 64)
    assert t is not None and t["bytes"] > 0 and t["profiled_avg_us"] > 0
    assert t["source"] == os.path.join("profiles", "r1_tb_summary.json")
    assert bench.pmc_traffic(os.path.join(ROOT, "profiles", "missing.json"), "bwd_coalesce", 64) is None
    assert bench.pmc_traffic(None, "bwd_coalesce", 64) is None


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
