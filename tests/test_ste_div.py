"""The STE division the HIP kernels use (csrc/dqrm_internal.h SteDiv: reciprocal, two fma
residual corrections) equals the IEEE division (g*s)/s of quant_utils.py:349-363 bit for
bit on its fast range. Host-side check of the same arithmetic in C (gcc, no contraction),
over random and structured significands; the GPU parity tests cover the kernels."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc not available")
def test_ste_division_matches_ieee(tmp_path):
    exe = str(tmp_path / "ste_div_check")
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", os.path.join(HERE, "native", "ste_div_check.c"),
                    "-o", exe, "-lm"], check=True)
    for seed in (1, 2, 3):
        out = subprocess.run([exe, "4000000", str(seed)], check=True, capture_output=True, text=True).stdout
        assert out.strip().splitlines()[-1] == "0", out
