"""The driver's build check, end to end on the CPU: __graft_entry__.build() compiles what is
stale (hipcc cross-compiles gfx950 here), relinks libdqrm.so, builds the oracle's C checker
and loads the library, whose ABI version must equal include/dqrm.h's and _lib.py's. Run in a
fresh interpreter so a library already loaded by another test cannot mask a stale build."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_graft_entry_build_end_to_end():
    code = ("import __graft_entry__ as g; g.build(); "
            "import deep_quantized_recommendation_model_dqrm_amd as dq; "
            "print('abi', dq._lib.load().dqrm_abi_version(), g.header_abi_version())")
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True, timeout=1500)
    assert r.returncode == 0, r.stderr[-4000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("abi ")][-1]
    _, lib_abi, hdr_abi = line.split()
    assert lib_abi == hdr_abi


def test_header_abi_matches_binding():
    sys.path.insert(0, ROOT)
    import __graft_entry__ as g
    from deep_quantized_recommendation_model_dqrm_amd import _lib as L

    assert g.header_abi_version() == L.DQRM_ABI_VERSION
