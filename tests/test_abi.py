"""CPU checks of the C-ABI library: it loads, exports every symbol include/dqrm.h declares,
and rejects bad arguments without touching a device."""
import ctypes as C
import os
import re

import pytest

import deep_quantized_recommendation_model_dqrm_amd as dq
from deep_quantized_recommendation_model_dqrm_amd import _lib as L
from deep_quantized_recommendation_model_dqrm_amd.comm import payload_bytes

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def lib():
    dq.build(verbose=False)
    return L.load()


def header_functions():
    src = open(os.path.join(ROOT, "include", "dqrm.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(dqrm_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_what_binding_expects():
    assert header_functions() == sorted(L.EXPORTED_SYMBOLS)


def test_library_exports_every_header_symbol(lib):
    for name in header_functions():
        assert hasattr(lib, name), name
    assert lib.dqrm_abi_version() == L.DQRM_ABI_VERSION


def test_payload_bytes_agree(lib):
    for T, cap, D, bits in [(26, 3328, 16, 8), (26, 53248, 64, 8), (4, 7, 4, 16), (3, 0, 32, 32), (1, 1, 256, 2)]:
        assert lib.dqrm_payload_bytes(T, cap, D, bits) == payload_bytes(T, cap, D, bits)


def test_struct_layouts():
    # dqrm_table_set: 2 x i32 + 3 x i64 + 15 pointers (the last a host array); dqrm_batch: 3 pointers + 2 x i64
    assert C.sizeof(L.TableSet) == 8 + 24 + 15 * 8
    assert C.sizeof(L.Batch) == 6 * 8
    # dqrm_exchange: 2 pointers + 2 x i32 + 17 eight-byte fields
    assert C.sizeof(L.Exchange) == 2 * 8 + 8 + 17 * 8


def test_invalid_arguments_rejected_without_device(lib):
    assert lib.dqrm_refresh_absmax(None, None) == L.DQRM_E_INVALID
    assert b"null table set" in lib.dqrm_last_error()
    ts = L.TableSet()
    ts.num_tables, ts.dim = 2, 12  # dim must be 4 * 2^k
    assert lib.dqrm_emb_fwd(C.byref(ts), None, 4, 0, None, 0, 0, None) == L.DQRM_E_INVALID
    assert b"dim" in lib.dqrm_last_error()
    assert lib.dqrm_grad_quant_pack(0, 16, None, 0, None, None, None, None, 1, 8, None, 0, None, None, None) == L.DQRM_E_INVALID
    assert lib.dqrm_grad_quant_pack(2, 16, None, 0, None, None, None, None, 1, 37, None, 0, None, None, None) == L.DQRM_E_INVALID


def test_exchange_and_comm_reject_bad_arguments_without_device(lib):
    """The N > 1 exchange entry points validate before touching RCCL or a device."""
    assert lib.dqrm_exchange_grad(None, None, None, 0, 0, 1, None) == L.DQRM_E_INVALID
    assert b"null exchange" in lib.dqrm_last_error()
    x = L.Exchange()
    ts = L.TableSet()
    x.set = C.pointer(ts)
    x.num_ranks = 2  # no communicator: only world size 1 is valid
    assert lib.dqrm_exchange_apply(C.byref(x), 0.1, L.DQRM_UPD_DP, 0, None) == L.DQRM_E_INVALID
    assert b"num_ranks" in lib.dqrm_last_error()
    assert lib.dqrm_comm_init(None, 1, 0, None) == L.DQRM_E_INVALID
    assert lib.dqrm_comm_allgather(None, None, None, 0, None) == L.DQRM_E_INVALID
    assert lib.dqrm_comm_destroy(None) == L.DQRM_OK
    assert lib.dqrm_emb_bwd_lookup_grad_presum(None, None, None, 0, 0, 1, None, None, None) == L.DQRM_E_INVALID


def test_check_exchange_errors_without_device(lib):
    """dqrm_exchange_grad / _apply reject an inconsistent exchange before any kernel or
    collective: num_ranks against the communicator's size, missing gather buffers, a payload
    size that is not dqrm_payload_bytes, bad grad_bits, a missing coalesce workspace. The
    communicator here is a caller-served one (dqrm_comm_init_external), which needs no device."""
    calls = []
    fn = L.ALLGATHER_FN(lambda send, recv, n, stream, user: calls.append((send, recv, n)) or 0)
    h = C.c_void_p()
    assert lib.dqrm_comm_init_external(C.byref(h), 2, 1, fn, None) == L.DQRM_OK
    try:
        assert lib.dqrm_comm_size(h) == 2
        ts = L.TableSet()
        ts.num_tables, ts.dim = 3, 16
        T, cap, D = 3, 100, 16
        x = L.Exchange()
        x.set = C.pointer(ts)
        x.comm = h
        x.grad_bits = 8
        x.cap_total, x.cap_base = cap, 0x1000
        x.payload, x.s_avg = 0x2000, 0x3000
        x.absmax_all, x.gathered = 0x4000, 0x5000
        x.ws_cap_base, x.ws_rows, x.ws_vals, x.ws_ucount, x.ws_absmax = 0x10, 0x20, 0x30, 0x40, 0x50
        x.payload_bytes = lib.dqrm_payload_bytes(T, cap, D, 8)

        def expect(field, value, msg, grad=False):
            old = getattr(x, field)
            setattr(x, field, value)
            try:
                fn_ = (lambda: lib.dqrm_exchange_grad(C.byref(x), None, None, 0, 0, 1, None)) if grad else \
                    (lambda: lib.dqrm_exchange_apply(C.byref(x), 0.1, L.DQRM_UPD_DP, 0, None))
                assert fn_() == L.DQRM_E_INVALID, field
                assert msg in lib.dqrm_last_error(), (field, lib.dqrm_last_error())
            finally:
                setattr(x, field, old)

        x.num_ranks = 2
        expect("num_ranks", 1, b"num_ranks")        # the communicator has 2 ranks
        expect("num_ranks", 3, b"num_ranks")
        expect("comm", None, b"num_ranks")          # no communicator: world size 1 only
        expect("absmax_all", None, b"gather buffers")
        expect("gathered", None, b"gather buffers")
        expect("payload", None, b"null payload")
        expect("payload_bytes", x.payload_bytes + 16, b"payload_bytes")
        expect("grad_bits", 1, b"grad_bits")
        expect("grad_bits", 17, b"grad_bits")
        expect("ws_rows", None, b"coalesce workspace", grad=True)
        assert not calls  # nothing reached the transport
        # the caller-served all-gather is called with the device pointers, in order
        assert lib.dqrm_comm_allgather(h, 0x111, 0x222, 48, None) == L.DQRM_OK
        assert calls == [(0x111, 0x222, 48)]
        bad = L.ALLGATHER_FN(lambda *a: 1)
        h2 = C.c_void_p()
        assert lib.dqrm_comm_init_external(C.byref(h2), 2, 0, bad, None) == L.DQRM_OK
        assert lib.dqrm_comm_allgather(h2, 0x111, 0x222, 48, None) == L.DQRM_E_HIP
        assert b"all-gather failed" in lib.dqrm_last_error()
        assert lib.dqrm_comm_destroy(h2) == L.DQRM_OK
        assert lib.dqrm_comm_init_external(C.byref(h2), 2, 2, fn, None) == L.DQRM_E_INVALID  # rank >= nranks
        assert lib.dqrm_comm_init_external(C.byref(h2), 2, 0, L.ALLGATHER_FN(), None) == L.DQRM_E_INVALID
    finally:
        assert lib.dqrm_comm_destroy(h) == L.DQRM_OK


def test_fused_next_forward_rejects_bad_arguments_without_device(lib):
    """dqrm_emb_bwd_apply_fwd_local validates the next batch's forward as dqrm_emb_fwd does
    (before any launch)."""
    ts = L.TableSet()
    ts.num_tables, ts.dim = 2, 12  # dim must be 4 * 2^k
    args = [C.byref(ts), None, None, 0, 0, 1, None, 0, None, None, None, None, 8, None, 0.1, 0, None, 0]
    assert lib.dqrm_emb_bwd_apply_fwd_local(*args, None, 4, 0, None, 0, 0, None) == L.DQRM_E_INVALID
    assert b"dim" in lib.dqrm_last_error()
    assert lib.dqrm_bwd_apply_fwd_local_is_one_launch(None, None, None, 0, None) == L.DQRM_E_INVALID
    assert lib.dqrm_emb_bwd_sgd_fwd(C.byref(ts), None, None, 0, 0, 1, 0.1, 0, None, 0, None, 4, 0, None, 0, 0,
                                    None) == L.DQRM_E_INVALID
    assert lib.dqrm_bwd_sgd_fwd_is_one_launch(None, None, None, 0) == L.DQRM_E_INVALID


def test_apply_kernel_selector(lib):
    prev = lib.dqrm_set_apply_kernel(L.DQRM_APPLY_SLOT)
    try:
        assert lib.dqrm_set_apply_kernel(L.DQRM_APPLY_FLAT) == L.DQRM_APPLY_SLOT
        assert lib.dqrm_set_apply_kernel(L.DQRM_APPLY_RANGES) == L.DQRM_APPLY_FLAT
        assert lib.dqrm_set_apply_kernel(L.DQRM_APPLY_MERGE) == L.DQRM_APPLY_RANGES
        assert lib.dqrm_set_apply_kernel(L.DQRM_APPLY_FLAT) == L.DQRM_APPLY_MERGE
        assert lib.dqrm_set_apply_kernel(5) == L.DQRM_E_INVALID
        assert b"kind" in lib.dqrm_last_error()
        assert lib.dqrm_set_apply_kernel(L.DQRM_APPLY_AUTO) == L.DQRM_APPLY_FLAT
    finally:
        lib.dqrm_set_apply_kernel(prev)


def test_slot_caps_partition():
    from deep_quantized_recommendation_model_dqrm_amd.tables import slot_caps
    rows = [3, 1000, 10**7, 256 * 9]
    base = slot_caps(rows, 2048)
    S = L.DQRM_TABLE_SPLIT
    assert len(base) == len(rows) * S + 1 and base[0] == 0
    caps = [base[k + 1] - base[k] for k in range(len(rows) * S)]
    # every row of a table lands in exactly one slot; a slot holds <= min(max_lookups, its rows)
    assert sum(caps[0:S]) == 3 and sum(caps[S:2 * S]) == 1000
    assert all(c <= 2048 for c in caps)
    assert sum(caps[3 * S:4 * S]) == 256 * 9


def test_product_path_fails_loudly_without_library(tmp_path, monkeypatch):
    monkeypatch.setattr(L, "_lib", None)
    with pytest.raises(L.DQRMError):
        L.load(str(tmp_path / "missing.so"))
