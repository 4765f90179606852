"""INT8-quantized sparse-gradient all-reduce for data-parallel embedding training.

Reference: sgd_quantized_gradients_parallel_comm.py
  quantize_emb_grad            :850-890  (coalesce, scale, all_reduce(scale), quantize,
                                          all_reduce(sparse), * 1/N)
  grad_update_parallel_comm    :257-317  (26 tables, 2 blocking collectives each)
  weight_update_parallel_comm  :601-628  (W += -lr * grad * s)

MI355X design: the 52 per-table Gloo collectives of the reference become TWO collectives
per step for all tables together, both all-gathers over RCCL (torch.distributed "nccl"
on ROCm, xGMI point-to-point):
  1. all_gather of the [T] local scales  -> every rank sums them in rank order (the
     average is bit-identical on every rank);
  2. all_gather of one fixed-capacity payload per rank  {counts i32[T], rows i32[CAP],
     q int8[CAP, D]} -> every rank decodes all N payloads, unions rows and sums the
     integers exactly (= Gloo sparse all_reduce, torch-internal: coalesce, allgather,
     sum, coalesce), then applies the dequantized SGD update.
Kernels: dqrm_emb_bwd_coalesce (K4), dqrm_grad_quant_pack (K5), dqrm_apply_sparse_update (K6).
"""
from __future__ import annotations

import ctypes as C
from typing import Protocol

import torch
import torch.distributed as dist

from . import _lib as L
from .tables import CoalescedGrad, EmbeddingTableSet, LookupBatch, _ptr, _stream_handle, default_caps


class ExchangeKernels(Protocol):
    """The three device steps of the exchange (HIP by default; tests may inject a checker)."""

    def coalesce(self, batch: LookupBatch, dy: torch.Tensor, ws: CoalescedGrad, ste: bool,
                 grad_bits: int, layout: str) -> None: ...

    def quant_pack(self, ws: CoalescedGrad, s_all: torch.Tensor, num_ranks: int, grad_bits: int,
                   s_avg: torch.Tensor, payload: torch.Tensor) -> None: ...

    def apply(self, ws: CoalescedGrad, gathered: torch.Tensor, payload_bytes: int, num_ranks: int,
              grad_bits: int, s_avg: torch.Tensor, lr: float, mode: int, repack: bool) -> None: ...


class HipExchangeKernels:
    """libdqrm kernels; the only implementation the product uses."""

    def __init__(self, tables: EmbeddingTableSet):
        self.tables = tables
        self.lib = tables.lib

    def coalesce(self, batch, dy, ws, ste, grad_bits, layout):
        self.tables.backward_coalesce(batch, dy, ws, ste=ste, grad_bits=grad_bits if grad_bits <= 16 else 0,
                                      layout=layout)

    def quant_pack(self, ws, s_all, num_ranks, grad_bits, s_avg, payload):
        t = self.tables
        L.check(
            self.lib.dqrm_grad_quant_pack(
                t.T, t.D, _ptr(ws.cap_base), ws.cap_total, _ptr(ws.rows), _ptr(ws.vals), _ptr(ws.counts),
                _ptr(s_all), num_ranks, grad_bits, _ptr(s_avg), _ptr(payload), _stream_handle()),
            "dqrm_grad_quant_pack",
        )

    def apply(self, ws, gathered, payload_bytes, num_ranks, grad_bits, s_avg, lr, mode, repack):
        t = self.tables
        L.check(
            self.lib.dqrm_apply_sparse_update(
                C.byref(t.c), _ptr(ws.cap_base), ws.cap_total, _ptr(gathered), payload_bytes, num_ranks,
                grad_bits, _ptr(s_avg), float(lr), mode, 4 if repack else 0, _stream_handle()),
            "dqrm_apply_sparse_update",
        )


def payload_bytes(num_tables: int, cap_total: int, dim: int, grad_bits: int) -> int:
    """Bytes of one rank's wire payload (mirrors dqrm_payload_bytes)."""
    a16 = lambda x: (x + 15) & ~15  # noqa: E731
    elem = 1 if grad_bits <= 8 else (2 if grad_bits <= 16 else 4)
    return a16(4 * num_tables) + a16(4 * cap_total) + a16(cap_total * dim * elem)


class SparseGradExchange:
    """Per-step DP embedding update: coalesce -> scale all-gather -> quantize-pack ->
    payload all-gather -> decode + SGD.  One instance per rank, buffers reused every step.

    grad_bits: 8 (scripts' --embedding_bag_gradient_bit_num=8), 2..16, or 32 for the
    unquantized sparse path (emb_grad_quantized=False, s_q_g_p_c.py:319-327).
    """

    def __init__(self, tables: EmbeddingTableSet, caps, grad_bits: int = 8, group=None,
                 kernels: ExchangeKernels | None = None, device=None):
        if not (grad_bits == 32 or 2 <= grad_bits <= 16):
            raise ValueError("grad_bits must be 2..16 or 32")
        self.tables = tables
        self.grad_bits = grad_bits
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if self.world > 1 else 0
        dev = device if device is not None else tables.device
        self.device = torch.device(dev)
        self.kernels = kernels if kernels is not None else HipExchangeKernels(tables)
        self.ws = CoalescedGrad.allocate(caps, tables.D, self.device)
        T = tables.T
        self.payload_bytes = payload_bytes(T, self.ws.cap_total, tables.D, grad_bits)
        self.s_all = torch.zeros(self.world, T, dtype=torch.float32, device=self.device)
        self.s_avg = torch.zeros(T, dtype=torch.float32, device=self.device)
        self.payload = torch.zeros(self.payload_bytes, dtype=torch.uint8, device=self.device)
        self.gathered = torch.zeros(self.world, self.payload_bytes, dtype=torch.uint8, device=self.device)

    @classmethod
    def for_batch_shape(cls, tables: EmbeddingTableSet, max_lookups_per_table: int, **kw):
        return cls(tables, default_caps(tables.num_rows, max_lookups_per_table), **kw)

    # -------------------------------------------------------------- collectives
    def _all_gather(self, out: torch.Tensor, inp: torch.Tensor) -> None:
        if self.world == 1:
            out[0].copy_(inp)
            return
        backend = dist.get_backend(self.group)
        if backend == "nccl":  # RCCL on ROCm: one all-gather straight into the output
            dist.all_gather_into_tensor(out.view(-1), inp.view(-1), group=self.group)
        else:
            dist.all_gather(list(out.unbind(0)), inp, group=self.group)

    # -------------------------------------------------------------- the step
    def step(self, batch: LookupBatch, dy: torch.Tensor, lr: float, ste: bool = True,
             mode: int | None = None, repack: bool = False, layout: str = "tbd") -> None:
        """grad_update_parallel_comm + weight_update_parallel_comm for all tables."""
        gb = self.grad_bits
        if mode is None:
            mode = L.DQRM_UPD_FP32 if gb == 32 else L.DQRM_UPD_DP
        self.kernels.coalesce(batch, dy, self.ws, ste, gb, layout)
        if gb != 32:
            self._all_gather(self.s_all, self.ws.s_loc)
        self.kernels.quant_pack(self.ws, self.s_all, self.world, gb, self.s_avg, self.payload)
        if self.world == 1:
            gathered = self.payload.view(1, -1)
        else:
            self._all_gather(self.gathered, self.payload)
            gathered = self.gathered
        self.kernels.apply(self.ws, gathered, self.payload_bytes, self.world, gb, self.s_avg, lr, mode, repack)


def get_my_slice(n: int, my_size: int, my_rank: int) -> slice:
    """Contiguous per-rank batch slice (dlrm_s_pytorch_single_gpu.py:989-993)."""
    k, m = divmod(n, my_size)
    return slice(my_rank * k + min(my_rank, m), (my_rank + 1) * k + min(my_rank + 1, m), 1)


__all__ = ["SparseGradExchange", "HipExchangeKernels", "payload_bytes", "get_my_slice"]
