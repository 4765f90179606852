"""INT8-quantized gradient exchange of the dense (MLP) layers of the data-parallel step.

Reference: sgd_quantized_gradients_parallel_comm.py
  quantize_linear_grad   :892-929  per-channel scale = max(|row min|, |row max|)/127,
                                   all_reduce(scale)/N, q = SymmetricQuantFunction(g),
                                   all_reduce(q)/N
  quantize_bias_grad     :931-961  the same, one scale per bias vector
  grad_update_parallel_comm      MLP branch :337-409   (2 layers x 2 tensors x 2 collectives each)
  weight_update_parallel_comm    MLP branch :630-668   W += (-lr * grad) * s

MI355X design: every weight row and every bias vector of all bot_l / top_l layers is one
channel of ONE channel table, so each phase is one libdqrm launch for all layers and the
reference's 4 blocking collectives per layer become two per step:
  1. all-gather of the per-channel local scales s_loc [C] -> every rank averages them in
     the same (descending-rank) order, bit-identical on all ranks;
  2. all-reduce(SUM) of the quantized wire: integer-valued fp16 (exact: N * 128 <= 2048
     for N <= 16; int32 beyond), half the bytes of an FP32 gradient all-reduce.
Kernels: dqrm_dense_grad_scale, dqrm_dense_grad_quant, dqrm_dense_grad_decode,
dqrm_dense_update (csrc/dqrm_dense.hip).
"""
from __future__ import annotations

import ctypes as C
from typing import Protocol, Sequence

import numpy as np
import torch
import torch.distributed as dist
from torch import nn

from . import _lib as L
from .tables import _ptr, _stream_handle

_WIRE_DTYPE = {L.DQRM_WIRE_F16: torch.float16, L.DQRM_WIRE_I32: torch.int32, L.DQRM_WIRE_F32: torch.float32}


class DenseChannels:
    """The channel table of a list of Linear layers: layer k contributes its weight rows
    (one channel each, per_channel=True) then its bias vector (one channel).
    weight_slices[k] / bias_index[k] locate layer k's scales in the [C] scale vectors."""

    def __init__(self, layers: Sequence[nn.Module]):
        self.layers = list(layers)
        self.weight_slices: list[slice] = []
        self.bias_index: list[int] = []
        lens, c = [], 0
        for l in self.layers:
            out, inp = l.weight.shape
            if l.bias is None:
                raise ValueError("quantize_bias_grad needs every Linear layer to have a bias (s_q_g_p_c.py:931)")
            self.weight_slices.append(slice(c, c + out))
            lens += [inp] * out
            c += out
            self.bias_index.append(c)
            lens.append(out)
            c += 1
        self.num_channels = c
        self.len = np.asarray(lens, dtype=np.int32)
        self.wire_off = np.zeros(c, dtype=np.int64)
        if c:
            self.wire_off[1:] = np.cumsum(self.len[:-1], dtype=np.int64)
        self.total_elems = int(self.len.sum()) if c else 0
        self.max_len = int(self.len.max()) if c else 0

    def tensors(self):
        """[(grad, param)] per layer tensor, in channel order (weight, bias, weight, ...)."""
        out = []
        for l in self.layers:
            out.append((l.weight.grad, l.weight.data))
            out.append((l.bias.grad, l.bias.data))
        return out


class DenseKernels(Protocol):
    """The four device steps (HIP by default; CPU tests inject an oracle-backed checker).
    prepare() runs once per exchange()/apply() before the steps."""

    def prepare(self) -> None: ...

    def scale(self, bits: int, s_loc: torch.Tensor) -> None: ...

    def quant(self, bits: int, s_all: torch.Tensor, num_ranks: int, s_avg: torch.Tensor, wire_type: int,
              wire: torch.Tensor) -> None: ...

    def decode(self, wire: torch.Tensor, wire_type: int, num_ranks: int) -> None: ...

    def update(self, s: torch.Tensor | None, lr: float) -> None: ...


class HipDenseKernels:
    """libdqrm's dense kernels over a DenseChannels table; the only implementation the
    product uses. The device channel table (grad/param pointers per channel) is rebuilt
    whenever a layer's .grad or .data storage changes."""

    def __init__(self, channels: DenseChannels, device):
        self.ch = channels
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise L.DQRMError(f"libdqrm's dense kernels need the layers on a GPU (got {self.device}); "
                              "there is no CPU path")
        if self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        self.lib = L.load()
        self._key = None
        self._c = L.DenseSet()
        self._bufs: list[torch.Tensor] = []

    def prepare(self) -> None:
        """Rebuild the device channel table if a layer's .grad / .data storage moved."""
        ts = self.ch.tensors()
        key = tuple((g.data_ptr(), p.data_ptr()) for g, p in ts)
        if key == self._key:
            return
        for g, p in ts:
            if g.device != self.device or p.device != self.device:
                raise ValueError(f"dense layers must live on {self.device} (got {g.device} / {p.device})")
            if g.dtype != torch.float32 or p.dtype != torch.float32 or not g.is_contiguous() or not p.is_contiguous():
                raise ValueError("dense layers need contiguous float32 weights and gradients")
        gp, pp = [], []
        for l in self.ch.layers:
            out, inp = l.weight.shape
            g0, p0 = l.weight.grad.data_ptr(), l.weight.data.data_ptr()
            gp += [g0 + 4 * inp * r for r in range(out)]
            pp += [p0 + 4 * inp * r for r in range(out)]
            gp.append(l.bias.grad.data_ptr())
            pp.append(l.bias.data.data_ptr())
        host = [np.asarray(gp, np.uint64).view(np.int64), np.asarray(pp, np.uint64).view(np.int64),
                self.ch.len, self.ch.wire_off]
        self._bufs = [torch.from_numpy(np.ascontiguousarray(a)).to(self.device) for a in host]
        c = self._c
        c.num_channels = self.ch.num_channels
        c.max_len = self.ch.max_len
        c.total_elems = self.ch.total_elems
        c.grad, c.param, c.len, c.wire_off = (_ptr(b) for b in self._bufs)
        self._key = key

    def scale(self, bits, s_loc):
        L.check(self.lib.dqrm_dense_grad_scale(C.byref(self._c), bits, _ptr(s_loc), _stream_handle()),
                "dqrm_dense_grad_scale")

    def quant(self, bits, s_all, num_ranks, s_avg, wire_type, wire):
        L.check(self.lib.dqrm_dense_grad_quant(C.byref(self._c), bits, _ptr(s_all), num_ranks, _ptr(s_avg),
                                               wire_type, _ptr(wire), _stream_handle()),
                "dqrm_dense_grad_quant")

    def decode(self, wire, wire_type, num_ranks):
        L.check(self.lib.dqrm_dense_grad_decode(C.byref(self._c), _ptr(wire), wire_type, num_ranks,
                                                _stream_handle()),
                "dqrm_dense_grad_decode")

    def update(self, s, lr):
        L.check(self.lib.dqrm_dense_update(C.byref(self._c), _ptr(s), float(lr), _stream_handle()),
                "dqrm_dense_update")


class DenseGradExchange:
    """The MLP half of grad_update_parallel_comm / weight_update_parallel_comm for all
    bot_l + top_l Linear layers. One instance per rank; buffers reused every step.

    grad_bits: 8 (the reference hard-codes num_bits=8 for the MLP, s_q_g_p_c.py:341,350),
    2..16, or 32 for mlp_layer_quantized=False (FP32 all-reduce / N, :358-369).
    """

    def __init__(self, layers: Sequence[nn.Module], grad_bits: int = 8, group=None,
                 kernels: DenseKernels | None = None, device=None, wire_type: int | None = None,
                 force_collectives: bool = False):
        """force_collectives: issue the scale all-gather and the wire all-reduce at world
        size 1 too, through the process group's backend (the N > 1 code path)."""
        if not (grad_bits == 32 or 2 <= grad_bits <= 16):
            raise ValueError("grad_bits must be 2..16 or 32")
        self.channels = DenseChannels(layers)
        self.grad_bits = grad_bits
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if self.world > 1 else 0
        self.coll = self.world > 1 or bool(force_collectives)
        if self.coll and not (dist.is_available() and dist.is_initialized()):
            raise ValueError("force_collectives needs an initialised process group")
        if device is None:
            device = self.channels.layers[0].weight.device if self.channels.layers else "cpu"
        self.device = torch.device(device)
        self.kernels = kernels if kernels is not None else HipDenseKernels(self.channels, self.device)
        if wire_type is None:
            wire_type = L.load().dqrm_dense_wire_type(grad_bits, self.world) if kernels is None else \
                _wire_type(grad_bits, self.world)
        if wire_type < 0:
            raise ValueError(f"no exact wire type for {grad_bits} bits over {self.world} ranks")
        self.wire_type = wire_type
        C_ = self.channels.num_channels
        self.s_loc = torch.zeros(C_, dtype=torch.float32, device=self.device)
        self.s_all = torch.zeros(self.world, C_, dtype=torch.float32, device=self.device)
        self.s_avg = torch.zeros(C_, dtype=torch.float32, device=self.device)
        self.wire = torch.zeros(self.channels.total_elems, dtype=_WIRE_DTYPE[wire_type], device=self.device)

    # -------------------------------------------------------------- collectives
    def _backend(self) -> str:
        return dist.get_backend(self.group)

    def _all_gather_scales(self) -> None:
        if self._backend() == "nccl":
            dist.all_gather_into_tensor(self.s_all.view(-1), self.s_loc, group=self.group)
        elif self.s_all.is_cuda:  # Gloo gathers host tensors (rehearsal only)
            host = self.s_all.cpu()
            dist.all_gather(list(host.unbind(0)), self.s_loc.cpu(), group=self.group)
            self.s_all.copy_(host)
        else:
            dist.all_gather(list(self.s_all.unbind(0)), self.s_loc, group=self.group)

    def _all_reduce_wire(self) -> None:
        if self._backend() == "nccl" or not self.wire.is_cuda:
            dist.all_reduce(self.wire, dist.ReduceOp.SUM, group=self.group)
        else:
            host = self.wire.cpu()
            dist.all_reduce(host, dist.ReduceOp.SUM, group=self.group)
            self.wire.copy_(host)

    # -------------------------------------------------------------- the step
    def exchange(self) -> None:
        """grad_update_parallel_comm's MLP branch: afterwards every layer's .grad holds the
        rank-averaged quantized gradient and weight_scaling_factor / bias_scaling_factor
        the averaged scales (views into this exchange's s_avg)."""
        k, gb = self.kernels, self.grad_bits
        k.prepare()
        if gb != 32:
            k.scale(gb, self.s_loc)
            if self.coll:
                self._all_gather_scales()
                s_all = self.s_all
            else:
                s_all = self.s_loc.view(1, -1)
        else:
            s_all = None
        k.quant(gb, s_all, self.world, self.s_avg if gb != 32 else None, self.wire_type, self.wire)
        if self.coll:
            self._all_reduce_wire()
        k.decode(self.wire, self.wire_type, self.world)
        if gb != 32:
            for l, ws, bi in zip(self.channels.layers, self.channels.weight_slices, self.channels.bias_index):
                l.weight_scaling_factor = self.s_avg[ws]
                l.bias_scaling_factor = self.s_avg[bi]

    def apply(self, lr: float) -> None:
        """weight_update_parallel_comm's MLP branch: W += (-lr * grad) * s."""
        self.kernels.prepare()
        self.kernels.update(self.s_avg if self.grad_bits != 32 else None, lr)


def _wire_type(bits: int, num_ranks: int) -> int:
    """dqrm_dense_wire_type, for host-only (injected-kernel) runs."""
    if bits == 32:
        return L.DQRM_WIRE_F32
    if not 2 <= bits <= 16 or num_ranks < 1:
        return L.DQRM_E_INVALID
    return L.DQRM_WIRE_F16 if num_ranks << (bits - 1) <= 2048 else L.DQRM_WIRE_I32


__all__ = ["DenseChannels", "DenseKernels", "HipDenseKernels", "DenseGradExchange"]
