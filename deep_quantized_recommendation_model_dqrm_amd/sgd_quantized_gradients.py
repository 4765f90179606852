"""Drop-in for the reference's simulated data-parallel quantized SGD
(``sgd_quantized_gradients.py``): one device plays N ranks by running N micro-steps whose
INT8-quantized embedding gradients accumulate in a buffer, then one dequantized update.

    grad_buffer_update_added_quantization(model, number_of_gpus, emb_grad_quantized=True)  :56-94
    weights_update_added_quantization(model, lr, num_gpus, emb_grad_quantized, update_embedding) :349-379
    grad_buffer_zeroing(model)                                                                :231-258

Semantics (reference): the FIRST micro-step's scale s = max|coalesced grad| / 127 is kept
(``emb_scaling_factor`` is non-zero afterwards) and quantizes every later micro-step; the
buffer holds the exact integer sum; the update is W += -lr * (buffer * fl32(s / N)).
Here each micro-step is coalesced and quantize-packed on the device into its own payload
(dqrm_emb_bwd_coalesce + dqrm_grad_quant_pack with the first micro-step's per-slot
max|grad| as a one-rank scale input), and the update is dqrm_apply_sparse_update over the
N payloads in DQRM_UPD_SIMULATED mode (the integer sum is order-free, hence identical to
the reference's coalesced buffer).

Embedding modules must be built with ``grad_mode="dp"``.
"""
from __future__ import annotations

import torch

from . import _lib as L
from .comm import HipExchangeKernels, payload_bytes
from .quant_modules_not_quantize_grad import _QuantEmbeddingBase
from .tables import CoalescedGrad, LookupBatch, default_caps

GRAD_BITS = 8  # the reference hard-codes num_bits = 8 here (:77,:80)


class _MicroStepBuffer:
    """Per-module state of the simulated-DP buffer: N payloads + the first micro-step's
    per-slot max|grad| and scale."""

    def __init__(self, m: _QuantEmbeddingBase, max_lookups: int):
        ts = m._tset
        self.max_lookups = max_lookups
        self.ws = CoalescedGrad.allocate(ts.num_rows, max_lookups, ts.D, ts.device)
        caps = default_caps(ts.num_rows, max_lookups)
        base = [0]
        for c in caps:
            base.append(base[-1] + c)
        self.cap_total = base[-1]
        self.cap_base = torch.tensor(base, dtype=torch.int64, device=ts.device)
        self.payload_bytes = payload_bytes(ts.T, self.cap_total, ts.D, GRAD_BITS)
        self.payloads: list[torch.Tensor] = []
        self.first_absmax: torch.Tensor | None = None
        self.s_first = torch.zeros(ts.T, dtype=torch.float32, device=ts.device)
        self.kernels = HipExchangeKernels(ts)


def _emb_modules(model) -> list[_QuantEmbeddingBase]:
    emb = getattr(model, "emb_l", None)
    if emb is None:
        raise Warning("Cannot find the list of embedding tables")
    mods = [emb] if isinstance(emb, _QuantEmbeddingBase) else list(emb)
    for m in mods:
        if not isinstance(m, _QuantEmbeddingBase) or m.grad_mode != "dp":
            raise ValueError("simulated DP needs this package's embedding modules with grad_mode='dp'")
    return mods


def grad_buffer_update_added_quantization(model, number_of_gpus, emb_grad_quantized=True) -> None:
    """sgd_quantized_gradients.py:56-94 (embedding branch), one micro-step. Unquantized
    (emb_grad_quantized=False, :88-91): the micro-step's lookups and upstream gradient are
    kept on the device; the update applies buffer = sum of grad / N in the reference's order."""
    if not emb_grad_quantized:
        with torch.no_grad():
            for m in _emb_modules(model):
                if m._pending is None:
                    continue
                fb = getattr(m, "_sim_fp32", None)
                if fb is None:
                    fb = m._sim_fp32 = []
                fb.append((m._pending, int(number_of_gpus)))
                m._pending = None
        return
    with torch.no_grad():
        for m in _emb_modules(model):
            if m._pending is None:
                continue
            batch, dy, ste, layout = m._pending
            buf = getattr(m, "_sim_buffer", None)
            if buf is None or buf.max_lookups < batch.max_lookups:
                if buf is not None and buf.payloads:
                    raise ValueError("micro-step batch larger than the first one of this accumulation")
                buf = _MicroStepBuffer(m, max(batch.max_lookups, 1))
                m._sim_buffer = buf
            buf.kernels.coalesce(batch, dy, buf.ws, ste, layout)
            if buf.first_absmax is None:  # emb_scaling_factor == 0: this micro-step sets the scale
                buf.first_absmax = buf.ws.absmax.clone().view(1, -1)
            payload = torch.empty(buf.payload_bytes, dtype=torch.uint8, device=buf.ws.rows.device)
            buf.kernels.quant_pack(buf.ws, buf.first_absmax, 1, GRAD_BITS, buf.cap_base, buf.cap_total,
                                   buf.s_first, payload)
            buf.payloads.append(payload)
            m.emb_scaling_factor.copy_(buf.s_first.view_as(m.emb_scaling_factor))
            m._pending = None


def _apply_fp32_buffer(m: _QuantEmbeddingBase, lr: float) -> None:
    """The unquantized buffer's update (:374-377): W.add_(-lr * buffer), where the buffer is
    sum over the micro-steps, in order, of grad / N (grad_buffer_update_added_quantization,
    :88-91: buffer.add_(grad / N); buffer.coalesce()). The micro-steps' batches are joined
    bag after bag; one coalesce divides every lookup's gradient by N before the ordered sum
    (dqrm_emb_bwd_coalesce_scaled), and the FP32 payload path applies W + (-lr * buffer)."""
    items = m._sim_fp32
    ts = m._tset
    (_, _, ste, _), N = items[0]
    if any(it[1] != N for it in items) or any(it[0][2] != ste for it in items):
        raise ValueError("micro-steps of one accumulation differ in number_of_gpus or full precision")
    batch = LookupBatch.concat_bags([it[0][0] for it in items])

    def tbd(it):  # a micro-step's upstream gradient as [T, B_i, D] (the modules hand tbd or btd)
        b, g, _, lay = it[0]
        return g.reshape(ts.T, b.num_bags, ts.D) if lay == "tbd" else g.reshape(b.num_bags, ts.T, ts.D).transpose(0, 1)

    dy = torch.cat([tbd(it) for it in items], dim=1).contiguous()
    ws = CoalescedGrad.allocate(ts.num_rows, max(batch.max_lookups, 1), ts.D, ts.device)
    ts.backward_coalesce_scaled(batch, dy, ws, N, ste=ste)
    caps = default_caps(ts.num_rows, max(batch.max_lookups, 1))
    base = [0]
    for c in caps:
        base.append(base[-1] + c)
    cap_base = torch.tensor(base, dtype=torch.int64, device=ts.device)
    pb = payload_bytes(ts.T, base[-1], ts.D, 32)
    payload = torch.zeros(pb, dtype=torch.uint8, device=ts.device)
    k = HipExchangeKernels(ts)
    k.quant_pack(ws, None, 1, 32, cap_base, base[-1], None, payload)
    k.apply(cap_base, base[-1], payload.view(1, -1), pb, 1, 32, None, lr, L.DQRM_UPD_FP32, m._use_packed(False))


def weights_update_added_quantization(model, lr, num_gpus, emb_grad_quantized=True, update_embedding=True) -> None:
    """sgd_quantized_gradients.py:349-379 (embedding branch): W += -lr * buffer * (s / N);
    unquantized (:374-377): W += -lr * buffer."""
    if not emb_grad_quantized:
        with torch.no_grad():
            for m in _emb_modules(model):
                if update_embedding and getattr(m, "_sim_fp32", None):
                    _apply_fp32_buffer(m, lr)
        return
    with torch.no_grad():
        if not update_embedding:
            return
        for m in _emb_modules(model):
            buf = getattr(m, "_sim_buffer", None)
            if buf is None or not buf.payloads:
                continue
            if len(buf.payloads) != int(num_gpus):
                raise ValueError(f"{len(buf.payloads)} micro-steps accumulated but num_gpus={num_gpus}")
            gathered = torch.stack(buf.payloads)
            buf.kernels.apply(buf.cap_base, buf.cap_total, gathered, buf.payload_bytes, len(buf.payloads),
                              GRAD_BITS, buf.s_first, lr, L.DQRM_UPD_SIMULATED, m._use_packed(False))


def grad_buffer_zeroing(model) -> None:
    """sgd_quantized_gradients.py:231-258: empty the buffers and zero the scales."""
    for m in _emb_modules(model):
        buf = getattr(m, "_sim_buffer", None)
        if buf is not None:
            buf.payloads.clear()
            buf.first_absmax = None
        m._sim_fp32 = []
        m.emb_scaling_factor.zero_()


__all__ = ["grad_buffer_update_added_quantization", "weights_update_added_quantization", "grad_buffer_zeroing"]
