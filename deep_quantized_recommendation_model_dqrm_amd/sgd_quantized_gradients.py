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
from .tables import CoalescedGrad, default_caps

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
    """sgd_quantized_gradients.py:56-94 (embedding branch), one micro-step."""
    if not emb_grad_quantized:
        raise NotImplementedError("the unquantized simulated buffer (grad / N accumulation) is not built")
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


def weights_update_added_quantization(model, lr, num_gpus, emb_grad_quantized=True, update_embedding=True) -> None:
    """sgd_quantized_gradients.py:349-379 (embedding branch): W += -lr * buffer * (s / N)."""
    if not emb_grad_quantized:
        raise NotImplementedError("the unquantized simulated buffer (grad / N accumulation) is not built")
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
        m.emb_scaling_factor.zero_()


__all__ = ["grad_buffer_update_added_quantization", "weights_update_added_quantization", "grad_buffer_zeroing"]
