"""Drop-in for the reference's grad-comm hooks (``sgd_quantized_gradients_parallel_comm.py``)
used by the data-parallel drivers (dlrm_s_pytorch_tb_dp_one_parallel_comm.py:1853-1907):

    clear_gradients(model)                                        s_q_g_p_c.py:714-734
    grad_update_parallel_comm(model, number_of_gpus, ...)         s_q_g_p_c.py:257-409
    weight_update_parallel_comm(model, lr, ...)                   s_q_g_p_c.py:601-668
    weight_syncc(dlrm, num_gpus)                                  s_q_g_p_c.py:963-970

``model`` exposes ``emb_l`` / ``bot_l`` / ``top_l`` as the reference's DLRM_Net does. The
embedding tables must be this package's modules built with ``grad_mode="dp"``: their
backward leaves the upstream gradient on the device, and the embedding branch below runs
the fused exchange (libdqrm kernels + two all-gathers for ALL tables of a module) instead of
the reference's 2 blocking Gloo collectives per table. Results per table are the
reference's: the averaged scale lands in ``emb_scaling_factor`` and the update applied by
``weight_update_parallel_comm`` is W += -lr * ((sum_r q_r) * 1/N) * s  (integer sums exact).

The MLP branch (QuantLinear / nn.Linear layers of bot_l, top_l) is dense PyTorch on the
layers' own device -- it is not part of the accelerated path -- and
follows quantize_linear_grad / quantize_bias_grad (s_q_g_p_c.py:892-961) op for op, with
every layer's scales in one all-reduce and every layer's gradients in one all-reduce.
"""
from __future__ import annotations

import torch
import torch.distributed as dist
from torch import nn

from . import _lib as L
from .comm import SparseGradExchange
from .quant_modules_not_quantize_grad import _QuantEmbeddingBase


# ---------------------------------------------------------------------------- helpers
def _world(group=None) -> int:
    return dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1


def _emb_modules(model) -> list[_QuantEmbeddingBase]:
    emb = getattr(model, "emb_l", None)
    if emb is None:
        raise Warning("Cannot find the list of embedding tables")
    mods = [emb] if isinstance(emb, _QuantEmbeddingBase) else list(emb)
    for m in mods:
        if not isinstance(m, _QuantEmbeddingBase):
            raise TypeError("emb_l must hold this package's QuantEmbeddingBag modules")
    return mods


def _linear_layers(model, name: str) -> list[nn.Module]:
    seq = getattr(model, name, None)
    if seq is None:
        raise Warning("Cannot find the list of {} linear layers".format("bottom" if name == "bot_l" else "top"))
    return [l for l in seq if isinstance(l, nn.Linear) or hasattr(l, "weight_scaling_factor")]


def _detach_grad(g: torch.Tensor) -> None:
    if g.grad_fn is not None:
        g.detach_()
    else:
        g.requires_grad_(False)


def _all_reduce_mean(tensors: list[torch.Tensor], n: int, group=None) -> None:
    """dist.all_reduce(SUM) then mul_(1/n), for a list of same-device tensors in one call."""
    if not tensors:
        return
    if _world(group) > 1:
        flat = torch.cat([t.reshape(-1) for t in tensors])
        dist.all_reduce(flat, dist.ReduceOp.SUM, group=group)
        off = 0
        for t in tensors:
            k = t.numel()
            t.copy_(flat[off: off + k].view_as(t))
            off += k
    for t in tensors:
        t.mul_(1.0 / n)


def _sym_quantize(x: torch.Tensor, scale: torch.Tensor, bits: int) -> torch.Tensor:
    """SymmetricQuantFunction.forward (quant_utils.py:322-346 with linear_quantize :75-101):
    round(1/scale * x + 0), clamped to [-2^(b-1), 2^(b-1)-1]; per-row scale for 2-D x."""
    n = 2 ** (bits - 1) - 1
    if x.dim() == 2 and (scale.dim() != 1 or scale.shape[0] != 1):
        scale = scale.view(-1, 1)
    else:
        scale = scale.view(-1)
    return torch.clamp(torch.round(1.0 / scale * x + 0.0), -n - 1, n)


def _sym_scale(absmax: torch.Tensor, bits: int) -> torch.Tensor:
    """symmetric_linear_quantization_params (quant_utils.py:196-220)."""
    return torch.clamp(absmax, min=1e-8) / (2 ** (bits - 1) - 1)


# ---------------------------------------------------------------------------- embedding branch
def _exchange_module(m: _QuantEmbeddingBase, number_of_gpus: int, grad_bits: int, group) -> None:
    if m.grad_mode != "dp":
        raise ValueError("grad_update_parallel_comm needs embedding modules built with grad_mode='dp'")
    if m._pending is None:
        return  # no backward since the last update: nothing to communicate
    if _world(group) != number_of_gpus:
        raise ValueError(f"number_of_gpus={number_of_gpus} but the process group has {_world(group)} ranks")
    batch, dy, ste, layout = m._pending
    ex = m._exchange
    if ex is None or ex.grad_bits != grad_bits or ex.max_lookups < batch.max_lookups or ex.group is not group:
        ex = SparseGradExchange(m._tset, max(batch.max_lookups, 1), grad_bits=grad_bits, group=group,
                                device=m._tset.device)
        m._exchange = ex
    s_avg = ex.exchange(batch, dy, ste=ste, layout=layout)
    if grad_bits != 32:
        m.emb_scaling_factor.copy_(s_avg.view_as(m.emb_scaling_factor))
    m._pending = None
    m._ready = grad_bits


def grad_update_parallel_comm(model, number_of_gpus, emb_grad_quantized=True, num_bits=16, ranking_range=False,
                              rank_for_debug=None, iteration_count=None, mlp_layer_quantized=True, group=None):
    """s_q_g_p_c.py:257-409. Embedding tables: fused coalesce -> scale all-gather ->
    quantize-pack -> payload all-gather (emb_grad_quantized=False: FP32 payloads, the
    unquantized sparse all_reduce of :319-327). MLP layers: see module docstring."""
    if ranking_range:
        raise NotImplementedError("ranking_range mixed-precision gradients are not built yet (SURVEY.md 8(f) #3)")
    if emb_grad_quantized and not 2 <= int(num_bits) <= 16:
        raise ValueError("num_bits must be in 2..16 for quantized embedding gradients")
    with torch.no_grad():
        for m in _emb_modules(model):
            _exchange_module(m, number_of_gpus, int(num_bits) if emb_grad_quantized else 32, group)
        _mlp_grad_update(model, number_of_gpus, mlp_layer_quantized, group)


def _mlp_grad_update(model, n: int, quantized: bool, group) -> None:
    layers = _linear_layers(model, "bot_l") + _linear_layers(model, "top_l")
    layers = [l for l in layers if l.weight.grad is not None]
    for l in layers:
        _detach_grad(l.weight.grad)
        if l.bias is not None and l.bias.grad is not None:
            _detach_grad(l.bias.grad)
    if not quantized:  # :358-369 / :385-396
        grads = [l.weight.grad for l in layers] + [l.bias.grad for l in layers
                                                    if l.bias is not None and l.bias.grad is not None]
        _all_reduce_mean(grads, n, group)
        return
    # quantize_linear_grad (per-channel, 8 bits) + quantize_bias_grad (:892-961)
    scales = []
    for l in layers:
        g = l.weight.grad
        w_min, _ = torch.min(g, dim=1)
        w_max, _ = torch.max(g, dim=1)
        scales.append(_sym_scale(torch.max(torch.stack([w_min.abs(), w_max.abs()], dim=1), dim=1)[0], 8))
        b = l.bias.grad
        scales.append(_sym_scale(torch.max(b.min().abs(), b.max().abs()), 8).reshape(1))
    _all_reduce_mean(scales, n, group)
    qs = []
    for k, l in enumerate(layers):
        qs.append(_sym_quantize(l.weight.grad, scales[2 * k], 8))
        qs.append(_sym_quantize(l.bias.grad, scales[2 * k + 1], 8))
    _all_reduce_mean(qs, n, group)
    for k, l in enumerate(layers):
        l.weight_scaling_factor = scales[2 * k]
        l.weight.grad.zero_()
        l.weight.grad.add_(qs[2 * k])
        l.bias_scaling_factor = scales[2 * k + 1].view(())
        l.bias.grad.zero_()
        l.bias.grad.add_(qs[2 * k + 1])


def weight_update_parallel_comm(model, lr, emb_grad_quantized=True, update_embedding=True, num_gpus=1,
                                rank_for_debug=None, ranking_range=False, use_ec=False, mlp_layer_quantized=True):
    """s_q_g_p_c.py:601-668: W += -lr * grad * s for the tables (one libdqrm launch for all
    tables of a module) and the MLP layers."""
    if ranking_range:
        raise NotImplementedError("ranking_range mixed-precision gradients are not built yet (SURVEY.md 8(f) #3)")
    if use_ec:
        raise NotImplementedError("error compensation (use_ec) is off in the reference's scripts and not built")
    with torch.no_grad():
        for m in _emb_modules(model):
            ready = getattr(m, "_ready", None)
            if ready is None:
                continue
            if update_embedding:
                if (ready != 32) != bool(emb_grad_quantized):
                    raise ValueError("emb_grad_quantized differs from the one used by grad_update_parallel_comm")
                mode = L.DQRM_UPD_DP if ready != 32 else L.DQRM_UPD_FP32
                m._exchange.apply(lr, mode=mode, repack=m._use_packed(False))
            m._ready = None
        for l in _linear_layers(model, "bot_l") + _linear_layers(model, "top_l"):
            if l.weight.grad is None:
                continue
            if mlp_layer_quantized:
                l.weight.data.add_(-lr * l.weight.grad * l.weight_scaling_factor.view(-1, 1))
                l.bias.data.add_(-lr * l.bias.grad * l.bias_scaling_factor)
            else:
                l.weight.data.add_(-lr * l.weight.grad)
                l.bias.data.add_(-lr * l.bias.grad)


def clear_gradients(model) -> None:
    """s_q_g_p_c.py:714-734, plus dropping any not-yet-exchanged embedding gradient."""
    with torch.no_grad():
        for _, param in model.named_parameters():
            if param.grad is not None:
                _detach_grad(param.grad)
                param.grad.zero_()
        emb = getattr(model, "emb_l", None)
        if emb is not None:
            for m in _emb_modules(model):
                m._pending = None
                m._ready = None


def weight_syncc(dlrm, num_gpus, group=None) -> None:
    """s_q_g_p_c.py:963-970: all_reduce(SUM) * 1/N of every parameter, tables included.
    (Replicas initialised from the same seed are bit-identical, and for N = 2^k the sum
    then 1/N is exact, so this is then a no-op; it is kept for drop-in behaviour.) The
    tables' |W| hierarchy and INT4 rows are rebuilt afterwards."""
    with torch.no_grad():
        for _, param in dlrm.named_parameters():
            param.requires_grad_(False)
            if _world(group) > 1:
                dist.all_reduce(param, dist.ReduceOp.SUM, group=group)
            param.mul_(1.0 / num_gpus)
            param.requires_grad_(True)
        emb = getattr(dlrm, "emb_l", None)
        if emb is not None:
            for m in _emb_modules(dlrm):
                m._tset.refresh_absmax()
                if m._tset.packed is not None:
                    m._tset.refresh_scale_and_pack(m.embedding_bit)


def quantized_gradients_update(model, arg, lr, num_gpus) -> None:
    """s_q_g_p_c.py:687-712: dense all_reduce(SUM) / N of every parameter's gradient and
    param += update * (-lr[-1]). Embedding modules in grad_mode="dp" carry no dense
    gradient (their update goes through grad_update/weight_update_parallel_comm)."""
    with torch.no_grad():
        for _, param in model.named_parameters():
            if param.grad is None or param.grad.is_sparse:
                continue
            update = param.grad
            if _world() > 1:
                dist.all_reduce(update, op=dist.ReduceOp.SUM)
            update = update / num_gpus
            param.add_(update * (-lr[-1]))


def grad_precision_and_scale(*args, **kwargs):
    """s_q_g_p_c.py:158-255 (ranking-range per-table bit widths): not built yet."""
    raise NotImplementedError("ranking_range mixed-precision gradients are not built yet (SURVEY.md 8(f) #3)")


# the DP driver imports this misspelled name (dlrm_s_pytorch_tb_dp_one_parallel_comm.py:121)
grad_upduate_parallel_comm = grad_update_parallel_comm

__all__ = ["grad_update_parallel_comm", "grad_upduate_parallel_comm", "weight_update_parallel_comm",
           "clear_gradients", "weight_syncc", "quantized_gradients_update", "grad_precision_and_scale"]
