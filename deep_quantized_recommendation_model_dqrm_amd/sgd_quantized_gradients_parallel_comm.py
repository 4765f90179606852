"""Drop-in for the reference's grad-comm hooks (``sgd_quantized_gradients_parallel_comm.py``)
used by the data-parallel drivers (dlrm_s_pytorch_tb_dp_one_parallel_comm.py:1853-1907):

    clear_gradients(model)                                        s_q_g_p_c.py:714-734
    grad_update_parallel_comm(model, number_of_gpus, ...)         s_q_g_p_c.py:257-409
    weight_update_parallel_comm(model, lr, ...)                   s_q_g_p_c.py:601-668
    weight_syncc(dlrm, num_gpus)                                  s_q_g_p_c.py:963-970

``model`` exposes ``emb_l`` / ``bot_l`` / ``top_l`` as the reference's DLRM_Net does. The
embedding tables must be this package's modules built with ``grad_mode="dp"``: their
backward leaves the upstream gradient on the device, and the embedding branch below runs
ONE fused exchange for all modules of ``emb_l`` -- a QuantEmbeddingBagCollection or the
unchanged driver's ModuleList of 26 QuantEmbeddingBagTwo alike (comm.MultiSetExchange:
libdqrm kernels + two all-gathers per step) -- instead of the reference's 2 blocking Gloo
collectives per table. Results per table are the reference's: the averaged scale lands in
``emb_scaling_factor`` and the update applied by ``weight_update_parallel_comm`` is
W += -lr * ((sum_r q_r) * 1/N) * s  (integer sums exact). After the update the hooks read
the tables' device error flags (one shared word, one read per step; every
``set_error_check_interval`` steps) and raise DQRMError if a kernel flagged bad input.

The MLP branch (QuantLinear-like layers of bot_l, top_l -- those carrying
``weight_scaling_factor``, as the reference's isinstance(QuantLinear / LinearCompressedGrad)
checks select, s_q_g_p_c.py:339,376,632,652; plain nn.Linear only after
``set_mlp_plain_linear(True)``) runs
quantize_linear_grad / quantize_bias_grad (s_q_g_p_c.py:892-961) for all layers as one
channel table through libdqrm's dense kernels (dense.DenseGradExchange): one all-gather of
the per-channel scales and one exact integer-valued fp16 all-reduce per step instead of 4
blocking collectives per layer. The layers must live on the GPU (no CPU path).
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist
from torch import nn

from . import _lib as L
from .comm import ConsolidatedExchange, MultiSetExchange, SparseGradExchange
from .dense import DenseGradExchange
from .quant_modules_not_quantize_grad import (_QuantEmbeddingBase, can_consolidate, consolidate_tables,
                                              error_check_due, poll_device_errors, set_error_check_interval)

_MLP_PLAIN_LINEAR = False


def set_mlp_plain_linear(include: bool) -> None:
    """Also exchange/update plain nn.Linear MLP layers (the reference touches only
    QuantLinear / LinearCompressedGrad layers and leaves plain Linear ones alone)."""
    global _MLP_PLAIN_LINEAR
    _MLP_PLAIN_LINEAR = bool(include)


# ---------------------------------------------------------------------------- helpers
def _world(group=None) -> int:
    return dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1


def _mset(model, name: str, value) -> None:
    """The hooks' per-step bookkeeping on the driver's model: a plain instance attribute
    (nn.Module.__setattr__'s checks are a measurable share of the hooks' host time)."""
    model.__dict__[name] = value


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
    return [l for l in seq if type(l).__name__ in ("QuantLinear", "LinearCompressedGrad")
            or (isinstance(l, nn.Linear) and _MLP_PLAIN_LINEAR)]


def _detach_grad(g: torch.Tensor) -> None:
    if g.grad_fn is not None:
        g.detach_()
    else:
        g.requires_grad_(False)


# ---------------------------------------------------------------------------- embedding branch
def _ensure_exchange(m: _QuantEmbeddingBase, grad_bits: int, group) -> SparseGradExchange:
    batch = m._pending[0]
    ex = m._exchange
    fresh = ex is None or ex.grad_bits != grad_bits or ex.group is not group or ex.tables is not m._tset
    if fresh or _outgrown([batch.max_lookups], [ex.max_lookups], group):
        need = max(batch.max_lookups, 1) if fresh else max(batch.max_lookups, ex.max_lookups)
        cap = _agreed_caps([need], group, m._tset.device)[0]
        ex = SparseGradExchange(m._tset, cap, grad_bits=grad_bits, group=group, device=m._tset.device)
        m._exchange = ex
    return ex


_CONSOLIDATE = True


def set_consolidate_tables(enable: bool) -> None:
    """Whether the hooks move a ModuleList of per-table modules into one table set the first
    time they see it (quant_modules_not_quantize_grad.consolidate_tables; skipped anyway when
    a second copy of the tables would not fit in device memory). On by default."""
    global _CONSOLIDATE
    _CONSOLIDATE = bool(enable)


_MAX_LOOKUPS = 0


def set_max_lookups(n: int) -> None:
    """Lookups per table and rank the embedding exchange plans its payload for (0: the
    first step's, taken as the maximum over the ranks). The payload layout must agree on
    every rank, so with N > 1 a later batch with more lookups than planned raises instead of
    resizing one rank alone; drivers with variable-size bags (random multi-hot data) set
    B * max_pooling here on every rank."""
    global _MAX_LOOKUPS
    _MAX_LOOKUPS = max(0, int(n))


def _agreed_caps(need: list[int], group, dev) -> list[int]:
    """Element-wise max of `need` over the ranks (one small all-reduce and one host read,
    when the exchange is built -- not per step), so every rank sizes the same payload."""
    need = [max(n, _MAX_LOOKUPS) for n in need]
    if _world(group) == 1:
        return need
    on_dev = dist.get_backend(group) == "nccl"
    t = torch.tensor(need, dtype=torch.int64, device=dev if on_dev else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return [int(x) for x in t.cpu().tolist()]


def _outgrown(need, caps, group) -> bool:
    """A batch beyond the planned capacity: rebuild at N = 1; at N > 1 only this rank knows,
    so raise rather than resize one rank's payload alone."""
    if not any(n > c for n, c in zip(need, caps)):
        return False
    if _world(group) > 1:
        raise L.DQRMError(f"a batch has {max(need)} lookups per table, beyond the {max(caps)} the embedding "
                          "exchange planned on every rank: call set_max_lookups(n) on all ranks")
    return True


def _all_ranks_agree(ok: bool, group, dev) -> bool:
    """True only if `ok` holds on every rank of the group (one all-reduce MIN, at setup)."""
    if _world(group) == 1:
        return ok
    on_dev = dist.get_backend(group) == "nccl"
    t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev if on_dev else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    return bool(t.item())


def _consolidated_set(model, mods, group=None):
    """The one set holding every module's table (consolidating on first use), or None. The
    choice changes the payload layout (one consolidated set vs one payload section per set),
    so at N > 1 the tables are consolidated only if EVERY rank can (free device memory may
    differ between ranks)."""
    big = getattr(model, "_dqrm_consolidated", None)
    if big is None:
        big = False
        if len(mods) > 1:
            ok = _all_ranks_agree(_CONSOLIDATE and can_consolidate(mods), group, mods[0]._tset.device)
            if ok:
                big = consolidate_tables(mods, force=True) or False
        _mset(model, "_dqrm_consolidated", big)
    if big is False:
        first = mods[0]._tset.parent
        if first is not None and len(mods) == first.T and all(
                m._tset.parent is first and m._tset.parent_index == t for t, m in enumerate(mods)):
            return first  # consolidated by the caller
        return None
    if all(m._tset.parent is big for m in mods):
        return big
    return None


def _emb_exchange(model, mods: list[_QuantEmbeddingBase], grad_bits: int, group):
    """The model's one exchange over all its embedding modules (cached; rebuilt when the
    modules, bits, group or a batch beyond the planned lookups change). The modules' table
    sets share one device error word so one read per step covers them all. A ModuleList of
    per-table modules is consolidated into one set (ConsolidatedExchange: one launch per
    phase); otherwise one MultiSetExchange over the modules' sets."""
    big = _consolidated_set(model, mods, group) if len(mods) > 1 else None
    if big is not None and all(m._pending is not None for m in mods) \
            and len({m._pending[0].num_bags for m in mods}) == 1:
        need = max(max(m._pending[0].max_lookups, 1) for m in mods)
        key = ("consolidated", id(big), grad_bits, id(group), _world(group))
        ex = getattr(model, "_dqrm_emb_exchange", None)
        fresh = ex is None or ex[0] != key
        if fresh or _outgrown([need], ex[1].max_lookups[:1], group):
            cap = _agreed_caps([need if fresh else max(need, ex[1].max_lookups[0])], group, big.device)[0]
            ex = (key, ConsolidatedExchange(big, cap, grad_bits=grad_bits, group=group))
            _mset(model, "_dqrm_emb_exchange", ex)
            for t, m in enumerate(mods):  # the modules' emb_scaling_factor: views of the averaged scales
                m.emb_scaling_factor = ex[1].scales[t]
        return ex[1]
    need = [max(m._pending[0].max_lookups if m._pending is not None else 1, 1) for m in mods]
    key = (tuple(id(m._tset) for m in mods), grad_bits, id(group), _world(group))
    ex = getattr(model, "_dqrm_emb_exchange", None)
    fresh = ex is None or ex[0] != key
    if fresh or _outgrown(need, ex[1].max_lookups, group):
        caps = _agreed_caps(need if fresh else [max(n, c) for n, c in zip(need, ex[1].max_lookups)], group,
                            mods[0]._tset.device)
        ex = (key, MultiSetExchange([m._tset for m in mods], caps, grad_bits=grad_bits, group=group,
                                    device=mods[0]._tset.device))
        _mset(model, "_dqrm_emb_exchange", ex)
        word = mods[0]._tset.err
        for m in mods[1:]:
            m._tset.share_error_word(word)
    return ex[1]


def _check_device_errors(model, mods: list[_QuantEmbeddingBase]) -> None:
    """Raise if a kernel flagged bad input (out-of-range index or offset, understated
    max_lookups): the reference would have raised in ATen instead of training on. One
    non-blocking poll per distinct error word (the flags of a step surface a step or two
    later; no host synchronisation)."""
    if not error_check_due(model):
        return
    seen = set()
    for m in mods:
        ptr = m._tset.err.data_ptr()
        if ptr in seen:
            continue
        seen.add(ptr)
        poll_device_errors(m._tset)


def grad_update_parallel_comm(model, number_of_gpus, emb_grad_quantized=True, num_bits=16, ranking_range=False,
                              rank_for_debug=None, iteration_count=None, mlp_layer_quantized=True, group=None):
    """s_q_g_p_c.py:257-409. Embedding tables: fused coalesce -> scale all-gather ->
    quantize-pack -> payload all-gather (emb_grad_quantized=False: FP32 payloads, the
    unquantized sparse all_reduce of :319-327). MLP layers: see module docstring."""
    if emb_grad_quantized and not ranking_range and not 2 <= int(num_bits) <= 16:
        raise ValueError("num_bits must be in 2..16 for quantized embedding gradients")
    with torch.no_grad():
        if ranking_range and emb_grad_quantized:  # :280-301, per-table bits from grad_precision_and_scale
            for m in _emb_modules(model):
                if m._pending is None:
                    continue
                if m._rr is None:
                    raise RuntimeError("ranking_range=True needs grad_precision_and_scale(...) first "
                                       "(dlrm_s_pytorch_tb_dp_one_parallel_comm.py:1897-1898)")
                m._exchange.exchange_ranked(m._rr[1], m._rr[2])
                m._ready = "ranked"
        else:
            mods = _emb_modules(model)
            for m in mods:
                if m.grad_mode != "dp":
                    raise ValueError("grad_update_parallel_comm needs embedding modules built with grad_mode='dp'")
            if any(m._pending is not None for m in mods):
                if _world(group) != number_of_gpus:
                    raise ValueError(f"number_of_gpus={number_of_gpus} but the process group has "
                                     f"{_world(group)} ranks")
                bits = int(num_bits) if emb_grad_quantized else 32
                ex = _emb_exchange(model, mods, bits, group)
                s_avg = ex.exchange([m._pending for m in mods])
                for m, s in zip(mods, s_avg):
                    if bits != 32 and s.data_ptr() != m.emb_scaling_factor.data_ptr():
                        m.emb_scaling_factor.copy_(s.view_as(m.emb_scaling_factor))
                    m._pending = None
                    m._ready = bits
                _mset(model, "_dqrm_emb_ready", (ex, bits, mods))
        _mlp_grad_update(model, number_of_gpus, mlp_layer_quantized, group)


def _mlp_exchange(model, n: int, quantized: bool, group) -> DenseGradExchange | None:
    layers = _linear_layers(model, "bot_l") + _linear_layers(model, "top_l")
    layers = [l for l in layers if l.weight.grad is not None]
    if not layers:
        return None
    bits = 8 if quantized else 32  # the reference hard-codes num_bits=8 (s_q_g_p_c.py:341,350)
    key = (tuple(id(l) for l in layers), bits, id(group), _world(group))
    ex = getattr(model, "_dqrm_dense_exchange", None)
    if ex is None or ex[0] != key:
        ex = (key, DenseGradExchange(layers, grad_bits=bits, group=group))
        _mset(model, "_dqrm_dense_exchange", ex)
    return ex[1]


def _mlp_grad_update(model, n: int, quantized: bool, group) -> None:
    """MLP branch (s_q_g_p_c.py:337-409): quantize_linear_grad / quantize_bias_grad for
    every layer, as one channel table (libdqrm dense kernels + 2 collectives)."""
    if _world(group) != n:
        raise ValueError(f"number_of_gpus={n} but the process group has {_world(group)} ranks")
    ex = _mlp_exchange(model, n, quantized, group)
    if ex is None:
        return
    for l in ex.channels.layers:
        _detach_grad(l.weight.grad)
        _detach_grad(l.bias.grad)
    ex.exchange()
    _mset(model, "_dqrm_dense_ready", ex)


def weight_update_parallel_comm(model, lr, emb_grad_quantized=True, update_embedding=True, num_gpus=1,
                                rank_for_debug=None, ranking_range=False, use_ec=False, mlp_layer_quantized=True):
    """s_q_g_p_c.py:601-668: W += -lr * grad * s for the tables (one libdqrm launch for all
    tables of a module) and the MLP layers."""
    if use_ec:
        raise NotImplementedError("error compensation (use_ec) is off in the reference's scripts and not built")
    with torch.no_grad():
        mods = _emb_modules(model)
        batched = getattr(model, "_dqrm_emb_ready", None)
        if batched is not None:  # the one exchange of grad_update_parallel_comm (:601-628)
            ex, bits, bmods = batched
            if (bits != 32) != bool(emb_grad_quantized):
                raise ValueError("emb_grad_quantized differs from the one used by grad_update_parallel_comm")
            if update_embedding:
                ex.apply(lr, mode=L.DQRM_UPD_DP if bits != 32 else L.DQRM_UPD_FP32,
                         repack=[m._use_packed(False) for m in bmods])
            elif hasattr(ex, "discard"):  # no update: settle the scales, release (batch, dy)
                ex.discard()
            for m in bmods:
                m._ready = None
            _mset(model, "_dqrm_emb_ready", None)
        for m in mods:
            ready = getattr(m, "_ready", None)
            if ready is None:
                continue
            if ready == "ranked":  # :610-622
                if not (ranking_range and emb_grad_quantized):
                    raise ValueError("ranking_range differs from the one used by grad_update_parallel_comm")
                if update_embedding:
                    bits_h, bits_d, scale_d = m._rr
                    repack = m._use_packed(False)
                    m._exchange.apply_ranked(lr, scale_d, repack=repack)  # 8-bit tables: W += -lr * (g * s)
                    if (bits_h == 32).any():  # 32-bit tables: W.add_(-lr * grad), the rank's own gradient
                        batch, dy, ste, layout = m._pending
                        mask = (bits_d == 32).to(torch.int32)
                        m._exchange.kernels.local_update(batch, dy, ste, layout, lr, mask, repack)
                m._pending = None
                m._ready = None
                m._rr = None
        _check_device_errors(model, mods)
        ex = getattr(model, "_dqrm_dense_ready", None)
        if ex is not None:  # MLP branch (:630-668), one libdqrm launch for all layers
            if (ex.grad_bits != 32) != bool(mlp_layer_quantized):
                raise ValueError("mlp_layer_quantized differs from the one used by grad_update_parallel_comm")
            ex.apply(lr)
            _mset(model, "_dqrm_dense_ready", None)


def clear_gradients(model) -> None:
    """s_q_g_p_c.py:714-734, plus dropping any not-yet-exchanged embedding gradient."""
    _mset(model, "_dqrm_emb_ready", None)
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
                m._rr = None


def _checksums(params, dev) -> torch.Tensor | None:
    """One position-dependent 64-bit checksum per parameter (dqrm_checksum64), int64 [P] on
    `dev`; None if a parameter cannot be hashed in place (not f32 / 16-B aligned / on dev)."""
    lib = L.load()
    out = torch.zeros(len(params), dtype=torch.int64, device=dev)
    for i, p in enumerate(params):
        if p.dtype != torch.float32 or not p.is_contiguous() or p.device != dev or p.data_ptr() % 16:
            return None
        L.check(lib.dqrm_checksum64(p.data_ptr(), p.numel(), out[i:].data_ptr(), _stream()), "dqrm_checksum64")
    return out


def _stream() -> int:
    from .tables import _stream_handle
    return _stream_handle()


def _replicas_identical(params, dev, group) -> bool:
    """Whether every rank holds the same bits in every parameter: one all-gather of the
    per-parameter checksums and one host read per weight_syncc call."""
    cs = _checksums(params, dev)
    if cs is None:
        return False
    world = _world(group)
    nccl = dist.get_backend(group) == "nccl"
    mine = cs if nccl else cs.cpu()
    allcs = torch.zeros(world, mine.numel(), dtype=torch.int64, device=mine.device)
    dist.all_gather_into_tensor(allcs.view(-1), mine, group=group) if nccl else \
        dist.all_gather(list(allcs.unbind(0)), mine, group=group)
    allcs = allcs.cpu()
    return bool((allcs == allcs[0]).all())


def _ring_mean_is_identity(p: torch.Tensor, world: int, num_gpus: int, absmax: float) -> bool:
    """The all-reduce of `world` identical copies times 1/num_gpus returns x unchanged for
    world = num_gpus in {1, 2, 4} (dqrm_replica_mean; checked exhaustively over the f32
    mantissas) unless world * |x| overflows."""
    return world == num_gpus and world in (1, 2, 4) and absmax * world < 3.0e38


def _sync_params(params, num_gpus: int, group, table_of: dict) -> set:
    """weight_syncc's arithmetic over `params`; table_of maps a table parameter's data_ptr to
    its table set (whose tmax bounds |W| without a pass over W). Returns the data_ptrs of
    the parameters whose values changed."""
    world = _world(group)
    if not params:
        return set()
    dev = params[0].device
    identical = world == 1 or (dev.type == "cuda" and _replicas_identical(params, dev, group))
    inv = float(np.float32(1.0 / num_gpus))
    absmax = [0.0] * len(params)
    if identical and world == num_gpus and world in (1, 2, 4):  # |x| bound of the identity check
        mx = []
        for p in params:
            ts = table_of.get(p.data_ptr())
            if ts is not None:  # a table: its exact max |W| (the hierarchy's, no pass over W)
                mx.append(ts.tmax.max())
            else:
                mx.append(p.detach().abs().max() if p.numel() else p.new_zeros(()))
        absmax = torch.stack(mx).float().cpu().tolist()
    changed = set()
    lib = L.load()
    for i, param in enumerate(params):
        rg = param.requires_grad
        param.requires_grad_(False)
        if not identical:  # the reference's all-reduce
            dist.all_reduce(param, dist.ReduceOp.SUM, group=group)
            param.mul_(1.0 / num_gpus)
            changed.add(param.data_ptr())
        elif not _ring_mean_is_identity(param, world, num_gpus, absmax[i]):
            if param.dtype == torch.float32 and param.is_contiguous() and param.data_ptr() % 16 == 0:
                L.check(lib.dqrm_replica_mean(param.data_ptr(), param.numel(), world, inv, _stream()),
                        "dqrm_replica_mean")
            else:  # same arithmetic in torch (element-wise, IEEE-rounded)
                acc = param.clone()
                for _ in range(world - 1):
                    acc.add_(param)
                param.copy_(acc.mul_(inv))
            changed.add(param.data_ptr())
        param.requires_grad_(rg)
    return changed


def _refresh_tables(sets_bits) -> None:
    """|W| hierarchy rebuild (and INT4 repack) of table sets whose W changed outside the
    update kernels."""
    for ts, bits in sets_bits:
        ts.refresh_absmax()
        if ts.packed is not None:
            ts.repack_all(bits)


def weight_syncc(dlrm, num_gpus, group=None) -> None:
    """s_q_g_p_c.py:963-970: all_reduce(SUM) * 1/N of every parameter, tables included,
    every 200 iterations of the DP driver (dlrm_s_pytorch_tb_dp_one_parallel_comm.py:1924-1936).

    The DP step keeps replicas bit-identical by construction, and the reference's result on
    identical replicas is computable locally: a ring all-reduce (Gloo's ring_chunked on the
    reference's CPU ranks, RCCL's ring here) adds the ranks one after another, so every
    element becomes fl(fl(...fl(x + x) + x ...) * 1/N) (dqrm_replica_mean) -- x itself for
    N = 1, 2, 4, an ulp away for about half of the elements at N = 3 or 8 (pinned against
    real Gloo at N = 3, 5, 6, 8 by tests/golden/syncc_gloo.npz). So: one
    all-gather of per-parameter checksums (dqrm_checksum64); if every rank holds the same
    bits, that local map (skipped where it is the identity) instead of the all-reduce --
    bit-exact with the reference and a few streaming passes over HBM instead of an
    all-reduce of the whole model (198 GB of tables at the config-5 shape); otherwise (e.g.
    ranks initialised from different random tables, as the reference's are before training,
    dlrm_s_pytorch_tb_dp_one_parallel_comm.py:1801) the reference's all-reduce. The
    tables' |W| hierarchy and INT4 rows are rebuilt when W changed."""
    with torch.no_grad():
        params = [p for _, p in dlrm.named_parameters()]
        mods = _emb_modules(dlrm) if getattr(dlrm, "emb_l", None) is not None else []
        table_of = {m.embedding_bag.weight.data_ptr(): m._tset for m in mods}
        changed = _sync_params(params, num_gpus, group, table_of)
        todo, seen = [], set()
        for m in mods:
            if m.embedding_bag.weight.data_ptr() not in changed:
                continue
            ts = m._tset.parent if m._tset.parent is not None else m._tset
            if id(ts) not in seen:
                seen.add(id(ts))
                todo.append((ts, m.embedding_bit))
        _refresh_tables(todo)


def sync_table_set(ts, num_gpus: int, group=None, bits: int = 4) -> bool:
    """weight_syncc for one resident table set (the bench's, or a QuantEmbeddingBagCollection's
    ``_tset``): returns whether W changed."""
    with torch.no_grad():
        changed = _sync_params([ts.W], num_gpus, group, {ts.W.data_ptr(): ts})
        if changed:
            _refresh_tables([(ts, bits)])
        return bool(changed)


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


def _rr_thresholds(T: int):
    """Last positions of the 0-bit and 8-bit groups in the sampled order: (8, 22) for the
    reference's 26 tables (:228-236); other table counts keep the same proportions."""
    if T == 26:
        return 8, 22
    return int(round(T * 9 / 26)) - 1, int(round(T * 23 / 26)) - 1


def grad_precision_and_scale(model, number_of_gpus, rank_for_debug=None, output_flag=False, group=None):
    """s_q_g_p_c.py:158-255, ranking-range mixed precision (called after backward, before
    grad_update/weight_update_parallel_comm(..., ranking_range=True)).

    Per table: range = max |coalesced grad| (finding_range_for_gradient), all-reduced / N
    (one all-gather of all tables' per-slot maxima, summed in descending rank order);
    emb_scaling_factor = range. Rank 0 ranks the tables with numpy's global RNG,
    np.random.choice(T, T, replace=False, p=range/(eb_scale*7) normalised)[::-1], and gives
    the first 9 positions 0 bits, the next 14 8 bits and the rest 32 bits; the widths are
    broadcast, and 8-bit tables get emb_scaling_factor = clamp(range, 1e-8) / 127."""
    import numpy as np

    with torch.no_grad():
        if _world(group) != number_of_gpus:
            raise ValueError(f"number_of_gpus={number_of_gpus} but the process group has {_world(group)} ranks")
        per, range_list = [], []
        for m in _emb_modules(model):
            if m.grad_mode != "dp":
                raise ValueError("grad_precision_and_scale needs embedding modules built with grad_mode='dp'")
            if m._pending is None:
                raise RuntimeError("grad_precision_and_scale needs a backward pass since the last update")
            batch, dy, ste, layout = m._pending
            ex = _ensure_exchange(m, 8, group)
            rg = ex.coalesce_ranges(batch, dy, ste=ste, layout=layout)
            eb = m._tset.scale.cpu().numpy().astype(np.float32)  # eb_scaling_factor of each table
            range_list += [float(x) for x in (rg / (eb * np.float32(7))).astype(np.float32)]
            per.append((m, rg))
        Tt = len(range_list)
        bits = torch.zeros(Tt, dtype=torch.int32)
        rank = dist.get_rank(group) if _world(group) > 1 else 0
        if rank == 0:
            prob_l = np.asarray(range_list) / (np.sum(range_list))
            list_id = np.random.choice(Tt, Tt, replace=False, p=prob_l)
            list_id = list_id[::-1]
            if rank_for_debug == 0 and output_flag:
                print("rank {} ranking from least wide range to the widest range {}".format(rank_for_debug, list_id))
            z, e = _rr_thresholds(Tt)
            for j, t in enumerate(list_id):
                bits[t] = 0 if j <= z else (8 if j <= e else 32)
        if _world(group) > 1:
            dist.barrier(group=group)
            dev = per[0][0]._tset.device if dist.get_backend(group) == "nccl" else torch.device("cpu")
            bd = bits.to(dev)
            dist.broadcast(bd, 0, group=group)
            bits = bd.cpu()
        off = 0
        for m, rg in per:
            b = bits[off: off + len(rg)].numpy()
            off += len(rg)
            n = np.float32(127.0)  # 2 ** (8 - 1) - 1: the only quantized width ranking assigns
            scale = np.where(b == 8, (np.maximum(rg, np.float32(1e-8)) / n).astype(np.float32), rg).astype(np.float32)
            m.emb_scaling_factor.copy_(torch.from_numpy(scale).view_as(m.emb_scaling_factor))
            m.gradient_bit_width.copy_(torch.from_numpy(b.astype(np.float32)).view_as(m.gradient_bit_width))
            dev = m._tset.device
            m._rr = (b.copy(), torch.from_numpy(b.copy()).to(dev), torch.from_numpy(scale).to(dev))


# the DP driver imports this misspelled name (dlrm_s_pytorch_tb_dp_one_parallel_comm.py:121)
grad_upduate_parallel_comm = grad_update_parallel_comm

__all__ = ["grad_update_parallel_comm", "grad_upduate_parallel_comm", "weight_update_parallel_comm",
           "clear_gradients", "weight_syncc", "quantized_gradients_update", "grad_precision_and_scale",
           "set_mlp_plain_linear", "set_error_check_interval", "set_consolidate_tables", "set_max_lookups",
           "sync_table_set"]
