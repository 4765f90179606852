"""Drop-in for the reference's ``quantization_supp/quant_modules_not_quantize_grad.py``
embedding module, backed by libdqrm's HIP kernels (no CPU fallback).

``QuantEmbeddingBagTwo`` keeps the reference constructor and forward signature
(quant_modules_not_quantize_grad.py:240-248, :317), its attribute / buffer names and
state-dict keys (:258-280, :288), and its semantics (:317-398):

  * training forward: s = clamp(max|W|, 1e-8) / (2^(b-1)-1) over the WHOLE table
    (recomputed on every call, as the live snapshot does: the period counters only advance
    in stringified code, F4 in SURVEY.md), out = EmbeddingBag-sum, y = clamp(round(out/s))*s;
  * test_mode forward: the last training scale is reused (:331);
  * full_precision_flag: plain FP32 EmbeddingBag sum;
  * backward: STE (g*s)/s (quant_utils.py:349-363), then one of
      grad_mode="sparse"    -> the uncoalesced sparse COO ``embedding_bag.weight.grad``
                               nn.EmbeddingBag(sparse=True) produces (one entry per
                               lookup), for torch.optim.SGD; by default each row's entries
                               are pre-summed into its first one so the optimizer's
                               scatter-add is deterministic (set_sparse_grad_form),
      grad_mode="fused_sgd" -> the update W -= lr * grad is applied inside the backward
                               kernel with torch.optim.SGD's rounding (per lookup, in order),
      grad_mode="dp"        -> the gradient is kept on device for
                               sgd_quantized_gradients_parallel_comm.grad_update_parallel_comm.

``QuantEmbeddingBagCollection`` is the fused T-table form used to replace the per-table
loop of DLRM_Net.apply_emb (dlrm_s_pytorch_single_gpu.py:609-674): one launch per step for
all tables instead of 26.
"""
from __future__ import annotations

import os
import weakref
from typing import Sequence

import numpy as np
import torch
from torch import nn

from . import _lib as L
from .tables import EmbeddingTableSet, LookupBatch


_DEFAULT_GRAD_MODE = "sparse"
# every 8th training call polls the device error flags: a poll is a stream-ordered snapshot
# (event + pinned copy, ~20 us of host time), and the reference's driver calls 26 per-table
# modules per step
_ERROR_CHECK_EVERY = 8


_POOLING_ONE_HINT = False


def set_error_check_interval(steps: int) -> None:
    """Poll the tables' device error flags (out-of-range index, bad offsets) every `steps`
    training calls -- in the module's forward for grad_mode "sparse" / "fused_sgd", in
    weight_update_parallel_comm for "dp" -- and raise DQRMError when one is set (ATen raises
    on such input). Default 8; 0 = never. A poll never synchronises the host: it reads the
    last completed asynchronous snapshot of the flag word (EmbeddingTableSet.poll_errors) and
    takes the next one, so a flag raised just after a snapshot is read two polls later: a bad
    batch raises within about 2 * `steps` + 1 calls after the call that consumed it. Calls
    inside a HIP graph capture do not poll (the capture records device work only)."""
    global _ERROR_CHECK_EVERY
    _ERROR_CHECK_EVERY = max(0, int(steps))


def set_pooling_one_inputs(promise: bool) -> None:
    """Promise that every batch the modules see is in the Criteo form (one index per bag,
    offsets == arange(B), dlrm_data_pytorch.py:328-345) even when the offsets already live
    on the GPU (host offsets are checked without it); the kernels then never read the
    offsets. Off by default: nn.EmbeddingBag accepts any offsets."""
    global _POOLING_ONE_HINT
    _POOLING_ONE_HINT = bool(promise)


def _pooling_one_arg():
    return True if _POOLING_ONE_HINT else None


def error_check_due(owner) -> bool:
    d = owner.__dict__  # a plain attribute (nn.Module.__setattr__ is slow on the per-call path)
    n = d.get("_dqrm_err_calls", 0) + 1
    d["_dqrm_err_calls"] = n
    return _ERROR_CHECK_EVERY > 0 and n % _ERROR_CHECK_EVERY == 0


def poll_device_errors(tset) -> None:
    """Raise DQRMError if the last completed snapshot of `tset`'s error word is non-zero
    (the flags are then cleared); never blocks."""
    flags = tset.poll_errors()
    if flags:
        tset.read_errors(clear=True)
        raise_device_errors(flags)


def raise_device_errors(flags: int) -> None:
    if flags:
        raise L.DQRMError(f"embedding kernels flagged device errors 0x{flags:x} (1 = index out of range, "
                          "2 = bad offsets, 4 = more lookups than max_lookups)")


# grad_mode "sparse": the COO handed to the optimizer -- "presummed" (default: each row's
# gradient summed in lookup order into its first lookup, zeros after it, so the optimizer's
# scatter-add is deterministic) or "per_lookup" (one STE'd dy row per lookup, exactly what
# nn.EmbeddingBag(sparse=True) yields; ATen's atomic scatter-add of duplicate rows then varies
# in its last bits run to run on the GPU)
_SPARSE_GRAD_FORM = os.environ.get("DQRM_SPARSE_GRAD", "presummed")


def set_sparse_grad_form(form: str) -> None:
    """The COO form of grad_mode="sparse" modules: "presummed" (deterministic optimizer step;
    default) or "per_lookup" (nn.EmbeddingBag's own per-lookup entries)."""
    global _SPARSE_GRAD_FORM
    if form not in ("presummed", "per_lookup"):
        raise ValueError("form must be 'presummed' or 'per_lookup'")
    _SPARSE_GRAD_FORM = form


def set_default_grad_mode(mode: str) -> None:
    """Default ``grad_mode`` of modules constructed afterwards, so a driver can switch its
    unmodified ``QuantEmbeddingBagTwo(n, m, bit, embedding_id=i)`` calls
    (dlrm_s_pytorch_tb_dp_one_parallel_comm.py:380) to the DP path with one line."""
    global _DEFAULT_GRAD_MODE
    if mode not in _QuantEmbeddingBase.grad_modes:
        raise ValueError(f"grad_mode must be one of {_QuantEmbeddingBase.grad_modes}")
    _DEFAULT_GRAD_MODE = mode


# grad_mode "sparse" under torch.optim.SGD: when a plain SGD step (no momentum, weight decay,
# nesterov or maximize) is about to add a module's COO -- the one its last backward produced,
# untouched since (no accumulation, no in-place edit) -- the module applies that update itself
# with the reference's rounding: torch's sparse SGD adds -lr * g of every lookup to its row in
# lookup order (dlrm_s_pytorch_single_gpu.py:1943-1950), which dqrm_emb_bwd_sgd reproduces bit for
# bit (deterministic; ATen's GPU scatter-add orders duplicate rows by atomics), and then clears
# .grad so the optimizer skips it. Any other optimizer, or a modified grad, gets the COO as is.
# DQRM_SGD_HOOK=0 turns this off (the optimizer then adds the COO).
_SGD_HOOK = os.environ.get("DQRM_SGD_HOOK", "1") != "0"
_SGD_OWNERS: dict = {}  # id(embedding_bag.weight) -> (weakref(weight), weakref(module)); tensors
                        # compare elementwise, so a WeakKeyDictionary cannot key them
_SGD_HOOK_HANDLE = None


def set_fused_optimizer_step(enabled: bool) -> None:
    """Whether plain torch.optim.SGD steps on grad_mode="sparse" modules run as the module's own
    per-lookup SGD kernel (default; bit-exact with torch's sparse SGD in lookup order) or as
    the optimizer's add of the COO."""
    global _SGD_HOOK
    _SGD_HOOK = bool(enabled)


def _plain_sgd_group(opt, g) -> bool:
    return (isinstance(opt, torch.optim.SGD) and not g.get("momentum", 0) and not g.get("weight_decay", 0)
            and not g.get("nesterov", False) and not g.get("maximize", False))


def _sgd_step_pre_hook(opt, args, kwargs):
    """torch.optim global step pre-hook: the fused per-lookup SGD of every pending module whose
    weight this optimizer steps with plain SGD (see _SGD_HOOK)."""
    if not _SGD_HOOK or not _SGD_OWNERS:
        return None
    for g in opt.param_groups:
        if not _plain_sgd_group(opt, g):
            continue
        for p in g["params"]:
            ent = _SGD_OWNERS.get(id(p))
            if ent is None or ent[0]() is not p:
                continue
            m = ent[1]()
            if m is not None:
                m._apply_pending_sgd(p, float(g["lr"]))
    return None


def _register_sgd_owner(module, weight: nn.Parameter) -> None:
    global _SGD_HOOK_HANDLE
    if _SGD_HOOK_HANDLE is None:
        from torch.optim.optimizer import register_optimizer_step_pre_hook

        _SGD_HOOK_HANDLE = register_optimizer_step_pre_hook(_sgd_step_pre_hook)
    key = id(weight)
    _SGD_OWNERS[key] = (weakref.ref(weight, lambda _r, k=key: _SGD_OWNERS.pop(k, None)), weakref.ref(module))
    mref = weakref.ref(module)

    def _post_accumulate(p):
        m = mref()
        pend = m.__dict__.get("_sgd_pend") if m is not None else None
        if pend is None:
            return
        if pend["gid"] is None:  # the COO of the last backward, now p.grad
            pend["gid"], pend["gver"] = id(p.grad), p.grad._version
        else:  # accumulated into again: the optimizer adds the sum itself
            m._sgd_pend = None

    weight.register_post_accumulate_grad_hook(_post_accumulate)


# grad_mode "sparse": the rows an optimizer changed are synced by the next forward's own launch
# (dqrm_emb_fwd_after_update); DQRM_FUSE_SYNC=0 issues dqrm_rows_changed as a call of its own (A/B)
_FUSE_SYNC = os.environ.get("DQRM_FUSE_SYNC", "1") != "0"


def _on(x: torch.Tensor, device: torch.device) -> bool:
    """x already lives where the kernels launch: an index-less "cuda" device means the
    current device (the kernels' stream), so inputs on any other GPU are copied over."""
    d = x.device
    if d.type != device.type:
        return False
    idx = device.index
    if idx is None and device.type == "cuda":
        idx = torch.cuda.current_device()
    return idx is None or d.index == idx


def _batch_from_input(input: torch.Tensor, offsets: torch.Tensor | None, device) -> LookupBatch:
    """nn.EmbeddingBag input conventions: 1-D input + offsets, or 2-D [B, L] fixed bags."""
    if (input.dim() == 1 and offsets is not None and offsets.dim() == 1 and _on(input, device)
            and _on(offsets, device)):  # the drivers' per-table call: one table, no copies
        p1 = _pooling_one_arg() if input.numel() == offsets.numel() else False
        return LookupBatch.one_table(input, offsets, pooling_one=p1)
    if input.dim() == 2:
        if offsets is not None:
            raise ValueError("if input is 2D, then offsets has to be None")
        B, Lb = input.shape
        offsets = torch.arange(0, B * Lb, Lb, dtype=torch.int64, device=input.device)
        input = input.reshape(-1)
    elif offsets is None:
        raise ValueError("offsets has to be a 1D Tensor but got None")
    flat_off = offsets.reshape(-1)
    p1 = _pooling_one_arg() if input.numel() == flat_off.numel() else False
    return LookupBatch([input.reshape(-1)], [flat_off], device=device, pooling_one=p1)


class _EmbeddingFn(torch.autograd.Function):
    """Autograd bridge: forward = dqrm_emb_fwd; backward per the module's grad_mode."""

    @staticmethod
    def forward(ctx, weight, owner, batches, bits, flags_refresh, full_precision, layout, changed=None):
        tset: EmbeddingTableSet = owner._tset
        one = layout == "bd"  # one table: its [B, D] output itself (no select node after the Function)
        layout = "tbd" if one else layout
        y = tset.forward(batches, bits=bits, refresh_scale=flags_refresh, use_packed=owner._use_packed(full_precision),
                         full_precision=full_precision, layout=layout, changed_rows=changed)
        if one:
            y = y.view(y.shape[1], y.shape[2])
        ctx.one = one
        ctx.owner = owner
        ctx.batches = batches
        ctx.ste = not full_precision
        ctx.layout = layout
        return y

    @staticmethod
    def backward(ctx, dy):
        owner = ctx.owner
        dy = dy.contiguous()
        if ctx.one:
            dy = dy.view(1, dy.shape[0], dy.shape[1])
        grad_w = owner._backward(ctx.batches, dy, ctx.ste, ctx.layout)
        return grad_w, None, None, None, None, None, None, None


class _WeightHolder(nn.Module):
    """Carries ``weight`` so that the reference's attribute path
    ``module.embedding_bag.weight`` (and the state-dict key) is unchanged."""

    def __init__(self, weight: nn.Parameter, mode: str = "sum", sparse: bool = True):
        super().__init__()
        self.weight = weight
        self.mode = mode
        self.sparse = sparse


# per-call bookkeeping attributes of the modules: plain instance attributes, written without
# nn.Module.__setattr__'s parameter / buffer / submodule checks (the drivers call 26 modules a
# step, and the hooks reset these for every module)
_PLAIN_ATTRS = frozenset({"_pending", "_ready", "_rr", "_ext_rows", "_counters", "_exchange", "_dqrm_err_calls",
                          "_sgd_pend"})


class _QuantEmbeddingBase(nn.Module):
    grad_modes = ("sparse", "fused_sgd", "dp")

    def __setattr__(self, name, value):
        if name in _PLAIN_ATTRS:
            self.__dict__[name] = value
        else:
            super().__setattr__(name, value)

    def _init_common(self, grad_mode, lr, scale_period, use_packed_int4):
        if grad_mode is None:
            grad_mode = _DEFAULT_GRAD_MODE
        if grad_mode not in self.grad_modes:
            raise ValueError(f"grad_mode must be one of {self.grad_modes}")
        self.grad_mode = grad_mode
        self.lr = lr
        # period P of the (stringified in the snapshot) periodic scale refresh,
        # quant_modules_not_quantize_grad.py:303-315,354-363; 0 = every training call (live code)
        self.scale_period = int(scale_period)
        self.use_packed_int4 = bool(use_packed_int4)
        self._pending = None      # (batch, dy, ste, layout) for grad_mode == "dp"
        self._exchange = None     # SparseGradExchange of the ranking-range hooks
        self._ready = None        # grad bits of an exchanged, not yet applied update
        self._counters = None     # host mirror of (now_iteration, iteration_bound, iteration_nt)
        self._rr = None           # ranking range: (bits host int32 [T], bits dev, scale dev) of this step
        self._ext_rows = []       # rows of the sparse grads handed to an optimizer since the last sync
                                  # (grad_mode "sparse"; several with gradient accumulation)
        self._sgd_pend = None     # grad_mode "sparse": the last backward's (batch, dy, ...) for the
                                  # fused optimizer step (_sgd_step_pre_hook)

    def _sync_external_update(self) -> None:
        """grad_mode "sparse": the optimizer stepped W on the rows of the last COO outside
        libdqrm; bring their maxima (the refreshing forward's full-table scale) and INT4 rows
        up to date before the next forward reads them."""
        if self._ext_rows:
            rows = self._ext_rows[0] if len(self._ext_rows) == 1 else torch.cat(self._ext_rows)
            self._tset.rows_changed(rows, repack=self._use_packed(False))
            self._ext_rows = []

    def _check_errors(self, test_mode: bool) -> None:
        """grad_mode "sparse" / "fused_sgd": flags raised by the previous call's kernels
        surface here, at the next training call (the DP hooks check them for "dp")."""
        if (self.grad_mode != "dp" and not test_mode and error_check_due(self)
                and not torch.cuda.is_current_stream_capturing()):
            poll_device_errors(self._tset)

    # ------------------------------------------------------------ scale refresh logic
    def _refresh_due(self, fp: bool, test_mode: bool) -> bool:
        """q_m_n_q_g.py:331-363: recompute when training (or first call); with a period the
        counters now_iteration / iteration_bound / iteration_nt follow the reference code."""
        first = tuple(self.eb_scaling_factor.shape) == (self.batch_size, 1)
        if not ((not fp and not test_mode) or first):
            return False
        if self.scale_period <= 0:
            return True  # live snapshot: the counters never advance, now == bound == 0
        if self._counters is None:  # one host read after construction / load_state_dict
            self._counters = [int(self.now_iteration.item()), int(self.iteration_bound.item()),
                              int(self.iteration_nt.item())]
        now, bound, nt = self._counters
        due = now == bound
        if due:  # update period info + set_iteration_bound (q_m_n_q_g.py:303-315,354-363)
            nt += 1
            now = 0
            if nt == 1 and bound == 0:
                bound += self.scale_period
        else:
            nt += 1
            now += 1
        self._counters = [now, bound, nt]
        self.now_iteration.fill_(now)
        self.iteration_bound.fill_(bound)
        self.iteration_nt.fill_(nt)
        return due

    def _use_packed(self, full_precision: bool) -> bool:
        return self.use_packed_int4 and not full_precision and self._tset.packed is not None

    # ------------------------------------------------------------ backward
    def _backward(self, batch: LookupBatch, dy: torch.Tensor, ste: bool, layout: str):
        ts = self._tset
        if self.grad_mode == "fused_sgd":
            if self.lr is None:
                raise RuntimeError("grad_mode='fused_sgd' needs module.lr")
            ts.backward_sgd(batch, dy, self.lr, ste=ste, repack=self._use_packed(False), layout=layout)
            return None
        if self.grad_mode == "dp":
            self._pending = (batch, dy, ste, layout)
            return None
        return self._sparse_grad(batch, dy, ste, layout)

    def _sparse_grad(self, batch, dy, ste, layout):
        """The uncoalesced COO nn.EmbeddingBag(sparse=True) yields: one entry per lookup, in
        lookup order (one libdqrm launch, no host sync), which torch.optim.SGD adds to W as it
        adds the reference's own embedding gradient. Form "presummed" (default): each row's
        entries summed into its first one (the others +0.0), so that add is deterministic;
        "per_lookup": one STE'd dy row per lookup (set_sparse_grad_form)."""
        rows, vals = self._tset.lookup_grad(batch, dy, ste=ste, layout=layout,
                                            presum=_SPARSE_GRAD_FORM == "presummed")
        self._ext_rows.append(rows)
        # the fused optimizer step applies this update if the COO reaches a plain SGD step as
        # the weight's whole gradient (nothing accumulated before it: .grad is None now)
        self._sgd_pend = (dict(batch=batch, dy=dy, ste=ste, layout=layout, rows=rows, gid=None, gver=None)
                          if _SGD_HOOK and self.embedding_bag.weight.grad is None else None)
        return torch.sparse_coo_tensor(rows.view(1, -1), vals, (self._tset.R, self._tset.D), is_coalesced=False)

    def _apply_pending_sgd(self, p: nn.Parameter, lr: float) -> bool:
        """Called before a plain torch.optim.SGD step over `p` (this module's weight): if p.grad
        is still exactly the COO of the last backward, apply W -= lr * grad with torch's sparse
        SGD rounding per lookup in lookup order (dqrm_emb_bwd_sgd: the |W| hierarchy and INT4
        rows kept too), and clear p.grad so the optimizer skips it. Returns whether it did."""
        pend, self._sgd_pend = self._sgd_pend, None
        g = p.grad
        if (pend is None or g is None or pend["gid"] != id(g) or g._version != pend["gver"]
                or self.grad_mode != "sparse"):
            return False
        self._ext_rows = [r for r in self._ext_rows if r is not pend["rows"]]
        self._sync_external_update()  # rows an earlier optimizer step changed, first
        self._tset.backward_sgd(pend["batch"], pend["dy"], lr, ste=pend["ste"], repack=self._use_packed(False),
                                layout=pend["layout"])
        p.grad = None
        return True


class QuantEmbeddingBagTwo(_QuantEmbeddingBase):
    """quant_modules_not_quantize_grad.py:220-398, one table, on libdqrm."""

    def __init__(self, num_embeddings, embedding_dim, embedding_bit=4, full_precision_flag=False,
                 quant_mode="symmetric", fix_flag=False, weight_percentile=0, embedding_id=None, *,
                 device="cuda", weight: torch.Tensor | None = None, init: str = "numpy",
                 grad_mode: str | None = None, lr: float | None = None, scale_period: int = 0,
                 use_packed_int4: bool = False):
        super().__init__()
        self.num_embeddings = num_embeddings
        self.embedding_dim = embedding_dim
        self.embedding_bit = embedding_bit
        self.full_precision_flag = full_precision_flag
        self.quant_mode = quant_mode
        self.fix_flag = fix_flag
        self.weight_percentile = weight_percentile
        self.batch_size = 128
        self.embedding_id = embedding_id
        self._init_common(grad_mode, lr, scale_period, use_packed_int4)
        if weight is None and init == "numpy":
            # q_m_n_q_g.py:273-275: numpy global RNG, U(-sqrt(1/n), sqrt(1/n)), f32
            weight = torch.from_numpy(np.random.uniform(
                low=-np.sqrt(1 / num_embeddings), high=np.sqrt(1 / num_embeddings),
                size=(num_embeddings, embedding_dim)).astype(np.float32))
        self._tset = EmbeddingTableSet([num_embeddings], embedding_dim, device=device, packed=use_packed_int4,
                                       init=None if weight is not None else "uniform",
                                       weights=[weight] if weight is not None else None)
        dev = self._tset.device
        self.register_buffer("eb_scaling_factor", torch.zeros(self.batch_size, 1, device=dev), persistent=True)
        self.register_buffer("output_integer", torch.zeros((1, 16), device=dev), persistent=False)
        self.register_buffer("embedding_bound", torch.sqrt(torch.tensor(1 / num_embeddings, device=dev)) * 4.0,
                             persistent=False)
        self.register_buffer("now_iteration", torch.zeros(1, device=dev), persistent=True)
        self.register_buffer("iteration_bound", torch.zeros(1, device=dev), persistent=True)
        self.register_buffer("iteration_nt", torch.zeros(1, device=dev), persistent=True)
        self.register_buffer("emb_scaling_factor", torch.zeros(1, device=dev), persistent=True)
        self.register_buffer("gradient_bit_width", torch.zeros(1, device=dev), persistent=True)
        self.embedding_bag = _WeightHolder(nn.Parameter(self._tset.W, requires_grad=True))
        _register_sgd_owner(self, self.embedding_bag.weight)

    def __repr__(self):
        s = super().__repr__()
        return "(" + s + " embedding_bit = {}, full_precision_flag = {}, quant_mode = {})".format(
            self.embedding_bit, self.full_precision_flag, self.quant_mode)

    def fix(self):
        self.fix_flag = True

    def unfix(self):
        self.fix_flag = False

    def forward(self, input, offsets=None, per_sample_weights=None, full_precision_flag=False, test_mode=False):
        fp = bool(full_precision_flag or self.full_precision_flag)
        self._check_errors(test_mode)
        fuse_sync = _FUSE_SYNC and bool(self._ext_rows) and not self._use_packed(False)  # synced by the forward's launch
        if not fuse_sync:
            self._sync_external_update()
        if self.quant_mode not in ("symmetric", "speed_symmetric", "asymmetric"):
            raise ValueError("unknown quant mode: {}".format(self.quant_mode))
        refresh = self._refresh_due(fp, test_mode)
        if refresh and self.quant_mode != "symmetric":
            raise Exception("for embedding weights, we only support symmetric quantization")
        if per_sample_weights is not None:
            print("Warning: Embedding Table Assumes per_sample_weights to be None but it is not")
        batch = _batch_from_input(input, offsets, self._tset.device)
        if refresh and self._use_packed(fp):
            self._tset.refresh_scale_and_pack(self.embedding_bit)
            refresh_in_fwd = False
        else:
            refresh_in_fwd = refresh
        changed = None
        if fuse_sync:
            changed = self._ext_rows[0] if len(self._ext_rows) == 1 else torch.cat(self._ext_rows)
            self._ext_rows = []
        y = _EmbeddingFn.apply(self.embedding_bag.weight, self, batch, self.embedding_bit, refresh_in_fwd, fp, "bd",
                               changed)
        if refresh:
            # 0-d scale, as the reference stores it: a view of the set's scale, which every
            # refreshing forward rewrites in place (the buffer entry, without __setattr__)
            sv = self.__dict__.get("_scale0")
            if sv is None or sv[0] is not self._tset:
                sv = (self._tset, self._tset.scale.view(()))
                self.__dict__["_scale0"] = sv
            if self._buffers["eb_scaling_factor"] is not sv[1]:
                self._buffers["eb_scaling_factor"] = sv[1]
        return y

    def load_state_dict(self, state_dict, strict=True, assign=False):
        out = super().load_state_dict(state_dict, strict=strict, assign=assign)
        self._tset.refresh_absmax()  # W changed outside the kernels: rebuild the |W| hierarchy
        if self._tset.packed is not None:  # the loaded rows, packed with their own scales
            self._tset.repack_all(self.embedding_bit)
        self._counters = None
        return out


def can_consolidate(modules) -> bool:
    """Whether consolidate_tables(modules) would move the tables: at least two single-table
    modules, not yet one set, alike (device, dim, packed rows), and room on the device for a
    second copy of the tables while they move. Data-parallel callers agree this over the ranks
    before consolidating (the payload layout depends on it)."""
    mods = list(modules)
    if len(mods) < 2 or any(not isinstance(m, QuantEmbeddingBagTwo) for m in mods):
        return False
    first = mods[0]._tset
    if first.parent is not None and all(m._tset.parent is first.parent for m in mods):
        return False  # already one set
    dev, D = first.device, first.D
    packed = first.packed is not None
    if any(m._tset.device != dev or m._tset.D != D or (m._tset.packed is not None) != packed for m in mods):
        return False
    rows = [m._tset.num_rows[0] for m in mods]
    need = sum(rows) * (D * 4 + (D // 2 if packed else 0) + 4)  # W, INT4 rows, row maxima
    if dev.type == "cuda":
        free, _ = torch.cuda.mem_get_info(dev)
        if need * 1.1 + (256 << 20) > free:
            return False
    return True


def consolidate_tables(modules, force: bool = False) -> EmbeddingTableSet | None:
    """Move the tables of several single-table modules (the DP driver's ModuleList of
    QuantEmbeddingBagTwo, dlrm_s_pytorch_tb_dp_one_parallel_comm.py:380) into ONE table set:
    one slab per array, each module then running on a one-table view of it
    (EmbeddingTableSet.view) and each ``embedding_bag.weight`` Parameter keeping its identity
    with its data a view of the slab. The grad-comm hooks then launch once per phase for all
    tables instead of once per module. State is copied exactly (W, INT4 rows, scales; the
    |W| hierarchy is rebuilt from the same W, so it is bit-identical).

    Needs room for a second copy of the tables while they are moved (checked against the
    device's free memory unless force=True); returns the set, or None when the modules are
    already consolidated, are not all alike (device, dim, packed rows), or do not fit."""
    mods = list(modules)
    if len(mods) < 2 or any(not isinstance(m, QuantEmbeddingBagTwo) for m in mods):
        return None
    first = mods[0]._tset
    if first.parent is not None and all(m._tset.parent is first.parent for m in mods):
        return None  # already one set
    dev, D = first.device, first.D
    packed = first.packed is not None
    if any(m._tset.device != dev or m._tset.D != D or (m._tset.packed is not None) != packed for m in mods):
        return None
    rows = [m._tset.num_rows[0] for m in mods]
    need = sum(rows) * (D * 4 + (D // 2 if packed else 0) + 4)  # W, INT4 rows, row maxima
    if not force and dev.type == "cuda":
        free, _ = torch.cuda.mem_get_info(dev)
        if need * 1.1 + (256 << 20) > free:
            return None
    big = EmbeddingTableSet(rows, D, device=dev, packed=packed, init=None)
    with torch.no_grad():
        for t, m in enumerate(mods):
            old = m._tset
            big.table_weight(t).copy_(old.W)
            if packed:
                big.table_packed(t).copy_(old.packed)
            big.scale[t: t + 1].copy_(old.scale)
            big.pscale[t: t + 1].copy_(old.pscale)
    big.refresh_absmax()
    for t, m in enumerate(mods):
        m._tset = big.view(t)
        m.embedding_bag.weight.data = m._tset.W
        m._exchange = None
    return big


class QuantEmbeddingBagCollection(_QuantEmbeddingBase):
    """All tables of a DLRM in one resident slab; forward(lS_o, lS_i) replaces the per-table
    loop of DLRM_Net.apply_emb (dlrm_s_pytorch_single_gpu.py:609-674) with ONE launch."""

    def __init__(self, ln: Sequence[int], m: int, embedding_bit: int = 4, full_precision_flag: bool = False,
                 *, device="cuda", init: str = "numpy", weights: Sequence[torch.Tensor] | None = None,
                 grad_mode: str | None = None, lr: float | None = None, scale_period: int = 0,
                 use_packed_int4: bool = False, seed: int = 123):
        super().__init__()
        self.ln = [int(n) for n in ln]
        self.embedding_dim = int(m)
        self.embedding_bit = embedding_bit
        self.full_precision_flag = full_precision_flag
        self.quant_mode = "symmetric"
        self.batch_size = 128
        self._init_common(grad_mode, lr, scale_period, use_packed_int4)
        if weights is None and init == "numpy":
            weights = [torch.from_numpy(np.random.uniform(low=-np.sqrt(1 / n), high=np.sqrt(1 / n),
                                                          size=(n, m)).astype(np.float32)) for n in self.ln]
        self._tset = EmbeddingTableSet(self.ln, m, device=device, packed=use_packed_int4,
                                       init=None if weights is not None else "uniform", seed=seed, weights=weights)
        dev = self._tset.device
        T = len(self.ln)
        self.register_buffer("eb_scaling_factor", torch.zeros(self.batch_size, 1, device=dev), persistent=True)
        self.register_buffer("now_iteration", torch.zeros(1, device=dev), persistent=True)
        self.register_buffer("iteration_bound", torch.zeros(1, device=dev), persistent=True)
        self.register_buffer("iteration_nt", torch.zeros(1, device=dev), persistent=True)
        self.register_buffer("emb_scaling_factor", torch.zeros(T, device=dev), persistent=True)
        self.register_buffer("gradient_bit_width", torch.zeros(T, device=dev), persistent=True)
        self.embedding_bag = _WeightHolder(nn.Parameter(self._tset.W, requires_grad=True))
        _register_sgd_owner(self, self.embedding_bag.weight)

    def table_weight(self, t: int) -> torch.Tensor:
        return self._tset.table_weight(t)

    def forward(self, lS_o, lS_i, full_precision_flag=False, test_mode=False, layout="list"):
        """lS_o / lS_i: per-table lists or stacked [T, B] tensors (dlrm_data_pytorch.py:328-345).
        layout "list" -> list of T [B, D] tensors (apply_emb's ly); "btd" -> [B, T, D]."""
        fp = bool(full_precision_flag or self.full_precision_flag)
        self._check_errors(test_mode)
        self._sync_external_update()
        refresh = self._refresh_due(fp, test_mode)
        batch = LookupBatch(lS_i, lS_o, device=self._tset.device, pooling_one=_pooling_one_arg())
        if refresh and self._use_packed(fp):
            self._tset.refresh_scale_and_pack(self.embedding_bit)
            refresh_in_fwd = False
        else:
            refresh_in_fwd = refresh
        kl = "btd" if layout == "btd" else "tbd"
        y = _EmbeddingFn.apply(self.embedding_bag.weight, self, batch, self.embedding_bit, refresh_in_fwd, fp, kl)
        if refresh:
            self.eb_scaling_factor = self._tset.scale
        return list(y.unbind(0)) if layout == "list" else y

    def load_state_dict(self, state_dict, strict=True, assign=False):
        out = super().load_state_dict(state_dict, strict=strict, assign=assign)
        self._tset.refresh_absmax()
        if self._tset.packed is not None:  # the loaded rows, packed with their own scales
            self._tset.repack_all(self.embedding_bit)
        self._counters = None
        return out


__all__ = ["QuantEmbeddingBagTwo", "QuantEmbeddingBagCollection", "set_default_grad_mode", "set_sparse_grad_form",
           "set_fused_optimizer_step",
           "set_error_check_interval", "set_pooling_one_inputs", "consolidate_tables", "can_consolidate"]
