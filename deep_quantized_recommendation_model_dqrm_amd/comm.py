"""INT8-quantized sparse-gradient all-reduce for data-parallel embedding training.

Reference: sgd_quantized_gradients_parallel_comm.py
  quantize_emb_grad            :850-890  (coalesce, scale, all_reduce(scale), quantize,
                                          all_reduce(sparse), * 1/N)
  grad_update_parallel_comm    :257-317  (26 tables, 2 blocking collectives each)
  weight_update_parallel_comm  :601-628  (W += -lr * grad * s)

MI355X design: the 52 per-table Gloo collectives of the reference become TWO collectives
per step for all tables together, both all-gathers over RCCL (torch.distributed "nccl"
on ROCm, xGMI point-to-point):
  1. all_gather of the per-slot max|grad| [T*8] -> every rank derives each rank's
     local scale and averages them in Gloo's order (bit-identical on every rank);
  2. all_gather of one fixed-capacity payload per rank  {counts i32[T*8] (per table and
     row-range slot), rows i32[CAP], q int8[CAP, D]} -> every rank decodes all N payloads, unions rows and sums the
     integers exactly (= Gloo sparse all_reduce, torch-internal: coalesce, allgather,
     sum, coalesce), then applies the dequantized SGD update.
Kernels: dqrm_emb_bwd_coalesce (K4), dqrm_grad_quant_pack (K5), dqrm_apply_sparse_update (K6).
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Protocol

import torch
import torch.distributed as dist

from . import _lib as L
from .tables import CoalescedGrad, EmbeddingTableSet, LookupBatch, _ptr, _stream_handle, default_caps


class ExchangeKernels(Protocol):
    """The three device steps of the exchange (HIP by default; tests may inject a checker)."""

    def coalesce(self, batch: LookupBatch, dy: torch.Tensor, ws: CoalescedGrad, ste: bool,
                 layout: str) -> None: ...

    def quant_pack(self, ws: CoalescedGrad, absmax_all: torch.Tensor, num_ranks: int, grad_bits: int,
                   cap_base: torch.Tensor, cap_total: int, s_avg: torch.Tensor, payload: torch.Tensor) -> None: ...

    def apply(self, cap_base: torch.Tensor, cap_total: int, gathered: torch.Tensor, payload_bytes: int,
              num_ranks: int, grad_bits: int, s_avg: torch.Tensor, lr: float, mode: int, repack: bool) -> None: ...

    def quant_pack_ranked(self, ws: CoalescedGrad, table_bits: torch.Tensor, table_scale: torch.Tensor,
                          cap_base: torch.Tensor, cap_total: int, payload: torch.Tensor) -> None: ...

    def local_update(self, batch: LookupBatch, dy: torch.Tensor, ste: bool, layout: str, lr: float,
                     table_mask: torch.Tensor, repack: bool) -> None: ...

    def coalesce_apply_local(self, batch: LookupBatch, dy: torch.Tensor, ws: CoalescedGrad, ste: bool, layout: str,
                             grad_bits: int, s_avg: torch.Tensor, lr: float, repack: bool) -> None: ...


class HipExchangeKernels:
    """libdqrm kernels; the only implementation the product uses."""

    def __init__(self, tables: EmbeddingTableSet):
        self.tables = tables
        self.lib = tables.lib

    def coalesce(self, batch, dy, ws, ste, layout):
        self.tables.backward_coalesce(batch, dy, ws, ste=ste, layout=layout)

    def quant_pack(self, ws, absmax_all, num_ranks, grad_bits, cap_base, cap_total, s_avg, payload):
        """absmax_all [N, T*S] may be a column slice of a wider gathered buffer (its row
        stride is passed as the pitch); payload a 16-B aligned slice of a wider one."""
        t = self.tables
        pitch = absmax_all.stride(0) if absmax_all is not None and absmax_all.dim() == 2 else t.T * L.DQRM_TABLE_SPLIT
        L.check(
            self.lib.dqrm_grad_quant_pack_strided(
                t.T, t.D, _ptr(ws.slot_cap_base), ws.cap_total, _ptr(ws.rows), _ptr(ws.vals), _ptr(ws.ucount),
                _ptr(absmax_all), pitch, num_ranks, grad_bits, _ptr(cap_base), cap_total, _ptr(s_avg),
                _ptr(payload), _stream_handle()),
            "dqrm_grad_quant_pack",
        )

    def apply(self, cap_base, cap_total, gathered, payload_bytes, num_ranks, grad_bits, s_avg, lr, mode, repack,
              workspace=None):
        """gathered [N, payload_bytes] may be a column slice of a wider gathered buffer. workspace:
        the merge apply's positions (dqrm_apply_workspace_bytes; allocated here when None and the
        merge kernels would take N > 1 ranks)."""
        t = self.tables
        pitch = gathered.stride(0) if gathered.dim() == 2 else payload_bytes
        if num_ranks > 1:
            if workspace is None:
                n = int(self.lib.dqrm_apply_workspace_bytes(num_ranks, cap_total))
                workspace = torch.zeros(max(n, 16), dtype=torch.uint8, device=t.device)
            self.apply_fwd(cap_base, cap_total, gathered, payload_bytes, num_ranks, grad_bits, s_avg, lr, mode, repack,
                           None, None, workspace=workspace)
            return
        L.check(
            self.lib.dqrm_apply_sparse_update_strided(
                C.byref(t.c), _ptr(cap_base), cap_total, _ptr(gathered), payload_bytes, pitch, num_ranks,
                grad_bits, _ptr(s_avg), float(lr), mode, 4 if repack else 0, _stream_handle()),
            "dqrm_apply_sparse_update",
        )

    def apply_fwd(self, cap_base, cap_total, gathered, payload_bytes, num_ranks, grad_bits, s_avg, lr, mode, repack,
                  next_batch, out, bits=4, refresh_scale=True, full_precision=False, layout="tbd", workspace=None):
        """apply() followed by the next batch's forward (dqrm_apply_sparse_update_fwd): the update
        and the forward in one update launch when the merge kernels take the apply
        (apply_fwd_is_one_launch; N > 1 needs `workspace`, dqrm_apply_workspace_bytes). next_batch
        None: the apply alone, with the workspace. Returns out."""
        t = self.tables
        pitch = gathered.stride(0) if gathered.dim() == 2 else payload_bytes
        nb = C.byref(next_batch.c) if next_batch is not None else None
        B = next_batch.num_bags if next_batch is not None else 0
        ost, osb = (B * t.D, t.D) if layout == "tbd" else (t.D, t.T * t.D)
        L.check(
            self.lib.dqrm_apply_sparse_update_fwd(
                C.byref(t.c), _ptr(cap_base), cap_total, _ptr(gathered), payload_bytes, pitch, num_ranks,
                grad_bits, _ptr(s_avg), float(lr), mode, 4 if repack else 0, _ptr(workspace),
                workspace.numel() if workspace is not None else 0, nb, int(bits),
                t._fwd_flags(refresh_scale, False, full_precision), _ptr(out), ost, osb, _stream_handle()),
            "dqrm_apply_sparse_update_fwd",
        )
        return out

    def apply_local(self, ws, grad_bits, s_avg, lr, repack):
        """world size 1: quant_pack + apply fused, straight from the workspace (no payload)."""
        t = self.tables
        L.check(
            self.lib.dqrm_apply_local(
                C.byref(t.c), _ptr(ws.slot_cap_base), ws.cap_total, _ptr(ws.rows), _ptr(ws.vals), _ptr(ws.ucount),
                _ptr(ws.absmax), grad_bits, _ptr(s_avg), float(lr), 4 if repack else 0, _stream_handle()),
            "dqrm_apply_local",
        )

    def coalesce_apply_local(self, batch, dy, ws, ste, layout, grad_bits, s_avg, lr, repack):
        """world size 1: coalesce + apply_local, one launch for Criteo-form batches."""
        self.tables.backward_apply_local(batch, dy, ws, grad_bits, s_avg, lr, repack=repack, ste=ste, layout=layout)

    def quant_pack_ranked(self, ws, table_bits, table_scale, cap_base, cap_total, payload):
        t = self.tables
        L.check(
            self.lib.dqrm_grad_quant_pack_ranked(
                t.T, t.D, _ptr(ws.slot_cap_base), ws.cap_total, _ptr(ws.rows), _ptr(ws.vals), _ptr(ws.ucount),
                _ptr(table_bits), _ptr(table_scale), _ptr(cap_base), cap_total, _ptr(payload), _stream_handle()),
            "dqrm_grad_quant_pack_ranked",
        )

    def local_update(self, batch, dy, ste, layout, lr, table_mask, repack):
        self.tables.local_update(batch, dy, lr, table_mask, ste=ste, repack=repack, layout=layout)


def payload_bytes(num_tables: int, cap_total: int, dim: int, grad_bits: int) -> int:
    """Bytes of one rank's wire payload (mirrors dqrm_payload_bytes)."""
    a16 = lambda x: (x + 15) & ~15  # noqa: E731
    elem = 1 if grad_bits <= 8 else (2 if grad_bits <= 16 else 4)
    return a16(4 * num_tables * L.DQRM_TABLE_SPLIT) + a16(4 * cap_total) + a16(cap_total * dim * elem)


def all_gather_into(out: torch.Tensor, inp: torch.Tensor, group=None, world: int | None = None,
                    force: bool = False) -> None:
    """out [N, ...] <- every rank's inp, in rank order. nccl (RCCL on ROCm): one
    all_gather_into_tensor straight into `out` over xGMI; gloo: staged through host memory
    when the tensors live on the GPU (functional rehearsal only). World size 1 is a local
    copy unless `force` (a process group must exist then): the collective itself runs, as on
    N > 1 (exercises the RCCL leg on a one-GPU box)."""
    world = world if world is not None else (dist.get_world_size(group) if dist.is_initialized() else 1)
    if world == 1 and not force:
        out.view(-1)[: inp.numel()].copy_(inp.view(-1))
        return
    backend = dist.get_backend(group)
    if backend == "nccl":
        # RCCL reads/writes raw device memory: a dtype, layout or size mismatch would be
        # silent corruption, so check what the collective assumes before issuing it
        if out.dtype != inp.dtype:
            raise TypeError(f"all_gather dtype mismatch: out {out.dtype}, inp {inp.dtype}")
        if not (out.is_contiguous() and inp.is_contiguous()):
            raise ValueError("all_gather needs contiguous tensors")
        if out.numel() != world * inp.numel():
            raise ValueError(f"all_gather size mismatch: out {out.numel()} != {world} x {inp.numel()}")
        if not (out.is_cuda and inp.is_cuda and out.device == inp.device):
            raise ValueError("RCCL all_gather needs both tensors on this rank's GPU")
        dist.all_gather_into_tensor(out.view(-1), inp.view(-1), group=group)
    elif out.is_cuda:  # Gloo gathers host tensors: stage through host memory (debug / rehearsal)
        host = out.cpu()
        dist.all_gather(list(host.unbind(0)), inp.cpu(), group=group)
        out.copy_(host)
    else:
        dist.all_gather(list(out.unbind(0)), inp, group=group)


class DqrmComm:
    """libdqrm's own RCCL communicator (dqrm_comm) over the ranks of a torch.distributed
    group: rank 0 draws RCCL's unique id, the group broadcasts it, every rank joins
    (ncclCommInitRank, collective). The exchange then issues its two all-gathers from C, on
    the compute stream between its kernels (dqrm_exchange_grad): no Python or c10d work per
    collective. One per (group, world size, rank, device), shared by every exchange on that
    group; released by close() / close_all() (registered at exit), and dropped from the cache
    when its group is no longer the live one of that key (destroy_process_group + re-init)."""

    _cache: dict = {}
    _atexit = False

    def __init__(self, group=None, device=None):
        self.lib = L.load()
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.group = group
        dev = torch.device(device if device is not None else "cuda")
        idbuf = torch.zeros(128, dtype=torch.uint8)
        if self.rank == 0:
            L.check(self.lib.dqrm_comm_unique_id(idbuf.data_ptr()), "dqrm_comm_unique_id")
        src = dist.get_global_rank(group, 0) if group is not None else 0
        if dist.get_backend(group) == "nccl":  # RCCL broadcasts device tensors
            t = idbuf.to(dev)
            dist.broadcast(t, src=src, group=group)
            idbuf = t.cpu()
        else:
            dist.broadcast(idbuf, src=src, group=group)
        h = C.c_void_p()
        with torch.cuda.device(dev):
            L.check(self.lib.dqrm_comm_init(C.byref(h), self.world, self.rank, idbuf.data_ptr()), "dqrm_comm_init")
        self.handle = h

    @staticmethod
    def _key(group, device):
        pg = group if group is not None else dist.distributed_c10d._get_default_group()
        return (id(pg), dist.get_world_size(group), dist.get_rank(group), str(device))

    @classmethod
    def get(cls, group=None, device=None) -> "DqrmComm":
        if not cls._atexit:
            import atexit

            atexit.register(cls.close_all)
            cls._atexit = True
        key = cls._key(group, device)
        pg = group if group is not None else dist.distributed_c10d._get_default_group()
        c = cls._cache.get(key)
        if c is not None and (c.handle is None or c._pg is not pg):  # a stale entry (group re-created)
            c.close()
            c = None
        if c is None:
            c = cls(group, device)
            c._pg = pg
            cls._cache[key] = c
        return c

    def close(self) -> None:
        if getattr(self, "handle", None) is not None:
            self.lib.dqrm_comm_destroy(self.handle)
            self.handle = None

    @classmethod
    def close_all(cls) -> None:
        for c in cls._cache.values():
            c.close()
        cls._cache.clear()


class TorchServedComm:
    """A dqrm_comm whose all-gathers torch.distributed serves (dqrm_comm_init_external): the
    exchange's C orchestration (dqrm_exchange_grad / _apply: coalesce, all-gather of the
    maxima, quantize-pack, all-gather of the payloads, apply) is the one the RCCL communicator
    runs, and each of its two all-gathers calls back here with the device buffers and the
    stream; they are gathered with all_gather_into over the process group (nccl: c10d's own
    RCCL communicator; gloo: staged through host memory -- the reference's Gloo transport).
    One per exchange: the callback maps the exchange's (send, recv) pointers to its tensors."""

    def __init__(self, group, world: int, buffers):
        self.lib = L.load()
        self.group, self.world = group, world
        self.rank = dist.get_rank(group)
        self._bufs = {(inp.data_ptr(), out.data_ptr()): (inp, out) for inp, out in buffers}
        self.exc = None
        self.calls = 0

        def _gather(send, recv, nbytes, stream, user):  # called by libdqrm on this thread
            try:
                inp, out = self._bufs[(send or 0, recv or 0)]
                if inp.numel() * inp.element_size() != nbytes or out.numel() != self.world * inp.numel():
                    raise ValueError(f"all-gather of {nbytes} bytes does not match the registered buffers")
                all_gather_into(out, inp, self.group, self.world, force=True)
                self.calls += 1
                return 0
            except BaseException as e:  # noqa: BLE001 -- re-raised by check() after the C call
                self.exc = e
                return 1

        self._fn = L.ALLGATHER_FN(_gather)  # kept alive as long as the communicator
        h = C.c_void_p()
        L.check(self.lib.dqrm_comm_init_external(C.byref(h), world, self.rank, self._fn, None),
                "dqrm_comm_init_external")
        self.handle = h

    def check(self, rc: int, what: str) -> None:
        if rc != L.DQRM_OK and self.exc is not None:
            e, self.exc = self.exc, None
            raise L.DQRMError(f"{what}: the torch.distributed all-gather failed: {e!r}") from e
        L.check(rc, what)

    def close(self) -> None:
        if getattr(self, "handle", None) is not None:
            self.lib.dqrm_comm_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001 -- interpreter shutdown
            pass


TRANSPORTS = ("rccl", "torch", "python")


def exchange_transport(group=None, world: int | None = None) -> str:
    """How an exchange over `group` runs its N > 1 step (also forced at world size 1):
      rccl    libdqrm's C orchestration on its own RCCL communicator (DqrmComm): both
              all-gathers issued from C between the kernels (nccl backend only);
      torch   the same C orchestration, the all-gathers served by torch.distributed through
              a callback (TorchServedComm: c10d's communicator, or Gloo staged via host);
      python  the kernels and all-gathers issued one by one from Python (round-4 form, A/B).
    DQRM_C_COMM=rccl|torch|python (0 = python) overrides. Default: rccl at world size 1 on nccl
    (the forced N > 1 path on a one-GPU box, the library's measured form), torch otherwise --
    with several ranks the drop-in hooks keep c10d's one RCCL communicator, which also carries
    the MLP's all-reduces (bench.py selects rccl explicitly: --comm)."""
    env = os.environ.get("DQRM_C_COMM", "").strip().lower()
    if env in ("0", "python"):
        return "python"
    if not (dist.is_available() and dist.is_initialized()):
        return "python"
    nccl = dist.get_backend(group) == "nccl"
    if env in ("rccl", "1"):
        return "rccl" if nccl else "torch"
    if env == "torch":
        return "torch"
    w = world if world is not None else dist.get_world_size(group)
    return "rccl" if nccl and w == 1 else "torch"


def use_library_collectives(group=None) -> bool:
    """Whether an exchange over `group` issues its collectives from libdqrm's own RCCL
    communicator (exchange_transport(group) == "rccl")."""
    return exchange_transport(group) == "rccl"


class SparseGradExchange:
    """Per-step DP embedding update: coalesce -> all-gather of per-slot max|grad| ->
    scale average + quantize-pack -> payload all-gather -> decode + SGD.
    One instance per rank, buffers reused every step.

    grad_bits: 8 (scripts' --embedding_bag_gradient_bit_num=8), 2..16, or 32 for the
    unquantized sparse path (emb_grad_quantized=False, s_q_g_p_c.py:319-327).
    max_lookups: upper bound of any table's lookups per rank per step (B x pooling).
    """

    def __init__(self, tables: EmbeddingTableSet, max_lookups: int, grad_bits: int = 8, group=None,
                 kernels: ExchangeKernels | None = None, device=None, absmax_buf: torch.Tensor | None = None,
                 payload_buf: torch.Tensor | None = None, force_collectives: bool = False,
                 transport: str | None = None):
        """absmax_buf / payload_buf: caller-owned slices of buffers several sets gather
        together (MultiSetExchange); the per-set gather buffers are then not allocated.
        force_collectives: run the N > 1 step (both all-gathers, quantize-pack, payload
        decode) at world size 1 too, through the process group's backend.
        transport: "rccl" | "torch" | "python" (exchange_transport; None = its default). An
        "rccl" communicator that cannot be created falls back to "torch" (self.transport says
        which runs)."""
        if not (grad_bits == 32 or 2 <= grad_bits <= 16):
            raise ValueError("grad_bits must be 2..16 or 32")
        self.tables = tables
        self.grad_bits = grad_bits
        self.max_lookups = int(max_lookups)
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if self.world > 1 else 0
        # exchange through the collectives (N > 1, or forced at N = 1)
        self.coll = self.world > 1 or bool(force_collectives)
        if self.coll and not (dist.is_available() and dist.is_initialized()):
            raise ValueError("force_collectives needs an initialised process group")
        dev = torch.device(device if device is not None else tables.device)
        self.device = dev
        self.kernels = kernels if kernels is not None else HipExchangeKernels(tables)
        T = tables.T
        self.ws = CoalescedGrad.allocate(tables.num_rows, max_lookups, tables.D, dev, absmax=absmax_buf)
        self.caps = default_caps(tables.num_rows, max_lookups)
        base = [0]
        for c in self.caps:
            base.append(base[-1] + c)
        self.cap_total = base[-1]
        self.cap_base = torch.tensor(base, dtype=torch.int64, device=dev)
        self.payload_bytes = payload_bytes(T, self.cap_total, tables.D, grad_bits)
        self.s_avg = torch.zeros(T, dtype=torch.float32, device=dev)
        shared = payload_buf is not None
        if shared and (payload_buf.numel() != self.payload_bytes or payload_buf.dtype != torch.uint8
                       or payload_buf.data_ptr() % 16):
            raise ValueError("payload_buf must be a 16-B aligned uint8 [payload_bytes] tensor")
        self.payload = payload_buf if shared else torch.zeros(self.payload_bytes, dtype=torch.uint8, device=dev)
        self.absmax_all = None if shared else torch.zeros(self.world, T * L.DQRM_TABLE_SPLIT, dtype=torch.float32,
                                                          device=dev)
        self.gathered = None if shared else torch.zeros(self.world, self.payload_bytes, dtype=torch.uint8,
                                                        device=dev)
        # the merge apply's positions (N > 1; dqrm_apply_workspace_bytes), caller-owned
        nws = (int(L.load().dqrm_apply_workspace_bytes(self.world, self.cap_total))
               if self.coll and isinstance(self.kernels, HipExchangeKernels) else 0)
        self.apply_ws = torch.zeros(max(nws, 16), dtype=torch.uint8, device=dev)
        # the library-issued step (dqrm_exchange_grad / _apply): two host calls per step, the
        # collectives from C on a dqrm_comm (libdqrm's RCCL communicator, or torch.distributed
        # through a callback); only with the HIP kernels and unshared buffers
        self._x = None
        self.dcomm = None
        self.transport = "local" if not self.coll else "python"
        if self.coll and not shared and isinstance(self.kernels, HipExchangeKernels):
            tr = transport if transport is not None else exchange_transport(group, self.world)
            if tr not in TRANSPORTS:
                raise ValueError(f"transport must be one of {TRANSPORTS}")
            if tr == "rccl" and dist.get_backend(group) != "nccl":
                raise ValueError("the rccl transport needs the nccl backend")
            if tr == "rccl":
                try:
                    self.dcomm = DqrmComm.get(group, dev)
                except L.DQRMError as e:  # e.g. RCCL missing: the same C step over torch.distributed
                    import warnings

                    warnings.warn(f"libdqrm's RCCL communicator is unavailable ({e}); using torch.distributed")
                    tr = "torch"
            if tr == "torch":
                self.dcomm = TorchServedComm(group, self.world, [(self.ws.absmax, self.absmax_all),
                                                                 (self.payload, self.gathered)])
            self.transport = tr
            if self.dcomm is not None:
                self._x = self._make_exchange(self.dcomm.handle)

    def _make_exchange(self, comm_handle) -> "L.Exchange":
        x = L.Exchange()
        x.set = C.pointer(self.tables.c)
        x.comm = comm_handle
        x.num_ranks = self.world
        x.grad_bits = self.grad_bits
        ws = self.ws
        x.ws_cap_base, x.ws_cap_total = _ptr(ws.slot_cap_base), ws.cap_total
        x.ws_rows, x.ws_vals, x.ws_ucount, x.ws_absmax = _ptr(ws.rows), _ptr(ws.vals), _ptr(ws.ucount), _ptr(ws.absmax)
        x.absmax_all = _ptr(self.absmax_all)
        x.cap_base, x.cap_total = _ptr(self.cap_base), self.cap_total
        x.s_avg, x.payload, x.gathered = _ptr(self.s_avg), _ptr(self.payload), _ptr(self.gathered)
        x.payload_bytes = self.payload_bytes
        w = self.tables.bwd_workspace(self.max_lookups)
        x.workspace, x.workspace_bytes = w.data_ptr(), w.numel()
        x.apply_ws, x.apply_ws_bytes = _ptr(self.apply_ws), self.apply_ws.numel()
        return x

    def _check(self, rc: int, what: str) -> None:
        if isinstance(self.dcomm, TorchServedComm):
            self.dcomm.check(rc, what)
        else:
            L.check(rc, what)

    # -------------------------------------------------------------- collectives
    def _all_gather(self, out: torch.Tensor, inp: torch.Tensor) -> None:
        all_gather_into(out, inp, self.group, self.world, force=self.coll)

    # -------------------------------------------------------------- the step
    def exchange(self, batch: LookupBatch, dy: torch.Tensor, ste: bool = True, layout: str = "tbd") -> torch.Tensor:
        """grad_update_parallel_comm's embedding branch (s_q_g_p_c.py:278-315 via :850-890):
        coalesce, all-gather the scale inputs, quantize-pack, all-gather the payloads.
        Returns the per-table averaged gradient scale (emb_scaling_factor)."""
        gb = self.grad_bits
        if self._x is not None:  # one library call: coalesce, all-gather, quantize-pack, all-gather
            t = self.tables
            st, sb = t._dy_strides(dy, layout, t.T, batch.num_bags, t.D)
            w = t.bwd_workspace(batch.max_lookups)
            x = self._x
            if x.workspace != w.data_ptr():  # a larger batch grew the scratch
                x.workspace, x.workspace_bytes = w.data_ptr(), w.numel()
            self._check(t.lib.dqrm_exchange_grad(C.byref(x), C.byref(batch.c), _ptr(dy), st, sb, int(ste),
                                                 _stream_handle()), "dqrm_exchange_grad")
            return self.s_avg
        k = self.kernels
        k.coalesce(batch, dy, self.ws, ste, layout)
        if gb != 32 and self.coll:
            self._all_gather(self.absmax_all, self.ws.absmax)
            absmax_all = self.absmax_all
        else:
            absmax_all = self.ws.absmax.view(1, -1)
        k.quant_pack(self.ws, absmax_all, self.world, gb, self.cap_base, self.cap_total, self.s_avg, self.payload)
        if self.coll:
            self._all_gather(self.gathered, self.payload)
        return self.s_avg

    def apply(self, lr: float, mode: int | None = None, repack: bool = False) -> None:
        """weight_update_parallel_comm's embedding branch (s_q_g_p_c.py:601-628)."""
        gb = self.grad_bits
        if mode is None:
            mode = L.DQRM_UPD_FP32 if gb == 32 else L.DQRM_UPD_DP
        if self._x is not None:
            self._check(self.tables.lib.dqrm_exchange_apply(C.byref(self._x), float(lr), int(mode),
                                                            4 if repack else 0, _stream_handle()),
                        "dqrm_exchange_apply")
            return
        gathered = self.gathered if self.coll else self.payload.view(1, -1)
        kw = {"workspace": self.apply_ws} if isinstance(self.kernels, HipExchangeKernels) else {}
        self.kernels.apply(self.cap_base, self.cap_total, gathered, self.payload_bytes, self.world, gb, self.s_avg,
                           lr, mode, repack, **kw)

    def apply_fwd_is_one_launch(self, next_batch: LookupBatch) -> bool:
        """Whether apply_forward runs the update and the next batch's forward as ONE launch
        (dqrm_apply_fwd_is_one_launch: the merge kernel takes this exchange's apply)."""
        t = self.tables
        rc = t.lib.dqrm_apply_fwd_is_one_launch(C.byref(t.c), self.world if self.coll else 1, self.cap_total,
                                                self.apply_ws.numel(), C.byref(next_batch.c),
                                                t._fwd_flags(True, False, False))
        if rc < 0:
            L.check(rc, "dqrm_apply_fwd_is_one_launch")
        return rc == 1

    def apply_fwd_form(self, next_batch: LookupBatch) -> str:
        """The launches apply_forward issues (dqrm_apply_fwd_form): "one_launch" (the merge kernel:
        update and forward together), "fin_fwd" (the flat apply, then its finalize and the forward in
        one launch) or "separate" (the apply's launches, then the forward's)."""
        t = self.tables
        rc = t.lib.dqrm_apply_fwd_form(C.byref(t.c), self.world if self.coll else 1, self.cap_total,
                                       self.apply_ws.numel(), C.byref(next_batch.c), t._fwd_flags(True, False, False))
        if rc < 0:
            L.check(rc, "dqrm_apply_fwd_form")
        return {L.DQRM_APPLY_FWD_ONE_LAUNCH: "one_launch", L.DQRM_APPLY_FWD_FIN_FWD: "fin_fwd"}.get(rc, "separate")

    def apply_forward(self, lr: float, next_batch: LookupBatch, out: torch.Tensor | None = None, bits: int = 4,
                      refresh_scale: bool = True, full_precision: bool = False, layout: str = "tbd",
                      mode: int | None = None, repack: bool = False) -> torch.Tensor:
        """apply(lr) followed by tables.forward(next_batch): weight_update_parallel_comm of step i
        and apply_emb of step i+1, adjacent in the DP loop (dlrm_s_pytorch_tb_dp_one_parallel_comm.py
        :1888-1904); the same results, one launch when the merge kernel takes the apply
        (dqrm_apply_sparse_update_fwd / dqrm_exchange_apply_fwd). Returns the next batch's output."""
        gb = self.grad_bits
        if mode is None:
            mode = L.DQRM_UPD_FP32 if gb == 32 else L.DQRM_UPD_DP
        t = self.tables
        B = next_batch.num_bags
        if out is None:
            out = torch.empty((t.T, B, t.D) if layout == "tbd" else (B, t.T, t.D), dtype=torch.float32,
                              device=t.device)
        if self._x is not None:
            ost, osb = (B * t.D, t.D) if layout == "tbd" else (t.D, t.T * t.D)
            self._check(t.lib.dqrm_exchange_apply_fwd(
                C.byref(self._x), float(lr), int(mode), 4 if repack else 0, C.byref(next_batch.c), int(bits),
                t._fwd_flags(refresh_scale, False, full_precision), _ptr(out), ost, osb, _stream_handle()),
                "dqrm_exchange_apply_fwd")
            return out
        fwd = getattr(self.kernels, "apply_fwd", None)
        if fwd is None:
            self.apply(lr, mode=mode, repack=repack)
            return t.forward(next_batch, bits=bits, refresh_scale=refresh_scale, full_precision=full_precision,
                             out=out, layout=layout)
        gathered = self.gathered if self.coll else self.payload.view(1, -1)
        return fwd(self.cap_base, self.cap_total, gathered, self.payload_bytes, self.world if self.coll else 1, gb,
                   self.s_avg, lr, mode, repack, next_batch, out, bits=bits, refresh_scale=refresh_scale,
                   full_precision=full_precision, layout=layout, workspace=self.apply_ws)

    def step(self, batch: LookupBatch, dy: torch.Tensor, lr: float, ste: bool = True,
             mode: int | None = None, repack: bool = False, layout: str = "tbd") -> None:
        """grad_update_parallel_comm + weight_update_parallel_comm for all tables.

        At world size 1 with quantized DP gradients the quantize-pack and the apply run as
        one fused kernel (dqrm_apply_local, bit-identical; no payload is produced)."""
        gb = self.grad_bits
        fused = getattr(self.kernels, "apply_local", None)
        if (fused is not None and not self.coll and 2 <= gb <= 16
                and (mode is None or mode == L.DQRM_UPD_DP)):
            one = getattr(self.kernels, "coalesce_apply_local", None)
            if one is not None:  # the whole local step in one launch (Criteo-form batches)
                one(batch, dy, self.ws, ste, layout, gb, self.s_avg, lr, repack)
                return
            self.kernels.coalesce(batch, dy, self.ws, ste, layout)
            fused(self.ws, gb, self.s_avg, lr, repack)
            return
        self.exchange(batch, dy, ste=ste, layout=layout)
        self.apply(lr, mode=mode, repack=repack)

    # -------------------------------------------------------------- ranking range
    def coalesce_ranges(self, batch: LookupBatch, dy: torch.Tensor, ste: bool = True, layout: str = "tbd"):
        """grad_precision_and_scale's per-table range (s_q_g_p_c.py:184-193): coalesce, then
        the all-gathered max |grad| of every rank, summed in descending rank order * 1/N.
        Returns host f32 [T] (the reference reads each with .item())."""
        import numpy as np

        self.kernels.coalesce(batch, dy, self.ws, ste, layout)
        if self.world > 1:
            self._all_gather(self.absmax_all, self.ws.absmax)
            am = self.absmax_all
        else:
            am = self.ws.absmax.view(1, -1)
        a = am.view(self.world, self.tables.T, L.DQRM_TABLE_SPLIT).amax(dim=2).cpu().numpy().astype(np.float32)
        acc = a[-1].copy()
        for r in range(self.world - 2, -1, -1):
            acc = (acc + a[r]).astype(np.float32)
        return (acc * np.float32(1.0 / self.world)).astype(np.float32)

    def exchange_ranked(self, table_bits: torch.Tensor, table_scale: torch.Tensor) -> None:
        """grad_update_parallel_comm(ranking_range=True)'s embedding branch (:280-309,
        quantize_emb_grad_two :836-848): 2..8-bit tables quantized with their own scale,
        0 / 32-bit tables send nothing; one payload all-gather. Needs grad_bits == 8."""
        if self.grad_bits != 8:
            raise ValueError("the ranking-range exchange uses the 8-bit payload layout")
        self.kernels.quant_pack_ranked(self.ws, table_bits, table_scale, self.cap_base, self.cap_total, self.payload)
        if self.world > 1:
            self._all_gather(self.gathered, self.payload)

    def apply_ranked(self, lr: float, table_scale: torch.Tensor, repack: bool = False) -> None:
        """weight_update_parallel_comm(ranking_range=True) for the quantized tables (:617-622)."""
        gathered = self.payload.view(1, -1) if self.world == 1 else self.gathered
        self.kernels.apply(self.cap_base, self.cap_total, gathered, self.payload_bytes, self.world, 8, table_scale,
                           lr, L.DQRM_UPD_DP, repack)

    def local_scales(self) -> torch.Tensor:
        """This rank's per-table gradient scale s_loc (host-side view for inspection)."""
        import numpy as np

        a = self.ws.absmax.view(self.tables.T, L.DQRM_TABLE_SPLIT).max(dim=1).values.cpu().numpy()
        a = np.maximum(a.astype(np.float32), np.float32(1e-8))
        return torch.from_numpy(a / np.float32(2 ** (self.grad_bits - 1) - 1))


class MultiSetExchange:
    """One exchange for several table sets: the unchanged DP driver's ModuleList of 26
    single-table QuantEmbeddingBagTwo modules (dlrm_s_pytorch_tb_dp_one_parallel_comm.py:380)
    gets the same TWO collectives per step as one 26-table set, instead of the reference's
    2 blocking collectives per table (s_q_g_p_c.py:278-315):
      per set   coalesce into its workspace, its per-slot max|grad| landing in its slice
                of one concatenated [sum T*S] buffer
      1 x       all-gather of the concatenated maxima
      per set   quantize-pack into its slice of one concatenated payload (the strided
                quant-pack reads its column of the gathered maxima)
      1 x       all-gather of the concatenated payloads
      per set   decode its column of the gathered payloads + SGD (strided apply)
    Per-set results are bit-identical to a SparseGradExchange per set."""

    def __init__(self, sets, max_lookups, grad_bits: int = 8, group=None, kernels=None, device=None):
        sets = list(sets)
        if not sets:
            raise ValueError("no table sets")
        ml = list(max_lookups) if isinstance(max_lookups, (list, tuple)) else [int(max_lookups)] * len(sets)
        self.sets = sets
        self.grad_bits = grad_bits
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1
        self.max_lookups = [int(m) for m in ml]
        dev = torch.device(device if device is not None else sets[0].device)
        S = L.DQRM_TABLE_SPLIT
        ts_n = [s.T * S for s in sets]
        pb_n = [payload_bytes(s.T, sum(default_caps(s.num_rows, m)), s.D, grad_bits) for s, m in zip(sets, ml)]
        self.am_off = [sum(ts_n[:i]) for i in range(len(sets) + 1)]
        self.pl_off = [sum(pb_n[:i]) for i in range(len(sets) + 1)]
        self.absmax = torch.zeros(self.am_off[-1], dtype=torch.float32, device=dev)
        self.payload = torch.zeros(self.pl_off[-1], dtype=torch.uint8, device=dev)
        self.absmax_all = torch.zeros(self.world, self.am_off[-1], dtype=torch.float32, device=dev)
        self.gathered = torch.zeros(self.world, self.pl_off[-1], dtype=torch.uint8, device=dev)
        ks = kernels if kernels is not None else [None] * len(sets)
        self.parts = [
            SparseGradExchange(s, m, grad_bits=grad_bits, group=group, kernels=k, device=dev,
                               absmax_buf=self.absmax[self.am_off[i]: self.am_off[i + 1]],
                               payload_buf=self.payload[self.pl_off[i]: self.pl_off[i + 1]])
            for i, (s, m, k) in enumerate(zip(sets, ml, ks))]

    def exchange(self, items) -> list[torch.Tensor]:
        """items[i] = (batch, dy, ste, layout) of set i, or None (no backward: the set sends
        no rows). Returns each set's averaged gradient scale (emb_scaling_factor)."""
        gb, N = self.grad_bits, self.world
        for p, it in zip(self.parts, items):
            if it is None:
                p.ws.ucount.zero_()
                p.ws.absmax.zero_()
            else:
                batch, dy, ste, layout = it
                p.kernels.coalesce(batch, dy, p.ws, ste, layout)
        if gb != 32 and N > 1:
            all_gather_into(self.absmax_all, self.absmax, self.group, N)
        for i, p in enumerate(self.parts):
            am = (self.absmax_all[:, self.am_off[i]: self.am_off[i + 1]] if gb != 32 and N > 1
                  else p.ws.absmax.view(1, -1))
            p.kernels.quant_pack(p.ws, am, N, gb, p.cap_base, p.cap_total, p.s_avg, p.payload)
        if N > 1:
            all_gather_into(self.gathered, self.payload, self.group, N)
        return [p.s_avg for p in self.parts]

    def apply(self, lr: float, mode: int | None = None, repack=False) -> None:
        """weight_update_parallel_comm's embedding branch for every set; repack: bool or
        one bool per set."""
        gb, N = self.grad_bits, self.world
        if mode is None:
            mode = L.DQRM_UPD_FP32 if gb == 32 else L.DQRM_UPD_DP
        rp = list(repack) if isinstance(repack, (list, tuple)) else [bool(repack)] * len(self.parts)
        for i, p in enumerate(self.parts):
            g = self.gathered[:, self.pl_off[i]: self.pl_off[i + 1]] if N > 1 else p.payload.view(1, -1)
            kw = {"workspace": p.apply_ws} if isinstance(p.kernels, HipExchangeKernels) else {}
            p.kernels.apply(p.cap_base, p.cap_total, g, p.payload_bytes, N, gb, p.s_avg, lr, mode, rp[i], **kw)

    @property
    def collective_bytes(self) -> tuple[int, int]:
        """Bytes each rank contributes to the two all-gathers (maxima, payloads)."""
        return self.absmax.numel() * 4, self.payload.numel()


class ConsolidatedExchange:
    """The exchange of a ModuleList of per-table modules whose tables live in ONE
    consolidated set (quant_modules_not_quantize_grad.consolidate_tables): the modules'
    pending (batch, dy) pairs are concatenated on the device (one copy each for the
    indices, offsets and dy) and the step runs as ONE coalesce, ONE quantize-pack and ONE
    apply for all tables (two collectives at N > 1) -- the launch count of a single
    26-table set. At world size 1 with quantized gradients the whole local step -- coalesce,
    quantize and apply -- runs at apply time as ONE launch (dqrm_emb_bwd_apply_local), which
    also produces the averaged scales (emb_scaling_factor holds them from then on; the
    reference sets them in grad_update_parallel_comm, s_q_g_p_c.py:296, and reads them in
    weight_update_parallel_comm, :618-622, so the update sees the same values)."""

    def __init__(self, tables: EmbeddingTableSet, max_lookups: int, grad_bits: int = 8, group=None):
        self.tables = tables
        self.grad_bits = grad_bits
        self.max_lookups = [int(max_lookups)] * tables.T
        self.inner = SparseGradExchange(tables, max_lookups, grad_bits=grad_bits, group=group)
        self.world = self.inner.world
        self.fused = self.world == 1 and 2 <= grad_bits <= 16
        self.scales = [self.inner.s_avg[t: t + 1] for t in range(tables.T)]
        self._args = None

    def exchange(self, items) -> list[torch.Tensor]:
        batch = LookupBatch.concat([it[0] for it in items])
        dy = torch.cat([it[1].reshape(1, batch.num_bags, -1) for it in items], dim=0)
        ste, layout = items[0][2], items[0][3]
        if any(it[2] != ste for it in items):
            raise ValueError("modules differ in full_precision (STE) within one step")
        if self.fused:
            self._args = (batch, dy, ste)  # the one-launch step runs at apply time
        else:
            self.inner.exchange(batch, dy, ste=ste, layout="tbd")
        return self.scales

    def apply(self, lr: float, mode: int | None = None, repack=False) -> None:
        rp = any(repack) if isinstance(repack, (list, tuple)) else bool(repack)
        if self.fused:
            if self._args is None:
                raise RuntimeError("apply() without a preceding exchange()")
            batch, dy, ste = self._args
            if mode is None or mode == L.DQRM_UPD_DP:
                self.inner.kernels.coalesce_apply_local(batch, dy, self.inner.ws, ste, "tbd", self.grad_bits,
                                                        self.inner.s_avg, lr, rp)
            else:  # another update rule: the exchange's coalesce, then the payload path
                self.inner.exchange(batch, dy, ste=ste, layout="tbd")
                self.inner.apply(lr, mode=mode, repack=rp)
        else:
            self.inner.apply(lr, mode=mode, repack=rp)
        self._args = None

    def discard(self) -> None:
        """weight_update_parallel_comm(update_embedding=False): no update this step. The fused
        form deferred the whole step to apply(); its exchange runs now (coalesce + scales, no
        update) so emb_scaling_factor holds this step's scales as in the reference (set in
        grad_update_parallel_comm, s_q_g_p_c.py:296), and the pending (batch, dy) is released."""
        if self.fused and self._args is not None:
            batch, dy, ste = self._args
            self.inner.exchange(batch, dy, ste=ste, layout="tbd")
        self._args = None

    @property
    def scales_ready_after_apply(self) -> bool:
        """True when the scales (emb_scaling_factor) are produced by apply() / discard() rather
        than by exchange(): the world-size-1 one-launch form computes them with the update."""
        return self.fused


def get_my_slice(n: int, my_size: int, my_rank: int) -> slice:
    """Contiguous per-rank batch slice (dlrm_s_pytorch_single_gpu.py:989-993)."""
    k, m = divmod(n, my_size)
    return slice(my_rank * k + min(my_rank, m), (my_rank + 1) * k + min(my_rank + 1, m), 1)


__all__ = ["DqrmComm", "TorchServedComm", "exchange_transport", "TRANSPORTS", "use_library_collectives", "SparseGradExchange", "MultiSetExchange", "ConsolidatedExchange", "HipExchangeKernels", "payload_bytes",
           "get_my_slice", "all_gather_into"]
