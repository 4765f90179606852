"""Resident embedding-table state and lookup batches, driven through libdqrm's C ABI.

Memory layout in HBM (one slab per array, all T tables back to back):
    W       f32 [R, D]      FP32 master rows (table t: rows row_base[t] .. +num_rows[t])
    packed  u8  [R, D/2]    INT4 rows, offset-binary nibbles, element 2j in the low nibble
    rowmax  f32 [R]         max_d |W[r, d]|
    blkmax  f32 [NB]        per 256-row block,   sblkmax f32 [NS] per 65536-row superblock
    tmax    f32 [T]         max |W_t|  (=> reference scale s_t = max(tmax_t, 1e-8)/7)

Reference semantics: quantization_supp/quant_modules_not_quantize_grad.py:240-398 (module),
quantization_supp/quant_utils.py:75-101,141-194,316-363 (math).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import Sequence

import torch

from . import _lib as L


def _ptr(t: torch.Tensor | None) -> int | None:
    return None if t is None else t.data_ptr()


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def _stream_handle(stream: torch.cuda.Stream | None = None) -> int:
    """hipStream_t of `stream` (default: torch's current stream on the current device)."""
    if stream is not None:
        return stream.cuda_stream
    if _raw_stream is not None:  # no Stream object construction on the launch path
        return _raw_stream(torch.cuda.current_device())
    return torch.cuda.current_stream().cuda_stream


def _ceil_div(a: int, b: int) -> int:
    return (a + b - 1) // b


_BASE_CACHE: dict = {}


def _device_base(base: list[int], dev: torch.device) -> torch.Tensor:
    """Device copy of a batch's idx_base, created once per distinct (lookup counts, device):
    steady-state steps reuse it instead of a pageable host-to-device copy per call."""
    key = (tuple(base), dev.type, dev.index)
    t = _BASE_CACHE.get(key)
    if t is None:
        if len(_BASE_CACHE) > 256:
            _BASE_CACHE.clear()
        t = torch.tensor(base, dtype=torch.int64, device=dev)
        _BASE_CACHE[key] = t
    return t


class LookupBatch:
    """All tables' lookups of one batch in the reference's (lS_i, lS_o) form.

    Accepted inputs (dlrm_data_pytorch.py:328-345 Criteo collate, :1099-1157 random bags):
      * ``indices``: list of T int64 tensors (ragged) or an int64 tensor [T, L];
      * ``offsets``: list of T int64 tensors [B] or an int64 tensor [T, B].
    Offsets are nn.EmbeddingBag offsets (bag b = [off[b], off[b+1]), last bag ends at L_t).
    """

    def __init__(self, indices, offsets, device: torch.device | str | None = None,
                 pooling_one: bool | None = False):
        """pooling_one: promise that every table has one lookup per bag (offsets = arange(B),
        the Criteo collate form) -- the kernels then skip reading the offsets. None: detect it
        when the offsets are host tensors (no device read, hence no host sync)."""
        if isinstance(indices, torch.Tensor):
            if indices.dim() != 2:
                raise ValueError("stacked indices must be [T, L]")
            T = indices.shape[0]
            lens = [indices.shape[1]] * T
            idx = indices.reshape(-1)
        else:
            T = len(indices)
            lens = [int(x.numel()) for x in indices]
            idx = (indices[0].reshape(-1) if T == 1 else  # one table (a per-table module): no copy
                   torch.cat([x.reshape(-1) for x in indices]) if T else torch.empty(0, dtype=torch.int64))
        if isinstance(offsets, torch.Tensor):
            if offsets.dim() != 2 or offsets.shape[0] != T:
                raise ValueError("stacked offsets must be [T, B]")
            off = offsets
        else:
            if len(offsets) != T:
                raise ValueError("need one offsets tensor per table")
            B0 = int(offsets[0].numel()) if T else 0
            if any(int(o.numel()) != B0 for o in offsets):
                raise ValueError("all tables must have the same number of bags")
            off = (offsets[0].reshape(1, -1) if T == 1 else
                   torch.stack([o.reshape(-1) for o in offsets]) if T else torch.empty(0, 0, dtype=torch.int64))
        dev = torch.device(device) if device is not None else idx.device
        self.num_tables = T
        self.num_bags = int(off.shape[1]) if T else 0
        self.lookups = lens
        self.max_lookups = max(lens) if lens else 0
        base = [0]
        for n in lens:
            base.append(base[-1] + n)
        self.idx_base_host = base
        self.idx = idx.to(device=dev, dtype=torch.int64).contiguous()
        self.off = off.to(device=dev, dtype=torch.int64).contiguous()
        self.idx_base = _device_base(base, dev)
        if pooling_one is None:  # auto: provable only from host offsets (a device copy would sync)
            pooling_one = (all(n == self.num_bags for n in lens) and off.device.type == "cpu"
                           and bool(torch.equal(off, torch.arange(self.num_bags, dtype=off.dtype).expand_as(off))))
        if pooling_one and any(n != self.num_bags for n in lens):
            raise ValueError("pooling_one needs exactly one lookup per bag in every table")
        self.pooling_one = bool(pooling_one)
        self._c = L.Batch(
            _ptr(self.idx), _ptr(self.off), _ptr(self.idx_base), self.num_bags, self.max_lookups,
            L.DQRM_BATCH_POOLING_ONE if pooling_one else 0, 0,
        )

    @property
    def c(self) -> L.Batch:
        return self._c

    @classmethod
    def concat(cls, batches: Sequence["LookupBatch"]) -> "LookupBatch":
        """One batch holding the tables of several batches in order (the per-table batches
        of a ModuleList's modules, for one launch over their consolidated set). All must
        have the same number of bags. Device concatenation only, no host sync."""
        B = batches[0].num_bags
        if any(b.num_bags != B for b in batches):
            raise ValueError("all batches must have the same number of bags")
        idx = [b.idx[b.idx_base_host[t]: b.idx_base_host[t + 1]] for b in batches for t in range(b.num_tables)]
        off = torch.cat([b.off for b in batches], dim=0)
        return cls(idx, off, pooling_one=all(b.pooling_one for b in batches))

    @classmethod
    def concat_bags(cls, batches: Sequence["LookupBatch"]) -> "LookupBatch":
        """The bags of several batches of the same tables back to back (batch i's bags after
        batch i-1's, per table; lookups likewise): the simulated-DP micro-steps as one batch.
        Device concatenation and an offset shift per (batch, table); no host sync."""
        T = batches[0].num_tables
        if any(b.num_tables != T for b in batches):
            raise ValueError("all batches must have the same tables")
        idx, off = [], []
        shift = [0] * T
        for b in batches:
            off.append(b.off + _device_base(list(shift), b.off.device).view(T, 1))
            for t in range(T):
                shift[t] += b.lookups[t]
        for t in range(T):
            idx.append(torch.cat([b.idx[b.idx_base_host[t]: b.idx_base_host[t + 1]] for b in batches]))
        return cls(idx, torch.cat(off, dim=1), pooling_one=all(b.pooling_one for b in batches))

    @classmethod
    def one_table(cls, idx: torch.Tensor, off: torch.Tensor, pooling_one: bool | None = False) -> "LookupBatch":
        """A one-table batch from a 1-D index and offsets tensor already on the device (the
        per-table module call of DLRM_Net.apply_emb): the same fields as the constructor,
        without its general-case work (no concatenation, no copies of int64 contiguous
        inputs). pooling_one None is taken as False (device offsets cannot be checked)."""
        if idx.dtype != torch.int64 or not idx.is_contiguous():
            idx = idx.to(torch.int64).contiguous()
        if off.dtype != torch.int64 or not off.is_contiguous():
            off = off.to(torch.int64).contiguous()
        b = cls.__new__(cls)
        n = idx.numel()
        B = off.numel()
        if pooling_one and n != B:
            raise ValueError("pooling_one needs exactly one lookup per bag in every table")
        b.num_tables, b.num_bags, b.lookups, b.max_lookups = 1, B, [n], n
        b.idx_base_host = [0, n]
        b.idx = idx
        b.off = off.view(1, B)
        b.idx_base = _device_base(b.idx_base_host, idx.device)
        b.pooling_one = bool(pooling_one)
        b._c = L.Batch(idx.data_ptr(), off.data_ptr(), b.idx_base.data_ptr(), B, n,
                       L.DQRM_BATCH_POOLING_ONE if pooling_one else 0, 0)
        return b

    @classmethod
    def pooling_one(cls, indices: torch.Tensor) -> "LookupBatch":
        """Criteo form: one index per (table, sample); offsets = arange(B) per table."""
        T, B = indices.shape
        off = torch.arange(B, dtype=torch.int64, device=indices.device).expand(T, B)
        return cls(indices, off.contiguous(), pooling_one=True)


class EmbeddingTableSet:
    """T embedding tables of dim D resident in one set of HBM slabs."""

    def __init__(
        self,
        num_rows: Sequence[int],
        dim: int,
        device: torch.device | str = "cuda",
        packed: bool = False,
        init: str | None = "uniform",
        seed: int = 123,
        weights: Sequence[torch.Tensor] | None = None,
    ):
        self.lib = L.load()
        self.parent, self.parent_index = None, 0  # set on views (EmbeddingTableSet.view)
        self.num_rows = [int(n) for n in num_rows]
        self.T = len(self.num_rows)
        self.D = int(dim)
        if self.T <= 0 or self.T > 256:
            raise ValueError("1..256 tables supported")
        if self.D < 4 or self.D > 256 or self.D % 4 or (self.D // 4) & (self.D // 4 - 1):
            raise ValueError("embedding dim must be 4*2^k <= 256")
        self.device = torch.device(device)
        T, D = self.T, self.D
        self.row_base = [0]
        for n in self.num_rows[:-1]:
            self.row_base.append(self.row_base[-1] + n)
        nblk = [_ceil_div(n, L.DQRM_BLOCK_ROWS) for n in self.num_rows]
        nsblk = [_ceil_div(b, L.DQRM_SBLOCK_ROWS // L.DQRM_BLOCK_ROWS) for b in nblk]
        self.blk_base = [0]
        for b in nblk[:-1]:
            self.blk_base.append(self.blk_base[-1] + b)
        self.sblk_base = [0]
        for b in nsblk[:-1]:
            self.sblk_base.append(self.sblk_base[-1] + b)
        self.R = sum(self.num_rows)
        NB, NS = sum(nblk), sum(nsblk)
        dev = self.device
        f32 = torch.float32
        self.W = torch.empty(self.R, D, dtype=f32, device=dev)
        self.packed = torch.empty(self.R, D // 2, dtype=torch.uint8, device=dev) if packed else None
        self.rowmax = torch.zeros(self.R, dtype=f32, device=dev)
        self.blkmax = torch.zeros(NB, dtype=f32, device=dev)
        self.sblkmax = torch.zeros(NS, dtype=f32, device=dev)
        self.tmax = torch.zeros(T, dtype=f32, device=dev)
        self.scale = torch.zeros(T, dtype=f32, device=dev)
        self.pscale = torch.full((T,), float("nan"), dtype=f32, device=dev)
        self.meta = torch.tensor(
            [self.row_base, self.num_rows, self.blk_base, self.sblk_base], dtype=torch.int64, device=dev
        ).contiguous()
        self.err = torch.zeros(1, dtype=torch.int32, device=dev)
        self.tflags = torch.zeros(T, dtype=torch.int32, device=dev)
        # flag arrays padded to whole 32-bit words (the kernels set / read them word-wise)
        self.sdirty = torch.zeros(_ceil_div(NS, 4) * 4, dtype=torch.uint8, device=dev)
        self.bdirty = torch.zeros(_ceil_div(NB, 4) * 4, dtype=torch.uint8, device=dev)
        # per-table arrival counters of the in-launch finalize, one per 256 bytes
        self.sync = torch.zeros(T * L.DQRM_SYNC_STRIDE, dtype=torch.int32, device=dev)
        self._bws: torch.Tensor | None = None  # backward workspace, grown to the largest batch seen
        self._err_host: torch.Tensor | None = None  # pinned snapshot of the error word (poll_errors)
        self._err_evt = None
        self._err_pending = False
        self._rows_host = (C.c_int64 * T)(*self.num_rows)  # kept alive with the struct
        self._c = L.TableSet(
            T, D, self.R, NB, NS,
            _ptr(self.W), _ptr(self.packed), _ptr(self.rowmax), _ptr(self.blkmax), _ptr(self.sblkmax),
            _ptr(self.tmax), _ptr(self.scale), _ptr(self.pscale), _ptr(self.meta), _ptr(self.err),
            _ptr(self.tflags), _ptr(self.sdirty), _ptr(self.bdirty), _ptr(self.sync),
            C.addressof(self._rows_host),
        )
        if weights is not None:
            if len(weights) != T:
                raise ValueError("one weight tensor per table")
            for t, w in enumerate(weights):
                self.table_weight(t).copy_(w.to(device=dev, dtype=f32))
        elif init == "uniform":
            L.check(self.lib.dqrm_init_uniform(C.byref(self._c), seed, _stream_handle()), "dqrm_init_uniform")
        self.refresh_absmax()

    # ------------------------------------------------------------------ views / state
    @property
    def c(self) -> L.TableSet:
        return self._c

    def view(self, t: int) -> "EmbeddingTableSet":
        """Table t of this set as a one-table set over the SAME device memory (its rows,
        packed rows, |W| maxima, scale, flags and arrival counter; the error word is shared).
        Kernels launched on the view see and update exactly table t's part of the slabs, so a
        ModuleList of per-table modules can run on views of one consolidated set while the
        grad-comm hooks launch once for all tables on the set itself."""
        if not 0 <= t < self.T:
            raise IndexError(t)
        v = object.__new__(EmbeddingTableSet)
        n = self.num_rows[t]
        rb, bb, sbb = self.row_base[t], self.blk_base[t], self.sblk_base[t]
        nb = _ceil_div(n, L.DQRM_BLOCK_ROWS)
        ns = _ceil_div(nb, L.DQRM_SBLOCK_ROWS // L.DQRM_BLOCK_ROWS)
        v.lib, v.num_rows, v.T, v.D, v.device = self.lib, [n], 1, self.D, self.device
        v.row_base, v.blk_base, v.sblk_base, v.R = [0], [0], [0], n
        v.parent, v.parent_index = self, t
        v.W = self.W[rb: rb + n]
        v.packed = self.packed[rb: rb + n] if self.packed is not None else None
        v.rowmax = self.rowmax[rb: rb + n]
        v.blkmax = self.blkmax[bb: bb + nb]
        v.sblkmax = self.sblkmax[sbb: sbb + ns]
        v.tmax, v.scale, v.pscale = self.tmax[t: t + 1], self.scale[t: t + 1], self.pscale[t: t + 1]
        v.meta = torch.tensor([[0], [n], [0], [0]], dtype=torch.int64, device=self.device)
        v.err = self.err
        v.tflags = self.tflags[t: t + 1]
        v.sdirty = self.sdirty[sbb:]  # to the end: word-wise flag reads stay inside the allocation
        v.bdirty = self.bdirty[bb:]
        v.sync = self.sync[t * L.DQRM_SYNC_STRIDE: (t + 1) * L.DQRM_SYNC_STRIDE]
        v._bws, v._err_host, v._err_evt, v._err_pending = None, None, None, False
        v._rows_host = (C.c_int64 * 1)(n)
        v._c = L.TableSet(
            1, self.D, n, nb, ns,
            _ptr(v.W), _ptr(v.packed), _ptr(v.rowmax), _ptr(v.blkmax), _ptr(v.sblkmax),
            _ptr(v.tmax), _ptr(v.scale), _ptr(v.pscale), _ptr(v.meta), _ptr(v.err),
            _ptr(v.tflags), _ptr(v.sdirty), _ptr(v.bdirty), _ptr(v.sync),
            C.addressof(v._rows_host),
        )
        return v

    def table_weight(self, t: int) -> torch.Tensor:
        b = self.row_base[t]
        return self.W[b : b + self.num_rows[t]]

    def table_packed(self, t: int) -> torch.Tensor:
        b = self.row_base[t]
        return self.packed[b : b + self.num_rows[t]]

    # ------------------------------------------------------------------ maintenance
    def refresh_absmax(self) -> None:
        """Recompute the |W| max hierarchy from W (after any external write to W)."""
        L.check(self.lib.dqrm_refresh_absmax(C.byref(self._c), _stream_handle()), "dqrm_refresh_absmax")

    def repack_all(self, bits: int = 4) -> None:
        """After W was rewritten outside the kernels (weight_syncc, load_state_dict): new
        scales from the |W| hierarchy and EVERY table's INT4 rows repacked (a table whose
        scale happens not to move still has new rows)."""
        self.pscale.fill_(float("nan"))
        self.refresh_scale_and_pack(bits)

    def refresh_scale_and_pack(self, bits: int = 4) -> None:
        L.check(
            self.lib.dqrm_refresh_scale_and_pack(C.byref(self._c), bits, _stream_handle()),
            "dqrm_refresh_scale_and_pack",
        )

    def share_error_word(self, word: torch.Tensor) -> None:
        """Raise this set's device error flags into `word` (int32 [1] on the same device)
        from the next call on, so one read covers several sets (the DP hooks over a
        ModuleList of per-table modules read one word per step). Pending flags carry over."""
        if word.dtype != torch.int32 or word.numel() != 1 or word.device != self.err.device:
            raise ValueError("the shared error word must be one int32 on the set's device")
        if word.data_ptr() == self.err.data_ptr():
            return
        word.bitwise_or_(self.err)
        self.err = word
        self._c.err = _ptr(word)

    def poll_errors(self) -> int:
        """Non-blocking read of the device error flags: the value of the last snapshot whose
        copy has completed (0 when none has), then a new asynchronous snapshot (pinned host
        memory, stream-ordered, no host synchronisation) if none is in flight. Flags are
        sticky on the device until read_errors(clear=True)."""
        if self._err_host is None:
            self._err_host = torch.zeros(1, dtype=torch.int32).pin_memory()
            self._err_evt = torch.cuda.Event()
            self._err_pending = False
        flags = 0
        if self._err_pending:
            if not self._err_evt.query():
                return 0  # the previous snapshot is still in flight
            flags = int(self._err_host[0])
            self._err_pending = False
        if flags == 0:
            self._err_host.copy_(self.err, non_blocking=True)
            self._err_evt.record()
            self._err_pending = True
        return flags

    def read_errors(self, clear: bool = True) -> int:
        f = C.c_uint32(0)
        L.check(self.lib.dqrm_read_errors(C.byref(self._c), C.byref(f), int(clear), _stream_handle()),
                "dqrm_read_errors")
        return int(f.value)

    # ------------------------------------------------------------------ forward
    def forward(
        self,
        batch: LookupBatch,
        bits: int = 4,
        refresh_scale: bool = True,
        use_packed: bool = False,
        full_precision: bool = False,
        out: torch.Tensor | None = None,
        layout: str = "tbd",
        nt_store: bool | None = None,
        changed_rows: torch.Tensor | None = None,
    ) -> torch.Tensor:
        """Fused T-table fake-quant EmbeddingBag (q_m_n_q_g.py:317-398 for every table).

        layout "tbd" -> out [T, B, D]; "btd" -> out [B, T, D] (DLRM interaction order).
        changed_rows: slab rows rewritten outside the kernels since the last call (an
        optimizer's step on the lookup_grad COO): rows_changed(changed_rows) first, in the
        same launch when the set and batch are small (dqrm_emb_fwd_after_update).
        """
        if batch.num_tables != self.T:
            raise ValueError("batch has %d tables, set has %d" % (batch.num_tables, self.T))
        B, T, D = batch.num_bags, self.T, self.D
        if out is None:
            shape = (T, B, D) if layout == "tbd" else (B, T, D)
            out = torch.empty(shape, dtype=torch.float32, device=self.device)
        if layout == "tbd":
            st, sb = B * D, D
        else:
            st, sb = D, T * D
        flags = 0
        if refresh_scale:
            flags |= L.DQRM_FWD_REFRESH_SCALE
        if use_packed:
            flags |= L.DQRM_FWD_USE_PACKED
        if full_precision:
            flags |= L.DQRM_FWD_FULL_PRECISION
        if nt_store is None:
            # stream the output past the caches once it cannot stay in the 256 MiB
            # Infinity Cache anyway (measured: +10-27% at 0.4-1.7 GB, -9% at 109 MB)
            nt_store = B * T * D * 4 > (192 << 20)
        if nt_store:
            flags |= L.DQRM_FWD_NT_STORE
        if changed_rows is not None and changed_rows.numel() > 0:
            rows = changed_rows
            if rows.dtype != torch.int64 or not rows.is_contiguous() or rows.device != self.device:
                rows = rows.to(device=self.device, dtype=torch.int64).contiguous()
            L.check(
                self.lib.dqrm_emb_fwd_after_update(C.byref(self._c), C.byref(batch.c), bits, flags, _ptr(out), st,
                                                   sb, _ptr(rows), rows.numel(), 0, _stream_handle()),
                "dqrm_emb_fwd_after_update",
            )
            return out
        L.check(
            self.lib.dqrm_emb_fwd(C.byref(self._c), C.byref(batch.c), bits, flags, _ptr(out), st, sb,
                                  _stream_handle()),
            "dqrm_emb_fwd",
        )
        return out

    # ------------------------------------------------------------------ backward
    def bwd_workspace(self, max_lookups: int) -> torch.Tensor:
        """Device scratch of the backward's per-table lookup sort (dqrm_bwd_workspace_bytes);
        allocated once per batch-size high-water mark, never on a steady-state step."""
        need = int(self.lib.dqrm_bwd_workspace_bytes(self.T, int(max_lookups)))
        if need <= 0:
            raise ValueError("bad workspace request (%d tables, max_lookups %d)" % (self.T, max_lookups))
        if self._bws is None or self._bws.numel() < need:  # zero-filled: the library's list counters
            self._bws = torch.zeros(need, dtype=torch.uint8, device=self.device)
        return self._bws

    @staticmethod
    def _dy_strides(dy: torch.Tensor, layout: str, T: int, B: int, D: int) -> tuple[int, int]:
        if dy.stride(-1) != 1:
            raise ValueError("dy must be contiguous in D")
        if layout == "tbd":
            if tuple(dy.shape) != (T, B, D):
                raise ValueError("dy must be [T, B, D]")
            return dy.stride(0), dy.stride(1)
        if tuple(dy.shape) != (B, T, D):
            raise ValueError("dy must be [B, T, D]")
        return dy.stride(1), dy.stride(0)

    def _ws_args(self, batch: LookupBatch) -> tuple[int, int]:
        w = self.bwd_workspace(batch.max_lookups)
        return w.data_ptr(), w.numel()

    def backward_sgd(self, batch: LookupBatch, dy: torch.Tensor, lr: float, ste: bool = True,
                     repack: bool = False, layout: str = "tbd") -> None:
        """Fused STE + sparse backward + SGD (torch.optim.SGD semantics, in lookup order)."""
        st, sb = self._dy_strides(dy, layout, self.T, batch.num_bags, self.D)
        L.check(
            self.lib.dqrm_emb_bwd_sgd(C.byref(self._c), C.byref(batch.c), _ptr(dy), st, sb, int(ste),
                                      float(lr), 4 if repack else 0, *self._ws_args(batch), _stream_handle()),
            "dqrm_emb_bwd_sgd",
        )

    def backward_sgd_forward(self, batch: LookupBatch, dy: torch.Tensor, lr: float, next_batch: LookupBatch,
                             bits: int = 4, refresh_scale: bool = True, full_precision: bool = False,
                             out: torch.Tensor | None = None, layout: str = "tbd", ste: bool = True,
                             repack: bool = False, dy_layout: str = "tbd") -> torch.Tensor:
        """backward_sgd(batch, dy, lr) followed by forward(next_batch): the single-GPU
        driver's SGD step and its next apply_emb, adjacent in the loop, with the same results;
        one launch for small batches (dqrm_emb_bwd_sgd_fwd). Returns the next batch's output."""
        if next_batch.num_tables != self.T:
            raise ValueError("batch has %d tables, set has %d" % (next_batch.num_tables, self.T))
        B, T, D = next_batch.num_bags, self.T, self.D
        if out is None:
            out = torch.empty((T, B, D) if layout == "tbd" else (B, T, D), dtype=torch.float32, device=self.device)
        ost, osb = (B * D, D) if layout == "tbd" else (D, T * D)
        st, sb = self._dy_strides(dy, dy_layout, self.T, batch.num_bags, self.D)
        L.check(
            self.lib.dqrm_emb_bwd_sgd_fwd(
                C.byref(self._c), C.byref(batch.c), _ptr(dy), st, sb, int(ste), float(lr), 4 if repack else 0,
                *self._ws_args(batch), C.byref(next_batch.c), int(bits),
                self._fwd_flags(refresh_scale, False, full_precision), _ptr(out), ost, osb, _stream_handle()),
            "dqrm_emb_bwd_sgd_fwd",
        )
        return out

    def sgd_fwd_is_one_launch(self, batch: LookupBatch, next_batch: LookupBatch, use_packed: bool = False) -> bool:
        """Whether backward_sgd_forward runs the SGD and the next batch's forward as ONE launch
        (dqrm_bwd_sgd_fwd_is_one_launch)."""
        rc = self.lib.dqrm_bwd_sgd_fwd_is_one_launch(C.byref(self._c), C.byref(batch.c), C.byref(next_batch.c),
                                                     self._fwd_flags(True, use_packed, False))
        if rc < 0:
            L.check(rc, "dqrm_bwd_sgd_fwd_is_one_launch")
        return rc == 1

    def local_update(self, batch: LookupBatch, dy: torch.Tensor, lr: float, table_mask: torch.Tensor | None = None,
                     ste: bool = True, repack: bool = False, layout: str = "tbd") -> None:
        """W.add_(-lr * grad) with the rank's own uncoalesced gradient, product rounded, in
        lookup order (ranking-range 32-bit tables, s_q_g_p_c.py:615-616); table_mask int32 [T]."""
        st, sb = self._dy_strides(dy, layout, self.T, batch.num_bags, self.D)
        L.check(
            self.lib.dqrm_emb_local_update(C.byref(self._c), C.byref(batch.c), _ptr(dy), st, sb, int(ste),
                                           float(lr), _ptr(table_mask), 4 if repack else 0,
                                           *self._ws_args(batch), _stream_handle()),
            "dqrm_emb_local_update",
        )

    def rows_changed(self, rows: torch.Tensor, repack: bool = False) -> None:
        """Rows (slab ids, device i64) rewritten outside the kernels, e.g. by torch.optim.SGD
        on the lookup_grad COO: refresh their maxima in the |W| hierarchy (and INT4 rows)."""
        rows = rows.to(device=self.device, dtype=torch.int64).contiguous()
        L.check(self.lib.dqrm_rows_changed(C.byref(self._c), _ptr(rows), rows.numel(), 4 if repack else 0,
                                           _stream_handle()), "dqrm_rows_changed")

    def backward_coalesce_scaled(self, batch: LookupBatch, dy: torch.Tensor, ws: "CoalescedGrad", divisor: int,
                                 ste: bool = True, layout: str = "tbd") -> None:
        """backward_coalesce with every lookup's gradient divided by `divisor` before the
        sum (dqrm_emb_bwd_coalesce_scaled; the simulated-DP buffer's grad / N)."""
        st, sb = self._dy_strides(dy, layout, self.T, batch.num_bags, self.D)
        L.check(
            self.lib.dqrm_emb_bwd_coalesce_scaled(
                C.byref(self._c), C.byref(batch.c), _ptr(dy), st, sb, int(ste), int(divisor), _ptr(ws.slot_cap_base),
                _ptr(ws.rows), _ptr(ws.vals), _ptr(ws.ucount), _ptr(ws.absmax), *self._ws_args(batch),
                _stream_handle()),
            "dqrm_emb_bwd_coalesce_scaled",
        )

    def lookup_grad(self, batch: LookupBatch, dy: torch.Tensor, ste: bool = True,
                    layout: str = "tbd", presum: bool = False) -> tuple[torch.Tensor, torch.Tensor]:
        """Uncoalesced per-lookup sparse gradient (dqrm_emb_bwd_lookup_grad): slab rows
        i64 [L] and STE'd dy rows f32 [L, D], in lookup order -- the COO that
        nn.EmbeddingBag(sparse=True)'s backward yields. presum: the same rows with each row's
        gradient summed (lookup order) into its first lookup and zeros after it
        (dqrm_emb_bwd_lookup_grad_presum) -- an optimizer's scatter-add of it is deterministic;
        batches of more than DQRM_PRESUM_MAX_LOOKUPS lookups per table take the per-lookup form."""
        if presum and 0 < batch.max_lookups <= L.DQRM_PRESUM_MAX_LOOKUPS and batch.num_bags > 0:
            st, sb = self._dy_strides(dy, layout, self.T, batch.num_bags, self.D)
            Lk = int(batch.idx.numel())
            rows = torch.empty(Lk, dtype=torch.int64, device=self.device)
            vals = torch.empty(Lk, self.D, dtype=torch.float32, device=self.device)
            L.check(
                self.lib.dqrm_emb_bwd_lookup_grad_presum(C.byref(self._c), C.byref(batch.c), _ptr(dy), st, sb,
                                                         int(ste), _ptr(rows), _ptr(vals), _stream_handle()),
                "dqrm_emb_bwd_lookup_grad_presum",
            )
            return rows, vals
        st, sb = self._dy_strides(dy, layout, self.T, batch.num_bags, self.D)
        Lk = int(batch.idx.numel())
        if batch.num_bags <= 0:  # no bag covers any lookup: an all-zero gradient on row 0
            return (torch.zeros(Lk, dtype=torch.int64, device=self.device),
                    torch.zeros(Lk, self.D, dtype=torch.float32, device=self.device))
        # every entry is written by the kernel (lookups before off[0] as zero rows, flagged)
        rows = torch.empty(Lk, dtype=torch.int64, device=self.device)
        vals = torch.empty(Lk, self.D, dtype=torch.float32, device=self.device)
        L.check(
            self.lib.dqrm_emb_bwd_lookup_grad(C.byref(self._c), C.byref(batch.c), _ptr(dy), st, sb, int(ste),
                                              _ptr(rows), _ptr(vals), _stream_handle()),
            "dqrm_emb_bwd_lookup_grad",
        )
        return rows, vals

    def backward_coalesce(self, batch: LookupBatch, dy: torch.Tensor, ws: "CoalescedGrad",
                          ste: bool = True, layout: str = "tbd") -> None:
        """STE + sparse backward + coalesce + per-slot max |grad| (s_q_g_p_c.py:850-861)."""
        st, sb = self._dy_strides(dy, layout, self.T, batch.num_bags, self.D)
        L.check(
            self.lib.dqrm_emb_bwd_coalesce(
                C.byref(self._c), C.byref(batch.c), _ptr(dy), st, sb, int(ste), _ptr(ws.slot_cap_base),
                _ptr(ws.rows), _ptr(ws.vals), _ptr(ws.ucount), _ptr(ws.absmax), *self._ws_args(batch),
                _stream_handle()),
            "dqrm_emb_bwd_coalesce",
        )

    def apply_local_is_one_launch(self, batch: LookupBatch) -> bool:
        """Whether backward_apply_local runs this batch as ONE launch on the current stream
        (Criteo form, <= 4096 lookups, <= 32 tables, and the grid resident at once: device CUs,
        occupancy and the stream's CU mask; dqrm_bwd_apply_local_is_one_launch)."""
        rc = self.lib.dqrm_bwd_apply_local_is_one_launch(C.byref(self._c), C.byref(batch.c), _stream_handle())
        if rc < 0:
            L.check(rc, "dqrm_bwd_apply_local_is_one_launch")
        return rc == 1

    def backward_apply_local(self, batch: LookupBatch, dy: torch.Tensor, ws: "CoalescedGrad", grad_bits: int,
                             s_avg: torch.Tensor, lr: float, repack: bool = False, ste: bool = True,
                             layout: str = "tbd") -> None:
        """World size 1: backward_coalesce + the local quantized update (dqrm_apply_local),
        one launch for Criteo-form batches (dqrm_emb_bwd_apply_local); same results."""
        st, sb = self._dy_strides(dy, layout, self.T, batch.num_bags, self.D)
        L.check(
            self.lib.dqrm_emb_bwd_apply_local(
                C.byref(self._c), C.byref(batch.c), _ptr(dy), st, sb, int(ste), _ptr(ws.slot_cap_base),
                ws.cap_total, _ptr(ws.rows), _ptr(ws.vals), _ptr(ws.ucount), _ptr(ws.absmax), int(grad_bits),
                _ptr(s_avg), float(lr), 4 if repack else 0, *self._ws_args(batch), _stream_handle()),
            "dqrm_emb_bwd_apply_local",
        )

    def _fwd_flags(self, refresh_scale: bool, use_packed: bool, full_precision: bool) -> int:
        flags = L.DQRM_FWD_REFRESH_SCALE if refresh_scale else 0
        if use_packed:
            flags |= L.DQRM_FWD_USE_PACKED
        if full_precision:
            flags |= L.DQRM_FWD_FULL_PRECISION
        return flags

    def apply_fwd_local_is_one_launch(self, batch: LookupBatch, next_batch: LookupBatch,
                                      use_packed: bool = False) -> bool:
        """Whether backward_apply_forward_local runs the update AND the next batch's forward
        as ONE launch (dqrm_bwd_apply_fwd_local_is_one_launch)."""
        rc = self.lib.dqrm_bwd_apply_fwd_local_is_one_launch(
            C.byref(self._c), C.byref(batch.c), C.byref(next_batch.c),
            self._fwd_flags(True, use_packed, False), _stream_handle())
        if rc < 0:
            L.check(rc, "dqrm_bwd_apply_fwd_local_is_one_launch")
        return rc == 1

    def backward_apply_forward_local(self, batch: LookupBatch, dy: torch.Tensor, ws: "CoalescedGrad",
                                     grad_bits: int, s_avg: torch.Tensor, lr: float, next_batch: LookupBatch,
                                     bits: int = 4, refresh_scale: bool = True, full_precision: bool = False,
                                     out: torch.Tensor | None = None, layout: str = "tbd", repack: bool = False,
                                     ste: bool = True, dy_layout: str = "tbd") -> torch.Tensor:
        """World size 1 at the step boundary: backward_apply_local(batch, dy, ...) followed by
        forward(next_batch, ...) -- the embedding update of step i and apply_emb of step i+1,
        adjacent in the training loop -- with the same results; for Criteo-form batches of one
        size the forward runs inside the update's launch, table by table as each table's update
        completes (dqrm_emb_bwd_apply_fwd_local). Returns the next batch's output."""
        if next_batch.num_tables != self.T:
            raise ValueError("batch has %d tables, set has %d" % (next_batch.num_tables, self.T))
        B, T, D = next_batch.num_bags, self.T, self.D
        if out is None:
            out = torch.empty((T, B, D) if layout == "tbd" else (B, T, D), dtype=torch.float32, device=self.device)
        ost, osb = (B * D, D) if layout == "tbd" else (D, T * D)
        st, sb = self._dy_strides(dy, dy_layout, self.T, batch.num_bags, self.D)
        L.check(
            self.lib.dqrm_emb_bwd_apply_fwd_local(
                C.byref(self._c), C.byref(batch.c), _ptr(dy), st, sb, int(ste), _ptr(ws.slot_cap_base),
                ws.cap_total, _ptr(ws.rows), _ptr(ws.vals), _ptr(ws.ucount), _ptr(ws.absmax), int(grad_bits),
                _ptr(s_avg), float(lr), 4 if repack else 0, *self._ws_args(batch), C.byref(next_batch.c), int(bits),
                self._fwd_flags(refresh_scale, False, full_precision), _ptr(out), ost, osb, _stream_handle()),
            "dqrm_emb_bwd_apply_fwd_local",
        )
        return out


def slot_caps(num_rows: Sequence[int], max_lookups: int) -> list[int]:
    """Exclusive prefix of the coalesce-slot capacities (dqrm_coalesce_slot_caps): slot
    t*S+s holds at most min(max_lookups, rows in row-range s of table t) entries."""
    lib = L.load()
    T = len(num_rows)
    nr = (C.c_int64 * T)(*[int(n) for n in num_rows])
    out = (C.c_int64 * (T * L.DQRM_TABLE_SPLIT + 1))()
    total = lib.dqrm_coalesce_slot_caps(nr, T, int(max_lookups), out)
    if total < 0:
        L.check(int(total), "dqrm_coalesce_slot_caps")
    return list(out)


@dataclass
class CoalescedGrad:
    """Coalesced sparse gradient of all tables (one rank), in row-range slots: slot
    k = t * DQRM_TABLE_SPLIT + s (include/dqrm.h)."""

    slot_base: list[int]        # host copy of slot_cap_base
    slot_cap_base: torch.Tensor  # i64 [T*S+1]
    rows: torch.Tensor           # i32 [WCAP]
    vals: torch.Tensor           # f32 [WCAP, D]
    ucount: torch.Tensor         # i32 [T*S]
    absmax: torch.Tensor         # f32 [T*S]

    @classmethod
    def allocate(cls, num_rows: Sequence[int], max_lookups: int, dim: int, device,
                 absmax: torch.Tensor | None = None) -> "CoalescedGrad":
        """absmax: caller-owned f32 [T*S] view to write the per-slot maxima into (a slice of
        a buffer several sets gather together), else allocated here."""
        base = slot_caps(num_rows, max_lookups)
        W = base[-1]
        TS = len(num_rows) * L.DQRM_TABLE_SPLIT
        if absmax is not None and (absmax.numel() != TS or absmax.dtype != torch.float32
                                   or not absmax.is_contiguous()):
            raise ValueError("absmax must be a contiguous f32 [T*S] tensor")
        return cls(
            slot_base=base,
            slot_cap_base=torch.tensor(base, dtype=torch.int64, device=device),
            rows=torch.zeros(max(W, 1), dtype=torch.int32, device=device),
            vals=torch.zeros(max(W, 1), dim, dtype=torch.float32, device=device),
            ucount=torch.zeros(TS, dtype=torch.int32, device=device),
            absmax=absmax if absmax is not None else torch.zeros(TS, dtype=torch.float32, device=device),
        )

    @property
    def cap_total(self) -> int:
        return self.slot_base[-1]


def default_caps(num_rows: Sequence[int], max_lookups: int) -> list[int]:
    """Payload capacity per table: cap_t = min(max lookups per table, n_t), the most
    unique rows one rank can send for table t."""
    return [min(int(max_lookups), int(n)) for n in num_rows]


def reference_scale(absmax: float, bits: int) -> float:
    """clamp(absmax, 1e-8) / (2^(bits-1)-1) in f32 (quant_utils.py:189-192), host helper."""
    import numpy as np

    a = np.float32(absmax)
    a = max(a, np.float32(1e-8))
    return float(np.float32(a) / np.float32(2 ** (bits - 1) - 1))


__all__ = ["LookupBatch", "EmbeddingTableSet", "CoalescedGrad", "default_caps", "slot_caps", "reference_scale"]
