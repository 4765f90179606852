"""Criteo input path feeding the QAT step.

Reference (data_loader_terabyte.py / dlrm_data_pytorch.py @ 2024-10-24):
  CriteoBinDataset (:197-240)   flat binary file of int32 records (label, 13 dense, 26
                                categorical), one batch per __getitem__, written by
                                numpy_to_binary (:243-280)
  _transform_features (:68-87)  x_cat % max_ind_range; X = log(x_int + 1); lS_i = x_cat.t();
                                y = label.view(-1, 1); lS_o = arange(B) per table
  collate_wrapper_criteo_offset (dlrm_data_pytorch.py:328-345)  the Kaggle collate, same outputs

MI355X design: the file is memory-mapped; a batch's raw records (160 B/sample) are copied
to HBM once (pinned staging, optional side stream) and ONE kernel (dqrm_criteo_unpack)
produces the dense features, labels and the transposed [26, B] int64 index tensor that the
embedding kernels consume directly as a Criteo-form LookupBatch (DQRM_BATCH_POOLING_ONE:
offsets are never read). The reference's host-side transpose, int64 cast, modulo and
log pass, and the H2D copy of 4x larger int64 indices, disappear.
"""
from __future__ import annotations

import math
import os

import numpy as np
import torch

from . import _lib as L
from .tables import LookupBatch, _ptr, _stream_handle

REC = L.DQRM_CRITEO_RECORD_INTS
DEN = L.DQRM_CRITEO_DENSE
CAT = L.DQRM_CRITEO_SPARSE


def transform_features(records: torch.Tensor, max_ind_range: int = -1, with_offsets: bool = True,
                       stream: torch.cuda.Stream | None = None):
    """_transform_features (data_loader_terabyte.py:68-87) of a device-resident record block
    records int32 [B, 40]. Returns (X [B,13] f32, lS_o [26,B] i64 or None, lS_i [26,B] i64,
    y [B,1] f32) on the records' device."""
    if not records.is_cuda:
        raise L.DQRMError("dqrm_criteo_unpack runs on the GPU (records must be a CUDA tensor; no CPU path)")
    if records.dtype != torch.int32 or records.dim() != 2 or records.shape[1] != REC:
        raise ValueError(f"records must be int32 [B, {REC}]")
    records = records.contiguous()
    B = records.shape[0]
    dev = records.device
    X = torch.empty(B, DEN, dtype=torch.float32, device=dev)
    lS_i = torch.empty(CAT, B, dtype=torch.int64, device=dev)
    y = torch.empty(B, 1, dtype=torch.float32, device=dev)
    lS_o = torch.empty(CAT, B, dtype=torch.int64, device=dev) if with_offsets else None
    mod = int(max_ind_range) if max_ind_range and max_ind_range > 0 else 0
    if mod > 0x7FFFFFFF:
        raise ValueError("max_ind_range must fit int32")
    with torch.cuda.device(dev):
        L.check(L.load().dqrm_criteo_unpack(_ptr(records), B, mod, _ptr(X), _ptr(lS_i), _ptr(y), _ptr(lS_o),
                                            _stream_handle(stream)),
                "dqrm_criteo_unpack")
    return X, lS_o, lS_i, y


class CriteoBinDataset:
    """data_loader_terabyte.CriteoBinDataset (:197-240) on the GPU: same constructor
    arguments, len() and __getitem__(idx) -> (X_int, lS_o, lS_i, y), as device tensors.

    The file is memory-mapped (no read() per batch); the last batch may be short, as in
    the reference (num_entries = ceil(file bytes / bytes per batch))."""

    def __init__(self, data_file, counts_file=None, batch_size=1, max_ind_range=-1, bytes_per_feature=4,
                 device: torch.device | str | None = None, pin_memory: bool = True):
        if bytes_per_feature != 4:
            raise ValueError("records are int32 (bytes_per_feature=4), as numpy_to_binary writes them")
        self.tar_fea, self.den_fea, self.spa_fea = 1, DEN, CAT
        self.tad_fea = self.tar_fea + self.den_fea
        self.tot_fea = self.tad_fea + self.spa_fea
        self.batch_size = int(batch_size)
        self.max_ind_range = max_ind_range
        self.bytes_per_entry = bytes_per_feature * self.tot_fea * self.batch_size
        size = os.path.getsize(data_file)
        if size % (bytes_per_feature * self.tot_fea):
            raise ValueError(f"{data_file}: size {size} is not a whole number of {self.tot_fea}-int32 records")
        self.num_entries = math.ceil(size / self.bytes_per_entry)
        self._mm = np.memmap(data_file, dtype=np.int32, mode="r").reshape(-1, self.tot_fea)
        self.counts = None
        if counts_file is not None:
            with np.load(counts_file) as data:  # allow_pickle=False (numpy default)
                self.counts = data["counts"]
        self.m_den = DEN
        self.device = torch.device(device) if device is not None else torch.device("cuda")
        self.pin_memory = pin_memory

    def __len__(self):
        return self.num_entries

    def records(self, idx: int) -> np.ndarray:
        """Host view of batch idx's raw records [b, 40] (b = batch_size except the last)."""
        if idx < 0:
            idx += self.num_entries
        if not 0 <= idx < self.num_entries:
            raise IndexError(idx)
        return self._mm[idx * self.batch_size: (idx + 1) * self.batch_size]

    def device_records(self, idx: int, stream: torch.cuda.Stream | None = None) -> torch.Tensor:
        src = self.records(idx)
        host = torch.empty(src.shape, dtype=torch.int32, pin_memory=self.pin_memory)
        np.copyto(host.numpy(), src)  # one copy: page cache -> (pinned) staging
        with torch.cuda.stream(stream) if stream is not None else _null():
            return host.to(self.device, non_blocking=self.pin_memory)

    def __getitem__(self, idx):
        return transform_features(self.device_records(idx), self.max_ind_range)

    def lookup_batch(self, lS_i: torch.Tensor) -> LookupBatch:
        """The Criteo-form batch the embedding kernels read (offsets implied)."""
        return LookupBatch.pooling_one(lS_i)


class _null:
    def __enter__(self):
        return None

    def __exit__(self, *a):
        return False


class CriteoPrefetcher:
    """Iterates a CriteoBinDataset with the next batch's H2D copy and unpack running on a
    side stream while the current batch trains; yields (X, lS_o, lS_i, y) ready on the
    consumer's current stream."""

    def __init__(self, dataset: CriteoBinDataset, start: int = 0, stop: int | None = None):
        self.ds = dataset
        self.start, self.stop = start, len(dataset) if stop is None else stop
        self.stream = torch.cuda.Stream(device=dataset.device)

    def _issue(self, i):
        with torch.cuda.stream(self.stream):
            rec = self.ds.device_records(i, self.stream)
            out = transform_features(rec, self.ds.max_ind_range, stream=self.stream)
            ev = torch.cuda.Event()
            ev.record(self.stream)
        return out, rec, ev

    def __iter__(self):
        nxt = self._issue(self.start) if self.start < self.stop else None
        for i in range(self.start, self.stop):
            out, rec, ev = nxt
            nxt = self._issue(i + 1) if i + 1 < self.stop else None
            torch.cuda.current_stream(self.ds.device).wait_event(ev)
            for t in (*out, rec):
                if t is not None:
                    t.record_stream(torch.cuda.current_stream(self.ds.device))
            yield out


def collate_wrapper_criteo_offset(list_of_tuples, device: torch.device | str | None = None):
    """dlrm_data_pytorch.collate_wrapper_criteo_offset (:328-345): (X_int, X_cat, y) tuples
    -> (X [B,13], lS_o [26,B], lS_i [26,B], T [B,1]) on the GPU (one record block, one
    unpack launch). Values must fit int32 (Criteo's do)."""
    B = len(list_of_tuples)
    rec = np.empty((B, REC), dtype=np.int64)
    for b, (x_int, x_cat, y) in enumerate(list_of_tuples):
        rec[b, 0] = y
        rec[b, 1:1 + DEN] = x_int
        rec[b, 1 + DEN:] = x_cat
    if rec.size and (rec.max() > np.iinfo(np.int32).max or rec.min() < np.iinfo(np.int32).min):
        raise ValueError("collate: values exceed int32")
    dev = torch.device(device) if device is not None else torch.device("cuda")
    return transform_features(torch.from_numpy(rec.astype(np.int32)).to(dev), -1)


def numpy_to_binary(arrays, output_file_path):
    """data_loader_terabyte.numpy_to_binary (:243-260) for in-memory arrays: a list of
    (y [n], X_int [n,13], X_cat [n,26]) written as int32 records (tests / tools)."""
    with open(output_file_path, "wb") as f:
        for y, x_int, x_cat in arrays:
            d = np.concatenate([np.asarray(y).reshape(-1, 1), x_int, x_cat], axis=1).astype(np.int32)
            f.write(d.tobytes())


__all__ = ["transform_features", "CriteoBinDataset", "CriteoPrefetcher", "collate_wrapper_criteo_offset",
           "numpy_to_binary"]
