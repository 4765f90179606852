"""Row-wise PTQ embedding formats of the reference's inference path.

After QAT the reference drivers convert each trained table to a row-wise quantized format
and serve it with fused gather ops:

    DLRM_Net.quantize_embedding  dlrm_s_pytorch_single_gpu_documentingp.py:689-704
        emb_l_q[k] = ops.quantized.embedding_bag_{4bit,byte}_prepack(emb_l[k].weight)
    DLRM_Net.apply_emb           dlrm_s_pytorch_single_gpu_documentingp.py:648-663
        ops.quantized.embedding_bag_{4bit,byte}_rowwise_offsets(emb_l_q[k], idx, off,
                                                               per_sample_weights=...)

(the same calls sit at dlrm_s_pytorch_tb_dp_one_parallel_comm.py:645-652,689-693). The
drivers import ``ops`` from ``torch._ops``; replacing that import with

    from deep_quantized_recommendation_model_dqrm_amd.quantized_ops import ops

routes exactly these four calls to libdqrm's HIP kernels (dqrm_rowwise_prepack /
dqrm_rowwise_bag). Packed rows are byte-identical to torch's CPU ops (FBGEMM fused row-wise
layout) and the gather adds in the same order with the same fused multiply-adds, so the
results are bit-identical. The packed tensor is a plain uint8 CUDA tensor [n, row_bytes].

Only mode=0 (sum), the path the reference drives, is built; other modes, pruned weights
and compressed index mappings raise NotImplementedError. Out-of-range indices raise
IndexError like the torch op (``check=False`` skips the device-side flag read).
"""
from __future__ import annotations

from types import SimpleNamespace

import torch

from . import _lib as L
from .tables import _stream_handle

SUPPORTED_DIMS = (8, 16, 32, 64, 128, 256)

_err_words: dict[int, torch.Tensor] = {}


def _err_word(device: torch.device) -> torch.Tensor:
    key = device.index if device.index is not None else torch.cuda.current_device()
    w = _err_words.get(key)
    if w is None:
        w = torch.zeros(1, dtype=torch.int32, device=torch.device("cuda", key))
        _err_words[key] = w
    return w


def _cuda(t: torch.Tensor, device: torch.device | None = None, dtype: torch.dtype | None = None) -> torch.Tensor:
    """`t` on the GPU (`device`) as a contiguous flat-or-2D tensor of `dtype`; a no-op for
    tensors already in that form (the common case on the serving path)."""
    if t.is_cuda and (device is None or t.device == device) and (dtype is None or t.dtype == dtype) \
            and t.is_contiguous():
        return t
    if not torch.cuda.is_available():
        raise L.DQRMError("row-wise quantized embedding ops run on the GPU only (no CPU path)")
    dev = device if device is not None else (t.device if t.is_cuda else torch.device("cuda"))
    return t.to(device=dev, dtype=dtype or t.dtype).contiguous()


def _prepack(weight: torch.Tensor, bits: int) -> torch.Tensor:
    if weight.dim() != 2:
        raise ValueError(f"embedding_bag prepack expects a 2-D weight, got {tuple(weight.shape)}")
    n, D = weight.shape
    if D not in SUPPORTED_DIMS:
        raise ValueError(f"embedding dim {D} unsupported (built for {SUPPORTED_DIMS})")
    lib = L.load()
    w = _cuda(weight.detach(), dtype=torch.float32)
    rb = int(lib.dqrm_rowwise_row_bytes(bits, D))
    out = torch.empty((n, rb), dtype=torch.uint8, device=w.device)
    with torch.cuda.device(w.device):
        L.check(lib.dqrm_rowwise_prepack(bits, w.data_ptr(), n, D, out.data_ptr(), _stream_handle()),
                "dqrm_rowwise_prepack")
    return out


def embedding_bag_4bit_prepack(weight: torch.Tensor) -> torch.Tensor:
    """torch.ops.quantized.embedding_bag_4bit_prepack: row = D/2 nibble bytes | fp16 scale | fp16 bias."""
    return _prepack(weight, 4)


def embedding_bag_byte_prepack(weight: torch.Tensor) -> torch.Tensor:
    """torch.ops.quantized.embedding_bag_byte_prepack: row = D bytes | f32 scale | f32 bias."""
    return _prepack(weight, 8)


def _rowwise_offsets(bits, weight, indices, offsets, scale_grad_by_freq, mode, pruned_weights,
                     per_sample_weights, compressed_indices_mapping, include_last_offset, check):
    if mode != 0:
        raise NotImplementedError("only mode=0 (sum) is built; the reference drives sum pooling")
    if pruned_weights or compressed_indices_mapping is not None:
        raise NotImplementedError("pruned row-wise tables are not built")
    if offsets is None:
        raise ValueError("offsets are required (the reference always passes them)")
    if weight.dtype != torch.uint8 or weight.dim() != 2 or not weight.is_cuda:
        raise ValueError("weight must be a packed uint8 CUDA tensor from the prepack op")
    n, rb = weight.shape
    D = (rb - 4) * 2 if bits == 4 else rb - 8
    if D not in SUPPORTED_DIMS:
        raise ValueError(f"packed row of {rb} bytes does not match a supported {bits}-bit dim")
    dev = weight.device
    idx = _cuda(indices, dev, torch.int64)
    off = _cuda(offsets, dev, torch.int64)
    if idx.dim() != 1 or off.dim() != 1:
        raise ValueError("indices and offsets must be 1-D")
    B = off.numel() - (1 if include_last_offset else 0)
    if B < 0:
        raise ValueError("include_last_offset needs at least one offset")
    psw = None
    if per_sample_weights is not None:
        psw = _cuda(per_sample_weights, dev, torch.float32)
        if psw.numel() != idx.numel():
            raise ValueError("per_sample_weights must have one weight per index")
    out = torch.empty((B, D), dtype=torch.float32, device=dev)
    lib = L.load()
    err = _err_word(dev)
    L.check(
        lib.dqrm_rowwise_bag(bits, weight.data_ptr(), n, D, idx.data_ptr() if idx.numel() else None,
                             idx.numel(), off.data_ptr(), B, int(bool(include_last_offset)),
                             psw.data_ptr() if psw is not None else None, out.data_ptr(), err.data_ptr(),
                             _stream_handle() if dev.index == torch.cuda.current_device()
                             else torch.cuda.current_stream(dev).cuda_stream),
        "dqrm_rowwise_bag",
    )
    if check:
        flags = int(err.item())
        if flags:
            err.zero_()
            if flags & L.DQRM_ERRF_INDEX:
                raise IndexError(f"embedding_bag: an index is out of range [0, {n})")
            raise ValueError("embedding_bag: offsets must be non-decreasing and within [0, len(indices)]")
    return out


def embedding_bag_4bit_rowwise_offsets(weight, indices, offsets=None, scale_grad_by_freq=False, mode=0,
                                       pruned_weights=False, per_sample_weights=None,
                                       compressed_indices_mapping=None, include_last_offset=False, *,
                                       check=True):
    """torch.ops.quantized.embedding_bag_4bit_rowwise_offsets (mode sum) -> [B, D] f32."""
    return _rowwise_offsets(4, weight, indices, offsets, scale_grad_by_freq, mode, pruned_weights,
                            per_sample_weights, compressed_indices_mapping, include_last_offset, check)


def embedding_bag_byte_rowwise_offsets(weight, indices, offsets=None, scale_grad_by_freq=False, mode=0,
                                       pruned_weights=False, per_sample_weights=None,
                                       compressed_indices_mapping=None, include_last_offset=False, *,
                                       check=True):
    """torch.ops.quantized.embedding_bag_byte_rowwise_offsets (mode sum) -> [B, D] f32."""
    return _rowwise_offsets(8, weight, indices, offsets, scale_grad_by_freq, mode, pruned_weights,
                            per_sample_weights, compressed_indices_mapping, include_last_offset, check)


def quantize_embedding(tables, bits: int) -> list[torch.Tensor]:
    """DLRM_Net.quantize_embedding (:689-704) over a list of [n, D] weights (or modules with
    ``.weight`` / ``.embedding_bag.weight``): returns emb_l_q."""
    fn = {4: embedding_bag_4bit_prepack, 8: embedding_bag_byte_prepack}.get(bits)
    if fn is None:
        raise ValueError(f"quantize_embedding: bits must be 4 or 8, got {bits}")
    out = []
    for t in tables:
        if isinstance(t, torch.Tensor):
            w = t
        elif hasattr(t, "embedding_bag"):
            w = t.embedding_bag.weight
        else:
            w = t.weight
        out.append(fn(w))
    return out


# `from ...quantized_ops import ops` replaces `from torch._ops import ops` in the drivers
ops = SimpleNamespace(quantized=SimpleNamespace(
    embedding_bag_4bit_prepack=embedding_bag_4bit_prepack,
    embedding_bag_byte_prepack=embedding_bag_byte_prepack,
    embedding_bag_4bit_rowwise_offsets=embedding_bag_4bit_rowwise_offsets,
    embedding_bag_byte_rowwise_offsets=embedding_bag_byte_rowwise_offsets,
))

__all__ = ["ops", "embedding_bag_4bit_prepack", "embedding_bag_byte_prepack",
           "embedding_bag_4bit_rowwise_offsets", "embedding_bag_byte_rowwise_offsets", "quantize_embedding"]
