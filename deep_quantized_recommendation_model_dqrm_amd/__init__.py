"""MI355X-native (gfx950 / CDNA4) DQRM data-parallel QAT embedding path.

Drop-in for the reference's hot path (YangZhou08/Deep_Quantized_Recommendation_Model_DQRM):
  * ``quant_modules_not_quantize_grad.QuantEmbeddingBagTwo``  (INT4 fake-quant EmbeddingBag)
  * ``sgd_quantized_gradients_parallel_comm`` hooks            (INT8 sparse-grad all-reduce + SGD,
                                                                and the MLP's per-channel INT8 grads)
  * ``sgd_quantized_gradients`` simulated-DP buffer helpers
  * ``quantized_ops.ops.quantized.embedding_bag_{4bit,byte}_*``  (row-wise PTQ inference formats)
backed by hand-written HIP kernels behind the C ABI in ``include/dqrm.h`` (libdqrm.so).
"""
from . import _lib
from ._build import LIB_PATH, build
from .tables import CoalescedGrad, EmbeddingTableSet, LookupBatch, default_caps, reference_scale
from .comm import MultiSetExchange, SparseGradExchange, get_my_slice, payload_bytes
from .dense import DenseGradExchange
from . import quant_modules_not_quantize_grad, sgd_quantized_gradients, sgd_quantized_gradients_parallel_comm
from .quant_modules_not_quantize_grad import QuantEmbeddingBagCollection, QuantEmbeddingBagTwo
from . import quantized_ops

__all__ = [
    "LIB_PATH",
    "build",
    "_lib",
    "EmbeddingTableSet",
    "LookupBatch",
    "CoalescedGrad",
    "default_caps",
    "reference_scale",
    "SparseGradExchange",
    "MultiSetExchange",
    "get_my_slice",
    "payload_bytes",
    "DenseGradExchange",
    "QuantEmbeddingBagTwo",
    "QuantEmbeddingBagCollection",
    "quant_modules_not_quantize_grad",
    "sgd_quantized_gradients",
    "sgd_quantized_gradients_parallel_comm",
    "quantized_ops",
]
