"""Bandwidth of the Criteo input-path kernel (dqrm_criteo_unpack) and the
end-to-end prefetched batch rate from a memory-mapped binary file.
Algorithmic bytes per sample: 160 read + 13*4 + 4 + 26*8 written (+ 26*8 with lS_o).
Prints one JSON line per batch size."""
import json
import os
import sys
import tempfile
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from deep_quantized_recommendation_model_dqrm_amd import criteo  # noqa: E402

for B in (2048, 65536, 1 << 20):
    rec = torch.randint(0, 1 << 30, (B, 40), dtype=torch.int32, device="cuda")
    for wo in (False, True):
        for _ in range(5):
            criteo.transform_features(rec, 10_000_000, with_offsets=wo)
        torch.cuda.synchronize()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(50)]
        for a, b in ev:
            a.record()
            criteo.transform_features(rec, 10_000_000, with_offsets=wo)
            b.record()
        torch.cuda.synchronize()
        ms = float(np.median([a.elapsed_time(b) for a, b in ev]))
        per = 160 + 13 * 4 + 4 + 26 * 8 + (26 * 8 if wo else 0)
        print(json.dumps({"kernel": "dqrm_criteo_unpack", "samples": B, "with_lS_o": wo, "ms": round(ms, 4),
                          "bytes_per_sample": per, "GBps": round(B * per / (ms * 1e-3) / 1e9, 1),
                          "Msamples_per_s": round(B / (ms * 1e-3) / 1e6, 1)}), flush=True)
# end to end: memory-mapped file -> pinned H2D -> unpack, prefetched on a side stream
with tempfile.TemporaryDirectory() as d:
    n, B = 1 << 20, 65536
    rs = np.random.RandomState(0)
    f = os.path.join(d, "train_data.bin")
    criteo.numpy_to_binary([(rs.randint(0, 2, n), rs.randint(0, 100, (n, 13)), rs.randint(0, 1 << 30, (n, 26)))], f)
    ds = criteo.CriteoBinDataset(f, batch_size=B, max_ind_range=10_000_000, device="cuda")
    list(criteo.CriteoPrefetcher(ds, 0, 2))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for out in criteo.CriteoPrefetcher(ds):
        pass
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    print(json.dumps({"path": "CriteoPrefetcher (memmap -> pinned -> H2D -> unpack)", "samples": n, "batch": B,
                      "s": round(el, 4), "Msamples_per_s": round(n / el / 1e6, 2),
                      "host_GBps": round(n * 160 / el / 1e9, 2)}), flush=True)
