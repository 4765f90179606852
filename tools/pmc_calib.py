"""Known byte counts for calibrating the memory-side counters (tools/pmc_tcc.py) on the
access shapes of the embedding kernels: random whole-row gathers of 32-, 64- and 128-B rows
(torch.index_select on half / float / double tables of 16 columns, distinct kernel names per
dtype) from 2 GiB tables (beyond the 256 MiB Infinity Cache), and a streaming elementwise pass.
Prints the algorithmic bytes per launch of each; pmc_tcc.py prints the counters.

usage: python tools/pmc_calib.py"""
import torch

M = 1 << 20          # rows gathered per launch
TABLE = 2 << 30      # bytes per table
REPS = 4

g = torch.Generator(device="cuda").manual_seed(0)
for dt in (torch.float16, torch.float32, torch.float64):
    row = 16 * torch.tensor([], dtype=dt).element_size()
    n = TABLE // row
    W = torch.empty(n, 16, dtype=dt, device="cuda").uniform_(generator=g)
    idx = torch.randint(0, n, (M,), device="cuda", generator=g)
    for _ in range(REPS):
        torch.index_select(W, 0, idx)
    torch.cuda.synchronize()
    print(f"gather {str(dt):14s} row {row:4d} B: reads {M * row + M * 8} B (rows + int64 idx), writes {M * row} B")
    del W
    torch.cuda.empty_cache()
x = torch.empty(128 << 20, dtype=torch.float32, device="cuda").uniform_(generator=g)
for _ in range(REPS):
    torch.neg(x)
torch.cuda.synchronize()
print(f"stream neg float32: reads {x.numel() * 4} B, writes {x.numel() * 4} B")
