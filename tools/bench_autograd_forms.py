"""Host cost of the ways a per-table module can hand its output's gradient to the library
(26 tables, Kaggle B=128, D=16): (a) a torch.autograd.Function node per module, (b) the
output as a leaf with requires_grad and a tensor hook, (c) a leaf whose .grad is read after
backward (no Python in the backward). The forward is one small device op per module in every
form; the backward of the downstream graph is a sum over the 26 outputs.
usage: python tools/bench_autograd_forms.py"""
import time

import torch

T, B, D, STEPS = 26, 128, 16, 200
dev = torch.device("cuda")
src = [torch.randn(B, D, device=dev) for _ in range(T)]
sink = [None] * T


class Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, w, t):
        ctx.t = t
        return src[t] * 1.0

    @staticmethod
    def backward(ctx, g):
        sink[ctx.t] = g
        return None, None


w = torch.zeros(1, device=dev, requires_grad=True)


def form_a():
    ys = [Fn.apply(w, t) for t in range(T)]
    torch.autograd.backward(ys, [torch.ones(B, D, device=dev)] * T)


def form_b():
    ys = []
    for t in range(T):
        y = src[t] * 1.0
        y.requires_grad_(True)
        y.register_hook(lambda g, t=t: sink.__setitem__(t, g))
        ys.append(y)
    torch.autograd.backward(ys, [torch.ones(B, D, device=dev)] * T)


def form_c():
    ys = []
    for t in range(T):
        y = src[t] * 1.0
        y.requires_grad_(True)
        ys.append(y)
    torch.autograd.backward(ys, [torch.ones(B, D, device=dev)] * T)
    for t in range(T):
        sink[t] = ys[t].grad


def form_c_cat():  # downstream: one cat, then a loss (the DLRM interaction's shape)
    ys = []
    for t in range(T):
        y = src[t] * 1.0
        y.requires_grad_(True)
        ys.append(y)
    z = torch.stack(ys, dim=1)
    z.sum().backward()
    for t in range(T):
        sink[t] = ys[t].grad


def form_a_cat():
    ys = [Fn.apply(w, t) for t in range(T)]
    z = torch.stack(ys, dim=1)
    z.sum().backward()


for name, f in [("a function node", form_a), ("b leaf + hook", form_b), ("c leaf, .grad read", form_c),
                ("a + stack/sum", form_a_cat), ("c + stack/sum", form_c_cat)]:
    for _ in range(20):
        f()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(STEPS):
        f()
    torch.cuda.synchronize()
    print(f"{name:22s} {(time.perf_counter() - t0) / STEPS * 1e6:8.1f} us/step")
