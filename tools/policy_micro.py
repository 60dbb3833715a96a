"""Micro-benchmark of the EgoAttention-2h forward pieces at 8192 envs (diagnostic)."""
import time
import torch
from torch.nn import functional as F

dev = torch.device("cuda:0")
x = torch.rand(8192, 15, 7, device=dev)
W1 = torch.rand(64, 7, device=dev)
b1 = torch.rand(64, device=dev)


def t(fn, n=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3


others = x[:, 1:, :]
print("linear 3D strided slice   %.1f us" % t(lambda: F.linear(others, W1, b1)))
oc = others.contiguous()
print("linear 3D contiguous      %.1f us" % t(lambda: F.linear(oc, W1, b1)))
o2 = oc.reshape(-1, 7)
print("linear 2D contiguous      %.1f us" % t(lambda: F.linear(o2, W1, b1)))
W8 = torch.zeros(64, 8, device=dev); W8[:, :7] = W1
o8 = torch.zeros(o2.shape[0], 8, device=dev); o8[:, :7] = o2
print("linear 2D K=8             %.1f us" % t(lambda: F.linear(o8, W8, b1)))
print("addmm 2D K=8              %.1f us" % t(lambda: torch.addmm(b1, o8, W8.t())))
print("matmul no bias 2D K=7     %.1f us" % t(lambda: o2 @ W1.t()))
W16 = torch.zeros(64, 16, device=dev); W16[:, :7] = W1
o16 = torch.zeros(o2.shape[0], 16, device=dev); o16[:, :7] = o2
print("linear 2D K=16            %.1f us" % t(lambda: F.linear(o16, W16, b1)))
h = torch.rand(o2.shape[0], 64, device=dev)
W2 = torch.rand(64, 64, device=dev)
print("linear 64x64 2D           %.1f us" % t(lambda: F.linear(h, W2, b1)))
