"""Fused EgoAttention-2h forward (ttrl_ego_attention_q) vs the torch forward at the config-5 batch:
time per call (HIP events on the current stream) and the largest |difference| (diagnostic)."""
import sys
import os

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from topotrafficrl_amd.agent import EgoAttentionNetwork  # noqa: E402


def t(fn, n=50):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3


def main(B=8192):
    dev = torch.device("cuda:0")
    net = EgoAttentionNetwork(5).reset(torch.Generator().manual_seed(0)).to(dev)
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.rand(B, 15, 7, device=dev, generator=g) * 2 - 1
    x[:, :, 0] = (torch.rand(B, 15, device=dev, generator=g) < 0.7).float()
    x[:, 0, 0] = 1.0
    with torch.no_grad():
        ref = net(x)
        got = net.fused_q(x)
        print(f"B={B}: fused {t(lambda: net.fused_q(x)):.1f} us, torch {t(lambda: net(x)):.1f} us, "
              f"max |diff| {float((got - ref).abs().max()):.2e} (max |q| {float(ref.abs().max()):.2e})")


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 8192)
