"""Per-phase shader clocks of the fused EgoAttention kernel (diagnostic).

  python3 tools/policy_clocks.py --build      # here: tools/_ab/lib_polclk.so (-DTTRL_POL_CLOCKS)
  python3 tools/policy_clocks.py [B]          # GPU box: one launch at batch B, phase medians / p95
"""
import ctypes as C
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
LIB = os.path.join(ROOT, "tools", "_ab", "lib_polclk.so")
PHASES = ["obs staging", "ego embedding", "query", "qk_h", "entity-loop weights", "entities", "Wv + Wc",
          "output MLP"]


def build():
    from __graft_entry__ import HIPCC, HIP_FLAGS
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    subprocess.run([HIPCC, *HIP_FLAGS, "-DTTRL_POL_CLOCKS", "-o", LIB,
                    os.path.join(ROOT, "topotrafficrl_amd", "csrc", "ttrl_policy.hip")], check=True)


def run(B):
    import numpy as np
    import torch
    from topotrafficrl_amd.agent import EgoAttentionNetwork
    lib = C.CDLL(LIB)
    dev = torch.device("cuda:0")
    net = EgoAttentionNetwork(5).reset(torch.Generator().manual_seed(0)).to(dev)
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.rand(B, 15, 7, device=dev, generator=g) * 2 - 1
    x[:, :, 0] = (torch.rand(B, 15, device=dev, generator=g) < 0.7).float()
    w = net.packed_weights()
    q = torch.empty(B, 5, device=dev)
    scratch = torch.empty(16, device=dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    for _ in range(3):
        assert lib.ttrl_ego_attention_q(C.c_void_p(x.data_ptr()), B, 15, 7, 2, C.c_void_p(w.data_ptr()), 5,
                                        C.c_void_p(scratch.data_ptr()), C.c_void_p(q.data_ptr()),
                                        C.c_void_p(st)) == 0
    torch.cuda.synchronize()
    nb = min((B + 3) // 4, 4096)
    out = np.zeros(nb * 9, dtype=np.int64)
    assert lib.ttrl_diag_policy_clocks(out.ctypes.data_as(C.c_void_p), out.size) == 0
    t = out.reshape(nb, 9)
    d = np.diff(t, axis=1)
    print(f"B={B}, {nb} waves; total cycles per wave median {np.median(t[:, 8]):.0f}, p95 "
          f"{np.percentile(t[:, 8], 95):.0f}")
    for i, name in enumerate(PHASES):
        print(f"  {name:22s} median {np.median(d[:, i]):8.0f}  p95 {np.percentile(d[:, i], 95):8.0f}")


if __name__ == "__main__":
    if sys.argv[1:] == ["--build"]:
        build()
    else:
        run(int(sys.argv[1]) if len(sys.argv) > 1 else 8192)
