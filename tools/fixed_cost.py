"""Diagnostic: fused-launch time vs frame count (0 frames = HBM load + LDS staging + store only)."""
import ctypes as C
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from topotrafficrl_amd import _lib  # noqa: E402
from topotrafficrl_amd.envs import VecHighwayEnv  # noqa: E402

dtype = sys.argv[1] if len(sys.argv) > 1 else "f64"
env = VecHighwayEnv({"num_envs": 4096, "vehicles_count": 64, "device": "cuda:0", "dtype": dtype})
env.reset(seed=12345)
dev = torch.device("cuda:0")
for _ in range(10):
    env.step(torch.randint(0, 5, (4096,), device=dev))
lib = _lib.load()
stream = torch.cuda.current_stream(dev).cuda_stream
acts = env.action_type._codes(torch.randint(0, 5, (4096,), device=dev))
base = env.state.clone()
for frames in (0, 1, 2, 4, 8, 15, 30):
    ts = []
    for r in range(8):
        env.state.copy_(base)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        rc = lib.ttrl_simulate(C.byref(env.state.struct()), C.byref(env.network.table), C.byref(env.params),
                               acts.data_ptr(), frames, 1 / 15, stream)
        e.record()
        torch.cuda.synchronize()
        assert rc == 0
        ts.append(s.elapsed_time(e))
    print(f"{dtype} frames {frames:3d}: {np.median(ts[2:]) * 1e3:8.1f} us")
