"""Phase clocks of reset_wave_kernel (build: -DTTRL_RESET_TRACE into tools/_ab/lib_rtrace.so,
then copy it over lib/libttrl_mi355x.so on the GPU box): one full reset of 4096 x 64 envs, then a
masked one of every 8th env."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from topotrafficrl_amd.envs import VecHighwayEnv  # noqa: E402

env = VecHighwayEnv({"num_envs": 4096, "vehicles_count": 64, "device": "cuda:0", "auto_reset": True})
env.reset(seed=1)
torch.cuda.synchronize()
term = torch.zeros(4096, dtype=torch.bool, device="cuda:0")
term[7::8] = True
for _ in range(3):
    env._auto_reset_step(term, torch.zeros_like(term))
torch.cuda.synchronize()
print("done")
