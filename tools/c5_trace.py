"""Diagnostic (timing only): the device launches of one config-5 step (policy act + env.step), by
phase, from torch.profiler, so every small launch beside the simulate and policy kernels is named.

  python tools/c5_trace.py
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from bench import CONFIGS
    from topotrafficrl_amd.agent import EgoAttentionPolicy
    from topotrafficrl_amd.envs import VecHighwayEnv
    C = CONFIGS[5]
    dev = torch.device("cuda:0")
    env = VecHighwayEnv({"num_envs": C["num_envs"], "vehicles_count": C["vehicles"], "observation": C["obs"],
                         "device": str(dev), "dtype": "f64"})
    policy = EgoAttentionPolicy(device=dev, seed=0)
    obs, _ = env.reset(seed=12345)
    for t in range(3):
        obs = env.step(policy.act(obs, t))[0]
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile, record_function
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
        for t in range(3, 5):
            with record_function("act"):
                a = policy.act(obs, t)
            with record_function("step"):
                obs = env.step(a)[0]
        torch.cuda.synchronize()
    print(prof.key_averages().table(sort_by="cuda_time_total", row_limit=40))
    for ev in prof.events():
        if ev.device_type.name == "CUDA" or "Memcpy" in ev.name or "copy" in ev.name.lower():
            print(f"{ev.name[:100]:100s} {ev.cpu_parent.name if ev.cpu_parent else '':30s}")


if __name__ == "__main__":
    main()
