"""Diagnostic (timing only): the intersection's fused 15-frame simulate launch at several batch
sizes (f64, 32 slots, EPW = 2 envs per workgroup), to see how the launch time follows the number
of workgroup rounds (LDS per workgroup bounds the workgroups resident per CU).

  python tools/ix_sim_time.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from bench import CONFIGS
    from topotrafficrl_amd.intersection import VecIntersectionEnv
    C = CONFIGS[6]
    dev = torch.device("cuda:0")
    for E in (256, 640, 1280, 1920, 2560, 3200, 3840, 4096, 5120):
        env = VecIntersectionEnv({"num_envs": E, "vehicle_slots": C["vehicles"], "observation": C["obs"],
                                  "device": str(dev), "dtype": os.environ.get("DT", "f64")})
        env.reset(seed=12345)
        codes = env.action_type._codes(torch.ones(E, dtype=torch.int32, device=dev))
        snap = env.state.clone()
        ts = []
        for r in range(6):
            env.state.copy_(snap)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            env.road.simulate(codes, 15, 1 / 15)
            e.record()
            torch.cuda.synchronize()
            ts.append(s.elapsed_time(e))
        ts = sorted(ts[1:])
        print(f"E {E:5d} workgroups {E // 2:5d}: {ts[len(ts) // 2]:.3f} ms per 15-frame launch", flush=True)


if __name__ == "__main__":
    main()
