"""Diagnostic (timing only): the config-6 step time against the spare resets' warm-up chunk size
(reset_chunk_frames; 0 = the whole 45-frame warm-up at once on two side streams), same seeds and
actions, bench-style timing (wall clock around synchronised steps).

  python tools/ix_chunks.py [steps]
"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(steps=60, warmup=10):
    from bench import CONFIGS
    from topotrafficrl_amd.intersection import VecIntersectionEnv
    C6 = CONFIGS[6]
    dev = torch.device("cuda:0")
    E = C6["num_envs"]
    for chunk in [int(c) for c in os.environ.get("CHUNKS", "15 9 5 0").split()]:
        env = VecIntersectionEnv({"num_envs": E, "vehicle_slots": C6["vehicles"], "observation": C6["obs"],
                                  "device": str(dev), "dtype": "f64", "auto_reset": True,
                                  "reset_chunk_frames": chunk})
        env.reset(seed=12345)
        g = torch.Generator(device=dev).manual_seed(1000)
        acts = torch.randint(0, 3, (warmup + steps, E), device=dev, generator=g, dtype=torch.int32)
        for t in range(warmup):
            env.step(acts[t])
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for t in range(warmup, warmup + steps):
            env.step(acts[t])
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / steps * 1e3
        print(f"reset_chunk_frames {chunk:3d} (effective {env._chunk}, {env._slots} spare slots): "
              f"{ms:.3f} ms per step", flush=True)
        env._join_sides()
        torch.cuda.synchronize()
        del env


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 60)
