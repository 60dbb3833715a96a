"""Diagnostic (timing only): is the config-6 step host-bound?  Enqueue time of N steps (no sync;
the host's Python + launch cost per step) against the wall time once the GPU has drained.

  python tools/ix_host.py [steps]
"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(steps=100):
    from bench import CONFIGS
    from topotrafficrl_amd.intersection import VecIntersectionEnv
    C6 = CONFIGS[6]
    dev = torch.device("cuda:0")
    E = C6["num_envs"]
    env = VecIntersectionEnv({"num_envs": E, "vehicle_slots": C6["vehicles"], "observation": C6["obs"],
                              "device": str(dev), "dtype": "f64", "auto_reset": True})
    env.reset(seed=12345)
    acts = torch.randint(0, 3, (steps + 10, E), device=dev, dtype=torch.int32,
                         generator=torch.Generator(device=dev).manual_seed(1))
    for t in range(10):
        env.step(acts[t])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for t in range(10, 10 + steps):
        env.step(acts[t])
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"{steps} steps: host enqueue {1e3 * (t1 - t0) / steps:.3f} ms per step, wall {1e3 * (t2 - t0) / steps:.3f} "
          f"ms per step", flush=True)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 100)
