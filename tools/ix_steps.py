"""Diagnostic (timing only): per-step wall time of config 6 (4096 intersection envs, auto-reset,
overlapped resets), from HIP events recorded on the main stream between steps, to show how the
episode-end reset waves (every env starts at reset(), so truncations cluster every `duration`
steps) spread over the steps.  Optional: the bench's live-vehicle count inside the loop.

  python tools/ix_steps.py [steps] [--live]
"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from bench import CONFIGS
    from topotrafficrl_amd.intersection import VecIntersectionEnv
    steps = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 100
    live_count = "--live" in sys.argv
    C = CONFIGS[6]
    dev = torch.device("cuda:0")
    env = VecIntersectionEnv({"num_envs": C["num_envs"], "vehicle_slots": C["vehicles"], "observation": C["obs"],
                              "device": str(dev), "dtype": "f64", "auto_reset": True,
                              "reset_streams": int(os.environ.get("IX_SIDES", "2"))})
    env.reset(seed=12345)
    g = torch.Generator(device=dev)
    g.manual_seed(1000)
    warm = 10
    acts = torch.randint(0, env.action_space.n, (warm + steps, C["num_envs"]), device=dev, generator=g,
                         dtype=torch.int32)
    live = torch.zeros((), dtype=torch.int64, device=dev)
    evs = []
    done_n = []
    t0 = None
    for t in range(warm + steps):
        if t == warm:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        evs.append(e)
        if live_count:
            live.add_((env.state["kind"] != 0).sum())
        _, _, term, trunc, _ = env.step(acts[t])
        done_n.append((term | trunc).sum())
    t_host = time.perf_counter() - t0
    torch.cuda.synchronize()
    t_all = time.perf_counter() - t0
    ms = np.array([evs[i].elapsed_time(evs[i + 1]) for i in range(warm, warm + steps - 1)])
    dn = np.array([int(d) for d in done_n[warm:warm + steps - 1]])
    print(f"wall {t_all / steps * 1e3:.3f} ms per step (host loop {t_host / steps * 1e3:.3f} ms per step)")
    print(f"mean {ms.mean():.3f} ms per step, median {np.median(ms):.3f}, max {ms.max():.3f}; done per step "
          f"mean {dn.mean():.0f} max {dn.max()}")
    for i in range(len(ms)):
        print(f"step {warm + i:3d} {ms[i]:7.3f} ms  done {dn[i]}")


if __name__ == "__main__":
    main()
