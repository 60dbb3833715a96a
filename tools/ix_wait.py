"""Diagnostic (timing only, results NOT the reference's): how much of a config-6 step is the main
stream waiting for the side stream's spare resets?  Times env.step at 4096 intersection envs
(a) as shipped, (b) with the spare-ready event recorded BEFORE the side stream's reset work (so the
main stream never waits for it; the swapped-in scenes are then not guaranteed to be ready), and
(c) with overlap_resets off (in-place resets on the main stream).  Measured with the one-deep spare
buffer (profiles/r02/r02r_ix_wait.txt): 1.25 / 0.96 / 1.66 ms -- the wait was the bound, hence the
two-deep queue (r02s: shipped 0.98 ms).

  python tools/ix_wait.py
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(mode: str, steps: int = 60, warm: int = 10) -> float:
    from bench import CONFIGS
    from topotrafficrl_amd.intersection import VecIntersectionEnv, ix_reset
    C = CONFIGS[6]
    dev = torch.device("cuda:0")
    env = VecIntersectionEnv({"num_envs": C["num_envs"], "vehicle_slots": C["vehicles"], "observation": C["obs"],
                              "device": str(dev), "dtype": "f64", "auto_reset": True,
                              "overlap_resets": mode != "in_place"})
    if mode == "no_side":  # the spare resets skipped entirely: the step without the side work (bound)
        def prepare(mask):
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(dev))
            env._spare_prev, env._spare_ready = env._spare_ready, ev
        env._prepare_spares = prepare
    if mode == "no_wait":
        def prepare(mask):
            main = torch.cuda.current_stream(dev)
            side = env._sides[env._side_i]
            env._side_i = (env._side_i + 1) % len(env._sides)
            side.wait_stream(main)
            ev = torch.cuda.Event()
            ev.record(side)  # before the work: the main stream does not wait for it
            with torch.cuda.stream(side):
                ix_reset(env._spare, env.network, env.params, env.ix, env._spare_ent, mask)
            if mask is not None:
                mask.record_stream(side)
            env._spare_prev, env._spare_ready = env._spare_ready, ev
        env._prepare_spares = prepare
    env.reset(seed=12345)
    g = torch.Generator(device=dev)
    g.manual_seed(1000)
    acts = torch.randint(0, env.action_space.n, (warm + steps, C["num_envs"]), device=dev, generator=g,
                         dtype=torch.int32)
    for t in range(warm):
        env.step(acts[t])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for t in range(warm, warm + steps):
        env.step(acts[t])
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps * 1e3


if __name__ == "__main__":
    for m in ("shipped", "no_wait", "no_side", "in_place", "shipped"):
        print(f"{m:10s} {run(m):.3f} ms per env.step", flush=True)
