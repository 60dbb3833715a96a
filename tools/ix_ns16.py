"""Diagnostic (timing only): the intersection's step launch on 16-slot rows (four envs per wave,
simulate_kernel<T, 16, 4, NET_GRAPH>) against the 32-slot rows (two envs per wave), and the mixed
launch on the 32-slot rows (simulate_mixed_kernel: the envs above 16 vehicles two to a wave, the
rest four to a wave), on the same in-loop config-6 scenes.

Runs the bench's config-6 env for a number of steps, then copies each env's first 16 slots (its
live vehicles are compacted at the front; an env with more than 16 keeps its first 16, for timing
only) into a 16-slot state, and times the fused 15-frame simulate launch and the env_step launch
(observation + step tail) on both, alternating, from the same snapshots.

  python tools/ix_ns16.py [steps]
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def timed(fn):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e)


def main(steps=30):
    from bench import CONFIGS
    from topotrafficrl_amd.intersection import VecIntersectionEnv
    from topotrafficrl_amd.road import BatchedRoad
    from topotrafficrl_amd.state import BatchState
    C6 = CONFIGS[6]
    dev = torch.device("cuda:0")
    E, N = C6["num_envs"], C6["vehicles"]
    dt = os.environ.get("DT", "f64")
    env = VecIntersectionEnv({"num_envs": E, "vehicle_slots": N, "observation": C6["obs"], "device": str(dev),
                              "dtype": dt, "auto_reset": True})
    env.reset(seed=12345)
    g = torch.Generator(device=dev).manual_seed(1000)
    for _ in range(steps):
        env.step(torch.randint(0, 3, (E,), device=dev, generator=g, dtype=torch.int32))
    env._join_sides()
    torch.cuda.synchronize()
    snap32 = env.state.clone()
    live = (snap32["kind"] != 0).sum(1).cpu().numpy()
    print(f"in-loop after {steps} steps: live per env mean {live.mean():.2f} p90 {np.percentile(live, 90):.0f} "
          f"max {live.max()}; envs with > 16: {int((live > 16).sum())}", flush=True)
    a32 = snap32.to_numpy()
    a16 = {k: (v if k in ("reg_steps", "rng") else v[:, :16].copy()) for k, v in a32.items()}
    snap16 = BatchState(E, 16, device=dev, dtype=dt).load_numpy(a16)
    codes = env.action_type._codes(torch.randint(0, 3, (E,), device=dev, generator=g, dtype=torch.int32))
    ot = env.observation_type
    kc = ot.fused_cfg()
    # the mixed order of the snapshot: envs by live vehicles, heaviest first; the count above 16
    lv = torch.from_numpy(live).to(dev)
    order = torch.argsort(lv, descending=True, stable=True).to(torch.int32)
    n_wide = (lv > 16).sum().to(torch.int32).view(1)
    pairs = torch.arange(E, device=dev).view(-1, 2)[torch.argsort(lv.view(-1, 2).sum(1), descending=True,
                                                                  stable=True)].flatten().to(torch.int32)
    runs = {"32-slot rows, 2 envs per wave (pair order)": (snap32, pairs, None),
            "16-slot rows, 4 envs per wave": (snap16, None, None),
            "32-slot rows, mixed launch": (snap32, order, n_wide)}
    res = {k: {"step": []} for k in runs}
    outs = {}
    for rep in range(7):
        for name, (snap, od, nw) in runs.items():
            work = snap.clone()
            road = BatchedRoad(env.network, work, env.params)
            t = env.time.clone()
            torch.cuda.synchronize()
            res[name]["step"].append(timed(lambda: road.env_step(codes, 15, 1 / 15, kc, env.reward_cfg, t, 1.0, od,
                                                                 None, nw)))
            outs[name] = work.to_numpy()
    for name in runs:
        print(f"{name}: env_step {np.median(res[name]['step'][1:]):.3f} ms (min {np.min(res[name]['step'][1:]):.3f})",
              flush=True)
    a, b = outs["32-slot rows, 2 envs per wave (pair order)"], outs["32-slot rows, mixed launch"]
    same = all(np.array_equal(a[k], b[k], equal_nan=True) for k in a)
    print(f"mixed launch == 32-slot launch, every field of every env: {same} (n_wide {int(n_wide)})", flush=True)
    # the 16-slot result equals the 32-slot one on every env that fits
    w32, w16 = snap32.clone(), snap16.clone()
    BatchedRoad(env.network, w32, env.params).simulate(codes, 15, 1 / 15)
    BatchedRoad(env.network, w16, env.params).simulate(codes, 15, 1 / 15)
    b32, b16 = w32.to_numpy(), w16.to_numpy()
    fit = live <= 16
    same = all(np.array_equal(b32[k][fit][:, :16], b16[k][fit]) for k in ("x", "y", "speed", "lane", "kind", "crashed"))
    print(f"16-slot state == 32-slot state on the {int(fit.sum())} envs with <= 16 live: {same}", flush=True)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 30)
