"""Per-step time of env.step with and without the bench's per-launch HIP events (diagnostic): the
timed loop of bench.py brackets every fused launch with two timing events; this measures what
those markers cost between back-to-back launches, interleaved in one process.

  python tools/gap_ab.py [config ...]     # on the GPU box; configs 2, 3, 4 (default 4)
"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from topotrafficrl_amd.envs import VecHighwayEnv  # noqa: E402
from topotrafficrl_amd.road import BatchedRoad  # noqa: E402


def run(cfg, steps=20, rounds=7):
    dev = torch.device("cuda:0")
    import bench
    obs = bench.CONFIGS[cfg]["obs"]
    env = VecHighwayEnv({"num_envs": 4096, "vehicles_count": bench.CONFIGS[cfg]["vehicles"], "observation": obs, "device": "cuda:0",
                         "dtype": "f64"})
    env.reset(seed=12345)
    g = torch.Generator(device=dev).manual_seed(1000)
    acts = torch.randint(0, env.action_space.n, (steps, 4096), device=dev, generator=g, dtype=torch.int32)
    orig = BatchedRoad.env_step

    def timed(self_road, *a, **kw):
        st_ = torch.cuda.current_stream(dev)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record(st_)
        r = orig(self_road, *a, **kw)
        e.record(st_)
        return r

    res = {"events": [], "plain": []}
    for t in range(5):
        env.step(acts[t])
    torch.cuda.synchronize()
    for r in range(rounds):
        for mode in ("events", "plain"):
            env.reset(seed=12345)  # the bench's episode: a fresh scene, 3 warm-up steps, then the timed ones
            for t in range(3):
                env.step(acts[t])
            BatchedRoad.env_step = timed if mode == "events" else orig
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for t in range(steps):
                env.step(acts[t])
            torch.cuda.synchronize()
            res[mode].append((time.perf_counter() - t0) / steps * 1e3)
            BatchedRoad.env_step = orig
    # host time of one env.step call
    env.reset(seed=12345)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for t in range(steps):
        env.step(acts[t])
    host = (time.perf_counter() - t0) / steps * 1e3  # before the sync: the host's own cost per call
    torch.cuda.synchronize()
    print(f"config {cfg}: ms per step, events {np.median(res['events']):.4f} (min {min(res['events']):.4f}), "
          f"plain {np.median(res['plain']):.4f} (min {min(res['plain']):.4f}); host enqueue {host:.4f} ms per call",
          flush=True)


if __name__ == "__main__":
    for c in (sys.argv[1:] or ["4"]):
        run(int(c))
