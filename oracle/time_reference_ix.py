"""Timing of the reference's own ``IntersectionEnv`` (config 6's scenario) against the float64 C
port -- TEST INFRASTRUCTURE, build container only.

bench.py's config-6 ``cpu_baseline`` times the C restatement (``cpu_baseline_ix``: oracle/ttrl_oracle.c,
OpenMP over envs) on the box's host cores; the reference itself cannot run there (/root/reference is
absent on the GPU box).  This script measures, on one core of this container, both

  * the unmodified reference ``IntersectionEnv`` (ttrl_env/envs/intersection_env.py) behind the
    name-only gymnasium / pygame / matplotlib stand-ins of oracle/gen_golden_envref.py:
    ``reset(seed)`` (abstract.py:188-214, intersection_env.py:131-318 with its 45 warm-up frames) and
    ``step(a)`` (abstract.py:224-282, intersection_env.py:135-139: 15 frames of Road.act /
    RegulatedRoad.step, the shuffled Kinematics observation through pandas, rewards, info,
    _clear_vehicles / _spawn_vehicle), a random action in {0, 1, 2} per step, the env reset when
    an episode ends -- the loop bench.py's config 6 runs, one env at a time;
  * ``bench.cpu_baseline_ix`` itself with OMP_NUM_THREADS=1 (the same per-step work over a batch),

in the same unit, live vehicle-steps/s (the vehicles present at each step's start x 15 frames, as
the GPU bench counts them), and prints the ratio port / reference.  bench.py reports
``reference_estimate`` = the port's value on the box / that ratio (REFERENCE_RATIO_IX there).

Usage:  PYTHONDONTWRITEBYTECODE=1 OMP_NUM_THREADS=1 python oracle/time_reference_ix.py [seconds]
"""
from __future__ import annotations

import os
import sys
import time

import numpy as np

os.environ["OMP_NUM_THREADS"] = "1"
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))


def reference_rate(seconds: float, seed0: int = 2000) -> tuple:
    """Live vehicle-frames and seconds of the reference IntersectionEnv's reset + step loop."""
    import gen_golden_envref as E  # noqa: E402  (installs the stand-ins, imports the unmodified env)
    env = E.ref_env()
    rng = np.random.default_rng(7)
    live = steps = episodes = 0
    el = 0.0
    seed = seed0
    t = time.perf_counter()
    env.reset(seed=seed)
    el += time.perf_counter() - t
    while el < seconds:
        n = len(env.road.vehicles)
        t = time.perf_counter()
        _, _, term, trunc, _ = env.step(int(rng.integers(0, 3)))
        if term or trunc:
            seed += 1
            episodes += 1
            env.reset(seed=seed)
        el += time.perf_counter() - t
        live += n
        steps += 1
    return live * 15, el, steps, episodes


def port_rate(seconds: float) -> dict:
    import bench
    return bench.cpu_baseline_ix(seconds_target=seconds)


def main(seconds: float = 60.0) -> None:
    rl = re = 0.0
    rs = rep = 0
    pv = []
    for _ in range(4):  # alternating rounds: the same machine state for both
        a, b, s, e = reference_rate(seconds / 4, seed0=2000 + 1000 * rs)
        rl, re, rs, rep = rl + a, re + b, rs + s, rep + e
        pv.append(port_rate(seconds / 4)["value"])
    ref = rl / re
    port = float(np.mean(pv))
    print(f"reference IntersectionEnv (reset + step, shuffled Kinematics 15x7, 1 core): {ref:.4g} live "
          f"vehicle-steps/s ({rs} steps, {rep} episodes ended, {re:.1f} s)")
    print(f"float64 C port (bench.cpu_baseline_ix, OMP_NUM_THREADS=1, 1024 envs): {port:.4g} live vehicle-steps/s "
          f"(rounds {', '.join(f'{v:.4g}' for v in pv)})")
    print(f"ratio port / reference = {port / ref:.1f}  (REFERENCE_RATIO_IX)")


if __name__ == "__main__":
    main(float(sys.argv[1]) if len(sys.argv) > 1 else 60.0)
