"""Diagnostic (timing only): where the config-6 step's time goes on IN-LOOP intersection scenes.

Runs the bench's config-6 env (4096 envs, auto-reset, overlapped resets) for a number of steps,
then, on snapshots of the in-loop state with no side-stream work pending, times
  * the fused simulate launch alone (ttrl_simulate, 15 frames),
  * the env.step launch (simulate + shuffled Kinematics observation + step tail; ttrl_env_step),
  * a fresh-reset scene's simulate launch (the 0.36 ms of profiles/r03/r03n),
and, with the phase-timing build (tools/_ab/lib_timing.so, -DTTRL_PHASE_TIMING), the per-phase
cycles per wave of the in-loop simulate launch, plus the live-vehicle count distribution.

  python tools/ix_inloop.py [steps]
"""
import ctypes as C
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def timed(fn):
    """One call of fn, timed with HIP events on the current stream (ms)."""
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e)


def main(steps=30):
    from bench import CONFIGS
    from phases import NAMES
    from topotrafficrl_amd import _lib
    from topotrafficrl_amd.intersection import VecIntersectionEnv
    C6 = CONFIGS[6]
    dev = torch.device("cuda:0")
    E, N = C6["num_envs"], C6["vehicles"]
    env = VecIntersectionEnv({"num_envs": E, "vehicle_slots": N, "observation": C6["obs"], "device": str(dev),
                              "dtype": os.environ.get("DT", "f64"), "auto_reset": True})
    env.reset(seed=12345)
    g = torch.Generator(device=dev).manual_seed(1000)
    fresh = env.state.clone()
    codes_fresh = env.action_type._codes(torch.ones(E, dtype=torch.int32, device=dev))
    for _ in range(steps):
        env.step(torch.randint(0, 3, (E,), device=dev, generator=g, dtype=torch.int32))
    env._join_sides()
    torch.cuda.synchronize()
    snap = env.state.clone()
    live = (snap["kind"] != 0).sum(1).cpu().numpy()
    print(f"in-loop after {steps} steps: live vehicles per env mean {live.mean():.2f} p50 {np.median(live):.0f} "
          f"p90 {np.percentile(live, 90):.0f} max {live.max()}; envs with <= 16: {np.mean(live <= 16) * 100:.1f}%; "
          f"fresh reset mean {(fresh['kind'] != 0).sum(1).float().mean().item():.2f}", flush=True)
    codes = env.action_type._codes(torch.randint(0, 3, (E,), device=dev, generator=g, dtype=torch.int32))
    road = env.road

    # copies are outside the timed region: time only the launch
    def launch_only(state, c):
        env.state.copy_(state)
        torch.cuda.synchronize()
        return timed(lambda: road.simulate(c, 15, 1 / 15))

    t_in = np.median([launch_only(snap, codes) for _ in range(5)][1:])
    t_fresh = np.median([launch_only(fresh, codes_fresh) for _ in range(5)][1:])
    ot = env.observation_type
    reps = []
    for _ in range(5):
        env.state.copy_(snap)
        t0 = env.time.clone()
        torch.cuda.synchronize()
        reps.append(timed(lambda: road.env_step(codes, 15, 1 / 15, ot.fused_cfg(), env.reward_cfg, env.time, 1.0)))
        env.time.copy_(t0)
    t_step = float(np.median(reps[1:]))
    print(f"simulate launch: in-loop {t_in:.3f} ms, fresh reset {t_fresh:.3f} ms; env_step launch (obs + tail) "
          f"in-loop {t_step:.3f} ms", flush=True)
    lib_path = os.path.join(ROOT, "tools", "_ab", "lib_timing.so")
    if not os.path.exists(lib_path):
        return
    lib = _lib.load(lib_path)
    sim = lib.ttrl_simulate
    sim.argtypes = [C.c_void_p] * 4 + [C.c_int32, C.c_double, C.c_void_p]
    rd = lib.ttrl_diag_phase_read
    rd.argtypes = [C.c_void_p]
    stream = torch.cuda.current_stream(dev).cuda_stream
    buf = np.zeros(20, dtype=np.uint64)
    for name, st_, c in (("in-loop", snap, codes), ("fresh", fresh, codes_fresh)):
        tot = np.zeros(20)
        for r in range(4):
            env.state.copy_(st_)
            torch.cuda.synchronize()
            rd(buf.ctypes.data)
            assert sim(C.byref(env.state.struct()), C.byref(env.network.table), C.byref(env.params), c.data_ptr(), 15,
                       1 / 15, stream) == 0
            torch.cuda.synchronize()
            rd(buf.ctypes.data)
            if r:
                tot += buf.astype(np.float64)
        per = tot / (3 * (E // 2))
        print(f"[{name}] cycles per wave per 15-frame launch, total {per.sum():.0f}")
        for n_, c_ in sorted(zip(NAMES, per), key=lambda t: -t[1]):
            if c_ > 0:
                print(f"  {n_:20s} {c_:10.0f}  {100 * c_ / per.sum():5.1f}%")


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 30)
