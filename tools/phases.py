"""Per-phase cycle breakdown of the fused simulate kernel (diagnostic build with
-DTTRL_PHASE_TIMING, see tools/variants.py 'timing'): mid-episode 4096x64 state."""
import ctypes as C
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from topotrafficrl_amd import _lib  # noqa: E402
from topotrafficrl_amd.envs import VecHighwayEnv  # noqa: E402

NAMES = ["meta", "act-setup", "scan", "mobil-bar+verdict", "abort", "steer/acc+bar", "kinematics", "project+bar",
         "candidates+bar", "sat+bar", "fold", "project-init", "idm-free(pow)", "mobil-queue+bar", "mobil-items",
         "hbm-load+stage", "store", "regulation-pairs", "regulation-predict", "follow_road"]


def main(dtype="f64", steps=30, frames=15, ix=False, E=4096):
    dev = torch.device("cuda:0")
    if ix:  # the intersection scenario (NET_GRAPH instance), 32 slots
        from topotrafficrl_amd.intersection import VecIntersectionEnv
        env = VecIntersectionEnv({"num_envs": 4096, "device": "cuda:0", "dtype": dtype})
    else:
        env = VecHighwayEnv({"num_envs": E, "vehicles_count": 64, "device": "cuda:0", "dtype": dtype})
    env.reset(seed=12345)
    n_act = env.action_space.n
    g = torch.Generator(device=dev).manual_seed(1000)
    lib = _lib.load(os.path.join(ROOT, "tools", "_variants", "lib_timing.so"))
    sim = lib.ttrl_simulate
    sim.argtypes = [C.c_void_p] * 4 + [C.c_int32, C.c_double, C.c_void_p]
    rd = lib.ttrl_diag_phase_read
    rd.argtypes = [C.c_void_p]
    stream = torch.cuda.current_stream(dev).cuda_stream
    buf = np.zeros(20, dtype=np.uint64)
    tot = np.zeros(20)
    for t in range(steps):
        a = env.action_type._codes(torch.randint(0, n_act, (E,), device=dev, generator=g))
        rd(buf.ctypes.data)
        sim(C.byref(env.state.struct()), C.byref(env.network.table), C.byref(env.params), a.data_ptr(), frames, 1 / 15,
            stream)
        torch.cuda.synchronize()
        rd(buf.ctypes.data)
        if t >= 10:
            tot += buf.astype(np.float64)
    waves = (E if not ix else 2048) * (steps - 10)  # ix: two envs per 64-lane workgroup
    per = tot / waves
    print(f"[{dtype}] E={E} cycles per wave per {frames}-frame launch (mean over {steps - 10} launches), total {per.sum():.0f}")
    for n, c in zip(NAMES, per):
        print(f"  {n:16s} {c:10.0f}  {100 * c / per.sum():5.1f}%  ({c / frames:8.0f} per frame)")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "f64", frames=int(sys.argv[2]) if len(sys.argv) > 2 else 15,
         ix="--ix" in sys.argv, E=int(os.environ.get("ENVS", "4096")))
