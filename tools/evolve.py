"""How the fused kernel time evolves over an episode (diagnostic)."""
import ctypes as C
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from topotrafficrl_amd import _lib  # noqa: E402
from topotrafficrl_amd.envs import VecHighwayEnv  # noqa: E402
from tools.ablate import VARIANTS  # noqa: E402


def main(dtype="f64", steps=40):
    dev = torch.device("cuda:0")
    env = VecHighwayEnv({"num_envs": 4096, "vehicles_count": 64, "device": "cuda:0", "dtype": dtype})
    env.reset(seed=12345)
    g = torch.Generator(device=dev).manual_seed(1000)
    # the ablation bits are compiled in only with -DTTRL_DIAG_ABLATE (tools/variants.py build)
    lib = _lib.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "_ab", "lib_ablate.so"))
    fn = lib.ttrl_diag_simulate
    fn.argtypes = [C.c_void_p] * 4 + [C.c_int32, C.c_double, C.c_int32, C.c_void_p]
    stream = torch.cuda.current_stream(dev).cuda_stream
    for t in range(steps):
        a = torch.randint(0, 5, (4096,), device=dev, generator=g)
        if t % 10 == 9:  # ablation snapshot of the current state
            base = env.state.clone()
            codes = env.action_type._codes(a)
            res = {}
            for name, ab in VARIANTS.items():
                env.state.copy_(base)
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                fn(C.byref(env.state.struct()), C.byref(env.network.table), C.byref(env.params), codes.data_ptr(),
                   15, 1 / 15, ab, stream)
                e.record()
                torch.cuda.synchronize()
                res[name] = s.elapsed_time(e)
            env.state.copy_(base)
            st = env.state.to_numpy()
            crashed = st["crashed"].mean()
            chg = (st["lane"] != st["target_lane"]).mean()
            print(f"step {t}: crashed frac {crashed:.3f} changing frac {chg:.3f} | " +
                  " ".join(f"{k}={v:.3f}" for k, v in res.items()), flush=True)
        env.step(a)


if __name__ == "__main__":
    main(*(sys.argv[1:2] or ["f64"]))
