"""Debug: run ONE fused simulate launch of a variant library (tools/_ab/lib_<name>.so) on an
intersection batch reset by the default library; its device printf reports any mismatch."""
import ctypes as C
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from topotrafficrl_amd import _lib  # noqa: E402
from topotrafficrl_amd.intersection import VecIntersectionEnv  # noqa: E402


def main(name, frames):
    lib = _lib.load(os.path.join(ROOT, "tools", "_ab", f"lib_{name}.so"))
    lib.ttrl_simulate.argtypes = [C.c_void_p] * 4 + [C.c_int32, C.c_double, C.c_void_p]
    for dtype in ("f64", "f32"):
        env = VecIntersectionEnv({"num_envs": 256, "device": "cuda:0", "dtype": dtype, "auto_reset": False})
        env.reset(seed=3)
        acts = env.action_type._codes(torch.ones(256, dtype=torch.int64, device="cuda:0"))
        torch.cuda.synchronize()
        print(dtype, "launch", frames, "frames", flush=True)
        rc = lib.ttrl_simulate(C.byref(env.state.struct()), C.byref(env.network.table), C.byref(env.params),
                               acts.data_ptr(), frames, 1 / 15, torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        st = env.state.to_numpy()
        print(dtype, "rc", rc, "finite x", bool(np.isfinite(st["x"]).all()), flush=True)


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]))
