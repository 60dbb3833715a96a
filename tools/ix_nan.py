"""Debug: step an f32 / f64 intersection batch and report the first non-finite state field."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from topotrafficrl_amd import _lib  # noqa: E402
from topotrafficrl_amd.intersection import VecIntersectionEnv  # noqa: E402


STEP_LIB = None


def main():
    for dtype in ("f32", "f64"):
        env = VecIntersectionEnv({"num_envs": 256, "device": "cuda:0", "dtype": dtype})
        obs, _ = env.reset(seed=3)
        if STEP_LIB is not None:  # reset with the default library, step with a variant
            _lib._lib = STEP_LIB
        print(dtype, "reset obs finite", bool(torch.isfinite(obs).all()))
        for t in range(int(os.environ.get("STEPS", "13"))):
            st = env.state.to_numpy()
            bad = {k: int((~np.isfinite(v)).sum()) for k, v in st.items() if v.dtype.kind == "f"}
            bad = {k: v for k, v in bad.items() if v}
            if bad:
                e = np.flatnonzero((~np.isfinite(st["x"])).any(1))
                print(f"  before step {t}: non-finite {bad}; envs {e[:8].tolist()}")
                if len(e):
                    print("   kind", st["kind"][e[0]].tolist(), "lane", st["lane"][e[0]].tolist())
                break
            obs, rew, term, trunc, info = env.step(torch.ones(256, dtype=torch.int64, device="cuda:0"))
            torch.cuda.synchronize()
            print("  step", t, flush=True)
            if not torch.isfinite(obs).all():
                rows = torch.nonzero(~torch.isfinite(obs).reshape(256, -1).all(1)).flatten().tolist()
                print(f"  step {t}: obs non-finite in envs {rows[:8]}")
        print(dtype, "done")


if __name__ == "__main__":
    if len(sys.argv) > 1:  # a variant build (tools/variants.py)
        lib = _lib.load(os.path.join(ROOT, "tools", "_ab", f"lib_{sys.argv[1]}.so"))
        if len(sys.argv) > 2 and sys.argv[2] == "step-only":
            _lib._lib = _lib.load(os.path.join(ROOT, "tools", "_ab", "lib_head.so"))
            STEP_LIB = lib
        else:
            _lib._lib = lib
        print("variant", sys.argv[1:], flush=True)
    main()
