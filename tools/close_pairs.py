"""Close vehicle pairs per env on the bench's highway scenes (the collision queue holds
every pair within the exact norm threshold before the SAT proofs, so an env with more than NS such
pairs takes the per-vehicle sweep).  Oracle scenes from seeds, random meta-actions, the pairs i < j
with |p_j - p_i| <= diag + v_i dt (objects.py:123-133) at each step's first frame.

  python tools/close_pairs.py [envs] [steps]
"""
import sys

import numpy as np

sys.path.insert(0, ".")
from oracle.oracle import HostState, Oracle  # noqa: E402
from topotrafficrl_amd import _abi  # noqa: E402


def main(E: int = 512, steps: int = 8) -> None:
    diag = np.sqrt(5 ** 2 + 2 ** 2)
    for N in (32, 64, 128):
        lanes, P = _abi.straight_lane_table(4), _abi.default_params()
        o = Oracle(lanes, P)
        h = HostState(E, N)
        o.reset_highway(h, _abi.reset_cfg(N, lanes), list(range(E)))
        rng = np.random.default_rng(0)
        worst = 0
        for step in range(steps):
            x, y, v, kind = h["x"], h["y"], h["speed"], h["kind"]
            cnts = []
            for e in range(E):
                n = int((kind[e] > 0).sum())
                dx = x[e, None, :n] - x[e, :n, None]
                dy = y[e, None, :n] - y[e, :n, None]
                m = (np.sqrt(dx * dx + dy * dy) <= diag + v[e, :n, None] / 15) & np.triu(np.ones((n, n), bool), 1)
                cnts.append(int(m.sum()))
            cnts = np.array(cnts)
            worst = max(worst, int(cnts.max()))
            print(f"N={N} step {step}: close pairs per env mean {cnts.mean():.2f} p99 {np.percentile(cnts, 99):.0f} "
                  f"max {cnts.max()}; envs over NS: {(cnts > N).mean() * 100:.2f}%")
            o.simulate(h, rng.integers(0, 5, size=E).astype(np.int32), 15, 1 / 15)
        print(f"N={N}: worst {worst} close pairs in an env over {steps} steps x {E} envs (queue capacity {N})")


if __name__ == "__main__":
    main(*(int(a) for a in sys.argv[1:]))
