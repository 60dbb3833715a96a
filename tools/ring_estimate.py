"""How many CircularLane projections a wave (2 intersection envs) needs per frame when a lane's
atan2 is skipped for vehicles outside its ring band (|r| > w/2 + 1 and |r| >= best distance):
an oracle replay of mid-episode intersection scenes (CPU only)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from oracle.oracle import HostState, Oracle  # noqa: E402
from test_ix_oracle import P_IX  # noqa: E402
from topotrafficrl_amd.intersection import VecIntersectionEnv, intersection_network, ix_cfg  # noqa: E402


def main(E=64, steps=12, margin=0.6):
    net = intersection_network()
    T = net.table
    o = Oracle(T, P_IX)
    cfg = ix_cfg(net, VecIntersectionEnv.default_config(), P_IX)
    h = HostState(E, 32)
    o.ix_reset(h, cfg, list(range(E)))
    nl = T.n_lanes
    circ = [l for l in range(nl) if T.type[l] == 2]
    print("lanes", nl, "circular", circ)
    hist = []
    rng = np.random.default_rng(0)
    for _ in range(steps):
        for _ in range(15):
            o.simulate(h, rng.integers(0, 3, E).astype(np.int32), 1, 1 / 15)
            kind, x, y = h["kind"], h["x"], h["y"]
            for w in range(E // 2):
                cnt = 0
                for l in circ:
                    need = False
                    for e in (2 * w, 2 * w + 1):
                        p = kind[e] > 0
                        rr = np.abs(T.radius[l] - np.hypot(x[e][p] - T.center_x[l], y[e][p] - T.center_y[l]))
                        need |= bool(np.any(rr <= T.width[l] / 2 + 1 + margin))
                    cnt += need
                hist.append(cnt)
        o.ix_clear_spawn(h, cfg)
    print("circular lanes needed per wave-frame: mean", np.mean(hist), "of", len(circ), np.bincount(hist).tolist())


if __name__ == "__main__":
    main()
