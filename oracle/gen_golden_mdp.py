"""Golden vectors of AbstractEnv.to_finite_mdp — TEST INFRASTRUCTURE, build container only.

Calls the reference's own ``finite_mdp(env, time_quantization, horizon)`` (finite_mdp.py:17-101:
compute_ttc_grid, transition_model / clip_position through np.fromfunction, the state reward,
action reward and terminal states) on highway scenes built from the unmodified reference sim core
(gen_golden.make_highway).  Its last step hands the tables to ``finite_mdp.mdp.DeterministicMDP``
from the third-party ``finite-mdp`` package, which is absent here: a recorder registered under
that module name keeps the arguments (transition, reward, terminal, state) — the reference's
outputs — and nothing else.  Recorded per observation point: the vehicle state and those tables.

Usage:  PYTHONDONTWRITEBYTECODE=1 python oracle/gen_golden_mdp.py
"""
from __future__ import annotations

import os
import sys
import types

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import gen_golden as G  # noqa: E402  (imports the reference sim core)

R = G.R


class _Recorder:  # stands in for finite_mdp.mdp.DeterministicMDP: records its arguments
    def __init__(self, transition, reward, terminal, state=None):
        self.transition, self.reward, self.terminal, self.state = transition, reward, terminal, state


_mod = types.ModuleType("finite_mdp.mdp")
_mod.DeterministicMDP = _Recorder
sys.modules.setdefault("finite_mdp", types.ModuleType("finite_mdp"))
sys.modules["finite_mdp.mdp"] = _mod

CONFIG = {"collision_reward": -1.0, "right_lane_reward": 0.1, "high_speed_reward": 0.4, "lane_change_reward": -0.05,
          "policy_frequency": 1}


def to_finite_mdp(road):
    ego = road.vehicles[0]
    env = types.SimpleNamespace(vehicle=ego, road=road, config=CONFIG, action_space=types.SimpleNamespace(n=5))
    return R.finite_mdp.finite_mdp(env, time_quantization=1 / CONFIG["policy_frequency"], horizon=10.0)


def main():
    for n in (8, 32, 64):
        for seed in (0, 1):
            road = G.make_highway(n, seed)
            rng = np.random.default_rng(4242 + seed)
            snaps, trans, rew, term, state, grids = [], [], [], [], [], []
            for p in range(4):
                mdp = to_finite_mdp(road)
                env = types.SimpleNamespace(vehicle=road.vehicles[0], road=road, config=CONFIG)
                grids.append(R.finite_mdp.compute_ttc_grid(env, time_quantization=1.0, horizon=10.0))
                snaps.append(G.snapshot(road))
                trans.append(mdp.transition); rew.append(mdp.reward); term.append(mdp.terminal)
                state.append(mdp.state)
                a = int(rng.integers(0, 5))
                for f in range(15):
                    if f == 0:
                        road.vehicles[0].act(G.ACTIONS_ALL[a])
                    road.act()
                    road.step(1 / 15)
            d = {k: np.stack([s[k] for s in snaps]) for k in G.FIELDS_F + G.FIELDS_I}
            d["transition"] = np.stack(trans).astype(np.int64)
            d["reward"] = np.stack(rew)
            d["terminal"] = np.stack(term)
            d["state"] = np.array(state, dtype=np.int64)
            d["grid"] = np.stack(grids)
            d["config"] = np.array([CONFIG[k] for k in ("collision_reward", "right_lane_reward",
                                                        "high_speed_reward", "lane_change_reward")])
            d["lane_table"] = np.array([[l.start[0], l.start[1], l.end[0], l.end[1], l.width, l.speed_limit]
                                        for l in road.network.lanes_list()])
            name = f"mdp_n{n}_s{seed}"
            print(name, "states", d["state"].tolist(), "collision cells", int((d["terminal"]).sum()))
            np.savez_compressed(os.path.join(G.OUT, name + ".npz"), **d)


if __name__ == "__main__":
    main()
