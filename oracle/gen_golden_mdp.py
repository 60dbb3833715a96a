"""Golden vectors of AbstractEnv.to_finite_mdp — TEST INFRASTRUCTURE, build container only.

The reference's ``finite_mdp(env, time_quantization, horizon)`` (finite_mdp.py:17-101) ends by
handing its tables to ``finite_mdp.mdp.DeterministicMDP`` from the third-party ``finite-mdp``
package, which is absent here (and stays absent: no stand-in is registered).  So the reference's
own functions compute the parts they own, on highway scenes built from the unmodified reference
sim core (gen_golden.make_highway):
  * the TTC grid: ``compute_ttc_grid`` (finite_mdp.py:104-167), called as is;
  * the transition: ``np.fromfunction(partial(transition_model, grid=grid), ...)`` with the
    reference's ``transition_model`` / ``clip_position`` (finite_mdp.py:170-208), called as is;
and the few assembly lines of finite_mdp.py:51-90 (state index, state / action rewards, terminal
cells) are restated line for line below.

Usage:  PYTHONDONTWRITEBYTECODE=1 python oracle/gen_golden_mdp.py
"""
from __future__ import annotations

import os
import sys
import types
from functools import partial

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import gen_golden as G  # noqa: E402  (imports the reference sim core)

R = G.R
FM = R.finite_mdp  # ttrl_env.envs.common.finite_mdp (imports only utils and Vehicle)

CONFIG = {"collision_reward": -1.0, "right_lane_reward": 0.1, "high_speed_reward": 0.4, "lane_change_reward": -0.05,
          "policy_frequency": 1}


def to_finite_mdp(road, time_quantization=1.0, horizon=10.0, n_actions=5):
    """finite_mdp.py:17-90 up to the DeterministicMDP call: (grid, transition, reward, terminal, state)."""
    ego = road.vehicles[0]
    env = types.SimpleNamespace(vehicle=ego, road=road, config=CONFIG, action_space=types.SimpleNamespace(n=n_actions))
    grid = FM.compute_ttc_grid(env, time_quantization, horizon)
    grid_state = (env.vehicle.speed_index, env.vehicle.lane_index[2], 0)
    state = np.ravel_multi_index(grid_state, grid.shape)
    transition_model_with_grid = partial(FM.transition_model, grid=grid)
    transition = np.fromfunction(transition_model_with_grid, grid.shape + (env.action_space.n,), dtype=int)
    transition = np.reshape(transition, (np.size(grid), env.action_space.n))
    v, l, t = grid.shape
    lanes = np.arange(l) / max(l - 1, 1)
    speeds = np.arange(v) / max(v - 1, 1)
    state_reward = (+env.config["collision_reward"] * grid
                    + env.config["right_lane_reward"] * np.tile(lanes[np.newaxis, :, np.newaxis], (v, 1, t))
                    + env.config["high_speed_reward"] * np.tile(speeds[:, np.newaxis, np.newaxis], (1, l, t)))
    state_reward = np.ravel(state_reward)
    action_reward = [env.config["lane_change_reward"], 0, env.config["lane_change_reward"], 0, 0]
    reward = np.fromfunction(np.vectorize(lambda s, a: state_reward[s] + action_reward[a]),
                             (np.size(state_reward), np.size(action_reward)), dtype=int)
    collision = grid == 1
    end_of_horizon = np.fromfunction(lambda h, i, j: j == grid.shape[2] - 1, grid.shape, dtype=int)
    terminal = np.ravel(collision | end_of_horizon)
    return grid, transition, reward, terminal, state


def main():
    for n in (8, 32, 64):
        for seed in (0, 1):
            road = G.make_highway(n, seed)
            rng = np.random.default_rng(4242 + seed)
            snaps, trans, rew, term, state, grids = [], [], [], [], [], []
            for p in range(4):
                grid, tr, rw, te, stt = to_finite_mdp(road)
                grids.append(grid)
                snaps.append(G.snapshot(road))
                trans.append(tr); rew.append(rw); term.append(te)
                state.append(stt)
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
