"""Batched AbstractEnv.to_finite_mdp (abstract.py:416-417 -> ttrl_env/envs/common/finite_mdp.py).

The reference builds, for its single env, the time-to-collision MDP of the ego: the grid of
``compute_ttc_grid`` (SPEED x LANES x TIME), a deterministic transition over its cells for the 5
meta-actions (``transition_model`` / ``clip_position``), a state reward mixing collision, right
lane and speed terms plus a per-action lane-change reward, and terminal cells (collisions and the
end of the horizon), then wraps them in the third-party ``finite_mdp.mdp.DeterministicMDP``.

Here every env of the batch at once: the grids come from the TTC HIP kernel (raw mode), the
tables are device tensors, and ``value_iteration`` solves all the MDPs in lockstep.  The transition
depends only on the grid shape and is shared by every env.
"""
from __future__ import annotations

from dataclasses import dataclass
from functools import lru_cache

import numpy as np
import torch

from . import _abi
from .observation import time_to_collision

ACTION_REWARD_KEYS = ("lane_change_reward", None, "lane_change_reward", None, None)  # finite_mdp.py:72-78


@lru_cache(maxsize=16)
def _transition_np(V: int, L: int, T: int, n_actions: int) -> np.ndarray:
    """transition_model (finite_mdp.py:170-192) over np.fromfunction, as [V*L*T, n_actions]."""
    h, i, j, a = np.indices((V, L, T, n_actions))

    def clip_position(h, i, j):  # finite_mdp.py:195-208
        return np.ravel_multi_index((np.clip(h, 0, V - 1), np.clip(i, 0, L - 1), np.clip(j, 0, T - 1)), (V, L, T))

    nxt = clip_position(h, i, j + 1)
    left, right = a == 0, a == 2
    faster, slower = (a == 3) & (j == 0), (a == 4) & (j == 0)
    nxt[left] = clip_position(h[left], i[left] - 1, j[left] + 1)
    nxt[right] = clip_position(h[right], i[right] + 1, j[right] + 1)
    nxt[faster] = clip_position(h[faster] + 1, i[faster], j[faster] + 1)
    nxt[slower] = clip_position(h[slower] - 1, i[slower], j[slower] + 1)
    return nxt.reshape(V * L * T, n_actions)


@dataclass
class BatchedFiniteMDP:
    """finite_mdp.mdp.DeterministicMDP fields, batched: transition [S, A] (shared), reward
    [E, S, A], terminal [E, S], state [E]; grid [E, V, L, T] and original_shape (V, L, T)."""
    transition: torch.Tensor
    reward: torch.Tensor
    terminal: torch.Tensor
    state: torch.Tensor
    grid: torch.Tensor
    original_shape: tuple

    def value_iteration(self, gamma: float = 1.0, iterations: int = 100) -> torch.Tensor:
        """Q-values [E, S, A]: Q = R + gamma * (1 - terminal[s']) * max_a' Q(s', a'), every env in
        lockstep.  A convenience for planners on top of the tables; the reference delegates
        solving to the absent finite-mdp package, so this solver itself is not a restatement."""
        nxt = self.transition.unsqueeze(0).expand(self.reward.shape[0], -1, -1)
        cont = (~self.terminal).to(self.reward.dtype)
        q = torch.zeros_like(self.reward)
        for _ in range(iterations):
            v = q.max(dim=2).values * cont                      # [E, S]
            q = self.reward + gamma * torch.gather(v, 1, nxt.reshape(v.shape[0], -1)).reshape(q.shape)
        return q


def finite_mdp(env, time_quantization: float = 1.0, horizon: float = 10.0) -> BatchedFiniteMDP:
    """finite_mdp(env, time_quantization, horizon) (finite_mdp.py:17-101) for every env of ``env``."""
    road, st = env.road, env.road.state
    cfg = _abi.ttc_cfg(horizon=horizon, policy_frequency=1.0 / time_quantization, raw=True)
    grid = time_to_collision(st, road.network, road.params, cfg).to(torch.float64)  # [E, V, L, T]
    E, V, L, T = grid.shape
    n_actions = env.action_space.n
    trans = torch.from_numpy(_transition_np(V, L, T, n_actions)).to(grid.device)
    c = env.config
    lanes = torch.arange(L, dtype=torch.float64, device=grid.device) / max(L - 1, 1)
    speeds = torch.arange(V, dtype=torch.float64, device=grid.device) / max(V - 1, 1)
    state_reward = (c["collision_reward"] * grid + c["right_lane_reward"] * lanes[None, None, :, None]
                    + c["high_speed_reward"] * speeds[None, :, None, None])       # [E, V, L, T]
    action_reward = torch.tensor([c[k] if k else 0.0 for k in ACTION_REWARD_KEYS], dtype=torch.float64,
                                 device=grid.device)
    if n_actions != len(action_reward):
        raise ValueError("finite_mdp's action reward covers the 5 DiscreteMetaAction actions (finite_mdp.py:72-78)")
    reward = state_reward.reshape(E, -1, 1) + action_reward[None, None, :]
    end = torch.zeros((V, L, T), dtype=torch.bool, device=grid.device)
    end[:, :, T - 1] = True
    terminal = ((grid == 1) | end[None]).reshape(E, -1)
    # grid_state = (speed_index, lane_index[2], 0) (finite_mdp.py:51-52); one road: lane id = slot lane
    state = (st.ego("speed_index").long() * L + st.ego("lane").long()) * T
    return BatchedFiniteMDP(trans, reward, terminal, state, grid, (V, L, T))
