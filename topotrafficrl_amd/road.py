"""Road network and the batched per-frame drop-in for ``Road.act`` / ``Road.step``.

Reference: ttrl_env/road/road.py — RoadNetwork (:21-389), Road (:392-516).
``BatchedRoad.act()`` / ``.step(dt)`` have the reference's meaning for every env of
the batch at once; ``simulate()`` is the fused ``AbstractEnv._simulate`` frame loop.
All work is enqueued on the current HIP stream of the state's device.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _abi, ops
from .state import BatchState


class RoadNetwork:
    """A single road "0" -> "1" with parallel lanes: StraightLanes (road.py:291-321) or the
    curved SineLane / CircularLane classes (lane.py:235-350)."""

    def __init__(self, table: _abi.LaneTable):
        self.table = table

    @classmethod
    def sine_road_network(cls, lanes: int = 4, length: float = 10000, amplitude: float = 5.0,
                          pulsation: float = 2 * 3.141592653589793 / 200, phase: float = 0.0,
                          speed_limit: float = 30) -> "RoadNetwork":
        return cls(_abi.sine_lane_table(lanes, length, amplitude, pulsation, phase, speed_limit))

    @classmethod
    def circular_road_network(cls, lanes: int = 3, center=(0.0, 0.0), radius: float = 200.0,
                              start_phase: float = -3.141592653589793 / 2, end_phase: float = 3.141592653589793 / 2,
                              clockwise: bool = True, speed_limit: float = 30) -> "RoadNetwork":
        return cls(_abi.circular_lane_table(lanes, center, radius, start_phase, end_phase, clockwise, speed_limit))

    @classmethod
    def straight_road_network(cls, lanes: int = 4, start: float = 0, length: float = 10000, angle: float = 0,
                              speed_limit: float = 30, nodes_str=None, net=None) -> "RoadNetwork":
        if net is not None:
            raise NotImplementedError("multi-segment networks are SURVEY.md §8(f) 'next'")
        return cls(_abi.straight_lane_table(lanes, start, length, angle, speed_limit))

    @property
    def lanes_count(self) -> int:
        return self.table.n_lanes

    def all_side_lanes(self, lane_index):
        """road.py:190-198"""
        return [("0", "1", i) for i in range(self.table.n_lanes)]

    def side_lanes(self, lane_index):
        """road.py:200-211"""
        _from, _to, _id = lane_index
        out = []
        if _id > 0:
            out.append((_from, _to, _id - 1))
        if _id < self.table.n_lanes - 1:
            out.append((_from, _to, _id + 1))
        return out

    def lanes_array(self) -> np.ndarray:
        t = self.table
        return np.array([[t.start_x[i], t.start_y[i], t.start_x[i] + t.length[i] * t.dir_x[i],
                          t.start_y[i] + t.length[i] * t.dir_y[i], t.width[i], t.speed_limit[i]]
                         for i in range(t.n_lanes)])


def _check_device(device: torch.device) -> None:
    if device.type != "cuda":
        raise RuntimeError("BatchedRoad runs on a HIP device only (no CPU fallback)")


class BatchedRoad:
    """Batched ``Road``: the vehicles of every env as one ``BatchState``.  Every method is one
    ``torch.ops.ttrl`` operator (csrc/ttrl_torch_ops.cpp) on the current HIP stream."""

    def __init__(self, network: RoadNetwork, state: BatchState, params: _abi.Params | None = None):
        self.network = network
        self.state = state
        self.params = params if params is not None else _abi.default_params()

    def _args(self):
        _check_device(self.state.device)
        return self.state.tensors(), ops.st(self.network.table), ops.st(self.params)

    def act(self) -> None:
        """Road.act (road.py:461-464): every vehicle decides, in list order."""
        ops.T.road_act_(*self._args())

    def step(self, dt: float) -> None:
        """Road.step (road.py:466-478): kinematics, lane update, collisions."""
        ops.T.road_step_(*self._args(), float(dt))

    def meta_action(self, actions: torch.Tensor) -> None:
        """DiscreteMetaAction.act for the ego of every env (action.py:259-260)."""
        ops.T.meta_action_(*self._args(), self._actions(actions))

    def simulate(self, actions: torch.Tensor | None, frames: int = 15, dt: float = 1 / 15) -> None:
        """Fused AbstractEnv._simulate (abstract.py:252-282) for `frames` frames."""
        a = None if actions is None else self._actions(actions)
        ops.T.simulate_(*self._args(), a, int(frames), float(dt))

    def env_step(self, actions: torch.Tensor | None, frames: int, dt: float, kin_cfg: _abi.KinCfg | None,
                 reward_cfg: _abi.RewardCfg, time: torch.Tensor, time_inc: float, order: torch.Tensor | None = None,
                 action_lut: list[int] | None = None, grid_cfg: _abi.GridCfg | None = None):
        """AbstractEnv.step (abstract.py:224-250) in one launch (ttrl_env_step): the fused frames, the
        Kinematics observation of the final state (``kin_cfg``; else obs / ids are empty; ``grid_cfg``
        instead: obs is the OccupancyGrid [E, F, W, H] of ttrl_env_step_grid, ids empty) and the step
        tail (time += time_inc, reward, terminated, truncated, components, the info's ego speed /
        crashed).  Returns those 8 tensors.  ``order``: an optional dispatch order of the envs (int32
        permutation, ix_step_tail_ writes it; road networks only, results unchanged).  It must be a
        permutation: an env named twice would be written by two workgroups (not checked on the
        device: that would need a host sync); a negative entry is an idle slot.
        ``action_lut``: ``actions`` are action indices and this maps them to meta-action codes inside
        the launch (DiscreteMetaAction._indices)."""
        a = None if actions is None else self._actions(actions)
        kc = None if kin_cfg is None else ops.kin_cfg_tensor(kin_cfg)
        gc = None if grid_cfg is None else ops.st(grid_cfg)
        return ops.T.env_step_(*self._args(), a, int(frames), float(dt), kc, ops.st(reward_cfg), time,
                               float(time_inc), order, action_lut, gc)

    def ix_env_step(self, cfg: _abi.IxCfg, actions: torch.Tensor | None, frames: int, dt: float,
                    kin_cfg: _abi.KinCfg, reward_cfg: _abi.RewardCfg, time: torch.Tensor, time_inc: float,
                    spare: BatchState, spare_parity: torch.Tensor, entropy: torch.Tensor,
                    spare_entropy: torch.Tensor, order: torch.Tensor | None = None,
                    action_lut: list[int] | None = None, live_count: torch.Tensor | None = None):
        """IntersectionEnv.step (intersection_env.py:135-139 over abstract.py:224-250) with the
        auto-reset from spare scenes, in one launch (ttrl_ix_env_step): env_step's launch, then for
        every env that goes on its _clear_vehicles / _spawn_vehicle (:320-362), and for every finished
        env its spare scene and first observation.  Returns env_step's 8 tensors, then done,
        spare_mask, obs_next, ids_next (ix_step_tail_'s outputs; spare / spare_parity / entropy /
        spare_entropy / order / live_count as ix_step_tail_ takes them)."""
        a = None if actions is None else self._actions(actions)
        return ops.T.ix_env_step_(*self._args(), ops.st(cfg), a, int(frames), float(dt), ops.kin_cfg_tensor(kin_cfg),
                                  ops.st(reward_cfg), time, float(time_inc), spare.tensors(), spare_parity, entropy,
                                  spare_entropy, order, action_lut, live_count)

    def neighbour_vehicles(self, query_lane: torch.Tensor | None = None):
        """Road.neighbour_vehicles (road.py:480-513) for every vehicle: (front, rear) slot ids, -1 = None."""
        st = self.state
        _check_device(st.device)
        if query_lane is not None and tuple(query_lane.shape) != (st.n_envs, st.n_veh):
            raise ValueError("query_lane must be [n_envs, n_veh]")
        return ops.T.neighbours(st.tensors(), ops.st(self.network.table), query_lane)

    def _actions(self, actions) -> torch.Tensor:
        a = torch.as_tensor(actions)
        if a.device != self.state.device or a.dtype != torch.int32:
            a = a.to(device=self.state.device, dtype=torch.int32)
        a = a.reshape(-1)
        if a.numel() != self.state.n_envs:
            raise ValueError(f"expected {self.state.n_envs} actions, got {a.numel()}")
        return a.contiguous()
