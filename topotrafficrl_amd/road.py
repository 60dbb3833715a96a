"""Road network and the batched per-frame drop-in for ``Road.act`` / ``Road.step``.

Reference: ttrl_env/road/road.py — RoadNetwork (:21-389), Road (:392-516).
``BatchedRoad.act()`` / ``.step(dt)`` have the reference's meaning for every env of
the batch at once; ``simulate()`` is the fused ``AbstractEnv._simulate`` frame loop.
All work is enqueued on the current HIP stream of the state's device.
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch

from . import _abi, _lib
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


def _stream(device: torch.device) -> int:
    if device.type != "cuda":
        raise RuntimeError("BatchedRoad runs on a HIP device only (no CPU fallback)")
    return torch.cuda.current_stream(device).cuda_stream


class BatchedRoad:
    """Batched ``Road``: the vehicles of every env as one ``BatchState``."""

    def __init__(self, network: RoadNetwork, state: BatchState, params: _abi.Params | None = None):
        self.network = network
        self.state = state
        self.params = params if params is not None else _abi.default_params()
        _lib.load()

    def _args(self):
        return C.byref(self.state.struct()), C.byref(self.network.table), C.byref(self.params)

    def act(self) -> None:
        """Road.act (road.py:461-464): every vehicle decides, in list order."""
        s, r, p = self._args()
        _lib.call("ttrl_road_act", s, r, p, _stream(self.state.device))

    def step(self, dt: float) -> None:
        """Road.step (road.py:466-478): kinematics, lane update, collisions."""
        s, r, p = self._args()
        _lib.call("ttrl_road_step", s, r, p, float(dt), _stream(self.state.device))

    def meta_action(self, actions: torch.Tensor) -> None:
        """DiscreteMetaAction.act for the ego of every env (action.py:259-260)."""
        a = self._actions(actions)
        s, r, p = self._args()
        _lib.call("ttrl_meta_action", s, r, p, a.data_ptr(), _stream(self.state.device))

    def simulate(self, actions: torch.Tensor | None, frames: int = 15, dt: float = 1 / 15, observe=None,
                 tail=None) -> None:
        """Fused AbstractEnv._simulate (abstract.py:252-282) for `frames` frames.  With ``observe`` =
        (KinCfg, out [E, V, F] float32, ids [E, V-1] int32) and / or ``tail`` = (RewardCfg, time [E] f64,
        time_inc, reward, terminated, truncated, components, ego_speed, ego_crashed) the same launch
        also writes the Kinematics observation and the step tail of the final state (ttrl_env_step)."""
        a = None if actions is None else self._actions(actions)
        s, r, p = self._args()
        ap = None if a is None else a.data_ptr()
        if observe is None and tail is None:
            _lib.call("ttrl_simulate", s, r, p, ap, int(frames), float(dt), _stream(self.state.device))
            return
        oc, oo, oi = (None, None, None) if observe is None else (C.byref(observe[0]), observe[1].data_ptr(),
                                                                   observe[2].data_ptr())
        if tail is None:
            rc, tail_ptrs = None, [None, 0.0] + [None] * 7
        else:
            rc = C.byref(tail[0])
            tail_ptrs = [tail[1].data_ptr(), float(tail[2])] + [t.data_ptr() for t in tail[3:]]
        _lib.call("ttrl_env_step", s, r, p, ap, int(frames), float(dt), oc, oo, oi, rc, *tail_ptrs,
                  _stream(self.state.device))

    def neighbour_vehicles(self, query_lane: torch.Tensor | None = None):
        """Road.neighbour_vehicles (road.py:480-513) for every vehicle: (front, rear) slot ids, -1 = None."""
        st = self.state
        front = torch.empty((st.n_envs, st.n_veh), dtype=torch.int32, device=st.device)
        rear = torch.empty_like(front)
        q = None
        if query_lane is not None:
            q = query_lane.to(device=st.device, dtype=torch.int32).contiguous()
            if q.shape != front.shape:
                raise ValueError("query_lane must be [n_envs, n_veh]")
        _lib.call("ttrl_neighbours", C.byref(st.struct()), C.byref(self.network.table),
                  None if q is None else q.data_ptr(), front.data_ptr(), rear.data_ptr(), _stream(st.device))
        return front, rear

    def _actions(self, actions) -> torch.Tensor:
        a = torch.as_tensor(actions).to(device=self.state.device, dtype=torch.int32).reshape(-1).contiguous()
        if a.numel() != self.state.n_envs:
            raise ValueError(f"expected {self.state.n_envs} actions, got {a.numel()}")
        return a
