"""Batched vehicle state: struct-of-arrays device tensors laid out [n_envs, n_veh].

One row per env, one column per slot of the reference's ``road.vehicles`` list
(the ego / ``env.vehicle`` is the env's first MDP slot: slot 0 on the highway).
The per-vehicle attributes of the reference objects map to fields as follows:

    position -> x, y            heading -> heading          speed -> speed
    target_speed, timer, DELTA -> target_speed, timer, delta
    action{steering, acceleration} -> steer, acc
    impact (None | ndarray)     -> has_impact, impact_x, impact_y
    lane_index[2], target_lane_index[2] -> lane, target_lane
    MDPVehicle.speed_index      -> speed_index
    class                       -> kind (ABSENT / MDP / IDM)
    crashed, enable_lane_change -> crashed, lane_change
    route (list of lane indexes | None) -> route_road, route_lane [.., ROUTE_MAX], route_n
    RegulatedRoad is_yielding / steps   -> yielding, reg_steps [n_envs]
    AbstractEnv.np_random (numpy Generator(PCG64)) -> rng [n_envs, 5] (uint64 words as int64)
"""
from __future__ import annotations

import numpy as np
import torch

from . import _abi

_TORCH = {"f32": torch.float32, "f64": torch.float64}


class BatchState:
    def __init__(self, n_envs: int, n_veh: int, device="cuda", dtype: str = "f64"):
        if dtype not in _TORCH:
            raise ValueError("dtype must be 'f32' or 'f64'")
        if not 1 <= n_veh <= 256:
            raise ValueError("n_veh must be in [1, 256]")
        self.n_envs, self.n_veh, self.device, self.dtype = int(n_envs), int(n_veh), torch.device(device), dtype
        tdt = _TORCH[dtype]
        shape = (self.n_envs, self.n_veh)
        self.t = {}
        for f in _abi.REAL_FIELDS:
            self.t[f] = torch.zeros(shape, dtype=tdt, device=self.device)
        for f in _abi.I32_FIELDS:
            self.t[f] = torch.zeros(shape, dtype=torch.int32, device=self.device)
        for f in _abi.U8_FIELDS:
            self.t[f] = torch.zeros(shape, dtype=torch.uint8, device=self.device)
        self.t["speed_index"].fill_(-1)
        self.t["delta"].fill_(4.0)
        for f in _abi.ROUTE_FIELDS:  # ControlledVehicle.route, RegulatedRoad state
            self.t[f] = torch.full(shape + (_abi.ROUTE_MAX,), -1, dtype=torch.int8, device=self.device)
        self.t["route_n"] = torch.full(shape, -1, dtype=torch.int8, device=self.device)
        self.t["yielding"] = torch.zeros(shape, dtype=torch.uint8, device=self.device)
        self.t["reg_steps"] = torch.zeros(self.n_envs, dtype=torch.int32, device=self.device)
        # AbstractEnv.np_random of each env (numpy Generator(PCG64) words, see _abi.RNG_WORDS)
        self.t["rng"] = torch.zeros((self.n_envs, _abi.RNG_WORDS), dtype=torch.int64, device=self.device)
        self._struct = None
        self._tensors = None

    def __getitem__(self, k: str) -> torch.Tensor:
        return self.t[k]

    @property
    def abi_dtype(self) -> int:
        return _abi.F64 if self.dtype == "f64" else _abi.F32

    def struct(self) -> _abi.State:
        if self._struct is None:
            self._struct = _abi.state_struct({k: v.data_ptr() for k, v in self.t.items()},
                                             self.n_envs, self.n_veh, self.abi_dtype)
        return self._struct

    def tensors(self) -> list:
        """The state tensors in _abi.ALL_FIELDS order (the ``state`` argument of torch.ops.ttrl)."""
        if self._tensors is None:
            self._tensors = [self.t[f] for f in _abi.ALL_FIELDS]
        return self._tensors

    def ego_index(self) -> torch.Tensor:
        """[E] slot of each env's controlled vehicle: its first MDP slot (AbstractEnv.vehicle)."""
        return (self.t["kind"] == _abi.MDP).to(torch.int8).argmax(dim=1)

    def ego(self, field: str) -> torch.Tensor:
        """[E] value of ``field`` for each env's controlled vehicle."""
        return self.t[field].gather(1, self.ego_index().unsqueeze(1)).squeeze(1)

    def nbytes(self) -> int:
        return sum(v.numel() * v.element_size() for v in self.t.values())

    def load_numpy(self, arrays: dict) -> "BatchState":
        """Copy host arrays (e.g. oracle.HostState.a) into the device tensors."""
        for k, v in self.t.items():
            a = np.ascontiguousarray(arrays[k])
            if a.dtype == np.uint64:
                a = a.view(np.int64)
            v.copy_(torch.as_tensor(a).to(v.dtype))
        return self

    def to_numpy(self) -> dict:
        out = {k: v.cpu().numpy() for k, v in self.t.items()}
        out["rng"] = out["rng"].view(np.uint64)
        return out

    def clone(self) -> "BatchState":
        b = BatchState.__new__(BatchState)
        b.n_envs, b.n_veh, b.device, b.dtype = self.n_envs, self.n_veh, self.device, self.dtype
        b.t = {k: v.clone() for k, v in self.t.items()}
        b._struct = b._tensors = None
        return b

    def rows(self, start: int, n: int) -> "BatchState":
        """A view of envs [start, start + n) sharing this state's storage."""
        b = BatchState.__new__(BatchState)
        b.n_envs, b.n_veh, b.device, b.dtype = int(n), self.n_veh, self.device, self.dtype
        b.t = {k: v[start:start + n] for k, v in self.t.items()}
        b._struct = b._tensors = None
        return b

    def copy_(self, other: "BatchState") -> "BatchState":
        for k, v in self.t.items():
            v.copy_(other.t[k])
        return self

    def state_dict(self) -> dict:
        """Checkpoint of the env state (the reference checkpoints the agent only)."""
        return {k: v.detach().cpu() for k, v in self.t.items()}

    def load_state_dict(self, sd: dict) -> "BatchState":
        for k, v in self.t.items():
            v.copy_(sd[k].to(v.device, v.dtype))
        return self
