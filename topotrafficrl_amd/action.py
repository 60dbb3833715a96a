"""Batched ego action type (drop-in for DiscreteMetaAction, ttrl_env/envs/common/action.py:199-298)."""
from __future__ import annotations

import numpy as np
import torch

from . import _abi
from .spaces import Discrete


class BatchedDiscreteMetaAction:
    ACTIONS_ALL = {0: "LANE_LEFT", 1: "IDLE", 2: "LANE_RIGHT", 3: "FASTER", 4: "SLOWER"}
    ACTIONS_LONGI = {0: "SLOWER", 1: "IDLE", 2: "FASTER"}
    ACTIONS_LAT = {0: "LANE_LEFT", 1: "IDLE", 2: "LANE_RIGHT"}
    _CODE = {"LANE_LEFT": _abi.LANE_LEFT, "IDLE": _abi.IDLE, "LANE_RIGHT": _abi.LANE_RIGHT,
             "FASTER": _abi.FASTER, "SLOWER": _abi.SLOWER}

    # Out-of-range action indices: the reference raises KeyError (self.actions[int(a)]).  CPU inputs
    # are always checked here.  Device-resident inputs are checked only when check_device_actions is
    # set (an asynchronous device assert, a few small launches per step); otherwise a device index
    # outside [0, n) is undefined (the kernel matches none of its meta-action branches: IDLE).
    check_device_actions = False

    def __init__(self, env, longitudinal: bool = True, lateral: bool = True, target_speeds=None, **kwargs):
        self.env = env
        self.longitudinal, self.lateral = longitudinal, lateral
        self.target_speeds = (np.array(target_speeds, dtype=np.float64) if target_speeds is not None
                              else np.linspace(20, 30, 3))
        self.actions = (self.ACTIONS_ALL if longitudinal and lateral else
                        self.ACTIONS_LONGI if longitudinal else self.ACTIONS_LAT if lateral else None)
        if self.actions is None:
            raise ValueError("At least longitudinal or lateral actions must be included")
        self.actions_indexes = {v: k for k, v in self.actions.items()}
        self._lut = None
        self._tab = None  # the index -> code table (_indices)

    def space(self) -> Discrete:
        return Discrete(len(self.actions))

    def _table(self) -> list[int]:
        """The meta-action code of each action index (ttrl_meta_action's codes)."""
        return [self._CODE[self.actions[i]] for i in range(len(self.actions))]

    def _indices(self, actions) -> tuple[torch.Tensor, list[int] | None]:
        """(int32 device action indices, the index -> code table, or None when index i is code i):
        ttrl_env_step maps the indices in its own launch, so the step needs no lookup launch."""
        if self._tab is None:
            self._tab = self._table()
        table = self._tab
        a = self._checked(actions)
        a = a.to(device=self.env.road.state.device, dtype=torch.int32).reshape(-1)
        return a, (None if table == list(range(len(table))) else table)

    def _checked(self, actions) -> torch.Tensor:
        a = torch.as_tensor(actions)
        if a.device.type == "cpu":
            an = a.numpy()
            if an.size and (an.min() < 0 or an.max() >= len(self.actions)):
                raise KeyError(f"action out of range [0, {len(self.actions)})")  # self.actions[int(a)] raises
        elif self.check_device_actions and a.numel():
            lo, hi = torch.aminmax(a)
            torch._assert_async((lo >= 0) & (hi < len(self.actions)), "action out of range")
        return a

    def _codes(self, actions) -> torch.Tensor:
        dev = self.env.road.state.device
        if self._lut is None or self._lut.device != dev:
            self._lut = torch.tensor(self._table(), dtype=torch.int32, device=dev)
            # the default action set maps index i to code i: no lookup launch then
            self._identity = bool(torch.equal(self._lut.cpu(), torch.arange(len(self.actions), dtype=torch.int32)))
        a = self._checked(actions)
        if self._identity:
            return a.to(device=dev, dtype=torch.int32).reshape(-1)
        a = a.to(dev).reshape(-1)
        return self._lut[a if a.dtype in (torch.int32, torch.int64) else a.long()]

    def act(self, actions) -> None:
        """DiscreteMetaAction.act (action.py:259-260) for every env's ego."""
        self.env.road.meta_action(self._codes(actions))

    def get_available_actions(self) -> torch.Tensor:
        """Batched get_available_actions (action.py:262-298) as an [E, n_actions] bool mask."""
        st, t = self.env.road.state, self.env.road.network.table
        lane = st.ego("lane").long()
        x, y = st.ego("x").double(), st.ego("y").double()
        E = st.n_envs
        mask = torch.zeros((E, len(self.actions)), dtype=torch.bool, device=st.device)
        mask[:, self.actions_indexes["IDLE"]] = True

        def reachable(lid):
            lid_c = lid.clamp(0, t.n_lanes - 1)
            sx = torch.tensor([t.start_x[i] for i in range(t.n_lanes)], device=st.device, dtype=torch.float64)[lid_c]
            sy = torch.tensor([t.start_y[i] for i in range(t.n_lanes)], device=st.device, dtype=torch.float64)[lid_c]
            dx = torch.tensor([t.dir_x[i] for i in range(t.n_lanes)], device=st.device, dtype=torch.float64)[lid_c]
            dy = torch.tensor([t.dir_y[i] for i in range(t.n_lanes)], device=st.device, dtype=torch.float64)[lid_c]
            s = (x - sx) * dx + (y - sy) * dy
            r = (x - sx) * (-dy) + (y - sy) * dx
            return (r.abs() <= 2 * t.width[0]) & (s >= 0) & (s < t.length[0] + 5.0) & (lid >= 0) & (lid < t.n_lanes)

        if self.lateral:
            if "LANE_LEFT" in self.actions_indexes:
                mask[:, self.actions_indexes["LANE_LEFT"]] = reachable(lane - 1)
            if "LANE_RIGHT" in self.actions_indexes:
                mask[:, self.actions_indexes["LANE_RIGHT"]] = reachable(lane + 1)
        if self.longitudinal:
            si = st.ego("speed_index")
            mask[:, self.actions_indexes["FASTER"]] = si < len(self.target_speeds) - 1
            mask[:, self.actions_indexes["SLOWER"]] = si > 0
        return mask


def action_factory(env, config: dict):
    """action.py:334-344 for the hot-path type."""
    t = config["type"]
    if t == "DiscreteMetaAction":
        return BatchedDiscreteMetaAction(env, **config)
    if t in ("ContinuousAction", "DiscreteAction", "MultiAgentAction"):
        raise NotImplementedError(f"action type {t!r} is out of the hot-path scope (SURVEY.md §2)")
    raise ValueError("Unknown action type")
