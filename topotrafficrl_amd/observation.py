"""Batched observation types (drop-ins for ttrl_env/envs/common/observation.py).

``BatchedKinematicObservation``     <- KinematicObservation      observation.py:154-275
``BatchedOccupancyGridObservation`` <- OccupancyGridObservation  observation.py:278-498
``BatchedTimeToCollisionObservation`` <- TimeToCollisionObservation observation.py:114-151
``BatchedLidarObservation``         <- LidarObservation          observation.py:677-768
``observation_factory``             <- observation_factory       observation.py:771-793

All accept the reference's config dict keys; ``observe()`` returns a float32 device
tensor [n_envs, ...] computed by the HIP kernels for every env's ego.
"""
from __future__ import annotations

import torch

from . import _abi, ops
from .spaces import Box


def _device_only(device):
    if device.type != "cuda":
        raise RuntimeError("observations run on a HIP device only (no CPU fallback)")


def kinematics(state, network, params, cfg: _abi.KinCfg, out=None, ids=None, mask=None):
    """KinematicObservation.observe for every env: ([E, V, F] float32, [E, V-1] int32 slot ids).
    ``mask`` (uint8/bool [E]): only those envs are observed (their np_random advanced); the other
    rows of ``out`` / ``ids`` are left as they were."""
    _device_only(state.device)
    if cfg.order_shuffled == 2 and state["rng"] is None:
        raise ValueError("np_random-shuffled observation needs the state's rng")
    args = (state.tensors(), ops.st(network.table), ops.st(params), ops.kin_cfg_tensor(cfg))
    if mask is None and out is None and ids is None:
        return ops.T.kinematics_obs(*args)
    E, V, F = state.n_envs, cfg.vehicles_count, cfg.n_features
    if out is None:
        out = torch.empty((E, V, F), dtype=torch.float32, device=state.device)
    if ids is None:
        ids = torch.empty((E, max(V - 1, 1)), dtype=torch.int32, device=state.device)
    if mask is None:
        mask = torch.ones(E, dtype=torch.uint8, device=state.device)
    elif mask.numel() != E:
        raise ValueError("mask must have one entry per env")
    elif mask.dtype == torch.bool:
        mask = mask.view(torch.uint8)
    ops.T.kinematics_obs_masked_(*args, mask, out, ids)
    return out, ids


def occupancy_grid(state, network, params, cfg: _abi.GridCfg):
    """OccupancyGridObservation.observe for every env: [E, F, W, H] float32."""
    _device_only(state.device)
    return ops.T.occupancy_grid(state.tensors(), ops.st(network.table), ops.st(params), ops.st(cfg))


def time_to_collision(state, network, params, cfg: _abi.TtcCfg):
    """TimeToCollisionObservation.observe for every env: [E, 3 speeds, 3 lanes, T] float32; with a
    raw cfg (obs_speeds = obs_lanes = 0) the whole compute_ttc_grid [E, speeds, lanes, T]."""
    _device_only(state.device)
    return ops.T.observe_ttc(state.tensors(), ops.st(network.table), ops.st(params), ops.st(cfg))


def lidar(state, network, params, cfg: _abi.LidarCfg):
    """LidarObservation.observe for every env: [E, cells, 2] float32 (distance, relative speed)."""
    _device_only(state.device)
    return ops.T.observe_lidar(state.tensors(), ops.st(network.table), ops.st(params), ops.st(cfg))


class BatchedObservationType:
    def __init__(self, env, **kwargs):
        self.env = env

    def space(self):
        raise NotImplementedError()

    def observe(self):
        raise NotImplementedError()


class BatchedKinematicObservation(BatchedObservationType):
    FEATURES = ["presence", "x", "y", "vx", "vy"]

    def __init__(self, env, features=None, vehicles_count=5, features_range=None, absolute=False,
                 order="sorted", normalize=True, clip=True, see_behind=False, observe_intentions=False,
                 include_obstacles=True, **kwargs):
        super().__init__(env)
        if observe_intentions and env.road.network.table.n_roads > 1:
            # with routes, cos_d / sin_d point to each vehicle's destination (kinematics.py:205-226);
            # the kernels emit the route-less value 0 (exact on a single road only)
            raise NotImplementedError("observe_intentions on a road network with routes")
        self.features = list(features or self.FEATURES)
        self.vehicles_count = vehicles_count
        self.features_range = features_range
        self.absolute, self.order, self.normalize, self.clip = absolute, order, normalize, clip
        self.see_behind, self.observe_intentions = see_behind, observe_intentions
        # the env's np_random drives the shuffle where the env keeps one on the device
        # (IntersectionEnv); elsewhere a counter-based Philox stream (seed, call count)
        self.cfg = _abi.kin_cfg(self.features, vehicles_count, features_range, absolute, order, normalize, clip,
                                see_behind, lanes_on_road=env.road.network.lanes_count,
                                shuffle_rng=getattr(env, "SHUFFLE_RNG", "philox"))
        self._out = self._ids = None
        self._calls = 0

    def space(self):
        return Box(low=-float("inf"), high=float("inf"), shape=(self.vehicles_count, len(self.features)),
                   dtype="float32")

    def observe(self, mask: torch.Tensor | None = None, out: torch.Tensor | None = None) -> torch.Tensor:
        """``mask``: re-observe only these envs into ``out`` (masked auto-reset)."""
        road = self.env.road
        if self.order == "shuffled" and self.cfg.order_shuffled == 1:
            self.cfg.shuffle_seed = int(self.env.shuffle_seed)
            self.cfg.shuffle_offset = self._calls
        self._calls += 1
        # a fresh output per call (the caching allocator makes it free): like the reference's
        # df.values.copy(), a returned observation is never overwritten by a later step
        # a masked call writes only the masked rows: the others keep their previous slot ids
        # (in place: the ids are this step's fresh tensor, and become the new episodes' for the masked envs)
        ids = self._ids if mask is not None and self._ids is not None else None
        self._out, self._ids = kinematics(road.state, road.network, road.params, self.cfg, out=out, ids=ids,
                                          mask=mask)
        return self._out

    def fused_cfg(self) -> _abi.KinCfg:
        """The cfg for an observation written by the env.step launch itself (BatchedRoad.env_step),
        with the same per-call bookkeeping as observe(); hand the outputs to fused_result()."""
        if self.order == "shuffled" and self.cfg.order_shuffled == 1:
            self.cfg.shuffle_seed = int(self.env.shuffle_seed)
            self.cfg.shuffle_offset = self._calls
        self._calls += 1
        return self.cfg

    def fused_result(self, out: torch.Tensor, ids: torch.Tensor) -> None:
        self._out, self._ids = out, ids

    @property
    def observed_ids(self) -> torch.Tensor:
        """Slot ids of rows 1.. of the last observation (sorted order), -1 for padding."""
        return self._ids


class BatchedOccupancyGridObservation(BatchedObservationType):
    FEATURES = ["presence", "vx", "vy", "on_road"]
    GRID_SIZE = [[-5.5 * 5, 5.5 * 5], [-5.5 * 5, 5.5 * 5]]
    GRID_STEP = [5, 5]

    def __init__(self, env, features=None, grid_size=None, grid_step=None, features_range=None, absolute=False,
                 align_to_vehicle_axes=False, clip=True, as_image=False, **kwargs):
        super().__init__(env)
        self.features = list(features if features is not None else self.FEATURES)
        self.cfg = _abi.grid_cfg(self.features, grid_size or self.GRID_SIZE, grid_step or self.GRID_STEP,
                                 features_range, absolute, align_to_vehicle_axes, clip, as_image)
        self._out = None

    def space(self):
        return Box(low=-float("inf"), high=float("inf"),
                   shape=(len(self.features), self.cfg.shape_x, self.cfg.shape_y), dtype="float32")

    def observe(self) -> torch.Tensor:
        road = self.env.road
        self._out = occupancy_grid(road.state, road.network, road.params, self.cfg)  # fresh per call
        return self._out


class BatchedTimeToCollisionObservation(BatchedObservationType):
    def __init__(self, env, horizon: int = 10, **kwargs):
        super().__init__(env)
        self.horizon = horizon
        self.cfg = _abi.ttc_cfg(horizon, env.config["policy_frequency"])

    def space(self):
        return Box(low=0, high=1, shape=(self.cfg.obs_speeds, self.cfg.obs_lanes, self.cfg.horizon_bins),
                   dtype="float32")

    def observe(self) -> torch.Tensor:
        road = self.env.road
        return time_to_collision(road.state, road.network, road.params, self.cfg)


class BatchedLidarObservation(BatchedObservationType):
    def __init__(self, env, cells: int = 16, maximum_range: float = 60, normalize: bool = True, **kwargs):
        super().__init__(env)
        self.cells, self.maximum_range, self.normalize = cells, maximum_range, normalize
        self.cfg = _abi.lidar_cfg(cells, maximum_range, normalize)

    def space(self):
        high = 1 if self.normalize else self.maximum_range
        return Box(low=-high, high=high, shape=(self.cells, 2), dtype="float32")

    def observe(self) -> torch.Tensor:
        road = self.env.road
        return lidar(road.state, road.network, road.params, self.cfg)


def observation_factory(env, config: dict) -> BatchedObservationType:
    """observation.py:771-793 for the hot-path types."""
    t = config["type"]
    if t == "Kinematics":
        return BatchedKinematicObservation(env, **config)
    if t == "OccupancyGrid":
        return BatchedOccupancyGridObservation(env, **config)
    if t == "TimeToCollision":
        return BatchedTimeToCollisionObservation(env, **config)
    if t == "LidarObservation":
        return BatchedLidarObservation(env, **config)
    if t in ("KinematicsGoal", "GrayscaleObservation", "AttributesObservation", "MultiAgentObservation",
             "TupleObservation", "ExitObservation"):
        raise NotImplementedError(f"observation type {t!r} is SURVEY.md §8(f) 'next' / out of scope")
    raise ValueError("Unknown observation type")
