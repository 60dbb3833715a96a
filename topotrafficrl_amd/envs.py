"""Batched gymnasium-style highway env: the drop-in for the reference's ``env.step()`` hot path.

Mirrors ttrl_env.envs.common.abstract.AbstractEnv (abstract.py:25-441): the same
``default_config`` / ``configure`` / ``define_spaces`` / ``reset`` / ``step`` /
``_simulate`` structure and config keys, batched over ``num_envs`` independent envs
that advance in lockstep on one HIP device.  Scene: the synthetic straight highway of
SURVEY.md §3.C (the reference registers no highway env; it is built from the
reference primitives RoadNetwork.straight_road_network, MDPVehicle, IDMVehicle.create_random).
Reward / termination follow IntersectionEnv._agent_reward (intersection_env.py:78-119).
"""
from __future__ import annotations

import copy

import numpy as np
import torch

from . import _abi, ops
from .action import action_factory
from .observation import BatchedKinematicObservation, BatchedOccupancyGridObservation, observation_factory
from .road import BatchedRoad, RoadNetwork
from .state import BatchState


def reset_highway(state: BatchState, network: RoadNetwork, params: _abi.Params, cfg: _abi.ResetCfg, seeds) -> None:
    """Scene generation on the device, bit-exact with ``np.random.default_rng(seed)`` per env."""
    seeds = [int(s) for s in seeds]
    if len(seeds) != state.n_envs:
        raise ValueError("one seed per env required")
    if all(0 <= s < 2 ** 32 for s in seeds):  # SeedSequence(seed) is the single entropy word: seeded on the device
        words = torch.tensor(np.asarray(seeds, dtype=np.uint32).view(np.int32), device=state.device).view(-1, 1)
        reset_highway_seeded(state, network, params, cfg, words)
        return
    _device_only(state)
    pcg = torch.from_numpy(_abi.pcg64_states(seeds).view(np.int64)).to(state.device)
    ops.T.reset_highway_(state.tensors(), ops.st(network.table), ops.st(params), ops.st(cfg), pcg)


def reset_highway_seeded(state: BatchState, network: RoadNetwork, params: _abi.Params, cfg: _abi.ResetCfg,
                         entropy: torch.Tensor, mask: torch.Tensor | None = None) -> None:
    """Device-seeded scene init: env e replays ``np.random.default_rng(list(entropy[e]))`` (uint32
    words, stored as int32), only where ``mask[e]`` (uint8/bool [E]) is set; no host round trip."""
    if entropy.dim() != 2 or entropy.shape[0] != state.n_envs or entropy.dtype != torch.int32:
        raise ValueError("entropy must be an int32 [n_envs, n_words] tensor of uint32 words")
    if entropy.device != state.device or (mask is not None and mask.device != state.device):
        raise ValueError("entropy / mask must live on the state's device")
    _device_only(state)
    ops.T.reset_highway_seeded_(state.tensors(), ops.st(network.table), ops.st(params), ops.st(cfg), entropy, mask)


def _device_only(state: BatchState) -> None:
    if state.device.type != "cuda":
        raise RuntimeError("the simulator runs on a HIP device only (no CPU fallback)")


def _keep_tail(env, outs):
    """outs = (reward, terminated, truncated, components, ego speed, ego crashed): kept for
    ``_info`` and returned as (reward, terminated, truncated)."""
    env._reward, env._term, env._trunc, env._components, env._ego_speed, env._ego_crashed = outs
    return outs[:3]


def rewards_and_dones(env, time_inc: float = 0.0):
    """The step tail in one launch (ttrl::rewards_step_): env.time += time_inc, then reward,
    terminated, truncated, env._components and the info's ego speed / crashed."""
    _device_only(env.state)
    outs = ops.T.rewards_step_(env.state.tensors(), ops.st(env.network.table), ops.st(env.reward_cfg), env.time,
                               float(time_inc))
    return _keep_tail(env, outs)


def _reward_terms(names, components: torch.Tensor) -> dict:
    """[E, 4] component block -> {name: [E] view} (float32; 0/1 for the boolean terms)."""
    return {n: components[:, i] for i, n in enumerate(names)}  # views of this step's fresh [E, 4]


class VecHighwayEnv:
    """``num_envs`` synthetic straight highways; vehicle 0 of each env is the controlled ego."""

    metadata = {"render_modes": []}
    PERCEPTION_DISTANCE = 5.0 * 40.0  # abstract.py:41

    def __init__(self, config: dict | None = None, render_mode: str | None = None) -> None:
        if render_mode is not None:
            raise NotImplementedError("rendering is out of scope (SURVEY.md §2)")
        self.config = self.default_config()
        self.configure(config)
        self.road = None
        self.observation_type = self.action_type = None
        self.observation_space = self.action_space = None
        self.time = None
        self.steps = 0
        self.done = False
        self.shuffle_seed = 0
        self._build()
        self.reset()

    @classmethod
    def default_config(cls) -> dict:
        """abstract.py:86-109 + highway scene keys + batching keys."""
        return {
            "observation": {"type": "Kinematics"},
            "action": {"type": "DiscreteMetaAction"},
            "simulation_frequency": 15,
            "policy_frequency": 1,
            "other_vehicles_type": "ttrl_env.vehicle.behavior.IDMVehicle",
            "manual_control": False,
            # scene
            "road": "straight",            # lane geometry: "straight" | "sine" | "circular" (lane.py:235-350)
            "road_params": {},             # sine: amplitude, pulsation, phase; circular: center, radius,
                                           # start_phase, end_phase, clockwise
            "lanes_count": 4,
            "road_length": 10000.0,
            "speed_limit": 30.0,
            "vehicles_count": 50,          # vehicles per env, ego included
            "vehicle_slots": None,         # padded row width (>= vehicles_count); None = vehicles_count
            "ego_lane": 1,
            "ego_x": 50.0,
            "ego_speed": 25.0,
            "spacing": 1.0,
            "enable_lane_change": True,
            "idm": {},                     # overrides of IDM/MOBIL constants (ttrl_params_t field names)
            # reward / termination (IntersectionEnv template)
            "duration": 40,
            "collision_reward": -1.0,
            "high_speed_reward": 0.4,
            "reward_speed_range": [20.0, 30.0],
            "normalize_reward": False,
            "offroad_terminal": False,
            # finite_mdp state reward terms (finite_mdp.py:64-78; highway-env defaults)
            "right_lane_reward": 0.1,
            "lane_change_reward": 0.0,
            # batching
            "num_envs": 1,
            "env_id_offset": 0,            # global id of env 0 (sharding: seeds = seed + global id)
            "device": "cuda",
            "dtype": "f64",
            "auto_reset": False,
            # an OccupancyGrid observation is written by the env.step launch (ttrl_env_step_grid);
            # False: the grid kernel runs after the step (A/B timing only, the same bits)
            "fuse_grid": True,
        }

    def configure(self, config: dict | None) -> None:
        if config:
            self.config.update(config)

    # ------------------------------------------------------------------ setup
    def _build(self):
        c = self.config
        if c["other_vehicles_type"] != "ttrl_env.vehicle.behavior.IDMVehicle":
            raise NotImplementedError("only IDMVehicle traffic is on the hot path (SURVEY.md §2)")
        self.num_envs = int(c["num_envs"])
        n = int(c["vehicles_count"])
        slots = int(c["vehicle_slots"] or n)
        if slots < n:
            raise ValueError("vehicle_slots < vehicles_count")
        self.device = torch.device(c["device"])
        lanes, rp, lim = int(c["lanes_count"]), dict(c["road_params"]), float(c["speed_limit"])
        if c["road"] == "straight":
            self.network = RoadNetwork.straight_road_network(lanes, length=float(c["road_length"]), speed_limit=lim,
                                                             **rp)
        elif c["road"] == "sine":
            self.network = RoadNetwork.sine_road_network(lanes, length=float(c["road_length"]), speed_limit=lim, **rp)
        elif c["road"] == "circular":
            self.network = RoadNetwork.circular_road_network(lanes, speed_limit=lim, **rp)
        else:
            raise ValueError(f"unknown road geometry {c['road']!r}")
        act_cfg = dict(c["action"])
        self.params = _abi.default_params(target_speeds=act_cfg.get("target_speeds"), **dict(c["idm"]))
        self.state = BatchState(self.num_envs, slots, device=self.device, dtype=c["dtype"])
        self.road = BatchedRoad(self.network, self.state, self.params)
        self.reset_cfg = _abi.reset_cfg(n, self.network.table, ego_lane=int(c["ego_lane"]), ego_x=float(c["ego_x"]),
                                        ego_speed=float(c["ego_speed"]), spacing=float(c["spacing"]),
                                        lane_change=bool(c["enable_lane_change"]))
        self.reward_cfg = _abi.reward_cfg(c["collision_reward"], c["high_speed_reward"], c["reward_speed_range"],
                                          c["normalize_reward"], c["offroad_terminal"], c["duration"])
        self.time = torch.zeros(self.num_envs, dtype=torch.float64, device=self.device)
        self._reward = torch.zeros(self.num_envs, dtype=torch.float32, device=self.device)
        self._term = torch.zeros(self.num_envs, dtype=torch.uint8, device=self.device)
        self._trunc = torch.zeros(self.num_envs, dtype=torch.uint8, device=self.device)
        self._components = torch.zeros((self.num_envs, 4), dtype=torch.float32, device=self.device)
        # auto-reset entropy per env: [seed lo word, seed hi word, episode]; episode k >= 1 of an env
        # reset with seed s replays np.random.default_rng([s & 0xffffffff, s >> 32, k])
        self._entropy = torch.zeros(self.num_envs, 3, dtype=torch.int32, device=self.device)
        self.define_spaces()

    @property
    def vehicle(self):
        """The controlled vehicles: slot 0 of every env (abstract.py:76-79)."""
        return {k: v[:, 0] for k, v in self.state.t.items() if k not in ("reg_steps", "rng")}

    def define_spaces(self) -> None:
        """abstract.py:123-130"""
        self.observation_type = observation_factory(self, self.config["observation"])
        self.action_type = action_factory(self, self.config["action"])
        self.observation_space = self.observation_type.space()
        self.action_space = self.action_type.space()

    # ------------------------------------------------------------------ API
    def _seeds(self, seed):
        if seed is None:
            seed = int(np.random.SeedSequence().generate_state(1)[0])
        if isinstance(seed, (list, tuple, np.ndarray, torch.Tensor)):
            s = [int(v) for v in (seed.tolist() if hasattr(seed, "tolist") else seed)]
            if len(s) != self.num_envs:
                raise ValueError("per-env seeds must have num_envs entries")
            return s
        base = int(seed) + int(self.config["env_id_offset"])
        return [base + e for e in range(self.num_envs)]

    def reset(self, *, seed=None, options: dict | None = None):
        """abstract.py:188-214.  ``seed``: int (env e gets seed + env_id_offset + e) or one per env."""
        if options and "config" in options:
            self.configure(options["config"])
            self._build()
        seeds = self._seeds(seed)
        self.shuffle_seed = seeds[0]
        self.time.zero_()
        self.steps = 0
        self.done = False
        reset_highway(self.state, self.network, self.params, self.reset_cfg, seeds)
        ent = np.zeros((self.num_envs, 3), dtype=np.uint32)
        ent[:, 0] = [s & 0xFFFFFFFF for s in seeds]
        ent[:, 1] = [(s >> 32) & 0xFFFFFFFF for s in seeds]
        self._entropy.copy_(torch.from_numpy(ent.view(np.int32)))
        obs = self.observation_type.observe()
        self._rewards_and_dones()  # abstract.py:211 reset's _info evaluates _rewards too
        return obs, self._info(obs, None)

    def step(self, action):
        """abstract.py:224-250: (obs, reward[E], terminated[E], truncated[E], info)."""
        if self.road is None:
            raise NotImplementedError("The road and vehicle must be initialized in the environment implementation")
        # one launch: _simulate, the Kinematics observation (or OccupancyGrid) of the final state and
        # the step tail (time += 1 / policy_frequency, abstract.py:239; rewards, dones, info),
        # ttrl_env_step / ttrl_env_step_grid
        obs, (reward, terminated, truncated) = self._simulate(action, tail=True)
        if obs is None:
            obs = self.observation_type.observe()
        info = self._info(obs, action)
        if self.config["auto_reset"]:
            # finished envs restart on the device; obs is the new episode's first observation and
            # info["final_observation"] the finished episode's last (no host round trip): only the
            # finished envs are regenerated and re-observed (masked launches)
            done = self._auto_reset_step(terminated, truncated)
            info["final_observation"], info["final_mask"] = obs, done
            if isinstance(self.observation_type, BatchedKinematicObservation):
                obs = self.observation_type.observe(mask=done, out=obs.clone())
            else:
                obs = self.observation_type.observe()
        return obs, reward, terminated, truncated, info

    def _simulate(self, action=None, tail: bool = False):
        """abstract.py:252-282 as one fused launch: meta-action at frame 0, then frames x (act, step).
        With ``tail`` the same launch also writes the step tail and, for a Kinematics observation, the
        observation of the final state (ttrl::env_step_); returns (obs or None, (reward, terminated,
        truncated))."""
        frames = int(self.config["simulation_frequency"] // self.config["policy_frequency"])
        dt = 1 / self.config["simulation_frequency"]
        act = action is not None and not self.config["manual_control"]
        self.steps += frames
        if not tail:
            self.road.simulate(self.action_type._codes(action) if act else None, frames, dt)
            return None
        # action indices: the launch maps them to meta-action codes (no lookup launch)
        idx, lut = self.action_type._indices(action) if act else (None, None)
        kin = isinstance(self.observation_type, BatchedKinematicObservation)
        grid = isinstance(self.observation_type, BatchedOccupancyGridObservation) and self.config["fuse_grid"]
        kc = self.observation_type.fused_cfg() if kin else None
        gc = self.observation_type.cfg if grid else None
        obs, ids, *outs = self.road.env_step(idx, frames, dt, kc, self.reward_cfg, self.time,
                                             1 / self.config["policy_frequency"], None, lut, gc)
        if kin:
            self.observation_type.fused_result(obs, ids)
        elif grid:
            self.observation_type._out = obs
        return (obs if kin or grid else None), _keep_tail(self, outs)

    REWARD_TERMS = ["collision_reward", "high_speed_reward", "arrived_reward", "on_road_reward"]

    def _rewards_and_dones(self, time_inc: float = 0.0):
        """reward, terminated, truncated [E]; the per-objective terms (_agent_rewards,
        intersection_env.py:95-104) go to self._components [E, 4] for info["rewards"]."""
        return rewards_and_dones(self, time_inc)

    def _info(self, obs, action) -> dict:
        """abstract.py:169-186 batched: device tensors [E]; info["rewards"] holds the per-objective
        terms of the last _rewards_and_dones (AbstractEnv._rewards)."""
        return {"speed": self._ego_speed, "crashed": self._ego_crashed,
                "action": action, "rewards": _reward_terms(self.REWARD_TERMS, self._components)}

    def _auto_reset_step(self, terminated: torch.Tensor, truncated: torch.Tensor) -> torch.Tensor:
        """The step's auto-reset in one launch (ttrl::auto_reset_highway_): done = terminated |
        truncated; the done envs' episode counters (entropy word 2) advance, their scenes are
        regenerated from default_rng([seed lo, seed hi, episode]) and their time zeroed."""
        _device_only(self.state)
        return ops.T.auto_reset_highway_(self.state.tensors(), ops.st(self.network.table), ops.st(self.params),
                                         ops.st(self.reset_cfg), self._entropy, 2, terminated, truncated, self.time)

    def _auto_reset(self, done: torch.Tensor) -> None:
        """Masked auto-reset of finished envs on the device."""
        d = done.view(torch.uint8) if done.dtype == torch.bool else done.to(torch.uint8)
        self._entropy[:, 2] += d
        reset_highway_seeded(self.state, self.network, self.params, self.reset_cfg, self._entropy, d)
        self.time.masked_fill_(done, 0.0)

    def get_available_actions(self):
        return self.action_type.get_available_actions()

    def to_finite_mdp(self):
        """abstract.py:416-417: the batched time-to-collision MDP of every env's ego."""
        from .finite_mdp import finite_mdp
        return finite_mdp(self, time_quantization=1 / self.config["policy_frequency"])

    def close(self) -> None:
        self.done = True

    def render(self):
        raise NotImplementedError("rendering is out of scope (SURVEY.md §2)")

    def __deepcopy__(self, memo):
        new = copy.copy(self)
        new.state = self.state.clone()
        new.road = BatchedRoad(self.network, new.state, self.params)
        new.time = self.time.clone()
        if self._entropy is not None:  # the fork's auto-resets must not advance our episode counters
            new._entropy = self._entropy.clone()
        new.define_spaces()
        return new


ENV_IDS = {"ttrl-highway-batched-v0": "topotrafficrl_amd.envs:VecHighwayEnv",
           "ttrl-intersection-batched-v0": "topotrafficrl_amd.intersection:VecIntersectionEnv",
           # single-env views (numpy out, one env) for gymnasium's checkers: single.py
           "ttrl-highway-single-v0": "topotrafficrl_amd.single:SingleHighwayEnv",
           "ttrl-intersection-single-v0": "topotrafficrl_amd.single:SingleIntersectionEnv"}
ALIASES = {"intersection-v0": "ttrl-intersection-batched-v0", "highway-v0": "ttrl-highway-batched-v0"}


def register(env_id: str | None = None) -> bool:
    """gymnasium.register(id, entry_point) as ttrl_env/__init__.py:28-56 does (intersection-v0 ->
    ttrl-intersection-batched-v0); no-op without gymnasium."""
    try:
        import gymnasium
    except ImportError:
        return False
    for i, entry in ENV_IDS.items():
        if env_id is None or i == env_id:
            gymnasium.register(id=i, entry_point=entry)
    return True


def resolve(env_id: str):
    """The env class registered under ``env_id`` (reference ids through ALIASES)."""
    env_id = ALIASES.get(env_id, env_id)
    if env_id not in ENV_IDS:
        raise KeyError(f"unknown env id {env_id!r}")
    mod, cls = ENV_IDS[env_id].split(":")
    import importlib
    return getattr(importlib.import_module(mod), cls)


def make(env_id: str, config: dict | None = None, **kwargs):
    """gym.make(id) + env.unwrapped.configure(config) (scripts/utils factory.py:72-91) without
    gymnasium: the batched env of ``env_id`` ("intersection-v0" / "highway-v0" map to ours)."""
    return resolve(env_id)(dict(config or {}, **kwargs))
