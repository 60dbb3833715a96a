"""Intersection episodes from the reference's own ``IntersectionEnv`` — TEST INFRASTRUCTURE, runs
only in the build container.

``oracle/gen_golden_ix.py`` records the intersection goldens (``tests/golden/ix_s*.npz``) through
``IxEnv``, a restatement of the env-level code of intersection_env.py over the reference's road
and vehicle classes, because ``intersection_env.py`` imports gymnasium (absent from the image).
This script closes that gap: it imports the unmodified ``ttrl_env.envs.intersection_env`` and
``abstract.py`` behind name-only stand-ins and drives the reference class itself:

  * ``AbstractEnv.reset(seed)``   abstract.py:188-214 (gymnasium's ``Env.reset`` seeding,
    ``define_spaces`` twice, ``_reset`` = ``_make_road`` + ``_make_vehicles`` intersection_env.py:131-133,
    141-318, the first ``observe`` and ``_info``)
  * ``IntersectionEnv.step(a)``   intersection_env.py:135-139 over ``AbstractEnv.step`` / ``_simulate``
    abstract.py:224-282, then ``_clear_vehicles`` / ``_spawn_vehicle`` :320-362
  * ``_reward`` / ``_agent_reward`` / ``_agent_rewards`` / ``_is_terminated`` / ``_is_truncated`` /
    ``_info`` / ``has_arrived``  intersection_env.py:61-129, 364-369
  * the shuffled Kinematics observation of ``scripts/configs/IntersectionEnv/env.json``

in lockstep with ``gen_golden_ix.IxEnv`` on the same seed and actions, and asserts, after reset
and after every step: the vehicle list (every field of every vehicle, in list order) after each
of the 15 frames and after the clear / spawn, the observation, reward, terminated, truncated, the
info dict (speed, crashed, the four reward terms, agents_rewards, agents_terminated) and the
state of ``np_random`` — all bit for bit.  The reference's outputs are committed as
``tests/golden/envref_ix_s<seed>.npz``; ``tests/test_ix_env_oracle.py`` holds the committed ix
goldens and the float64 oracle to them, and ``tests/test_gpu_ix_env.py`` the device env.

Episodes: seeds 0-11 draw their actions as ``gen_golden_ix.episode`` does (so seeds 0-5 are the
committed ix goldens' episodes); seeds 12-17 hold FASTER, which drives the ego to its exit (the
``arrived`` reward and termination).  The set must contain crashes, arrivals and rejected spawns
(asserted).

Stand-ins (names only; none is on the computed path):
  * ``gymnasium``: ``Env`` with gymnasium 0.29's seeding (``reset(seed)`` sets ``np_random`` to
    ``Generator(PCG64(SeedSequence(seed)))``, ``gymnasium/utils/seeding.py``), ``Wrapper``,
    ``spaces.{Space, Box, Discrete, Tuple, Dict, MultiDiscrete}`` (``Discrete.sample`` draws from
    its own generator, as gymnasium's spaces do, never from the env's), ``utils.RecordConstructorArgs``,
    ``wrappers.RecordVideo``, ``envs.registration.register``, ``logger``;
  * ``pygame`` and ``matplotlib.pyplot``: modules whose every attribute is an empty class
    (class statements in the graphics modules and ``dynamics.py``'s import need them).

Usage:  PYTHONDONTWRITEBYTECODE=1 python oracle/gen_golden_envref.py
"""
from __future__ import annotations

import json
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import gen_golden as G  # noqa: E402  (registers the reference package, imports the sim core)
import gen_golden_ix as X  # noqa: E402

OUT = G.OUT
REF_ENV_JSON = os.path.join(G.REF, "scripts", "configs", "IntersectionEnv", "env.json")
STEPS = 13
RANDOM_SEEDS = list(range(12))
FASTER_SEEDS = list(range(12, 18))
INFO_TERMS = ["collision_reward", "high_speed_reward", "arrived_reward", "on_road_reward"]


class _AnyName(types.ModuleType):
    def __getattr__(self, name):
        if name.startswith("__"):
            raise AttributeError(name)
        cls = type(name, (), {})
        setattr(self, name, cls)
        return cls


def _stand_ins():
    gym = types.ModuleType("gymnasium")

    class Env:
        spec = None
        _np_random = None
        metadata = {"render_modes": []}

        def reset(self, *, seed=None, options=None):
            if seed is not None:  # gymnasium.utils.seeding.np_random(seed)
                self._np_random = np.random.Generator(np.random.PCG64(np.random.SeedSequence(seed)))

        @property
        def np_random(self):
            if self._np_random is None:
                self._np_random = np.random.Generator(np.random.PCG64(np.random.SeedSequence(None)))
            return self._np_random

        @np_random.setter
        def np_random(self, value):
            self._np_random = value

        @property
        def unwrapped(self):
            return self

    class Wrapper:
        def __init__(self, env):
            self.env = env

        @classmethod
        def wrapper_spec(cls, **kwargs):
            return None

    spaces = types.ModuleType("gymnasium.spaces")

    class Space:
        def __init__(self, *a, **k):
            pass

    class Box(Space):
        def __init__(self, low=None, high=None, shape=None, dtype=np.float32):
            self.low, self.high, self.shape, self.dtype = low, high, tuple(shape), dtype

    class Discrete(Space):
        def __init__(self, n):
            self.n = int(n)
            self._rng = np.random.default_rng(12345)  # the space's own generator, not the env's

        def sample(self):
            return int(self._rng.integers(self.n))

    spaces.Space, spaces.Box, spaces.Discrete = Space, Box, Discrete
    spaces.Tuple = spaces.Dict = spaces.MultiDiscrete = Space
    utils = types.ModuleType("gymnasium.utils")

    class RecordConstructorArgs:
        def __init__(self, **kwargs):
            self._saved_kwargs = kwargs

    utils.RecordConstructorArgs = RecordConstructorArgs
    wrappers = types.ModuleType("gymnasium.wrappers")
    wrappers.RecordVideo = type("RecordVideo", (), {})
    envs = types.ModuleType("gymnasium.envs")
    registration = types.ModuleType("gymnasium.envs.registration")
    registration.register = lambda **kwargs: None
    envs.registration = registration
    logger = types.ModuleType("gymnasium.logger")
    logger.warn = lambda *a, **k: None
    gym.Env, gym.Wrapper, gym.spaces, gym.utils, gym.wrappers, gym.envs, gym.logger = (
        Env, Wrapper, spaces, utils, wrappers, envs, logger)
    for name, mod in (("gymnasium", gym), ("gymnasium.spaces", spaces), ("gymnasium.utils", utils),
                      ("gymnasium.wrappers", wrappers), ("gymnasium.envs", envs),
                      ("gymnasium.envs.registration", registration), ("gymnasium.logger", logger)):
        sys.modules[name] = mod
    sys.modules["pygame"] = _AnyName("pygame")
    mpl = _AnyName("matplotlib")
    mpl.pyplot = _AnyName("matplotlib.pyplot")
    sys.modules["matplotlib"], sys.modules["matplotlib.pyplot"] = mpl, mpl.pyplot


_stand_ins()
from ttrl_env.envs.intersection_env import IntersectionEnv  # noqa: E402  (the unmodified reference)


class CountingIxEnv(X.IxEnv):
    """IxEnv counting its spawn outcomes (drawn and placed, drawn and rejected by the 15 m test)."""

    def __init__(self, seed, order="shuffled"):
        self.spawns = {"placed": 0, "rejected": 0, "not_drawn": 0}
        super().__init__(seed, order)

    def _spawn_vehicle(self, longitudinal=0, position_deviation=1.0, speed_deviation=1.0, spawn_probability=0.6,
                       go_straight=False):
        state = self.np_random.bit_generator.state
        out = super()._spawn_vehicle(longitudinal, position_deviation, speed_deviation, spawn_probability,
                                     go_straight)
        if out is not None:
            self.spawns["placed"] += 1
        else:  # drew more than the spawn-probability uniform: placed, then rejected by the 15 m test
            self.spawns["rejected" if self._drew_placement(state) else "not_drawn"] += 1
        return out

    def _drew_placement(self, state) -> bool:
        g = np.random.default_rng()
        g.bit_generator.state = state
        g.uniform()
        return g.bit_generator.state != self.np_random.bit_generator.state

    def info(self):
        """IntersectionEnv._info (intersection_env.py:121-129) over AbstractEnv._info (abstract.py:169-186)."""
        v = self.vehicle
        scaled = G.R.utils.lmap(v.speed, self.config["reward_speed_range"], [0, 1])
        terms = {"collision_reward": v.crashed, "high_speed_reward": np.clip(scaled, 0, 1),
                 "arrived_reward": self.has_arrived(v), "on_road_reward": v.on_road}
        return {"speed": v.speed, "crashed": v.crashed, "rewards": terms, "agents_rewards": (self.reward(),),
                "agents_terminated": (v.crashed or self.has_arrived(v),)}


def ref_env() -> IntersectionEnv:
    cfg = json.load(open(REF_ENV_JSON))
    cfg = {k: v for k, v in cfg.items() if k not in ("id", "import_module")}  # factory.py:89-91 strips nothing
    return IntersectionEnv(config=cfg)


def rng_words(g) -> np.ndarray:
    """np_random's state in the layout of the device's ``state.rng`` row (_abi.RNG_WORDS words:
    state hi, lo, inc hi, lo, has_uint32 << 32 | uinteger)."""
    s = g.bit_generator.state
    st, inc = int(s["state"]["state"]), int(s["state"]["inc"])
    m = (1 << 64) - 1
    return np.array([st >> 64, st & m, inc >> 64, inc & m, (int(s["has_uint32"]) << 32) | int(s["uinteger"])],
                    dtype=np.uint64)


def assert_same_snapshot(a: dict, b: dict, what: str):
    assert a.keys() == b.keys(), what
    for k in a:
        assert np.array_equal(np.asarray(a[k]), np.asarray(b[k]), equal_nan=True), (what, k, a[k], b[k])


def info_row(info: dict) -> np.ndarray:
    """speed, crashed, the four terms, agents_rewards[0], agents_terminated[0] as float64."""
    return np.array([float(info["speed"]), float(bool(info["crashed"]))]
                    + [float(info["rewards"][t]) for t in INFO_TERMS]
                    + [float(info["agents_rewards"][0]), float(bool(info["agents_terminated"][0]))])


def assert_same_info(ref: dict, mine: dict, what: str):
    assert np.array_equal(info_row(ref), info_row(mine)), (what, info_row(ref), info_row(mine))
    assert list(ref["rewards"].keys()) == INFO_TERMS, what


def episode(env: IntersectionEnv, seed: int, actions: np.ndarray):
    """The reference env and IxEnv from reset(seed) through len(actions) steps, compared after every
    frame and step.  Returns the reference's record and IxEnv's spawn counts."""
    obs0, info0 = env.reset(seed=seed)
    mine = CountingIxEnv(seed, "shuffled")
    mine_obs0 = mine.observe()
    assert np.array_equal(obs0, mine_obs0) and obs0.dtype == mine_obs0.dtype, (seed, "reset obs")
    assert_same_snapshot(X.snapshot(env), X.snapshot(mine), f"s{seed} reset state")
    assert rng_words(env.np_random).tolist() == rng_words(mine.np_random).tolist(), (seed, "reset rng")
    rng_reset = rng_words(env.np_random)  # np_random after reset: the state step 0 starts from
    # AbstractEnv.reset's _info is evaluated on the reset scene (its sampled action is unused)
    assert_same_info(info0, mine.info(), f"s{seed} reset info")
    rec = {"pre": [], "frames": [], "post": [], "obs": [], "reward": [], "terminated": [], "truncated": [],
           "info": [], "rng": []}
    for p, a in enumerate(actions):
        rec["pre"].append(X.snapshot(env))
        frames = []
        road = env.road
        orig = road.step

        def step_and_record(dt, _orig=orig, _frames=frames):  # the reference's frame, then a snapshot
            _orig(dt)
            _frames.append(X.snapshot(env))

        road.step = step_and_record
        obs, rew, term, trunc, info = env.step(int(a))
        del road.step
        mrec = {"act": [], "frames": []}
        mobs, mrew, mterm, mtrunc = mine.step(int(a), mrec)
        minfo = mine.info()
        assert len(frames) == 15 and len(mrec["frames"]) == 15
        for f in range(15):
            assert_same_snapshot(frames[f], mrec["frames"][f], f"s{seed} step {p} frame {f}")
        assert np.array_equal(obs, mobs) and obs.dtype == mobs.dtype, (seed, p, "obs")
        assert rew == mrew, (seed, p, "reward", rew, mrew)
        assert bool(term) == mterm and bool(trunc) == mtrunc, (seed, p, "flags")
        assert_same_info(info, minfo, f"s{seed} step {p} info")
        assert_same_snapshot(X.snapshot(env), X.snapshot(mine), f"s{seed} step {p} post")
        assert rng_words(env.np_random).tolist() == rng_words(mine.np_random).tolist(), (seed, p, "rng")
        rec["frames"].append(frames)
        rec["post"].append(X.snapshot(env))
        rec["obs"].append(obs)
        rec["reward"].append(rew)
        rec["terminated"].append(bool(term))
        rec["truncated"].append(bool(trunc))
        rec["info"].append(info_row(info))
        rec["rng"].append(rng_words(env.np_random))
    rec["obs0"], rec["info0"] = obs0, info_row(info0)
    return rec, mine.spawns, rng_reset


def save(seed: int, actions: np.ndarray, rec: dict, rng0: np.ndarray, spawns: dict, rng_reset: np.ndarray):
    allsnaps = rec["pre"] + rec["post"] + [s for f in rec["frames"] for s in f]
    nmax = max(len(s["x"]) for s in allsnaps)
    d = {}
    for name in ("pre", "post"):
        for k, v in X.stack(rec[name], nmax).items():
            d[f"{name}_{k}"] = v
    st = X.stack([f[14] for f in rec["frames"]], nmax)  # the state entering the observation
    for k, v in st.items():
        d[f"end_{k}"] = v
    d["actions"] = actions.astype(np.int32)
    d["obs0"], d["info0"], d["rng0"] = rec["obs0"], rec["info0"], rng0
    d["obs"] = np.stack(rec["obs"])
    d["reward"] = np.array(rec["reward"], dtype=np.float64)
    d["terminated"] = np.array(rec["terminated"], dtype=np.uint8)
    d["truncated"] = np.array(rec["truncated"], dtype=np.uint8)
    d["info"] = np.stack(rec["info"])
    d["rng"] = np.stack(rec["rng"])
    d["rng_reset"] = rng_reset  # rng[p - 1] is the state step p starts from; rng_reset that of step 0
    d["meta"] = np.array([seed, len(actions), nmax], dtype=np.int64)
    # the episode's _spawn_vehicle outcomes (reset and steps): placed, rejected by the 15 m test
    # after its draws, not drawn (the spawn-probability uniform alone)
    d["spawns"] = np.array([spawns["placed"], spawns["rejected"], spawns["not_drawn"]], dtype=np.int64)
    np.savez_compressed(os.path.join(OUT, f"envref_ix_s{seed}.npz"), **d)
    return d


def main():
    env = ref_env()
    assert env.config["observation"]["order"] == "shuffled" and env.config["destination"] == "o1"
    totals = {"placed": 0, "rejected": 0, "not_drawn": 0, "crashed": 0, "arrived": 0}
    for seed in RANDOM_SEEDS + FASTER_SEEDS:
        if seed in RANDOM_SEEDS:  # gen_golden_ix.episode's action draw
            actions = np.random.default_rng(555 + seed).integers(0, 3, size=STEPS).astype(np.int32)
        else:
            actions = np.full(STEPS, 2, dtype=np.int32)
        rng0 = rng_words(np.random.default_rng(seed))
        rec, spawns, rng_reset = episode(env, seed, actions)
        d = save(seed, actions, rec, rng0, spawns, rng_reset)
        crashed = int(d["info"][:, 1].max())
        arrived = int((d["info"][:, 4] > 0).any())
        for k, v in spawns.items():
            totals[k] += v
        totals["crashed"] += crashed
        totals["arrived"] += arrived
        print(f"envref_ix_s{seed}: vehicles per step {(d['pre_kind'] > 0).sum(1).tolist()} spawns {spawns} "
              f"crashed {crashed} arrived {arrived} term {d['terminated'].tolist()} "
              f"reward {np.round(d['reward'], 3).tolist()}")
    print("totals", totals)
    assert totals["crashed"] > 0 and totals["arrived"] > 0 and totals["rejected"] > 0, totals


if __name__ == "__main__":
    main()
