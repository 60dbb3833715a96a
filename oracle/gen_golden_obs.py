"""Observation goldens from the reference's own observation classes — TEST INFRASTRUCTURE, runs
only in the build container.

``oracle/gen_golden.py`` records the observations of its golden scenes through a restatement of
the observation *assembly* (observation.py imports gymnasium and pygame, absent from the image),
built on the reference's own primitives.  This script closes that gap: it replays the same scenes
(``gen_golden.make_highway`` / ``make_dense`` / ``make_curved`` and ``gen_golden.rollout``'s frame
loop: same seeds, same actions) and calls the reference's unmodified observation classes on them:

  * ``KinematicObservation.observe``        observation.py:233-275  (pandas assembly, normalize_obs :205-231)
  * ``OccupancyGridObservation.observe``    observation.py:353-434  (+ fill_road_layer_by_lanes :453-483)
  * ``TimeToCollisionObservation.observe``  observation.py:126-151
  * ``LidarObservation.observe`` / ``trace`` observation.py:694-768
  * the intersection episodes of ``gen_golden_ix.py`` (absolute Kinematics 15x7, ``order="shuffled"``
    drawing ``env.np_random.shuffle(obs[1:])``, observation.py:272-273)

with the two configurations per class that ``gen_golden.py`` records.  Each output must equal the
restated one bit for bit (asserted here); ``tests/golden/obsref_<scene>.npz`` keeps the reference
outputs so that ``tests/test_oracle_golden.py`` can hold the committed fixtures to them.

Stand-ins.  ``observation.py`` imports ``gymnasium.spaces`` (``Box`` / ``Space`` for ``space()``)
and, through ``ttrl_env.envs.common.graphics`` (the ``EnvViewer`` it names for the grayscale
observation), ``pygame`` and ``gymnasium``-typed action classes.  None of them is on the computed
path of the four observers above.  The stand-ins provide those names only: ``spaces.Box`` records
shape and dtype (the Kinematic observation's final ``astype(self.space().dtype)`` reads them), and
``pygame`` is a module whose every attribute is an empty class (``WorldSurface(pygame.Surface)`` is
a class statement at import).  The env is a namespace with the attributes the observers read:
``road``, ``vehicle``, ``PERCEPTION_DISTANCE`` (abstract.py:41), ``config["policy_frequency"]``
and ``np_random``.

Usage:  PYTHONDONTWRITEBYTECODE=1 python oracle/gen_golden_obs.py
"""
from __future__ import annotations

import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import gen_golden as G  # noqa: E402  (imports the reference sim core, no stand-ins)

OUT = G.OUT


def _stand_ins():
    gym = types.ModuleType("gymnasium")
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

    spaces.Space, spaces.Box, spaces.Discrete = Space, Box, Discrete
    spaces.Tuple = spaces.Dict = spaces.MultiDiscrete = Space
    gym.spaces = spaces
    sys.modules["gymnasium"], sys.modules["gymnasium.spaces"] = gym, spaces

    class _AnyName(types.ModuleType):
        def __getattr__(self, name):
            if name.startswith("__"):
                raise AttributeError(name)
            cls = type(name, (), {})
            setattr(self, name, cls)
            return cls

    sys.modules["pygame"] = _AnyName("pygame")


_stand_ins()
from ttrl_env.envs.common import observation as O  # noqa: E402

CLASS_CFGS = {
    "kin5": (O.KinematicObservation, G.KIN_DEFAULT),
    "kin15": (O.KinematicObservation, G.KIN_ENVJSON),
    "grid7": (O.OccupancyGridObservation, G.GRID_DENSE),
    "grid_onroad": (O.OccupancyGridObservation, G.GRID_ONROAD),
    "ttc": (O.TimeToCollisionObservation, dict(horizon=10)),
    "lidar": (O.LidarObservation, dict(cells=16, maximum_range=60.0, normalize=True)),
}


def observers(road):
    env = types.SimpleNamespace(road=road, vehicle=road.vehicles[0],
                                PERCEPTION_DISTANCE=5.0 * G.R.Vehicle.MAX_SPEED,  # abstract.py:41
                                config={"policy_frequency": 1}, np_random=np.random.default_rng(0))
    # one instance per observer for the whole episode, as AbstractEnv keeps it (features_range is
    # filled lazily on the first observe, observation.py:212-225)
    return {k: cls(env, order="sorted", **cfg) for k, (cls, cfg) in CLASS_CFGS.items()}


def restated(road):
    o = {}
    o["kin5"], _ = G.kinematics_obs(road, G.KIN_DEFAULT)
    o["kin15"], _ = G.kinematics_obs(road, G.KIN_ENVJSON)
    o["grid7"] = G.grid_obs(road, G.GRID_DENSE)
    o["grid_onroad"] = G.grid_obs(road, G.GRID_ONROAD)
    o["ttc"] = G.ttc_obs(road)
    o["lidar"] = G.lidar_obs(road)
    return o


def replay(road, policy_steps: int, seed: int):
    """gen_golden.rollout's frame loop (same action draw), observing after reset and after each
    policy step with the reference classes."""
    rng = np.random.default_rng(7777 + seed)
    actions = rng.integers(0, 5, size=policy_steps).astype(np.int32)
    obs = observers(road)
    out = {k: [] for k in CLASS_CFGS}

    def observe():
        mine = restated(road)
        for k, ob in obs.items():
            ref = np.asarray(ob.observe())
            assert ref.shape == mine[k].shape, (k, ref.shape, mine[k].shape)
            assert np.array_equal(ref.astype(mine[k].dtype), mine[k]), k  # restatement == reference
            out[k].append(ref)

    observe()
    for p in range(policy_steps):
        for f in range(15):
            if f == 0:
                road.vehicles[0].act(G.ACTIONS_ALL[int(actions[p])])
            road.act()
            road.step(1 / 15)
        observe()
    return {k: np.stack(v) for k, v in out.items()}


def ix_episode(seed: int, steps: int = 13):
    """gen_golden_ix.episode's intersection episode (absolute Kinematics 15x7, order "shuffled"
    from env.json), observed by the reference's KinematicObservation on a clone of the env's
    generator: its output, and the generator state after its shuffle, must equal the restatement's."""
    import gen_golden_ix as X

    class RefObserved(X.IxEnv):
        def observe(self):
            clone = np.random.default_rng()
            clone.bit_generator.state = self.np_random.bit_generator.state
            env = types.SimpleNamespace(road=self.road, vehicle=self.vehicle, np_random=clone,
                                        PERCEPTION_DISTANCE=5.0 * G.R.Vehicle.MAX_SPEED)
            ref = O.KinematicObservation(env, order=self.order, **X.KIN_IX).observe()
            mine = super().observe()
            assert np.array_equal(ref, mine) and ref.dtype == mine.dtype
            assert clone.bit_generator.state == self.np_random.bit_generator.state  # same shuffle draws
            self.ref_obs.append(ref)
            return mine

    env = RefObserved.__new__(RefObserved)
    env.ref_obs = []
    X.IxEnv.__init__(env, seed, "shuffled")
    env.observe()  # AbstractEnv.reset observes once (abstract.py:210)
    rng = np.random.default_rng(555 + seed)  # gen_golden_ix.episode's action draw
    for a in rng.integers(0, 3, size=steps).astype(np.int32):
        env.step(int(a))
    return {"obs0": env.ref_obs[0], "obs": np.stack(env.ref_obs[1:])}


def main():
    for seed in range(6):
        d = ix_episode(seed)
        np.savez_compressed(os.path.join(OUT, f"obsref_ix_s{seed}.npz"), **d)
        print(f"ix_s{seed}", {k: v.shape for k, v in d.items()})
    cases = [("highway", n, s, 4 if n <= 64 else 2) for n in (8, 32, 64, 128) for s in (0, 1, 2)]
    cases += [("dense", n, s, 2) for n in (16, 64) for s in (0, 1)]
    cases += [(k, 32, s, 4) for k in ("sine", "arc") for s in (0, 1)]
    for kind, n, seed, steps in cases:
        road = (G.make_highway(n, seed) if kind == "highway" else
                G.make_dense(n, seed) if kind == "dense" else G.make_curved(kind, n, seed))
        d = replay(road, steps, seed)
        name = f"{kind}_n{n}_s{seed}"
        np.savez_compressed(os.path.join(OUT, "obsref_" + name + ".npz"), **d)
        print(name, {k: v.shape for k, v in d.items()})


if __name__ == "__main__":
    main()
