"""Single-env view of a batched env: the gymnasium ``Env`` contract of the reference
(abstract.py:188-250) with numpy observations and Python scalars, for gymnasium's env checkers and
for code written against one ``intersection-v0`` instance ("Env API").

``SingleEnv(VecIntersectionEnv, config)`` builds a batch of one env on the device and unwraps each
call: ``reset(seed=s)`` is ``IntersectionEnv.reset(seed=s)`` (the batched env seeds env 0 with ``s``),
``step(a)`` returns ``(obs float32 ndarray, float, bool, bool, info)`` with ``info`` as the
reference's ``_info`` (abstract.py:169-186, intersection_env.py:120-128): ``speed`` float,
``crashed`` bool, ``action``, ``rewards`` ({name: bool | float}, as ``_agent_rewards`` returns them)
and, for the intersection, ``agents_rewards`` / ``agents_terminated`` tuples.  Episodes end the
gymnasium way: the caller resets (the batched env's ``auto_reset`` is forced off).
"""
from __future__ import annotations

import numpy as np
import torch

# _agent_rewards returns vehicle.crashed / has_arrived / on_road as bools, the speed term as a float
_BOOL_TERMS = ("collision_reward", "arrived_reward", "on_road_reward")


class SingleEnv:
    metadata = {"render_modes": []}

    def __init__(self, env_cls, config: dict | None = None, render_mode: str | None = None) -> None:
        cfg = dict(config or {})
        if int(cfg.get("num_envs", 1)) != 1:
            raise ValueError("SingleEnv wraps exactly one env (num_envs = 1)")
        cfg.update(num_envs=1, auto_reset=False, env_id_offset=0)
        self.batched = env_cls(cfg, render_mode=render_mode)
        self.render_mode = render_mode

    # gymnasium attributes -------------------------------------------------------------------------
    @property
    def unwrapped(self):
        return self

    @property
    def config(self) -> dict:
        return self.batched.config

    @property
    def observation_space(self):
        return self.batched.observation_space

    @property
    def action_space(self):
        return self.batched.action_space

    @property
    def time(self) -> float:
        return float(self.batched.time[0])

    @property
    def vehicle(self) -> dict:
        """The controlled vehicle's fields as Python scalars."""
        return {k: v[0].item() for k, v in self.batched.vehicle.items()}

    def configure(self, config: dict) -> None:
        """abstract.py:118-121; takes effect at the next reset (as in the reference)."""
        cfg = dict(config)
        cfg.pop("num_envs", None)
        cfg.pop("auto_reset", None)
        self.batched.configure(cfg)

    # API ------------------------------------------------------------------------------------------
    def reset(self, *, seed: int | None = None, options: dict | None = None):
        if options and "config" in options:
            options = dict(options, config={k: v for k, v in options["config"].items()
                                            if k not in ("num_envs", "auto_reset")})
        obs, info = self.batched.reset(seed=seed, options=options)
        return self._obs(obs), self._info(info)

    def step(self, action):
        a = int(action)
        obs, reward, terminated, truncated, info = self.batched.step(torch.tensor([a], dtype=torch.int64))
        return (self._obs(obs), float(reward[0]), bool(terminated[0]), bool(truncated[0]),
                self._info(info, a))

    def render(self):
        return None

    def close(self) -> None:
        self.batched.close()

    # unwrapping -----------------------------------------------------------------------------------
    @staticmethod
    def _obs(obs):
        if isinstance(obs, torch.Tensor):
            return obs[0].cpu().numpy()
        if isinstance(obs, tuple):  # tuple observations (one per type)
            return tuple(SingleEnv._obs(o) for o in obs)
        return np.asarray(obs)[0]

    @staticmethod
    def _info(info: dict, action=None) -> dict:
        out = {"speed": float(info["speed"][0]), "crashed": bool(info["crashed"][0]), "action": action}
        if "rewards" in info:
            out["rewards"] = {n: (bool(v[0]) if n in _BOOL_TERMS else float(v[0]))
                              for n, v in info["rewards"].items()}
        if "agents_rewards" in info:
            out["agents_rewards"] = tuple(float(r[0]) for r in info["agents_rewards"])
            out["agents_terminated"] = tuple(bool(t[0]) for t in info["agents_terminated"])
        return out


class SingleHighwayEnv(SingleEnv):
    """ttrl-highway-single-v0: one synthetic highway (VecHighwayEnv, num_envs 1)."""

    def __init__(self, config: dict | None = None, render_mode: str | None = None) -> None:
        from .envs import VecHighwayEnv
        super().__init__(VecHighwayEnv, config, render_mode)


class SingleIntersectionEnv(SingleEnv):
    """ttrl-intersection-single-v0: one intersection-v0 (VecIntersectionEnv, num_envs 1)."""

    def __init__(self, config: dict | None = None, render_mode: str | None = None) -> None:
        from .intersection import VecIntersectionEnv
        super().__init__(VecIntersectionEnv, config, render_mode)


def make_single(env_id: str, config: dict | None = None) -> SingleEnv:
    """The single-env view of ``envs.make(env_id)`` (the same ids and aliases)."""
    from .envs import resolve
    cls = resolve(env_id)
    return cls(config) if issubclass(cls, SingleEnv) else SingleEnv(cls, config)
