"""One batched env.step — optionally closed through the policy — captured as a HIP graph.

The fused simulate kernel, the observation and reward kernels and the policy's torch
kernels are all stream-ordered, allocation-free at replay and host-sync-free, so the whole
closed loop  obs -> policy -> action -> env.step -> obs  records once and replays as one
graph launch: the per-step host work (ctypes marshalling, ~20 small torch launches of the
policy forward) disappears from the step time.  This is the MI355X replacement for a
tracing compiler on this path.

Graph semantics: the tensors a replay returns are static buffers overwritten by the next
replay (clone what you keep); ``epsilon`` and the exploration ``step`` are device scalars
refreshed before each replay, so the exploration schedule and the policy's draws keep advancing.  ``VecHighwayEnv`` must not auto-reset inside a
graph (use ``auto_reset=False``); ``VecIntersectionEnv`` may (``GRAPH_AUTO_RESET``): its
done mask, episode counters, seeds and masked resets are all device tensors and launches, so a
replay resets exactly the envs an eager step would.
"""
from __future__ import annotations

import torch


class StepGraph:
    """``replay()`` advances every env by one policy step; returns (obs, reward, terminated,
    truncated) static tensors.  ``policy``: an ``EgoAttentionPolicy`` (actions from the current
    observation) or None (then ``actions`` [steps?, E] device tensor rows are consumed in order
    from a static buffer the caller fills via ``set_actions``)."""

    def __init__(self, env, obs: torch.Tensor, policy=None, warmup: int = 2):
        if env.config.get("auto_reset") and not getattr(env, "GRAPH_AUTO_RESET", False):
            raise ValueError("StepGraph needs auto_reset=False for this env")
        self.env, self.policy = env, policy
        dev = env.device
        self.obs = obs.clone()
        self.actions = torch.zeros(env.num_envs, dtype=torch.int64, device=dev)
        self.epsilon = torch.zeros((), dtype=torch.float32, device=dev)
        self.step = torch.zeros((), dtype=torch.int64, device=dev)
        self.t = 0
        time0 = policy.time if policy is not None else 0  # warm-up and capture do not count as acts
        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):  # warm up allocator pools and lazy initialisation off-graph
            saved = env.state.clone(), env.time.clone(), self.obs.clone()
            entropy = getattr(env, "_entropy", None)
            saved_entropy = entropy.clone() if isinstance(entropy, torch.Tensor) else None
            for _ in range(warmup):
                self._body()
            env.state.copy_(saved[0])
            env.time.copy_(saved[1])
            self.obs.copy_(saved[2])
            if saved_entropy is not None:
                entropy.copy_(saved_entropy)
        torch.cuda.current_stream(dev).wait_stream(side)
        self.graph = torch.cuda.CUDAGraph()
        if policy is not None:
            self.graph.register_generator_state(policy.gen)
        with torch.cuda.graph(self.graph):
            self.out = self._body()
        if policy is not None:
            policy.time = time0

    def _body(self):
        if self.policy is not None:
            a = self.policy.act(self.obs, epsilon=self.epsilon, step=self.step, dtype=torch.int32)
            self.actions.copy_(a)
        obs, reward, terminated, truncated, _ = self.env.step(self.actions)
        self.obs.copy_(obs)
        return self.obs, reward, terminated, truncated

    def set_actions(self, actions: torch.Tensor) -> None:
        self.actions.copy_(actions)

    def replay(self):
        if self.policy is not None:  # AbstractDQNAgent.act steps the exploration time first
            self.policy.time += 1
            self.epsilon.fill_(self.policy.epsilon(self.policy.time))
            self.step.fill_(self.policy.time)
        self.graph.replay()
        self.t += 1
        return self.out
