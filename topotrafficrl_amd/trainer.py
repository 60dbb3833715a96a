"""Batched trainer hooks: the drop-in for ttrl_agent/trainer/evaluation.py:Evaluation.

Keeps the reference's hook names and call order (Evaluation.step, evaluation.py:163-194):
  agent.plan(obs) -> env.step(action) -> step_callback_fn(episode, env, agent, transition, writer)
  -> agent.record(previous_obs, action, reward, obs, done, info)
but every quantity is a batch over the env's ``num_envs`` (device tensors), so one call
advances thousands of episodes.  Differences, on purpose:
  * the reset seed is actually passed to the env (the reference computes it and drops it,
    evaluation.py:372-376);
  * rendering / video / tensorboard are out of scope: ``writer`` is any object with
    ``add_scalar`` (or None).
"""
from __future__ import annotations

import logging
import time
import warnings
from pathlib import Path

import numpy as np
import torch

from .agent import EgoAttentionPolicy
from .dqn import DEFAULT_CONFIG, DQNLearner

logger = logging.getLogger(__name__)


class BatchedDQNAgent:
    """DQNAgent (deep_q_network/pytorch.py, abstract.py) for batched observations: acting with
    the EgoAttention-2h value net and epsilon-greedy exploration, learning with the batched
    replay memory / double-DQN residual / Adam / target sync of ``dqn.DQNLearner``."""

    def __init__(self, device, n_actions: int = 5, seed: int = 0, config: dict | None = None, env_id_offset: int = 0):
        self.policy = EgoAttentionPolicy(device, n_actions=n_actions, seed=seed, env_id_offset=env_id_offset)
        self.config = {**DEFAULT_CONFIG, **(config or {})}
        self.seed_value = seed
        self.learner = None  # built on the first record (the observation shape is known then)
        self.training = True
        self.writer = None

    def plan(self, observation):
        """AbstractAgent.plan: a sequence of actions whose first element is applied (batched: [E])."""
        return [self.act(observation)]

    def act(self, observation):
        return self.policy.act(observation)

    def record(self, state, action, reward, next_state, done, info):
        """AbstractDQNAgent.record (abstract.py:37-63) for a batch of transitions.  With an
        auto-resetting env the finished envs' ``next_state`` is the episode's last observation
        (info["final_observation"]), not the next episode's first."""
        if not self.training:
            return None
        if info and "final_observation" in info and "final_mask" in info:
            m = info["final_mask"].view(-1, *[1] * (next_state.dim() - 1))
            next_state = torch.where(m, info["final_observation"], next_state)
        if self.learner is None:
            self.learner = DQNLearner(self.policy.value_net, tuple(state.shape[1:]), self.policy.device, self.config,
                                      seed=self.seed_value + 7)
        loss = self.learner.record(state, action, reward, next_state, done)
        if loss is not None and self.writer is not None:
            self.writer.add_scalar("agent/loss", float(loss), self.learner.steps)
        return loss

    def seed(self, seed=None):
        if seed is not None:
            self.policy.gen.manual_seed(int(seed))
        return [seed]

    def reset(self):
        pass

    def eval(self):
        self.training = False
        self.policy.value_net.eval()

    def set_writer(self, writer):
        self.writer = writer

    def save(self, filename):
        """DQNAgent.save (pytorch.py:82-86): {'state_dict', 'optimizer'}."""
        Path(filename).parent.mkdir(parents=True, exist_ok=True)
        opt = self.learner.optimizer.state_dict() if self.learner is not None else None
        torch.save({"state_dict": self.policy.value_net.state_dict(), "optimizer": opt}, filename)
        return filename

    def load(self, filename):
        """DQNAgent.load (pytorch.py:88-93), weights_only."""
        ckpt = torch.load(filename, map_location=self.policy.device, weights_only=True)
        self.policy.value_net.load_state_dict(ckpt["state_dict"])
        if self.learner is not None:
            self.learner.target_net.load_state_dict(ckpt["state_dict"])
            if ckpt.get("optimizer"):
                self.learner.optimizer.load_state_dict(ckpt["optimizer"])
        return filename


class BatchedEvaluation:
    def __init__(self, env, agent, num_episodes: int = 1, training: bool = True, sim_seed: int | None = None,
                 step_callback_fn=None, writer=None, directory: str | None = None, max_steps: int | None = None):
        self.env, self.agent = env, agent
        self.num_episodes, self.training = num_episodes, training
        self.sim_seed = sim_seed if sim_seed is not None else int(np.random.randint(0, 1e6))
        self.step_callback_fn = step_callback_fn
        self.writer = writer
        self.directory = Path(directory or "out") / type(env).__name__ / type(agent).__name__
        self.max_steps = max_steps
        self.episode = 0
        self.observation = None
        if hasattr(agent, "set_writer"):
            agent.set_writer(writer)
        if isinstance(getattr(agent, "policy", None), EgoAttentionPolicy) and hasattr(env, "config"):
            # the env's global ids (a data-parallel rank's shard): exploration keyed on them.  An
            # offset given to the agent explicitly is kept: an env left at offset 0 does not reset it,
            # and a different non-zero env offset is a conflict, not a silent override
            env_off = int(env.config.get("env_id_offset", 0) or 0)
            agent_off = int(agent.policy.env_id_offset)
            if agent_off == 0:
                agent.policy.env_id_offset = env_off
            elif env_off not in (0, agent_off):
                raise ValueError(f"the agent's env_id_offset {agent_off} conflicts with the env's {env_off}")
            elif env_off == 0:
                warnings.warn(f"keeping the agent's env_id_offset {agent_off} (the env's config has 0)")
        agent.evaluation = self

    # evaluation.py:115-121
    def train(self):
        self.training = True
        self.run_episodes()
        self.close()

    # evaluation.py:123-137
    def test(self):
        self.training = False
        try:
            self.agent.eval()
        except AttributeError:
            pass
        self.run_episodes()
        self.close()

    # evaluation.py:139-161, batched: an episode ends when every env has terminated or truncated
    def run_episodes(self):
        for self.episode in range(self.num_episodes):
            self.reset(seed=self.episode)
            done_mask = None
            rewards = []
            start = time.time()
            steps = 0
            while True:
                reward, terminal = self.step()
                live = ~done_mask if done_mask is not None else torch.ones_like(terminal)
                rewards.append(torch.where(live, reward, torch.zeros_like(reward)))
                done_mask = terminal if done_mask is None else (done_mask | terminal)
                steps += 1
                if bool(done_mask.all()) or (self.max_steps and steps >= self.max_steps):
                    break
            self.after_all_episodes(self.episode, torch.stack(rewards), time.time() - start)

    # evaluation.py:163-194
    def step(self):
        actions = self.agent.plan(self.observation)
        if actions is None or len(actions) == 0:
            raise Exception("The agent did not plan any action")
        previous_observation, action = self.observation, actions[0]
        transition = self.env.step(action)
        self.observation, reward, done, truncated, info = transition
        terminal = done | truncated
        if self.step_callback_fn is not None:
            self.step_callback_fn(self.episode, self.env, self.agent, transition, self.writer)
        try:
            self.agent.record(previous_observation, action, reward, self.observation, done, info)
        except NotImplementedError:
            pass
        return reward, terminal

    def rollout(self, steps: int):
        """Fixed-length batched collection (no episode bookkeeping): returns stacked rewards [steps, E]."""
        if self.observation is None:
            self.reset(seed=0)
        return torch.stack([self.step()[0] for _ in range(steps)])

    # evaluation.py:372-376 (the seed IS forwarded here)
    def reset(self, seed: int = 0):
        seed = self.sim_seed + seed
        self.observation, info = self.env.reset(seed=seed)
        if hasattr(self.agent, "seed"):
            self.agent.seed(seed)
        if hasattr(self.agent, "reset"):
            self.agent.reset()

    # evaluation.py:325-333 (per-env episode statistics, averaged)
    def after_all_episodes(self, episode, rewards: torch.Tensor, duration: float):
        gamma = getattr(self.agent, "config", {}).get("gamma", 1)
        r = rewards.double()
        disc = gamma ** torch.arange(r.shape[0], dtype=torch.float64, device=r.device)
        stats = {"episode/length": float(r.shape[0]), "episode/total_reward": float(r.sum(0).mean()),
                 "episode/return": float((r * disc[:, None]).sum(0).mean()),
                 "episode/fps": float(r.shape[0] / max(duration, 1e-6))}
        if self.writer is not None:
            for k, v in stats.items():
                self.writer.add_scalar(k, v, episode)
        logger.info("Episode %d mean score: %.2f", episode, stats["episode/total_reward"])
        self.last_stats = stats

    # evaluation.py:292-307
    def save_agent_model(self, identifier):
        try:
            return self.agent.save(filename=self.directory / "saved_models" / f"checkpoint-{identifier}.tar")
        except NotImplementedError:
            return None

    def close(self):
        if self.training:
            self.save_agent_model("final")
        if hasattr(self.env, "close"):
            self.env.close()
