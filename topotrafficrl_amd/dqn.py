"""Batched DQN training in the loop: replay memory in HBM, the
(double-)DQN Bellman residual, Adam, target-network sync and, across GPUs, one gradient
all-reduce per update over RCCL.

Restates ttrl_agent/agents:
  * ReplayMemory             common/memory.py:9-86 (ring buffer, n-step collapse :63-82)
  * AbstractDQNAgent.record  deep_q_network/abstract.py:37-63 (push, sample, residual, step, target)
  * DQNAgent                 deep_q_network/pytorch.py:14-73 (step_optimizer with grad clamp +-1,
                             compute_bellman_residual with the double-DQN target)
  * loss / optimizer factory common/optimizers.py:132-152

Batched on purpose: one ``record`` call carries one transition per env ([E, ...] device
tensors), written into the ring in one copy; ``updates_per_record`` gradient steps follow it
(the reference does one per transition: a batch of E transitions would otherwise mean E
updates).  Sampling is uniform without replacement, like ``random.sample``, drawn on the
device from the agent's generator.  With ``torch.distributed`` initialised every rank keeps
its own memory (its own envs) and the gradients are averaged across ranks before the
clamp and the Adam step, so all ranks hold identical networks (data-parallel DQN).
"""
from __future__ import annotations

import copy

import torch
import torch.distributed as dist
from torch.nn import functional as F

DEFAULT_CONFIG = {  # deep_q_network/abstract.py:23-37 with scripts/configs/.../DQNAgent/baseline.json
    "optimizer": {"type": "ADAM", "lr": 5e-4, "weight_decay": 0, "k": 5},
    "loss_function": "l2",
    "memory_capacity": 15000,
    "batch_size": 64,
    "gamma": 0.95,
    "n_steps": 1,
    "target_update": 512,
    "double": True,
    "updates_per_record": 1,
}


def loss_function_factory(name: str):
    """optimizers.py:132-142"""
    table = {"l2": F.mse_loss, "l1": F.l1_loss, "smooth_l1": F.smooth_l1_loss, "bce": F.binary_cross_entropy}
    if name not in table:
        raise ValueError(f"Unknown loss function : {name}")
    return table[name]


def optimizer_factory(optimizer_type: str, params, lr=None, weight_decay=None, k=None, **kwargs):
    """optimizers.py:145-152 (RANGER is not on the hot path)."""
    if optimizer_type == "ADAM":
        return torch.optim.Adam(params=params, lr=lr, weight_decay=weight_decay)
    if optimizer_type == "RMS_PROP":
        return torch.optim.RMSprop(params=params, weight_decay=weight_decay)
    raise ValueError(f"Unknown optimizer type: {optimizer_type}")


class ReplayMemory:
    """Device ring buffer of transitions (memory.py:9-86).  Transitions of one ``push`` are
    consecutive; n-step collapse follows each sampled transition's own env, which sits
    ``stride`` (= envs per push) slots later in the ring."""

    def __init__(self, capacity: int, obs_shape, device, n_steps: int = 1, gamma: float = 0.99):
        self.capacity, self.device = int(capacity), torch.device(device)
        self.n_steps, self.gamma = int(n_steps), float(gamma)
        self.state = torch.zeros((self.capacity, *obs_shape), dtype=torch.float32, device=self.device)
        self.next_state = torch.zeros_like(self.state)
        self.action = torch.zeros(self.capacity, dtype=torch.int64, device=self.device)
        self.reward = torch.zeros(self.capacity, dtype=torch.float32, device=self.device)
        self.terminal = torch.zeros(self.capacity, dtype=torch.bool, device=self.device)
        self.size, self.position, self.stride = 0, 0, None

    def __len__(self):
        return self.size

    def is_full(self):
        return self.size == self.capacity

    def is_empty(self):
        return self.size == 0

    def push(self, state, action, reward, next_state, terminal) -> None:
        """Store one transition per env; the oldest are overwritten once full (memory.py:29-38)."""
        b = state.shape[0]
        if b > self.capacity:
            raise ValueError("more envs than memory capacity")
        if self.stride is None:
            self.stride = b
        elif self.n_steps > 1 and b != self.stride:
            raise ValueError("n-step memory needs the same number of envs on every push")
        idx = (self.position + torch.arange(b, device=self.device)) % self.capacity
        self.state[idx] = state.to(self.device, torch.float32)
        self.next_state[idx] = next_state.to(self.device, torch.float32)
        self.action[idx] = action.to(self.device, torch.int64).reshape(-1)
        self.reward[idx] = reward.to(self.device, torch.float32).reshape(-1)
        self.terminal[idx] = terminal.to(self.device, torch.bool).reshape(-1)
        self.position = (self.position + b) % self.capacity
        self.size = min(self.size + b, self.capacity)

    def sample(self, batch_size: int, generator: torch.Generator | None = None):
        """``random.sample`` of transitions (without replacement), n-step collapsed
        (memory.py:63-82): returns (state, action, reward, next_state, terminal) tensors."""
        if batch_size > self.size:
            raise ValueError("not enough transitions")
        pick = torch.randperm(self.size, device=self.device, generator=generator)[:batch_size]
        return self.gather(pick)

    def gather(self, pick: torch.Tensor):
        """The n-step collapsed transitions starting at ages ``pick`` (0 = the oldest stored
        transition): ``collapse_n_steps`` (memory.py:63-82) of ``memory[i:i + n_steps]``."""
        oldest = (self.position - self.size) % self.capacity
        idx = (oldest + pick) % self.capacity
        s, a = self.state[idx], self.action[idx]
        r, s2, t = self.reward[idx].clone(), self.next_state[idx].clone(), self.terminal[idx].clone()
        if self.n_steps > 1:
            disc = torch.ones_like(r)
            pos = pick.clone()
            for _ in range(1, self.n_steps):
                pos = pos + self.stride
                live = (~t) & (pos < self.size)  # stop at a terminal state or the end of the trajectory
                j = (oldest + pos.clamp(max=self.size - 1)) % self.capacity
                disc = torch.where(live, disc * self.gamma, disc)
                r = torch.where(live, r + disc * self.reward[j], r)
                s2 = torch.where(live.view(-1, *[1] * (s2.dim() - 1)), self.next_state[j], s2)
                t = torch.where(live, self.terminal[j], t)
        return s, a, r, s2, t


class DQNLearner:
    """The learning side of DQNAgent for a batched value network (pytorch.py:14-73,
    abstract.py:37-63, 95-100)."""

    def __init__(self, value_net: torch.nn.Module, obs_shape, device, config: dict | None = None, seed: int = 0):
        self.config = copy.deepcopy(DEFAULT_CONFIG)
        for k, v in (config or {}).items():
            self.config[k] = {**self.config[k], **v} if isinstance(v, dict) and isinstance(self.config.get(k), dict) \
                else v
        c = self.config
        self.device = torch.device(device)
        self.value_net = value_net
        self.target_net = copy.deepcopy(value_net).eval()
        self.target_net.load_state_dict(self.value_net.state_dict())
        for p in self.target_net.parameters():
            p.requires_grad_(False)
        self.loss_function = loss_function_factory(c["loss_function"])
        self.optimizer = optimizer_factory(c["optimizer"]["type"], self.value_net.parameters(), **c["optimizer"])
        self.memory = ReplayMemory(c["memory_capacity"], obs_shape, self.device, c["n_steps"], c["gamma"])
        self.gen = torch.Generator(device=self.device)
        self.gen.manual_seed(int(seed))
        self.steps = 0
        self.last_loss = None

    # abstract.py:37-63
    def record(self, state, action, reward, next_state, done) -> torch.Tensor | None:
        self.memory.push(state, action, reward, next_state, done)
        loss = None
        for _ in range(int(self.config["updates_per_record"])):
            batch = self.sample_minibatch()
            if batch is None:
                break
            loss, _ = self.compute_bellman_residual(batch)
            self.step_optimizer(loss)
            self.update_target_network()
        self.last_loss = loss.detach() if loss is not None else self.last_loss
        return loss

    # abstract.py:83-87
    def sample_minibatch(self):
        if len(self.memory) < self.config["batch_size"]:
            return None
        return self.memory.sample(self.config["batch_size"], self.gen)

    # pytorch.py:40-73
    def compute_bellman_residual(self, batch, target_state_action_value=None):
        state, action, reward, next_state, terminal = batch
        state_action_values = self.value_net(state).gather(1, action.unsqueeze(1)).squeeze(1)
        if target_state_action_value is None:
            with torch.no_grad():
                next_state_values = torch.zeros(reward.shape, device=self.device)
                if self.config["double"]:
                    _, best_actions = self.value_net(next_state).max(1)
                    best_values = self.target_net(next_state).gather(1, best_actions.unsqueeze(1)).squeeze(1)
                else:
                    best_values, _ = self.target_net(next_state).max(1)
                next_state_values = torch.where(terminal, next_state_values, best_values)
                target_state_action_value = reward + self.config["gamma"] * next_state_values
        loss = self.loss_function(state_action_values, target_state_action_value)
        return loss, target_state_action_value

    # pytorch.py:32-38, plus the data-parallel gradient average (one RCCL bucket)
    def step_optimizer(self, loss: torch.Tensor) -> None:
        self.optimizer.zero_grad()
        loss.backward()
        params = [p for p in self.value_net.parameters() if p.grad is not None]
        if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
            flat = torch.cat([p.grad.reshape(-1) for p in params])
            dist.all_reduce(flat)
            flat /= dist.get_world_size()
            off = 0
            for p in params:
                n = p.grad.numel()
                p.grad.copy_(flat[off:off + n].view_as(p.grad))
                off += n
        for p in params:
            p.grad.data.clamp_(-1, 1)
        self.optimizer.step()

    # abstract.py:95-100
    def update_target_network(self) -> None:
        self.steps += 1
        if self.steps % self.config["target_update"] == 0:
            self.target_net.load_state_dict(self.value_net.state_dict())
