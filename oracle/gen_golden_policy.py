"""Golden-vector generator for the policy (config 5) and the DQN update — TEST INFRASTRUCTURE,
runs only in the build container.

It imports the reference agent package ``ttrl_agent`` from ``/root/reference`` and runs its own
code: ``EgoAttentionNetwork.forward`` (models.py:237-312, EgoAttention :157-194, attention
:370-388, MultiLayerPerceptron :50-76) built by ``model_factory`` from the reference's JSON
configs (scripts/configs/IntersectionEnv/agents/DQNAgent/ego_attention*.json over baseline.json),
``DQNAgent.compute_bellman_residual`` / ``step_optimizer`` (deep_q_network/pytorch.py:32-73),
``AbstractDQNAgent.update_target_network`` (deep_q_network/abstract.py:95-100),
``ReplayMemory.collapse_n_steps`` (common/memory.py:63-82) and ``EpsilonGreedy.update``
(exploration/epsilon_greedy.py:37-48).  Only the resulting ``tests/golden/policy_*.npz`` /
``dqn_*.npz`` data files are committed; nothing from the reference travels to the GPU box.

Stand-ins: gymnasium is absent from the image and the agent modules import
it only for type names — ``gymnasium.spaces.{Box, Discrete, Tuple}`` in isinstance checks
(models.py:404-428, epsilon_greedy.py:16-19, deep_q_network/abstract.py:14),
``gymnasium.core.Env`` (configuration.py:2, imported, unused) and ``gymnasium.utils.seeding``
(exploration seeding, unused by the fixtures).  The stand-ins below provide exactly those names
and carry no arithmetic.  The exploration modules import ``rl_agents.*``; that name is aliased
to ``ttrl_agent`` (§8(c).3).

Usage:  PYTHONDONTWRITEBYTECODE=1 python oracle/gen_golden_policy.py
"""
from __future__ import annotations

import copy
import json
import os
import sys
import types

import numpy as np
import torch

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "..", "tests", "golden")
CFG_DIR = os.path.join(REF, "scripts", "configs", "IntersectionEnv", "agents", "DQNAgent")


def _gymnasium_stand_in():
    """Type names only (see the module docstring)."""
    gym = types.ModuleType("gymnasium")
    spaces = types.ModuleType("gymnasium.spaces")

    class Space:
        pass

    class Box(Space):
        def __init__(self, low, high, shape, dtype=np.float32):
            self.low, self.high, self.shape, self.dtype = low, high, tuple(shape), dtype

    class Discrete(Space):
        def __init__(self, n):
            self.n = int(n)

    class Tuple(Space):
        def __init__(self, spaces_):
            self.spaces = tuple(spaces_)

    spaces.Space, spaces.Box, spaces.Discrete, spaces.Tuple = Space, Box, Discrete, Tuple
    core = types.ModuleType("gymnasium.core")

    class Env:
        pass

    core.Env = Env
    utils = types.ModuleType("gymnasium.utils")
    seeding = types.ModuleType("gymnasium.utils.seeding")

    def np_random(seed=None):
        ss = np.random.SeedSequence(seed)
        return np.random.Generator(np.random.PCG64(ss)), ss.entropy

    seeding.np_random = np_random
    utils.seeding = seeding
    gym.spaces, gym.core, gym.utils, gym.Env = spaces, core, utils, Env
    for name, mod in (("gymnasium", gym), ("gymnasium.spaces", spaces), ("gymnasium.core", core),
                      ("gymnasium.utils", utils), ("gymnasium.utils.seeding", seeding)):
        sys.modules[name] = mod
    return spaces


def _import_reference():
    sys.dont_write_bytecode = True
    spaces = _gymnasium_stand_in()
    sys.path.insert(0, REF)
    import ttrl_agent
    import ttrl_agent.configuration
    sys.modules["rl_agents"] = ttrl_agent  # §8(c).3: the exploration modules import rl_agents.*
    sys.modules["rl_agents.configuration"] = ttrl_agent.configuration
    ttrl_agent.configuration  # noqa: B018
    from ttrl_agent.agents.common import memory, models
    import ttrl_agent.agents.common.exploration.abstract as expl_abstract
    sys.modules["rl_agents.agents"] = sys.modules["ttrl_agent.agents"]
    sys.modules["rl_agents.agents.common"] = sys.modules["ttrl_agent.agents.common"]
    sys.modules["rl_agents.agents.common.exploration"] = sys.modules["ttrl_agent.agents.common.exploration"]
    sys.modules["rl_agents.agents.common.exploration.abstract"] = expl_abstract
    from ttrl_agent.agents.common.exploration import epsilon_greedy
    from ttrl_agent.agents.deep_q_network import pytorch as dqn
    return types.SimpleNamespace(spaces=spaces, models=models, memory=memory, dqn=dqn,
                                 epsilon_greedy=epsilon_greedy)


R = _import_reference()


def agent_config(name: str) -> dict:
    """Resolve the reference's base_config chain (factory.py:44-56) for one agent JSON."""
    with open(os.path.join(CFG_DIR, name)) as f:
        cfg = json.load(f)
    if "base_config" in cfg:
        base = agent_config(os.path.basename(cfg.pop("base_config")))
        R.models.Configurable.rec_update(base, cfg)
        cfg = base
    return cfg


class _Env:
    """What size_model_config / AbstractDQNAgent read: the spaces of the Kinematics 15x7
    observation and DiscreteMetaAction (n actions)."""

    def __init__(self, n_actions: int, shape=(15, 7)):
        self.observation_space = R.spaces.Box(-np.inf, np.inf, shape, np.float32)
        self.action_space = R.spaces.Discrete(n_actions)


def build_network(name: str, n_actions: int, seed: int, bias_scale: float):
    cfg = agent_config(name)["model"]
    R.models.size_model_config(_Env(n_actions), cfg)
    torch.manual_seed(seed)
    net = R.models.model_factory(cfg)
    net.reset()  # BaseModule._init_weights: xavier uniform, zero biases (models.py:24-33)
    if bias_scale:
        g = torch.Generator().manual_seed(seed + 1000)
        with torch.no_grad():
            for n, p in net.named_parameters():
                if n.endswith("bias"):
                    p.copy_((torch.rand(p.shape, generator=g) * 2 - 1) * bias_scale)
    return net.eval(), cfg


def policy_inputs(seed: int = 7) -> np.ndarray:
    """[1000, 15, 7] float32: real Kinematics 15x7 observations from the committed goldens
    (intersection episodes and highway kin15), the same rows with vehicles masked out
    (presence 0), fully masked rows (the ego's presence 0 too) and random rows."""
    rows = []
    for i in range(6):
        with np.load(os.path.join(OUT, f"ix_s{i}.npz")) as z:
            rows.append(z["obs0"][None])
            rows.append(z["obs"])
    for n in (8, 32, 64, 128):
        for s in range(3):
            with np.load(os.path.join(OUT, f"highway_n{n}_s{s}.npz")) as z:
                k = z["kin15"].copy()
                k[..., 0] = (k[..., 0] != 0).astype(np.float32)  # highway kin15 has no presence feature:
                rows.append(k)                                    # feature 0 becomes one for filled rows
    real = np.concatenate(rows).astype(np.float32)
    rng = np.random.default_rng(seed)
    masked = real.copy()
    drop = rng.random(masked.shape[:2]) < 0.4
    drop[:, 0] = False
    masked[..., 0] = np.where(drop, 0.0, masked[..., 0])
    full = real[: 16].copy()
    full[..., 0] = 0.0  # every entity absent, the ego included
    n_rand = 1000 - len(real) - len(masked) - len(full)
    rand = rng.uniform(-1, 1, size=(n_rand, 15, 7)).astype(np.float32)
    rand[..., 0] = (rng.random((n_rand, 15)) < 0.6).astype(np.float32)
    x = np.concatenate([real, masked, full, rand])[:1000]
    perm = rng.permutation(len(x))
    return np.ascontiguousarray(x[perm])


def gen_policy():
    x = policy_inputs()
    variants = [  # (file, agent json, actions, weight seed, bias scale)
        ("policy_2h_a5", "ego_attention_2h.json", 5, 11, 0.1),
        ("policy_2h_a3", "ego_attention_2h.json", 3, 12, 0.0),
        ("policy_1h_a3", "ego_attention.json", 3, 13, 0.05),
    ]
    for fname, cfgname, n_actions, seed, bias in variants:
        net, cfg = build_network(cfgname, n_actions, seed, bias)
        out = {"x": x, "heads": np.int32(cfg["attention_layer"]["heads"]), "n_actions": np.int32(n_actions)}
        for k, v in net.state_dict().items():
            out["w/" + k] = v.numpy()
        with torch.no_grad():
            for b in (1, 37, 1000):
                xb = torch.from_numpy(x[:b])
                out[f"q_b{b}"] = net(xb).numpy()
                out[f"att_b{b}"] = net.get_attention_matrix(xb).numpy()
        np.savez_compressed(os.path.join(OUT, fname + ".npz"), **out)
        print(fname, "params", sum(p.numel() for p in net.parameters()))


def gen_dqn():
    """DQNAgent updates: Bellman residual (double and plain), ±1 gradient clamp, Adam, target
    sync every 2 updates, over 4 successive minibatches (pytorch.py:32-73, abstract.py:95-100)."""
    x = policy_inputs(seed=21)
    rng = np.random.default_rng(5)
    for double in (True, False):
        cfg = agent_config("ego_attention_2h.json")
        cfg.update(device="cpu", double=double, target_update=2)
        torch.manual_seed(31 if double else 32)
        agent = R.dqn.DQNAgent(_Env(5), cfg)
        out = {"double": np.int32(double), "gamma": np.float64(agent.config["gamma"]),
               "lr": np.float64(agent.config["optimizer"]["lr"]), "target_update": np.int32(2)}
        for k, v in agent.value_net.state_dict().items():
            out["w0/" + k] = v.numpy().copy()
        B = agent.config["batch_size"]
        for step in range(4):
            idx = rng.choice(len(x), size=B, replace=False)
            nidx = rng.choice(len(x), size=B, replace=False)
            s, s2 = x[idx], x[nidx]
            a = rng.integers(0, 5, size=B)
            r = rng.uniform(0, 1, size=B)
            t = rng.random(B) < 0.25
            batch = R.memory.Transition(tuple(s), tuple(int(v) for v in a), tuple(float(v) for v in r),
                                        tuple(s2), tuple(bool(v) for v in t), tuple({} for _ in range(B)))
            loss, target, _ = agent.compute_bellman_residual(batch)
            agent.step_optimizer(loss)
            agent.update_target_network()
            out[f"s{step}/state"], out[f"s{step}/next_state"] = s, s2
            out[f"s{step}/action"], out[f"s{step}/reward"] = a.astype(np.int64), r.astype(np.float32)
            out[f"s{step}/terminal"] = t
            out[f"s{step}/loss"] = np.float32(loss.item())
            out[f"s{step}/target"] = target.numpy()
            for k, v in agent.value_net.state_dict().items():
                out[f"s{step}/w/" + k] = v.numpy().copy()
            for k, v in agent.target_net.state_dict().items():
                out[f"s{step}/tw/" + k] = v.numpy().copy()
        np.savez_compressed(os.path.join(OUT, f"dqn_{'double' if double else 'plain'}.npz"), **out)
        print("dqn", double, [float(out[f's{i}/loss']) for i in range(4)])


def gen_memory_and_exploration():
    """ReplayMemory.collapse_n_steps over trajectories with terminals (memory.py:63-82), and the
    EpsilonGreedy schedule / greedy action (epsilon_greedy.py:37-48)."""
    rng = np.random.default_rng(9)
    out = {}
    for n_steps in (1, 2, 3, 5):
        mem = R.memory.ReplayMemory({"memory_capacity": 64, "n_steps": n_steps, "gamma": 0.95})
        T = 40
        states = rng.integers(0, 1000, size=T + 1)
        actions = rng.integers(0, 5, size=T)
        rewards = rng.uniform(0, 1, size=T)
        dones = rng.random(T) < 0.15
        for i in range(T):
            mem.push(int(states[i]), int(actions[i]), float(rewards[i]), int(states[i + 1]), bool(dones[i]), {})
        coll = [mem.collapse_n_steps(mem.memory[i:i + n_steps]) for i in range(T)]
        out[f"n{n_steps}/state"], out[f"n{n_steps}/action"] = states, actions
        out[f"n{n_steps}/reward"], out[f"n{n_steps}/done"] = rewards, dones
        out[f"n{n_steps}/c_state"] = np.array([c[0] for c in coll])
        out[f"n{n_steps}/c_action"] = np.array([c[1] for c in coll])
        out[f"n{n_steps}/c_reward"] = np.array([c[2] for c in coll])
        out[f"n{n_steps}/c_next_state"] = np.array([c[3] for c in coll])
        out[f"n{n_steps}/c_done"] = np.array([c[4] for c in coll])
    cfg = copy.deepcopy(agent_config("baseline.json")["exploration"])
    eg = R.epsilon_greedy.EpsilonGreedy(R.spaces.Discrete(5), cfg)
    times = np.array([0, 1, 10, 100, 1000, 15000, 50000, 200000])
    eps, greedy = [], []
    vals = rng.normal(size=(len(times), 5))
    for t, v in zip(times, vals):
        eg.set_time(int(t))
        eg.update(v)
        eps.append(eg.epsilon)
        greedy.append(eg.optimal_action)
    out["eps/time"], out["eps/values"] = times, vals
    out["eps/epsilon"], out["eps/greedy"] = np.array(eps), np.array(greedy)
    out["eps/tau"] = np.float64(cfg["tau"])
    out["eps/temperature"] = np.float64(cfg["temperature"])
    out["eps/final_temperature"] = np.float64(eg.config["final_temperature"])
    np.savez_compressed(os.path.join(OUT, "dqn_memory.npz"), **out)
    print("memory / exploration fixtures written")


if __name__ == "__main__":
    torch.set_num_threads(1)  # deterministic CPU reductions for the fixtures
    gen_policy()
    gen_dqn()
    gen_memory_and_exploration()
