"""BatchedEvaluation keeps the reference trainer's hook names and call order
(Evaluation.step evaluation.py:163-194, reset :372-376, run_episodes :139-161).
A recording fake env/agent (CPU, duck-typed) captures the trace."""
import pytest
import torch

from topotrafficrl_amd.agent import EgoAttentionNetwork
from topotrafficrl_amd.trainer import BatchedDQNAgent, BatchedEvaluation


class FakeEnv:
    def __init__(self, trace, E=3, horizon=4):
        self.trace, self.E, self.h, self.t = trace, E, horizon, 0

    def reset(self, seed=None):
        self.trace.append(("env.reset", seed))
        self.t = 0
        return torch.zeros(self.E, 15, 7), {}

    def step(self, action):
        self.trace.append(("env.step", tuple(action.tolist())))
        self.t += 1
        done = torch.zeros(self.E, dtype=torch.bool)
        trunc = torch.full((self.E,), self.t >= self.h)
        return torch.full((self.E, 15, 7), float(self.t)), torch.ones(self.E), done, trunc, {"speed": torch.ones(self.E)}

    def close(self):
        self.trace.append(("env.close",))


class FakeAgent:
    config = {"gamma": 0.5}

    def __init__(self, trace):
        self.trace = trace

    def plan(self, obs):
        self.trace.append(("agent.plan", float(obs[0, 0, 0])))
        return [torch.arange(obs.shape[0])]

    def record(self, s, a, r, s2, done, info):
        self.trace.append(("agent.record", float(s[0, 0, 0]), float(s2[0, 0, 0])))

    def seed(self, seed):
        self.trace.append(("agent.seed", seed))

    def reset(self):
        self.trace.append(("agent.reset",))

    def set_writer(self, w):
        self.trace.append(("agent.set_writer",))

    def save(self, filename):
        self.trace.append(("agent.save", str(filename).split("/")[-1]))
        return filename


def test_hook_order_matches_reference(tmp_path):
    trace = []
    cb = lambda ep, env, agent, tr, writer: trace.append(("callback", ep))  # noqa: E731
    ev = BatchedEvaluation(FakeEnv(trace), FakeAgent(trace), num_episodes=1, sim_seed=100, step_callback_fn=cb,
                           directory=str(tmp_path))
    ev.train()
    assert trace[0] == ("agent.set_writer",)
    assert trace[1:4] == [("env.reset", 100), ("agent.seed", 100), ("agent.reset",)]
    step = trace[4:8]
    assert [t[0] for t in step] == ["agent.plan", "env.step", "callback", "agent.record"]
    assert step[3][1:] == (0.0, 1.0)  # record(previous_observation, ..., next observation)
    assert sum(1 for t in trace if t[0] == "env.step") == 4
    assert trace[-2:] == [("agent.save", "checkpoint-final.tar"), ("env.close",)]
    assert ev.last_stats["episode/length"] == 4 and ev.last_stats["episode/return"] == 1 + 0.5 + 0.25 + 0.125


def test_dqn_agent_checkpoint_roundtrip(tmp_path):
    a = BatchedDQNAgent("cpu", seed=1)
    b = BatchedDQNAgent("cpu", seed=2)
    x = torch.rand(4, 15, 7)
    assert not torch.equal(a.policy.q_values(x), b.policy.q_values(x))
    a.save(tmp_path / "m.tar")
    b.load(tmp_path / "m.tar")
    assert torch.equal(a.policy.q_values(x), b.policy.q_values(x))


def test_ego_attention_masks_absent_rows():
    """Rows with presence < 0.5 must not influence Q (models.py:294-300 mask, -1e9 fill)."""
    net = EgoAttentionNetwork(5).reset(torch.Generator().manual_seed(0))
    g = torch.Generator().manual_seed(1)
    x = torch.rand(2, 15, 7, generator=g)
    x[:, :5, 0] = 1.0  # present rows (with every row masked the softmax is uniform over all 15)
    x[:, 5:, 0] = 0.0
    y = x.clone()
    y[:, 5:, 1:] = torch.rand(2, 10, 6, generator=g) * 9
    assert torch.allclose(net(x), net(y), atol=1e-6)


def test_evaluation_keys_exploration_on_the_env_shard():
    """BatchedEvaluation hands the env's global id offset (a data-parallel rank's shard,
    env_id_offset) to the agent's policy, whose fused epsilon-greedy draws are keyed on global env
    ids: shards of one seed explore independently (ttrl_ego_attention_act's env_offset)."""
    from topotrafficrl_amd.trainer import BatchedDQNAgent

    class ShardEnv:
        config = {"env_id_offset": 8192}

    agent = BatchedDQNAgent("cpu", n_actions=3)
    assert agent.policy.env_id_offset == 0
    BatchedEvaluation(ShardEnv(), agent, num_episodes=1, sim_seed=0)
    assert agent.policy.env_id_offset == 8192


def test_evaluation_keeps_an_explicit_agent_offset():
    """An offset given to the agent explicitly survives an env left at offset 0 (with a warning),
    and a different non-zero env offset is an error rather than a silent override."""
    from topotrafficrl_amd.trainer import BatchedDQNAgent

    class Env:
        def __init__(self, off):
            self.config = {"env_id_offset": off}

    agent = BatchedDQNAgent("cpu", n_actions=3, env_id_offset=4096)
    with pytest.warns(UserWarning):
        BatchedEvaluation(Env(0), agent, num_episodes=1, sim_seed=0)
    assert agent.policy.env_id_offset == 4096
    BatchedEvaluation(Env(4096), agent, num_episodes=1, sim_seed=0)
    assert agent.policy.env_id_offset == 4096
    with pytest.raises(ValueError):
        BatchedEvaluation(Env(8192), agent, num_episodes=1, sim_seed=0)
