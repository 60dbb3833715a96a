"""Batched DQN training on CPU: replay memory ring / sampling / n-step
collapse (memory.py:9-86), the double-DQN Bellman residual (pytorch.py:40-73), the optimizer
step with the +-1 gradient clamp (:32-38), the target sync cadence (abstract.py:95-100), and
the data-parallel gradient average across 2 gloo ranks."""
import copy
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
from torch import nn

from topotrafficrl_amd.agent import EgoAttentionNetwork
from topotrafficrl_amd.dqn import DQNLearner, ReplayMemory
from topotrafficrl_amd.trainer import BatchedDQNAgent


def test_memory_ring_overwrites_oldest_and_samples_stored_transitions():
    m = ReplayMemory(10, (2,), "cpu")
    for k in range(4):  # 4 pushes of 3 envs = 12 transitions into a ring of 10
        s = torch.full((3, 2), float(k * 3)) + torch.arange(3.0).view(3, 1)
        m.push(s, torch.arange(3), s[:, 0], s + 100, torch.zeros(3, dtype=torch.bool))
    assert len(m) == 10 and m.is_full()
    g = torch.Generator().manual_seed(0)
    s, a, r, s2, t = m.sample(10, g)
    assert sorted(r.tolist()) == [float(v) for v in range(2, 12)]  # 0 and 1 were overwritten
    assert torch.equal(s2, s + 100) and len(set(r.tolist())) == 10  # without replacement
    with pytest.raises(ValueError):
        m.sample(11, g)


def reference_collapse(transitions, gamma):
    """memory.py:63-82, verbatim semantics on python tuples."""
    state, action, cumulated_reward, next_state, done = transitions[0]
    discount = 1
    for transition in transitions[1:]:
        if done:
            break
        _, _, reward, next_state, done = transition
        discount *= gamma
        cumulated_reward += discount * reward
    return state, action, cumulated_reward, next_state, done


def test_n_step_collapse_follows_each_env():
    E, T, n, gamma = 3, 6, 3, 0.9
    m = ReplayMemory(100, (1,), "cpu", n_steps=n, gamma=gamma)
    g = torch.Generator().manual_seed(1)
    traj = {e: [] for e in range(E)}
    for t in range(T):
        s = torch.tensor([[10.0 * e + t] for e in range(E)])
        r = torch.rand(E, generator=g)
        d = torch.rand(E, generator=g) < 0.25
        m.push(s, torch.zeros(E, dtype=torch.long), r, s + 1, d)
        for e in range(E):
            traj[e].append((float(s[e, 0]), 0, float(r[e]), float(s[e, 0] + 1), bool(d[e])))
    s, a, r, s2, t = m.sample(E * T, torch.Generator().manual_seed(2))
    for k in range(E * T):
        e, step = int(s[k, 0]) // 10, int(s[k, 0]) % 10
        ref = reference_collapse(traj[e][step:step + n], gamma)
        assert abs(float(r[k]) - ref[2]) < 1e-6 and float(s2[k, 0]) == ref[3] and bool(t[k]) == ref[4]


class Lin(nn.Module):
    def __init__(self):
        super().__init__()
        self.f = nn.Linear(2, 3)

    def forward(self, x):
        return self.f(x)


def test_bellman_residual_double_and_plain():
    torch.manual_seed(0)
    L = DQNLearner(Lin(), (2,), "cpu", {"gamma": 0.5, "batch_size": 4})
    with torch.no_grad():
        L.target_net.f.weight.add_(0.3)
    s, s2 = torch.randn(4, 2), torch.randn(4, 2)
    a, r = torch.tensor([0, 1, 2, 1]), torch.randn(4)
    t = torch.tensor([False, True, False, False])
    loss, target = L.compute_bellman_residual((s, a, r, s2, t))
    best = L.value_net(s2).argmax(1)
    nv = L.target_net(s2).gather(1, best[:, None]).squeeze(1).detach()
    ref = r + 0.5 * torch.where(t, torch.zeros(4), nv)
    assert torch.allclose(target, ref)
    q = L.value_net(s).gather(1, a[:, None]).squeeze(1)
    assert torch.allclose(loss, ((q - ref) ** 2).mean())
    L.config["double"] = False
    _, target = L.compute_bellman_residual((s, a, r, s2, t))
    ref = r + 0.5 * torch.where(t, torch.zeros(4), L.target_net(s2).max(1).values)
    assert torch.allclose(target, ref)


def test_optimizer_step_clamps_and_target_syncs_on_cadence():
    torch.manual_seed(1)
    L = DQNLearner(Lin(), (2,), "cpu", {"target_update": 3, "batch_size": 8, "optimizer": {"lr": 1e-2}})
    before = copy.deepcopy(L.value_net.state_dict())
    for k in range(5):
        L.record(torch.randn(4, 2) * 100, torch.randint(0, 3, (4,)), torch.randn(4) * 1e3, torch.randn(4, 2),
                 torch.zeros(4, dtype=torch.bool))
    assert L.steps == 4  # updates start once 8 transitions are stored (pushes 2..5)
    for p in L.value_net.parameters():
        assert p.grad.abs().max() <= 1.0  # grad.clamp_(-1, 1)
    assert not torch.equal(before["f.weight"], L.value_net.state_dict()["f.weight"])
    # target synced at step 3, not at step 4
    assert not torch.equal(L.target_net.f.weight, L.value_net.f.weight)


def test_q_learning_fits_a_fixed_target():
    torch.manual_seed(2)
    L = DQNLearner(Lin(), (2,), "cpu", {"batch_size": 32, "memory_capacity": 64, "gamma": 0.0,
                                        "optimizer": {"lr": 5e-2}})
    s = torch.randn(64, 2)
    a = torch.randint(0, 3, (64,))
    r = s[:, 0] * 2 - s[:, 1] + a.float()
    L.memory.push(s, a, r, s, torch.ones(64, dtype=torch.bool))
    first = None
    for _ in range(300):
        loss, _ = L.compute_bellman_residual(L.sample_minibatch())
        L.step_optimizer(loss)
        first = first if first is not None else float(loss)
    assert float(loss) < 0.05 * first


def test_agent_uses_final_observation_for_finished_envs():
    agent = BatchedDQNAgent("cpu", config={"batch_size": 2, "memory_capacity": 8})
    s, s_new, s_fin = torch.zeros(2, 15, 7), torch.ones(2, 15, 7), torch.full((2, 15, 7), 5.0)
    done = torch.tensor([True, False])
    agent.record(s, torch.tensor([0, 1]), torch.zeros(2), s_new, done,
                 {"final_observation": s_fin, "final_mask": done})
    mem = agent.learner.memory
    assert float(mem.next_state[0, 0, 0]) == 5.0 and float(mem.next_state[1, 0, 0]) == 1.0


def _port():
    so = socket.socket()
    so.bind(("127.0.0.1", 0))
    p = so.getsockname()[1]
    so.close()
    return p


def _dp_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)
    net = EgoAttentionNetwork(5).reset(torch.Generator().manual_seed(0))
    L = DQNLearner(net, (15, 7), "cpu", {"batch_size": 16, "memory_capacity": 64}, seed=rank)
    g = torch.Generator().manual_seed(100 + rank)  # each rank its own envs / data
    L.memory.push(torch.rand(32, 15, 7, generator=g), torch.randint(0, 5, (32,), generator=g),
                  torch.rand(32, generator=g), torch.rand(32, 15, 7, generator=g), torch.zeros(32, dtype=torch.bool))
    batch = L.sample_minibatch()
    loss, _ = L.compute_bellman_residual(batch)
    L.step_optimizer(loss)
    torch.save({"params": [p.detach().clone() for p in net.parameters()], "batch": batch}, f"{out}/r{rank}.pt")
    dist.destroy_process_group()


def test_data_parallel_gradient_average_keeps_ranks_identical(tmp_path):
    mp.spawn(_dp_worker, args=(2, _port(), str(tmp_path)), nprocs=2, join=True)
    r0 = torch.load(tmp_path / "r0.pt", weights_only=True)
    r1 = torch.load(tmp_path / "r1.pt", weights_only=True)
    for a, b in zip(r0["params"], r1["params"]):
        assert torch.equal(a, b)
    # equals one process stepping on the mean of the two ranks' gradients
    net = EgoAttentionNetwork(5).reset(torch.Generator().manual_seed(0))
    L = DQNLearner(net, (15, 7), "cpu", {"batch_size": 16, "memory_capacity": 64})
    grads = []
    for r in (r0, r1):
        L.optimizer.zero_grad()
        loss, _ = L.compute_bellman_residual(tuple(r["batch"]))
        loss.backward()
        grads.append([p.grad.clone() for p in net.parameters()])
    L.optimizer.zero_grad()
    for p, g0, g1 in zip(net.parameters(), *grads):
        p.grad = ((g0 + g1) / 2).clamp(-1, 1)
    L.optimizer.step()
    for a, p in zip(r0["params"], net.parameters()):
        assert torch.allclose(a, p.detach(), atol=1e-6)
