"""Config 5 (policy in the loop) and the DQN update, pinned to fixtures from the reference's own
code (oracle/gen_golden_policy.py runs ttrl_agent's EgoAttentionNetwork, DQNAgent,
ReplayMemory and EpsilonGreedy):

* EgoAttentionNetwork.forward      models.py:237-312, EgoAttention :157-194, attention :370-388
* compute_bellman_residual / step_optimizer / update_target_network
                                   deep_q_network/pytorch.py:32-73, abstract.py:95-100
* ReplayMemory.collapse_n_steps    common/memory.py:63-82
* EpsilonGreedy.update             exploration/epsilon_greedy.py:37-48

Tolerances: the torch restatement on the CPU against the reference forward: rtol 1e-5,
atol 1e-6 (same float32 operations, different summation order in the attention).  The fused
HIP forward (ttrl_ego_attention_q): rtol 1e-4, atol 1e-5 on Q-values (float32, MFMA and
online softmax).  DQN updates: loss / targets to 1e-5 relative; weights after each Adam step
to 1e-6 absolute (one Adam step moves a weight by at most lr = 5e-4).
"""
import copy
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN, load_golden
from topotrafficrl_amd.agent import EGO_ATTENTION_2H, EgoAttentionNetwork, EgoAttentionPolicy
from topotrafficrl_amd.dqn import DQNLearner, ReplayMemory

POLICY = ["policy_2h_a5", "policy_2h_a3", "policy_1h_a3"]


def _network(z, device="cpu"):
    cfg = copy.deepcopy(EGO_ATTENTION_2H)
    cfg["attention_layer"]["heads"] = int(z["heads"])
    net = EgoAttentionNetwork(int(z["n_actions"]), cfg)
    sd = {k[2:]: torch.from_numpy(v) for k, v in z.items() if k.startswith("w/")}
    net.load_state_dict(sd, strict=True)
    return net.to(device).eval()


def _state_dict(z, prefix):
    return {k[len(prefix):]: torch.from_numpy(v) for k, v in z.items() if k.startswith(prefix)}


@pytest.mark.parametrize("name", POLICY)
def test_torch_forward_matches_reference_network(name):
    z = load_golden(os.path.join(GOLDEN, name + ".npz"))
    net = _network(z)
    assert sum(p.numel() for p in net.parameters()) == sum(v.size for k, v in z.items() if k.startswith("w/"))
    with torch.no_grad():
        for b in (1, 37, 1000):
            x = torch.from_numpy(z["x"][:b])
            q = net(x).numpy()
            np.testing.assert_allclose(q, z[f"q_b{b}"], rtol=1e-5, atol=1e-6)
            ego, others = x[:, 0:1], x[:, 1:]
            mask = x[:, :, 0:1] < 0.5
            _, att = net.attention_layer(net.ego_embedding(ego), net.others_embedding(others), mask)
            np.testing.assert_allclose(att.numpy(), z[f"att_b{b}"], rtol=1e-5, atol=1e-6)


def test_policy_fixtures_cover_masks():
    z = load_golden(os.path.join(GOLDEN, "policy_2h_a5.npz"))
    pres = z["x"][..., 0]
    assert (pres.sum(1) == 0).sum() >= 10  # fully masked envs (uniform softmax over -1e9 scores)
    assert ((pres[:, 0] == 1) & (pres[:, 1:].sum(1) < 14) & (pres[:, 1:].sum(1) > 0)).sum() >= 100


@pytest.mark.gpu
@pytest.mark.parametrize("name", POLICY)
def test_fused_hip_forward_matches_reference_network(name, hip_device):
    z = load_golden(os.path.join(GOLDEN, name + ".npz"))
    net = _network(z, hip_device)
    for b in (1, 37, 1000):
        x = torch.from_numpy(z["x"][:b]).to(hip_device)
        q = net.fused_q(x).cpu().numpy()
        np.testing.assert_allclose(q, z[f"q_b{b}"], rtol=1e-4, atol=1e-5)
        with torch.no_grad():
            qt = net(x).cpu().numpy()
        np.testing.assert_allclose(qt, z[f"q_b{b}"], rtol=1e-4, atol=1e-5)
        # greedy actions agree wherever the reference's top two Q-values are apart
        ref = z[f"q_b{b}"]
        srt = np.sort(ref, axis=1)
        clear = (srt[:, -1] - srt[:, -2]) > 1e-4
        assert (q.argmax(1)[clear] == ref.argmax(1)[clear]).all()


def test_acting_steps_the_exploration_time_first():
    """AbstractDQNAgent.act (dqn/abstract.py:77-83) steps EpsilonGreedy.time before update: the
    k-th act of a fresh agent acts with epsilon(k); the schedule at the fixture's times."""
    z = load_golden(os.path.join(GOLDEN, "dqn_memory.npz"))
    pol = EgoAttentionPolicy("cpu", tau=float(z["eps/tau"]), temperature=float(z["eps/temperature"]),
                             final_temperature=float(z["eps/final_temperature"]), fused=False)
    x = torch.from_numpy(load_golden(os.path.join(GOLDEN, "policy_2h_a5.npz"))["x"][:8])
    for t, e in zip(z["eps/time"], z["eps/epsilon"]):
        if t == 0:
            continue  # no act runs at time 0: the first act is at time 1
        pol.time = int(t) - 1
        pol.act(x)
        assert pol.time == int(t) and abs(pol.last_epsilon - e) <= 1e-15


@pytest.mark.gpu
def test_fused_epsilon_greedy(hip_device):
    """The epsilon-greedy draw fused into the forward launch (ttrl::ego_attention_act):
    epsilon 0 is the reference network's argmax (where its top two Q-values are apart), epsilon 1
    is uniform over the actions (chi-square), epsilon 0.3 leaves the greedy action with probability
    0.3 (1 - 1/A); draws are a pure function of (seed, env, step); Q equals the plain forward."""
    from topotrafficrl_amd import ops
    z = load_golden(os.path.join(GOLDEN, "policy_2h_a5.npz"))
    net = _network(z, hip_device)
    w, A = net.packed_weights(), int(z["n_actions"])
    x = torch.from_numpy(z["x"][:1000]).to(hip_device)
    a0, q0 = ops.T.ego_attention_act(x, w, 2, A, 0.0, 3, 1)
    assert torch.equal(q0, net.fused_q(x))
    ref = z["q_b1000"]
    srt = np.sort(ref, axis=1)
    clear = (srt[:, -1] - srt[:, -2]) > 1e-4
    assert (a0.cpu().numpy()[clear] == ref.argmax(1)[clear]).all()
    assert torch.equal(a0, q0.argmax(1))  # first maximum, as np.argmax
    big = x.repeat(8, 1, 1)  # 8000 envs
    counts = np.zeros(A)
    for step in range(5):
        a1, _ = ops.T.ego_attention_act(big, w, 2, A, 1.0, 3, step)
        counts += np.bincount(a1.cpu().numpy(), minlength=A)
    n = counts.sum()
    chi2 = float(((counts - n / A) ** 2 / (n / A)).sum())
    assert chi2 < 20.5, (counts, chi2)  # p = 0.0004 at 4 degrees of freedom
    greedy = q0.argmax(1).repeat(8)
    moved = 0
    for step in range(5):
        a3, _ = ops.T.ego_attention_act(big, w, 2, A, 0.3, 3, step)
        moved += int((a3 != greedy).sum())
    p = 0.3 * (1 - 1 / A)
    m = 5 * big.shape[0]
    assert abs(moved / m - p) < 5 * np.sqrt(p * (1 - p) / m)
    r1, _ = ops.T.ego_attention_act(big, w, 2, A, 0.5, 11, 7)
    r2, _ = ops.T.ego_attention_act(big, w, 2, A, 0.5, 11, 7)
    r3, _ = ops.T.ego_attention_act(big, w, 2, A, 0.5, 11, 8)
    assert torch.equal(r1, r2) and not torch.equal(r1, r3)
    # env e's draw does not depend on the batch it is in: a prefix, and any other slice given its
    # global offset (a data-parallel rank's shard), draws the rows of the whole batch
    r4, _ = ops.T.ego_attention_act(big[:1000], w, 2, A, 0.5, 11, 7)
    assert torch.equal(r4, r1[:1000])
    r6, _ = ops.T.ego_attention_act(big[3000:5500], w, 2, A, 0.5, 11, 7, env_offset=3000)
    assert torch.equal(r6, r1[3000:5500])
    # the same rows at offset 0 (what every rank drew before the offset): other draws
    r7, _ = ops.T.ego_attention_act(big[3000:5500], w, 2, A, 1.0, 11, 7)
    r8, _ = ops.T.ego_attention_act(big[3000:5500], w, 2, A, 1.0, 11, 7, env_offset=3000)
    assert (r7 != r8).float().mean() > 0.5
    # device scalars override epsilon / step (the captured-graph path)
    eps = torch.tensor(0.5, device=hip_device)
    stp = torch.tensor(7, dtype=torch.int64, device=hip_device)
    r5, _ = ops.T.ego_attention_act(big, w, 2, A, 0.0, 11, 0, eps, stp)
    assert torch.equal(r5, r1)


@pytest.mark.gpu
def test_policy_act_is_one_launch_in_a_graph(hip_device):
    """EgoAttentionPolicy.act on the GPU: the fused launch; inside a StepGraph the replays draw
    with the schedule's epsilon and a fresh step each time, equal to eager acting."""
    from topotrafficrl_amd.envs import VecHighwayEnv
    from topotrafficrl_amd.graph import StepGraph
    KIN = {"type": "Kinematics", "vehicles_count": 15,
           "features": ["presence", "x", "y", "vx", "vy", "cos_h", "sin_h"],
           "features_range": {"x": [-100, 100], "y": [-100, 100], "vx": [-20, 20], "vy": [-20, 20]},
           "absolute": False, "order": "sorted"}
    cfg = {"num_envs": 64, "vehicles_count": 32, "observation": KIN, "device": hip_device}
    e1, e2 = VecHighwayEnv(cfg), VecHighwayEnv(cfg)
    o1, _ = e1.reset(seed=3)
    o2, _ = e2.reset(seed=3)
    p1 = EgoAttentionPolicy(hip_device, seed=0, tau=2.0)
    p2 = EgoAttentionPolicy(hip_device, seed=0, tau=2.0)
    sg = StepGraph(e2, o2, p2)
    assert p2.time == 0
    for t in range(4):
        a = p1.act(o1)
        o1, r1, *_ = e1.step(a)
        o2g, r2, *_ = sg.replay()
        assert torch.equal(a, sg.actions), t
        assert torch.equal(o1, o2g) and torch.equal(r1, r2), t
    assert p1.time == p2.time == 4


def _learner(z, device):
    net = EgoAttentionNetwork(5).to(device)
    net.load_state_dict({k: v.to(device) for k, v in _state_dict(z, "w0/").items()}, strict=True)
    cfg = {"double": bool(z["double"]), "gamma": float(z["gamma"]), "target_update": int(z["target_update"]),
           "optimizer": {"type": "ADAM", "lr": float(z["lr"]), "weight_decay": 0, "k": 5}}
    return DQNLearner(net, (15, 7), device, cfg)


def _check_dqn(name, device):
    z = load_golden(os.path.join(GOLDEN, name + ".npz"))
    lrn = _learner(z, device)
    for step in range(4):
        p = f"s{step}/"
        dev = lambda k, dt=None: torch.from_numpy(z[p + k]).to(device, dt)  # noqa: E731
        batch = (dev("state"), dev("action"), dev("reward"), dev("next_state"), dev("terminal"))
        loss, target = lrn.compute_bellman_residual(batch)
        np.testing.assert_allclose(target.detach().cpu().numpy(), z[p + "target"], rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(float(loss.detach()), float(z[p + "loss"]), rtol=1e-5)
        lrn.step_optimizer(loss)
        lrn.update_target_network()
        for k, v in lrn.value_net.state_dict().items():
            np.testing.assert_allclose(v.cpu().numpy(), z[p + "w/" + k], rtol=0, atol=1e-6, err_msg=k)
        for k, v in lrn.target_net.state_dict().items():
            np.testing.assert_allclose(v.cpu().numpy(), z[p + "tw/" + k], rtol=0, atol=1e-6, err_msg=k)


@pytest.mark.parametrize("name", ["dqn_double", "dqn_plain"])
def test_dqn_update_matches_reference_agent(name):
    _check_dqn(name, "cpu")


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["dqn_double", "dqn_plain"])
def test_dqn_update_matches_reference_agent_on_gpu(name, hip_device):
    _check_dqn(name, hip_device)


@pytest.mark.parametrize("n_steps", [1, 2, 3, 5])
def test_n_step_collapse_matches_reference_memory(n_steps):
    z = load_golden(os.path.join(GOLDEN, "dqn_memory.npz"))
    p = f"n{n_steps}/"
    T = len(z[p + "action"])
    mem = ReplayMemory(64, (1,), "cpu", n_steps=n_steps, gamma=0.95)
    st = torch.from_numpy(z[p + "state"].astype(np.float32))
    for i in range(T):  # one env: one transition per push, like the reference's push loop
        mem.push(st[i:i + 1, None], torch.tensor([int(z[p + "action"][i])]),
                 torch.tensor([float(z[p + "reward"][i])], dtype=torch.float64), st[i + 1:i + 2, None],
                 torch.tensor([bool(z[p + "done"][i])]))
    s, a, r, s2, t = mem.gather(torch.arange(T))
    np.testing.assert_array_equal(s[:, 0].numpy(), z[p + "c_state"])
    np.testing.assert_array_equal(a.numpy(), z[p + "c_action"])
    np.testing.assert_allclose(r.numpy(), z[p + "c_reward"], rtol=1e-6)
    np.testing.assert_array_equal(s2[:, 0].numpy(), z[p + "c_next_state"])
    np.testing.assert_array_equal(t.numpy(), z[p + "c_done"])


def test_epsilon_greedy_schedule_matches_reference():
    z = load_golden(os.path.join(GOLDEN, "dqn_memory.npz"))
    pol = EgoAttentionPolicy("cpu", tau=float(z["eps/tau"]), temperature=float(z["eps/temperature"]),
                             final_temperature=float(z["eps/final_temperature"]), fused=False)
    for t, e, v, g in zip(z["eps/time"], z["eps/epsilon"], z["eps/values"], z["eps/greedy"]):
        assert abs(pol.epsilon(int(t)) - e) <= 1e-15
        assert int(torch.from_numpy(v).argmax()) == g
