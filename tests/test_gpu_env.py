"""The batched env API on the GPU (VecHighwayEnv.reset/step, obs/reward/termination,
policy in the loop) against the float64 oracle driven through the same calls."""
import numpy as np
import pytest
import torch

from oracle.oracle import HostState, Oracle
from topotrafficrl_amd import _abi
from topotrafficrl_amd.agent import EgoAttentionPolicy
from topotrafficrl_amd.envs import VecHighwayEnv
from topotrafficrl_amd.trainer import BatchedDQNAgent, BatchedEvaluation

pytestmark = pytest.mark.gpu

KIN15 = {"type": "Kinematics", "vehicles_count": 15, "features": ["presence", "x", "y", "vx", "vy", "cos_h", "sin_h"],
         "features_range": {"x": [-100, 100], "y": [-100, 100], "vx": [-20, 20], "vy": [-20, 20]},
         "absolute": False, "order": "sorted"}


def make(E=16, N=40, obs=None, dtype="f64", **kw):
    cfg = {"num_envs": E, "vehicles_count": N, "observation": obs or KIN15, "device": "cuda:0", "dtype": dtype}
    cfg.update(kw)
    return VecHighwayEnv(cfg)


@pytest.mark.parametrize("road", ["straight", "sine", "circular"])
def test_env_step_matches_oracle(road, hip_device):
    E, N = 16, 40
    env = make(E, N, road=road, lanes_count=4 if road == "straight" else 3)
    obs, info = env.reset(seed=77)
    lanes = env.network.table
    o = Oracle(lanes, env.params)
    h = HostState(E, N)
    o.reset_highway(h, env.reset_cfg, [77 + e for e in range(E)])
    kin = _abi.kin_cfg(**{k: v for k, v in KIN15.items() if k != "type"})
    ref_obs, _ = o.observe_kinematics(h, kin)
    if road == "straight":
        assert np.array_equal(obs.cpu().numpy(), ref_obs)
    else:  # curved placement goes through device sin/cos (1 ulp): float32 features may round apart
        assert np.max(np.abs(obs.cpu().numpy() - ref_obs)) < 1e-6
    rng = np.random.default_rng(3)
    for t in range(1, 6):
        a = rng.integers(0, 5, size=E)
        obs, rew, term, trunc, info = env.step(torch.from_numpy(a))
        o.simulate(h, a.astype(np.int32), 15, 1 / 15)
        ref_obs, _ = o.observe_kinematics(h, kin)
        ref_r, ref_term, ref_trunc, ref_c = o.rewards(h, env.reward_cfg, float(t), components=True)
        assert np.max(np.abs(obs.cpu().numpy() - ref_obs)) < 1e-6
        assert np.allclose(rew.cpu().numpy(), ref_r, atol=1e-6)
        assert np.array_equal(term.cpu().numpy(), ref_term) and np.array_equal(trunc.cpu().numpy(), ref_trunc)
        assert np.allclose(info["speed"].cpu().numpy(), h["speed"][:, 0])
        assert np.array_equal(info["crashed"].cpu().numpy(), h["crashed"][:, 0] != 0)
        assert np.all(env.time.cpu().numpy() == float(t))  # time += 1 runs in the rewards launch
        for i, name in enumerate(env.REWARD_TERMS):  # info["rewards"] (abstract.py:182-185)
            assert np.allclose(info["rewards"][name].cpu().numpy(), ref_c[:, i], atol=1e-6), name


def test_truncation_and_auto_reset(hip_device):
    env = make(8, 20, duration=3, auto_reset=True)
    env.reset(seed=1)
    for t in range(3):
        _, _, term, trunc, _ = env.step(torch.ones(8, dtype=torch.int64))
    assert bool(trunc.all())
    assert float(env.time.max()) == 0.0  # every env was truncated at t=3 and auto-reset


def test_sharded_envs_equal_one_big_batch(hip_device):
    """env_id_offset sharding: two shards == one batch of the same global envs."""
    big = make(8, 30)
    big.reset(seed=5)
    a = make(4, 30, env_id_offset=0)
    b = make(4, 30, env_id_offset=4)
    a.reset(seed=5)
    b.reset(seed=5)
    acts = torch.tensor([0, 1, 2, 3, 4, 1, 3, 2])
    o1, *_ = big.step(acts)
    oa, *_ = a.step(acts[:4])
    ob, *_ = b.step(acts[4:])
    assert torch.equal(o1, torch.cat([oa, ob]))
    for k in ("x", "lane", "crashed"):
        assert torch.equal(big.state[k], torch.cat([a.state[k], b.state[k]]))


def test_policy_in_the_loop(hip_device):
    env = make(32, 64)
    pol = EgoAttentionPolicy(hip_device, seed=0)
    obs, _ = env.reset(seed=9)
    for t in range(3):
        act = pol.act(obs, t)
        assert act.shape == (32,) and act.device.type == "cuda"
        obs, rew, term, trunc, info = env.step(act)
    assert torch.isfinite(obs).all()
    ev = BatchedEvaluation(env, BatchedDQNAgent(hip_device), num_episodes=1, sim_seed=0, max_steps=3)
    ev.run_episodes()
    assert ev.last_stats["episode/length"] == 3


@pytest.mark.parametrize("dtype", ["f64", "f32"])
def test_occupancy_grid_env(dtype, hip_device):
    grid = {"type": "OccupancyGrid", "features": ["presence", "x", "y", "vx", "vy", "cos_h", "sin_h"],
            "features_range": {"x": [-100, 100], "y": [-100, 100], "vx": [-20, 20], "vy": [-20, 20]},
            "grid_size": [[-32, 32], [-32, 32]], "grid_step": [2, 2]}
    env = make(8, 128, obs=grid, dtype=dtype)
    obs, _ = env.reset(seed=2)
    assert obs.shape == (8, 7, 32, 32)
    obs, *_ = env.step(torch.ones(8, dtype=torch.int64))
    assert float(obs[:, 0].sum()) >= 8  # the ego occupies the centre cell of every env


def test_masked_auto_reset_replays_numpy_seed(hip_device):
    """Device-side auto-reset: env e reset with seed s restarts its k-th new episode as
    np.random.default_rng([s & 0xffffffff, s >> 32, k]) would, only where the mask is set."""
    E, N, s = 8, 24, 5
    env = make(E, N)
    env.reset(seed=s)
    for _ in range(2):
        env.step(torch.ones(E, dtype=torch.int64))
    before = env.state.to_numpy()
    mask = torch.tensor([1, 0, 1, 0, 0, 1, 0, 1], dtype=torch.bool, device=hip_device)
    env.time.fill_(2.0)
    env._auto_reset(mask)
    after = env.state.to_numpy()
    o = Oracle(env.network.table, env.params)
    ref = HostState(E, N)
    o.reset_highway(ref, env.reset_cfg, [[s + e, 0, 1] for e in range(E)])
    m = mask.cpu().numpy()
    for k in ("x", "y", "heading", "speed", "target_speed", "timer", "delta", "lane", "kind", "crashed"):
        assert np.array_equal(after[k][m], ref[k][m].astype(after[k].dtype)), k
        assert np.array_equal(after[k][~m], before[k][~m]), k
    assert torch.equal(env.time.cpu(), torch.where(mask.cpu(), 0.0, 2.0).double())
    env._auto_reset(mask)  # the second new episode of the same envs: k = 2
    o.reset_highway(ref, env.reset_cfg, [[s + e, 0, 2] for e in range(E)])
    assert np.array_equal(env.state.to_numpy()["x"][m], ref["x"][m])


def test_reset_with_seeds_beyond_32_bits(hip_device):
    """Seeds >= 2^32 (multi-word SeedSequence entropy) take the host-seeded path: same scenes."""
    E, N = 4, 16
    env = make(E, N)
    base = 2 ** 33 + 7
    env.reset(seed=base)
    o = Oracle(env.network.table, env.params)
    ref = HostState(E, N)
    o.reset_highway(ref, env.reset_cfg, [base + e for e in range(E)])
    got = env.state.to_numpy()
    for k in ("x", "y", "speed", "delta", "lane"):
        assert np.array_equal(got[k], ref[k]), k


def test_auto_reset_in_step_returns_new_first_observation(hip_device):
    env = make(8, 20, duration=2, auto_reset=True)
    env.reset(seed=3)
    env.step(torch.ones(8, dtype=torch.int64))
    obs, rew, term, trunc, info = env.step(torch.ones(8, dtype=torch.int64))
    assert bool(trunc.all())
    assert "final_observation" in info and not torch.equal(info["final_observation"], obs)
    fresh = make(8, 20)
    fresh.reset(seed=3)
    fresh._entropy.copy_(env._entropy)
    fresh._entropy[:, 2] -= 1  # _auto_reset advances the episode counter itself
    fresh._auto_reset(torch.ones(8, dtype=torch.bool, device=hip_device))
    assert torch.equal(obs, fresh.observation_type.observe())


def test_deepcopy_forks_an_independent_highway_env(hip_device):
    """copy.deepcopy forks state, time and the auto-reset seed words / episode counters: both
    copies follow the same trajectory through their auto-resets independently, and the fork's
    resets do not change which episode the original replays next."""
    import copy
    env = make(8, 20, duration=2, auto_reset=True)
    env.reset(seed=6)
    env.step(torch.ones(8, dtype=torch.int64))
    fork = copy.deepcopy(env)
    assert fork._entropy.data_ptr() != env._entropy.data_ptr()
    a = torch.full((8,), 3, dtype=torch.int64)
    for _ in range(4):  # lockstep through two auto-resets (shared counters would advance twice)
        r1, r2 = env.step(a), fork.step(a)
        assert torch.equal(r1[0], r2[0]) and torch.equal(r1[1], r2[1])


def test_returned_observations_are_not_overwritten(hip_device):
    """Like the reference's df.values.copy(), an obs kept by the caller survives later steps
    (a trainer records (s, a, r, s') pairs across steps)."""
    env = make(4, 20)
    o0, _ = env.reset(seed=4)
    keep = o0.clone()
    o1, *_ = env.step(torch.ones(4, dtype=torch.int64))
    assert torch.equal(o0, keep) and not torch.equal(o0, o1)


def test_dqn_training_in_the_loop(hip_device):
    """Trainer hooks + batched DQN learning on the device: replay memory fills from the env,
    the double-DQN residual is minimised, the target net syncs, finished envs auto-reset."""
    env = make(64, 32, duration=12, auto_reset=True)
    agent = BatchedDQNAgent(hip_device, config={"batch_size": 64, "memory_capacity": 2048, "target_update": 4})
    ev = BatchedEvaluation(env, agent, num_episodes=1, sim_seed=0, max_steps=10)
    params0 = [p.detach().clone() for p in agent.policy.value_net.parameters()]
    ev.run_episodes()
    L = agent.learner
    assert len(L.memory) == 640 and L.steps == 10 and torch.isfinite(L.last_loss)
    assert any(not torch.equal(a, b) for a, b in zip(params0, agent.policy.value_net.parameters()))
    assert float(env.time.max()) == 10.0


def test_step_graph_replays_the_same_rollout(hip_device):
    """A captured closed-loop step (policy -> env.step) replays the same trajectory as eager
    steps from the same state and RNG."""
    from topotrafficrl_amd.graph import StepGraph
    E, N = 16, 32
    eager = make(E, N)
    graphed = make(E, N)
    o1, _ = eager.reset(seed=11)
    o2, _ = graphed.reset(seed=11)
    p1 = EgoAttentionPolicy(hip_device, seed=3)
    p2 = EgoAttentionPolicy(hip_device, seed=3)
    sg = StepGraph(graphed, o2, p2, warmup=1)
    p2.gen.manual_seed(4)
    p1.gen.manual_seed(4)
    for t in range(4):
        a = p1.act(o1, t)
        o1, r1, te1, tr1, _ = eager.step(a)
        o2, r2, te2, tr2 = sg.replay()
        assert torch.equal(o1, o2) and torch.equal(r1, r2) and torch.equal(te1, te2)
    assert torch.equal(eager.state["x"], graphed.state["x"])


@pytest.mark.parametrize("B", [1, 5, 64, 1000])
def test_fused_ego_attention_matches_torch_forward(B, hip_device):
    """ttrl_ego_attention_q (fused HIP forward) == the torch EgoAttentionNetwork in float32."""
    from topotrafficrl_amd.agent import EgoAttentionNetwork
    net = EgoAttentionNetwork(5).reset(torch.Generator().manual_seed(B)).to(hip_device)
    g = torch.Generator(device=hip_device).manual_seed(B)
    x = torch.rand(B, 15, 7, device=hip_device, generator=g) * 2 - 1
    x[:, :, 0] = (torch.rand(B, 15, device=hip_device, generator=g) < 0.7).float()
    x[:, 0, 0] = 1.0
    if B >= 5:
        x[3, :, 0] = 0.0  # every entity masked: uniform softmax
    ref = net(x)
    got = net.fused_q(x)
    assert torch.allclose(got, ref, rtol=1e-4, atol=1e-5), float((got - ref).abs().max())
    # packed weights follow parameter updates
    with torch.no_grad():
        net.output_layer.predict.bias.add_(1.0)
    assert torch.allclose(net.fused_q(x), net(x), rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("heads,F_,NE,A,B", [(1, 7, 15, 5, 37), (2, 5, 2, 3, 9), (2, 7, 5, 5, 130), (2, 8, 32, 4, 66),
                                             (4, 7, 16, 5, 21), (8, 7, 8, 5, 13)])
def test_fused_ego_attention_shapes_and_biases(heads, F_, NE, A, B, hip_device):
    """Every supported head count / feature count / entity count (partial entity batches, partial
    last wave), with random nonzero biases in every layer."""
    import copy
    from topotrafficrl_amd.agent import EGO_ATTENTION_2H, EgoAttentionNetwork
    cfg = copy.deepcopy(EGO_ATTENTION_2H)
    cfg["embedding_layer"]["in"] = cfg["others_embedding_layer"]["in"] = F_
    cfg["attention_layer"]["heads"] = heads
    gen = torch.Generator().manual_seed(heads * 100 + NE)
    net = EgoAttentionNetwork(A, cfg).reset(gen)
    with torch.no_grad():
        for m in net.modules():
            if isinstance(m, torch.nn.Linear) and m.bias is not None:
                m.bias.uniform_(-0.3, 0.3, generator=gen)
    net = net.to(hip_device)
    g = torch.Generator(device=hip_device).manual_seed(NE)
    x = torch.rand(B, NE, F_, device=hip_device, generator=g) * 2 - 1
    x[:, :, 0] = (torch.rand(B, NE, device=hip_device, generator=g) < 0.6).float()
    x[0, 0, 0] = 0.0  # a masked ego
    ref = net(x)
    got = net.fused_q(x)
    assert torch.allclose(got, ref, rtol=1e-4, atol=1e-5), float((got - ref).abs().max())


@pytest.mark.parametrize("road,N,dtype,order", [("straight", 64, "f64", "sorted"), ("straight", 24, "f32", "sorted"),
                                                ("straight", 100, "f64", "shuffled"), ("sine", 40, "f64", "sorted")])
def test_fused_step_observation_equals_separate_observe(road, N, dtype, order, hip_device):
    """env.step in one launch (ttrl_env_step: simulate, then the observation and the step tail from
    the on-chip state) == ttrl_simulate, ttrl_observe_kinematics and ttrl_rewards_step, bit for bit
    (rows, observed slot ids, rewards, dones, info, time)."""
    obs_cfg = dict(KIN15, order=order)
    kw = dict(road=road, lanes_count=4 if road == "straight" else 3)
    a, b = make(16, N, obs=obs_cfg, dtype=dtype, **kw), make(16, N, obs=obs_cfg, dtype=dtype, **kw)
    a.reset(seed=21)
    b.reset(seed=21)
    rng = np.random.default_rng(4)
    for _ in range(4):
        act = torch.from_numpy(rng.integers(0, 5, size=16))
        oa, ra, ta, ua, ia = a.step(act)
        b._simulate(act)
        ob = b.observation_type.observe()
        rb, tb, ub = b._rewards_and_dones(1.0)
        ib = b._info(ob, act)
        assert torch.equal(oa, ob)
        assert torch.equal(a.observation_type.observed_ids, b.observation_type.observed_ids)
        assert torch.equal(a.state["x"], b.state["x"])
        assert torch.equal(ra, rb) and torch.equal(ta, tb) and torch.equal(ua, ub)
        assert torch.equal(ia["speed"], ib["speed"]) and torch.equal(ia["crashed"], ib["crashed"])
        assert torch.equal(a._components, b._components) and torch.equal(a.time, b.time)


GRID = {"type": "OccupancyGrid", "features": ["presence", "x", "y", "vx", "vy", "cos_h", "sin_h"],
        "features_range": {"x": [-100, 100], "y": [-100, 100], "vx": [-20, 20], "vy": [-20, 20]},
        "grid_size": [[-32, 32], [-32, 32]], "grid_step": [2, 2]}


GRID_ROAD = {"type": "OccupancyGrid", "features": ["presence", "vx", "vy", "on_road"]}  # the reference default


@pytest.mark.parametrize("obs_cfg,N,dtype,road", [(GRID, 128, "f64", "straight"), (GRID, 128, "f32", "straight"),
                                                  (GRID, 48, "f64", "straight"), (GRID_ROAD, 64, "f64", "straight"),
                                                  (GRID_ROAD, 100, "f32", "straight"), (GRID, 64, "f64", "sine"),
                                                  ({"type": "TimeToCollision", "horizon": 10}, 64, "f64", "straight")])
def test_fused_step_tail_without_kinematics(obs_cfg, N, dtype, road, hip_device):
    """With a non-Kinematics observation env.step runs the simulate launch with the reward-only step
    tail (the ego found and read from the on-chip final state); an OccupancyGrid is written by the
    same launch (ttrl_env_step_grid, straight roads of 64 / 128 slots; the sine road takes its two
    launches), another observer runs separately.  It must equal ttrl_simulate, the observer and
    ttrl_rewards_step bit for bit (observation, rewards, dones, terms, info, time)."""
    kw = dict(road=road, lanes_count=4 if road == "straight" else 3)
    a, b = make(16, N, obs=obs_cfg, dtype=dtype, **kw), make(16, N, obs=obs_cfg, dtype=dtype, **kw)
    a.reset(seed=8)
    b.reset(seed=8)
    rng = np.random.default_rng(6)
    for _ in range(4):
        act = torch.from_numpy(rng.integers(0, 5, size=16))
        oa, ra, ta, ua, ia = a.step(act)
        b._simulate(act)
        ob = b.observation_type.observe()
        rb, tb, ub = b._rewards_and_dones(1.0)
        ib = b._info(ob, act)
        assert torch.equal(oa, ob)
        assert torch.equal(a.state["x"], b.state["x"]) and torch.equal(a.state["crashed"], b.state["crashed"])
        assert torch.equal(ra, rb) and torch.equal(ta, tb) and torch.equal(ua, ub)
        assert torch.equal(ia["speed"], ib["speed"]) and torch.equal(ia["crashed"], ib["crashed"])
        assert torch.equal(a._components, b._components) and torch.equal(a.time, b.time)
