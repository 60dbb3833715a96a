"""VecIntersectionEnv on the MI355X: the device reset (seeding, spawns, 45 warm-up frames,
challenger, ego, removal), np_random-shuffled observations, rewards, clears and spawns, against
the golden intersection episodes captured from the reference (oracle/gen_golden_ix.py) and the
float64 oracle.  Tolerances as tests/test_ix_env_oracle.py; every discrete field exact."""
import numpy as np
import pytest
import torch

from conftest import golden_files, load_golden
from oracle.oracle import HostState, Oracle
import parity_log
from test_ix_env_oracle import EPISODE_TOL, KIN, check_obs, ref_step_input, reward_tol, same_state
from test_host_logic import _reward_from_terms
from test_ix_oracle import P_IX
from topotrafficrl_amd import _abi
from topotrafficrl_amd.intersection import VecIntersectionEnv, intersection_network, ix_cfg, ix_reset

pytestmark = pytest.mark.gpu

GOLD = [load_golden(p) for p in golden_files("ix_*")]
# scripts/configs/IntersectionEnv/env.json: the default Kinematics observation with order "shuffled"
ENV_JSON = {"observation": dict(VecIntersectionEnv.default_config()["observation"], order="shuffled")}


def env_view(d: dict, e: int) -> dict:
    return {k: v[e:e + 1] for k, v in d.items()}


def test_device_reset_matches_reference_scenes(hip_device):
    env = VecIntersectionEnv({**ENV_JSON, "num_envs": len(GOLD), "device": hip_device})
    obs, _ = env.reset(seed=0)   # env e: IntersectionEnv.reset(seed=e)
    st = env.state.to_numpy()
    for e, d in enumerate(GOLD):
        assert int(d["meta"][0]) == e
        same_state(env_view(st, e), HostState.from_ix(d, "pre", 0, pad_to=32), 1e-9, f"reset {e}")
        assert np.max(np.abs(obs[e].cpu().numpy() - d["obs0"])) <= 1e-6, e


def test_device_episodes_match_reference(hip_device):
    from test_ix_env_oracle import standstill_links
    # the ix goldens are the reference env's episodes of seeds 0-5 bit for bit
    # (test_ix_goldens_equal_the_reference_env): their standstill links come from those fixtures
    links = [standstill_links(load_golden(golden_files(f"envref_ix_s{e}.npz")[0])) for e in range(len(GOLD))]
    env = VecIntersectionEnv({**ENV_JSON, "num_envs": len(GOLD), "device": hip_device})
    env.reset(seed=0)
    steps = int(GOLD[0]["meta"][1])
    acts = np.stack([d["actions"] for d in GOLD], 1)  # [steps, E]
    for p in range(steps):
        obs, rew, term, trunc, info = env.step(torch.from_numpy(acts[p]).to(hip_device))
        st = env.state.to_numpy()
        for e, d in enumerate(GOLD):
            end = HostState.from_ix(d, "frame", (p, 14), pad_to=32)
            check_obs(obs[e].cpu().numpy(), d["obs"][p], end, EPISODE_TOL, f"env {e} step {p}", "device ix episodes from seed")
            assert abs(float(rew[e]) - d["reward"][p]) <= reward_tol(end, EPISODE_TOL), (e, p)
            assert bool(term[e]) == bool(d["terminated"][p]) and bool(trunc[e]) == bool(d["truncated"][p]), (e, p)
            same_state(env_view(st, e), HostState.from_ix(d, "post", p, pad_to=32), EPISODE_TOL, f"env {e} step {p}",
                       "device ix episodes from seed", links=links[e][p][1])
        # IntersectionEnv._info (intersection_env.py:120-128): the terms rebuild the reward
        terms = np.stack([info["rewards"][n].cpu().numpy() for n in env.REWARD_TERMS], 1)
        for e in range(len(GOLD)):
            assert abs(_reward_from_terms(env.reward_cfg, terms[e]) - float(rew[e])) <= 1e-6, (e, p)
        assert torch.equal(info["agents_rewards"][0], rew)
        # info speed / crashed come from the rewards launch; the step tail's clears leave the ego as it was
        assert torch.equal(info["speed"], env.state.ego("speed"))
        assert torch.equal(info["crashed"], env.state.ego("crashed").bool())
        assert np.all(env.time.cpu().numpy() == float(p + 1))
        assert torch.equal(info["agents_terminated"][0].cpu(), torch.from_numpy((terms[:, 0] != 0) | (terms[:, 2] != 0)))


def test_large_batch_reset_equals_oracle(hip_device):
    """4096 envs reset on the device; 64 of them replayed on the oracle."""
    E = 4096
    env = VecIntersectionEnv({"num_envs": E, "device": hip_device})
    env.reset(seed=12345)
    st = env.state.to_numpy()
    net = intersection_network()
    o = Oracle(net.table, P_IX)
    cfg = ix_cfg(net, VecIntersectionEnv.default_config(), P_IX)
    pick = np.arange(0, E, E // 64)
    h = HostState(len(pick), 32)
    o.ix_reset(h, cfg, [12345 + int(e) for e in pick])
    for i, e in enumerate(pick):
        same_state(env_view(st, int(e)), {k: v[i:i + 1] for k, v in h.a.items()}, 1e-9, f"env {e}")
    assert np.array_equal(st["rng"][pick], h["rng"])
    counts = (st["kind"] > 0).sum(1)
    assert counts.min() >= 2 and counts.max() <= 32


def test_masked_auto_reset(hip_device):
    """Finished envs restart as default_rng([seed, episode]); the others continue untouched."""
    E = 64
    env = VecIntersectionEnv({**ENV_JSON, "num_envs": E, "device": hip_device, "auto_reset": True, "duration": 3})
    env.reset(seed=7)
    g = torch.Generator().manual_seed(0)
    net = intersection_network()
    o = Oracle(net.table, P_IX)
    cfg = ix_cfg(net, VecIntersectionEnv.default_config(), P_IX)
    episodes = np.zeros(E, dtype=np.int64)
    for p in range(5):
        before = env.state.to_numpy()
        a = torch.randint(0, 3, (E,), generator=g).to(hip_device)
        obs, rew, term, trunc, info = env.step(a)
        done = (term | trunc).cpu().numpy()
        episodes += done
        st = env.state.to_numpy()
        if done.any():
            idx = np.nonzero(done)[0]
            h = HostState(len(idx), 32)
            o.ix_reset(h, cfg, [[7 + int(e), int(episodes[e])] for e in idx])
            ob, _ = o.observe_kinematics(h, KIN)
            for i, e in enumerate(idx):
                same_state(env_view(st, int(e)), {k: v[i:i + 1] for k, v in h.a.items()}, 1e-9, f"auto-reset {e}")
                assert np.max(np.abs(obs[e].cpu().numpy() - ob[i])) <= 1e-6
            assert float(env.time[idx].abs().max()) == 0.0
        assert not np.array_equal(before["x"], st["x"])
    assert episodes.sum() > 0


def test_f32_episode_runs(hip_device):
    env = VecIntersectionEnv({"num_envs": 256, "device": hip_device, "dtype": "f32"})
    obs, _ = env.reset(seed=3)
    for _ in range(13):
        obs, rew, term, trunc, info = env.step(torch.ones(256, dtype=torch.int64, device=hip_device))
    torch.cuda.synchronize()
    assert torch.isfinite(obs).all() and torch.isfinite(rew).all()
    assert bool(trunc.all())


def test_grid_and_lidar_observe_the_intersection_ego(hip_device):
    """OccupancyGrid (env_grid_dense.json) and Lidar of the intersection ego, which sits after the
    traffic in the vehicle list, on every golden step state: device == oracle."""
    from observation_helpers import batch_of_ix_states
    from topotrafficrl_amd.observation import lidar, occupancy_grid
    from topotrafficrl_amd.road import BatchedRoad
    from topotrafficrl_amd.state import BatchState
    h = batch_of_ix_states(GOLD)
    net = intersection_network()
    o = Oracle(net.table, P_IX)
    st = BatchState(h.E, h.N, device=hip_device).load_numpy(h.a)
    grid = _abi.grid_cfg(["presence", "x", "y", "vx", "vy", "cos_h", "sin_h"], [[-32, 32], [-32, 32]], [2, 2],
                         {"x": [-100, 100], "y": [-100, 100], "vx": [-20, 20], "vy": [-20, 20]})
    got = occupancy_grid(st, net, P_IX, grid).cpu().numpy()
    want = o.observe_grid(h, grid)
    assert np.max(np.abs(got - want)) <= 1e-6
    lc = _abi.lidar_cfg()
    got = lidar(st, net, P_IX, lc).cpu().numpy()
    want = o.observe_lidar(h, lc)
    assert np.max(np.abs(got - want)) <= 1e-6
    BatchedRoad(net, st, P_IX)  # the network table is a valid BatchedRoad network


def test_intersection_step_graph_equals_eager(hip_device):
    """graph.StepGraph captures the whole intersection step, auto-reset included (device-only
    masks, counters and masked resets); replays equal eager steps bit for bit."""
    from topotrafficrl_amd.graph import StepGraph
    cfg = {**ENV_JSON, "num_envs": 32, "device": hip_device, "auto_reset": True, "duration": 4,
           "overlap_resets": False}
    eager, graphed = VecIntersectionEnv(cfg), VecIntersectionEnv(cfg)
    o1, _ = eager.reset(seed=5)
    o2, _ = graphed.reset(seed=5)
    sg = StepGraph(graphed, o2, None, warmup=1)
    g = torch.Generator(device=hip_device).manual_seed(0)
    for t in range(9):  # two auto-reset rounds (duration 4) plus crashes / arrivals
        a = torch.randint(0, 3, (32,), device=hip_device, generator=g)
        o1, r1, te1, tr1, _ = eager.step(a)
        sg.set_actions(a)
        o2, r2, te2, tr2 = sg.replay()
        assert torch.equal(o1, o2) and torch.equal(r1, r2) and torch.equal(te1, te2) and torch.equal(tr1, tr2), t
    for k in ("x", "kind", "rng", "route_road"):
        assert torch.equal(eager.state[k], graphed.state[k]), k


def test_f32_intersection_frames_vs_oracle(hip_device):
    """fp32 fast path on the intersection, one frame at a time from every golden frame state (all
    6 episodes x 13 steps x 15 frames), against the float64 oracle on the same float32-rounded
    inputs, under the highway's rule (check_f32_flips): continuous fields within 1e-4 * (1 + |x|)
    per frame, every discrete difference (lanes, targets, routes, yields, crashes) traced to a
    float64 decision margin below 1e-5 -- its own, or through a causal link that of a flipped
    vehicle.  The decisions include the RegulatedRoad conflicts and priorities and follow_road.
    A slow vehicle's steering command is held to the steering law's 1 / v^2 gain on its
    position's rounding (f32_cont_tol); every other field to 1e-4 * (1 + |x|)."""
    from observation_helpers import batch_of_ix_states
    from test_gpu_parity import DISC as HW_DISC, check_f32_flips, f32_inputs, to_dev
    from test_ix_oracle import LONGI, ix_lanes
    from topotrafficrl_amd.road import BatchedRoad
    disc = HW_DISC + ["yielding", "route_n", "route_road", "route_lane", "kind"]
    lanes = ix_lanes(GOLD[0])
    net = intersection_network()
    o = Oracle(lanes, P_IX)
    flips = total = 0
    for f in range(15):
        if f == 0:
            h = batch_of_ix_states(GOLD, "pre")
            cases = [(d, p) for d in GOLD for p in range(int(d["meta"][1]))]
        else:
            golds = [(d, p) for d in GOLD for p in range(int(d["meta"][1]))]
            h = HostState(len(golds), 32)
            for e, (d, p) in enumerate(golds):
                g = HostState.from_ix(d, "frame", (p, f - 1), pad_to=32)
                for k in h.a:
                    h.a[k][e] = g.a[k][0]
            cases = golds
        g = f32_inputs(h)
        dev = to_dev(g, hip_device, dtype="f32")
        road = BatchedRoad(net, dev, P_IX)
        act = None
        if f == 0:
            act = [LONGI[int(d["actions"][p])] for d, p in cases]
            road.meta_action(torch.tensor(act, dtype=torch.int32))
        road.act()
        road.step(1 / 15)
        m, lk = o.frame_margins(g, act, links=True)
        torch.cuda.synchronize()
        flips += check_f32_flips(dev, g, m, lk, f"ix frame {f}", disc=disc)
        total += int((g["kind"] > 0).sum())
    assert flips <= max(3, total // 1000), (flips, total)  # flips are rare, not merely excused


def test_dqn_training_on_the_intersection(hip_device):
    """Trainer hooks + batched DQN learning on VecIntersectionEnv (3 longitudinal actions,
    auto-reset, the reference's env.json observation)."""
    from topotrafficrl_amd.trainer import BatchedDQNAgent, BatchedEvaluation
    env = VecIntersectionEnv({**ENV_JSON, "num_envs": 64, "device": hip_device, "auto_reset": True})
    agent = BatchedDQNAgent(hip_device, n_actions=3, config={"batch_size": 64, "memory_capacity": 2048,
                                                              "target_update": 4})
    ev = BatchedEvaluation(env, agent, num_episodes=1, sim_seed=0, max_steps=8)
    ev.run_episodes()
    L = agent.learner
    assert len(L.memory) == 512 and L.steps == 8 and torch.isfinite(L.last_loss)


@pytest.mark.parametrize("duration,dtype,streams,slots,chunk,init", [
    (1, "f64", 2, 32, 15, 10), (3, "f64", 2, 32, 15, 10), (3, "f32", 2, 32, 15, 10), (2, "f64", 1, 32, 15, 10),
    (2, "f64", 2, 96, 15, 10), (1, "f64", 2, 32, 9, 10), (2, "f64", 2, 32, 5, 10), (1, "f64", 2, 32, 0, 10),
    (3, "f64", 2, 32, 0, 10), (2, "f64", 1, 32, 0, 10), (1, "f64", 3, 32, 0, 10), (4, "f64", 2, 32, 15, 16),
    (4, "f32", 2, 32, 15, 16)])
def test_overlapped_resets_equal_in_place_resets(duration, dtype, streams, slots, chunk, init, hip_device):
    """overlap_resets (each env's next two episodes prepared on side streams, swapped in from
    alternating spare slots by ix_step_tail when an env finishes, the new episode observed in the
    same launch) gives the same trajectories, bit for bit, as the in-place composition of separate
    launches (simulate, observe, rewards, clear / spawn, reset, masked observe); duration 1
    finishes every env at every step (every spare slot in turn).  chunk: the warm-up frames per
    step of a spare reset (15: three chunks, four spare slots; 9: five chunks, six slots; 5: nine
    chunks, ten slots; 0: the whole warm-up at once on `streams` side streams, two slots).  96 slots: the new scenes are observed by the masked observation launch
    instead of the tail launch (one slot per lane there).  init 16: denser scenes (16 initial
    vehicles plus the challenger and the ego).  The
    tail's live-vehicle counter (the config-6 bench's count) equals the vehicles present after
    every step."""
    cfg = {**ENV_JSON, "num_envs": 48, "device": hip_device, "auto_reset": True, "duration": duration,
           "dtype": dtype, "reset_streams": streams, "vehicle_slots": slots, "reset_chunk_frames": chunk,
           "initial_vehicle_count": init}
    a = VecIntersectionEnv({**cfg, "overlap_resets": True})
    b = VecIntersectionEnv({**cfg, "overlap_resets": False})
    a.live_counter = torch.zeros((), dtype=torch.int64, device=hip_device)
    oa, _ = a.reset(seed=21)
    ob, _ = b.reset(seed=21)
    assert torch.equal(oa, ob)
    g = torch.Generator(device=hip_device).manual_seed(2)
    present = 0
    for t in range(8):
        act = torch.randint(0, 3, (48,), device=hip_device, generator=g)
        ra = a.step(act)
        rb = b.step(act)
        present += int((a.state["kind"] != 0).sum())
        for x, y in zip(ra[:4], rb[:4]):
            assert torch.equal(x, y), t
    for k in a.state.t:
        assert torch.equal(a.state[k], b.state[k]), k
    assert int(a.live_counter) == present
    # the next step's dispatch order: the envs in workgroup groups, heaviest group first
    order = a._order[:48].cpu()
    assert torch.equal(order.sort().values, torch.arange(48, dtype=torch.int32))
    G = 2 if slots <= 32 else 1
    assert torch.equal(order.view(-1, G), order.view(-1, G)[:, :1] + torch.arange(G, dtype=torch.int32))
    w = (a.state["kind"] != 0).sum(1).cpu()[order.long()].view(-1, G).sum(1)
    assert bool((w[:-1] >= w[1:]).all()), w


@pytest.mark.parametrize("duration,dtype,init,slots", [(1, "f64", 10, 32), (3, "f64", 10, 32), (4, "f64", 16, 32),
                                                      (4, "f32", 16, 32), (3, "f64", 10, 64), (5, "f64", 16, 20)])
def test_fused_tail_equals_the_separate_tail(duration, dtype, init, slots, hip_device):
    """fuse_tail (ttrl_ix_env_step: the envs that go on run _clear_vehicles / _spawn_vehicle inside
    the step launch, from its LDS rows; ix_step_tail_(cleared=True) swaps in the finished envs'
    spare scenes) against the two-launch step (ttrl_env_step, then ix_step_tail_'s clear / spawn):
    observations, rewards, flags, the info terms, the final observation, every state field, every
    np_random, the live-vehicle counter and the next dispatch order, bit for bit, step by step
    (duration 1: every env finishes every step; 20 slots: rows narrower than the 32 lanes of
    their half-wave; 64: one env per wavefront; init 16: dense scenes, full rows)."""
    cfg = {**ENV_JSON, "num_envs": 40, "device": hip_device, "auto_reset": True, "duration": duration,
           "dtype": dtype, "vehicle_slots": slots, "initial_vehicle_count": init}
    a = VecIntersectionEnv({**cfg, "fuse_tail": True})
    b = VecIntersectionEnv({**cfg, "fuse_tail": False})
    for e in (a, b):
        e.live_counter = torch.zeros((), dtype=torch.int64, device=hip_device)
    oa, _ = a.reset(seed=31)
    ob, _ = b.reset(seed=31)
    assert torch.equal(oa, ob)
    g = torch.Generator(device=hip_device).manual_seed(4)
    spawned = 0
    for t in range(10):
        act = torch.randint(0, 3, (40,), device=hip_device, generator=g)
        before = int((b.state["kind"] != 0).sum())
        ra, rb = a.step(act), b.step(act)
        for x, y in zip(ra[:4], rb[:4]):
            assert torch.equal(x, y), t
        for k in ("final_observation", "final_mask", "speed", "crashed"):
            assert torch.equal(ra[4][k], rb[4][k]), (t, k)
        for k in ra[4]["rewards"]:
            assert torch.equal(ra[4]["rewards"][k], rb[4]["rewards"][k]), (t, k)
        for k in a.state.t:
            assert torch.equal(a.state[k], b.state[k]), (t, k)
        assert torch.equal(a._order[:40], b._order[:40]), t
        assert int(a.live_counter) == int(b.live_counter), t
        spawned += int((b.state["kind"] != 0).sum()) - before
    assert spawned != 0


@pytest.mark.parametrize("E", [64, 63])
def test_dispatch_order_leaves_results_unchanged(E, hip_device):
    """The step launch's dispatch order (workgroup slot -> env) changes only which workgroup runs an
    env: every output and the state after the launch are the same for any permutation (63 envs: the
    last workgroup holds one env)."""
    env = VecIntersectionEnv({**ENV_JSON, "num_envs": E, "device": hip_device})
    env.reset(seed=5)
    g = torch.Generator(device=hip_device).manual_seed(4)
    for _ in range(3):
        env.step(torch.randint(0, 3, (E,), device=hip_device, generator=g))
    snap, t0 = env.state.clone(), env.time.clone()
    codes = env.action_type._codes(torch.randint(0, 3, (E,), device=hip_device, generator=g))
    kc = env.observation_type.fused_cfg()  # one cfg (shuffle words included) for the three launches
    runs = []
    for order in (None, torch.randperm(E, generator=torch.Generator().manual_seed(1)).to(torch.int32).to(hip_device),
                  torch.arange(E - 1, -1, -1, dtype=torch.int32, device=hip_device)):
        env.state.copy_(snap)
        env.time.copy_(t0)
        outs = env.road.env_step(codes, 15, 1 / 15, kc, env.reward_cfg, env.time, 1.0, order)
        runs.append(([o.clone() for o in outs], env.state.clone(), env.time.clone()))
    for outs, st, t in runs[1:]:
        for x, y in zip(outs, runs[0][0]):
            assert torch.equal(x, y)
        for k in st.t:
            assert torch.equal(st[k], runs[0][1][k]), k
        assert torch.equal(t, runs[0][2])


def test_deepcopy_forks_an_independent_env(hip_device):
    """copy.deepcopy (the reference's what-if simulations, abstract.py:342-429) forks state, seeds
    and spare scenes: both copies then follow the same trajectory independently."""
    import copy
    env = VecIntersectionEnv({**ENV_JSON, "num_envs": 16, "device": hip_device, "auto_reset": True, "duration": 1})
    env.reset(seed=9)
    a0 = torch.zeros(16, dtype=torch.int64, device=hip_device)
    env.step(a0)
    env.step(a0)  # spare resets in flight on both side streams when the fork clones them
    fork = copy.deepcopy(env)
    a = torch.ones(16, dtype=torch.int64, device=hip_device)
    for _ in range(4):
        r1 = env.step(a)
        r2 = fork.step(a)
        assert torch.equal(r1[0], r2[0]) and torch.equal(r1[1], r2[1])
    assert torch.equal(env.state["x"], fork.state["x"]) and env.state["x"].data_ptr() != fork.state["x"].data_ptr()


def test_regulation_chunks_with_yields_vs_oracle(hip_device):
    """RegulatedRoad.enforce_road_rules (regulation.py:34-103) with more live pairs in a wavefront
    than one chunk of RQ_PAIRS (256) holds, on crossing routes: two dense envs share the wave (16
    initial vehicles, a spawn every step), env 0's pairs first, env 1's after them, past the first
    chunk; reset and fourteen steps equal the oracle, the yielding flags and every other discrete
    field exact, and at steps with more than 256 pairs both envs yield (chunks that
    contain conflicting pairs, yields decided in different chunks)."""
    E = 2
    cfg = {**ENV_JSON, "num_envs": E, "device": hip_device, "initial_vehicle_count": 16, "spawn_probability": 1.0,
           "duration": 100}
    env = VecIntersectionEnv(cfg)
    env.reset(seed=11)
    net = intersection_network()
    o = Oracle(net.table, P_IX)
    icfg = ix_cfg(net, {**VecIntersectionEnv.default_config(), **cfg}, P_IX)
    h = HostState(E, 32)
    o.ix_reset(h, icfg, [11 + e for e in range(E)])
    o.observe_kinematics(h, KIN)
    from test_ix_oracle import LONGI
    acts = np.random.default_rng(3).integers(0, 3, size=(14, E))
    chunked = 0  # steps with more than RQ_PAIRS live pairs in the wave and yields in both envs
    for p in range(14):
        live = (h["kind"] > 0).sum(1)
        tot = int(sum(n * (n - 1) // 2 for n in live))
        a = torch.from_numpy(acts[p]).to(hip_device)
        env.step(a)
        o.simulate(h, [LONGI[int(x)] for x in acts[p]], 15, 1 / 15)
        chunked += tot > 256 and all(bool(h["yielding"][e].any()) for e in range(E))
        o.observe_kinematics(h, KIN)
        o.ix_clear_spawn(h, icfg)
        st = env.state.to_numpy()
        for e in range(E):
            same_state(env_view(st, e), {k: v[e:e + 1] for k, v in h.a.items()}, EPISODE_TOL, f"dense {e} {p}")
    assert chunked >= 2, chunked


@pytest.mark.parametrize("slots", [16, 96])
def test_slot_classes_match_the_oracle(slots, hip_device):
    """Other slot widths: 16 (tight: spawns beyond the last slot are dropped after their draws)
    and 96 (the 128-slot kernels, two 64-lane chunks in the scene kernels); reset and three
    steps equal the oracle's, which applies the same rules."""
    E = 8
    env = VecIntersectionEnv({**ENV_JSON, "num_envs": E, "device": hip_device, "vehicle_slots": slots})
    obs, _ = env.reset(seed=40)
    net = intersection_network()
    o = Oracle(net.table, P_IX)
    cfg = ix_cfg(net, VecIntersectionEnv.default_config(), P_IX)
    h = HostState(E, slots)
    o.ix_reset(h, cfg, [40 + e for e in range(E)])
    want, _ = o.observe_kinematics(h, KIN)
    assert np.max(np.abs(obs.cpu().numpy() - want)) <= 1e-6
    g = torch.Generator(device=hip_device).manual_seed(5)
    from test_ix_oracle import LONGI
    for p in range(3):
        a = torch.randint(0, 3, (E,), device=hip_device, generator=g)
        obs, rew, term, trunc, _ = env.step(a)
        o.simulate(h, [LONGI[int(x)] for x in a.cpu().numpy()], 15, 1 / 15)
        want, _ = o.observe_kinematics(h, KIN)
        o.ix_clear_spawn(h, cfg)
        st = env.state.to_numpy()
        for e in range(E):
            same_state(env_view(st, e), {k: v[e:e + 1] for k, v in h.a.items()}, EPISODE_TOL, f"{slots} {e} {p}")
        assert np.max(np.abs(obs.cpu().numpy() - want)) <= 1e-4


@pytest.mark.parametrize("streams", [2, 3])
def test_reset_right_after_step_joins_the_background_resets(streams, hip_device):
    """reset() straight after steps whose auto-resets keep every side stream busy: it waits for
    all of them (not only the latest) before replacing the spare buffers (or rebuilding with a new
    config), so the result equals a fresh env's."""
    cfg = {**ENV_JSON, "num_envs": 32, "device": hip_device, "auto_reset": True, "duration": 1,
           "reset_streams": streams}
    env = VecIntersectionEnv(cfg)
    env.reset(seed=3)
    a = torch.ones(32, dtype=torch.int64, device=hip_device)
    for _ in range(streams + 1):  # duration 1: every env finishes, every step launches spare resets
        env.step(a)
    obs, _ = env.reset(seed=11, options={"config": {"initial_vehicle_count": 8}})
    fresh = VecIntersectionEnv({**cfg, "initial_vehicle_count": 8})
    want, _ = fresh.reset(seed=11)
    assert torch.equal(obs, want)
    for _ in range(3):
        r1, r2 = env.step(a), fresh.step(a)
        assert torch.equal(r1[0], r2[0]) and torch.equal(r1[1], r2[1])
    obs, _ = env.reset(seed=11)  # same config, buffers kept: the spare reset is joined too
    want, _ = fresh.reset(seed=11)
    assert torch.equal(obs, want)


def test_masked_observation_keeps_the_other_envs_ids(hip_device):
    """An auto-reset step re-observes only the finished envs: observed_ids of the others stay those
    of their last full observation."""
    env = VecIntersectionEnv({**ENV_JSON, "num_envs": 16, "device": hip_device})
    env.reset(seed=4)
    ot = env.observation_type
    ot.observe()
    full = ot.observed_ids.clone()
    mask = torch.zeros(16, dtype=torch.int32, device=hip_device)
    mask[3] = 1
    ot.observe(mask=mask, out=torch.empty((16, ot.vehicles_count, len(ot.features)), device=hip_device))
    keep = torch.arange(16, device=hip_device) != 3
    assert torch.equal(ot.observed_ids[keep], full[keep])


def test_overlapped_resets_with_an_occupancy_grid(hip_device):
    """A non-Kinematics observation with overlapped resets: the finished envs' rows are their new
    scenes' grids, the others' the grid observed before clear / spawn -- as the in-place path."""
    grid = {"type": "OccupancyGrid", "features": ["presence", "vx", "vy"], "grid_size": [[-27.5, 27.5], [-27.5, 27.5]],
            "grid_step": [5, 5]}
    cfg = {"observation": grid, "num_envs": 32, "device": hip_device, "auto_reset": True, "duration": 2}
    a = VecIntersectionEnv({**cfg, "overlap_resets": True})
    b = VecIntersectionEnv({**cfg, "overlap_resets": False})
    a.reset(seed=5)
    b.reset(seed=5)
    g = torch.Generator(device=hip_device).manual_seed(9)
    for t in range(5):
        act = torch.randint(0, 3, (32,), device=hip_device, generator=g)
        ra, rb = a.step(act), b.step(act)
        for x, y in zip(ra[:4], rb[:4]):
            assert torch.equal(x, y), t
        assert torch.equal(ra[4]["final_observation"], rb[4]["final_observation"])


def test_single_vehicle_observation_has_padding_ids(hip_device):
    """vehicles_count 1 (the ego alone): observed_ids' placeholder column is -1, also for the envs
    the overlapped auto-reset re-observes."""
    obs1 = dict(ENV_JSON["observation"], vehicles_count=1)
    env = VecIntersectionEnv({"observation": obs1, "num_envs": 16, "device": hip_device, "auto_reset": True,
                              "duration": 1})
    env.reset(seed=2)
    assert torch.equal(env.observation_type.observed_ids.cpu(), torch.full((16, 1), -1, dtype=torch.int32))
    for _ in range(3):
        env.step(torch.ones(16, dtype=torch.int64, device=hip_device))
        assert torch.equal(env.observation_type.observed_ids.cpu(), torch.full((16, 1), -1, dtype=torch.int32))


def test_device_episodes_match_the_reference_env(hip_device):
    """All 18 episodes of the reference's own IntersectionEnv (envref fixtures: reset(seed) and 13
    env.json steps, crashes, arrivals and rejected spawns among them) replayed in one batch from
    their seeds: observation, reward, flags, the info dict, the state after clear / spawn, and
    each env's np_random state word for word after every step."""
    from test_ix_env_oracle import ENVREF, INFO_TERMS, standstill_links
    refs = [load_golden(p) for p in ENVREF]
    links = [standstill_links(d) for d in refs]  # the vehicles the standstill chaos reaches (CPU)
    E = len(refs)
    env = VecIntersectionEnv({**ENV_JSON, "num_envs": E, "device": hip_device})
    obs, info = env.reset(seed=[int(d["meta"][0]) for d in refs])
    st = env.state.to_numpy()
    for e, d in enumerate(refs):
        same_state(env_view(st, e), HostState.from_ix(d, "pre", 0, pad_to=32), 1e-9, f"reset {e}")
        assert np.max(np.abs(obs[e].cpu().numpy() - d["obs0"])) <= 1e-6, e
    steps = int(refs[0]["meta"][1])
    acts = np.stack([d["actions"] for d in refs], 1)
    for p in range(steps):
        obs, rew, term, trunc, info = env.step(torch.from_numpy(acts[p]).to(hip_device))
        st = env.state.to_numpy()
        terms = np.stack([info["rewards"][n].cpu().numpy() for n in INFO_TERMS], 1)
        speed, crashed = info["speed"].cpu().numpy(), info["crashed"].cpu().numpy()
        ar, at = info["agents_rewards"][0].cpu().numpy(), info["agents_terminated"][0].cpu().numpy()
        for e, d in enumerate(refs):
            end = HostState.from_ix(d, "end", p, pad_to=32)
            check_obs(obs[e].cpu().numpy(), d["obs"][p], end, EPISODE_TOL, f"env {e} step {p}",
                      "device envref episodes from seed")
            tol = reward_tol(end, EPISODE_TOL)  # the reward and the info terms follow the ego alone
            assert abs(float(rew[e]) - d["reward"][p]) <= tol, (e, p)
            assert bool(term[e]) == bool(d["terminated"][p]) and bool(trunc[e]) == bool(d["truncated"][p]), (e, p)
            want = d["info"][p]
            assert abs(float(speed[e]) - want[0]) <= tol * (1 + abs(want[0])) and bool(crashed[e]) == bool(want[1])
            assert terms[e, 0] == want[2] and terms[e, 2] == want[4] and terms[e, 3] == want[5], (e, p)
            assert abs(terms[e, 1] - want[3]) <= tol and abs(float(ar[e]) - want[6]) <= tol, (e, p)
            assert bool(at[e]) == bool(want[7]), (e, p)
            same_state(env_view(st, e), HostState.from_ix(d, "post", p, pad_to=32), EPISODE_TOL, f"env {e} step {p}",
                       "device envref episodes from seed", links=links[e][p][1])
            assert np.array_equal(st["rng"][e], d["rng"][p]), (e, p, "np_random state")


# one step (15 frames) from the reference's own state on the device, float64 against the reference:
# about 10x the worst values seen on the MI355X (round 5, profiles/r05/r05a_parity.json: steering
# 8.1e-9 on a 0.15 m/s vehicle -- numpy's float64 transcendentals against the device's through the
# steering law's 1 / v^2 gain, the oracle lands on the same value -- pose 2.7e-11, speed 2.1e-14,
# acceleration 4.6e-13, observations 2.2e-16, the reward the float32 rounding of the reference's);
# discrete fields, np_random and the flags exact
DEV_STEP_TOL = {"x": 1e-10, "y": 1e-10, "heading": 1e-10, "speed": 1e-12, "target_speed": 0.0, "timer": 0.0,
                "steer": 1e-7, "acc": 1e-11, "delta": 0.0}
DEV_STEP_OBS_TOL = 1e-14


def test_device_steps_from_reference_state(hip_device):
    """Every step of the 18 reference IntersectionEnv episodes (234 steps, the 12 episodes whose
    ego drives to its exit included), each started on the device from the reference's own state
    and np_random (``pre``; tests/test_ix_env_oracle.py::ref_step_input), all in one batch: the
    fused frames give the reference's ``end`` state; env.step gives its shuffled observation,
    reward, flags and info; clear / spawn its ``post`` state; and np_random's words after the step
    are the reference's.  No standstill allowance: one step holds every vehicle to DEV_STEP_TOL."""
    from test_ix_env_oracle import ENVREF, INFO_TERMS
    from test_ix_oracle import LONGI
    from topotrafficrl_amd.road import BatchedRoad
    from topotrafficrl_amd.state import BatchState
    chk = "device envref one step from reference state"
    refs = [load_golden(p) for p in ENVREF]
    cases = [(i, p) for i, d in enumerate(refs) for p in range(int(d["meta"][1]))]
    E = len(cases)
    big = HostState(E, 32)
    for e, (i, p) in enumerate(cases):
        h = ref_step_input(refs[i], p)
        for k in big.a:
            big.a[k][e] = h.a[k][0]
    acts = np.array([int(refs[i]["actions"][p]) for i, p in cases])
    env = VecIntersectionEnv({**ENV_JSON, "num_envs": E, "device": hip_device})
    env.reset(seed=0)
    # the frames alone: the state entering the observation
    frames = BatchState(E, 32, device=hip_device).load_numpy(big.a)
    BatchedRoad(env.network, frames, env.params).simulate(torch.tensor([LONGI[int(a)] for a in acts]), 15, 1 / 15)
    fr = frames.to_numpy()
    for e, (i, p) in enumerate(cases):
        same_state(env_view(fr, e), HostState.from_ix(refs[i], "end", p, pad_to=32), DEV_STEP_TOL,
                   f"envref_ix_s{int(refs[i]['meta'][0])} step {p}", chk, standstill=False)
    # the whole env.step from the same state
    env.state.load_numpy(big.a)
    env.time.copy_(torch.tensor([float(p) for _, p in cases], dtype=torch.float64))
    obs, rew, term, trunc, info = env.step(torch.from_numpy(acts).to(hip_device))
    st = env.state.to_numpy()
    obs = obs.cpu().numpy()
    terms = np.stack([info["rewards"][n].cpu().numpy() for n in INFO_TERMS], 1)
    speed, crashed = info["speed"].cpu().numpy(), info["crashed"].cpu().numpy()
    at = info["agents_terminated"][0].cpu().numpy()
    for e, (i, p) in enumerate(cases):
        d = refs[i]
        what = f"envref_ix_s{int(d['meta'][0])} step {p}"
        err = np.abs(obs[e].astype(np.float64) - d["obs"][p])
        parity_log.note(chk, "obs", err, what)
        assert err.max() <= DEV_STEP_OBS_TOL, (what, "obs", err.max())
        parity_log.note(chk, "reward", abs(float(rew[e]) - d["reward"][p]), what)
        assert rew[e].item() == float(np.float32(d["reward"][p])), (what, "reward: float32 of the reference's")
        assert bool(term[e]) == bool(d["terminated"][p]) and bool(trunc[e]) == bool(d["truncated"][p]), what
        want = d["info"][p]
        assert abs(float(speed[e]) - want[0]) <= DEV_STEP_TOL["speed"] * (1 + abs(want[0])), (what, "info speed")
        parity_log.note(chk, "info high_speed_reward", abs(terms[e, 1] - want[3]), what)
        assert bool(crashed[e]) == bool(want[1]) and bool(at[e]) == bool(want[7]), what
        assert terms[e, 0] == want[2] and terms[e, 2] == want[4] and terms[e, 3] == want[5], what
        assert terms[e, 1] == np.float32(want[3]), (what, "high_speed_reward: float32 of the reference's")
        same_state(env_view(st, e), HostState.from_ix(d, "post", p, pad_to=32), DEV_STEP_TOL, what, chk + " (post)",
                   standstill=False)
        assert np.array_equal(st["rng"][e], d["rng"][p]), (what, "np_random state")
    parity_log.count(chk, "steps", E)
    parity_log.count(chk, "arrived steps", int(sum(refs[i]["info"][p][4] > 0 for i, p in cases)))


def test_negative_dispatch_order_entry_is_an_idle_slot(hip_device):
    """A negative entry of the dispatch order is an idle workgroup slot (not row -1): the env it
    replaces is left untouched by the launch, every other env steps as under slot order."""
    E = 16
    env = VecIntersectionEnv({**ENV_JSON, "num_envs": E, "device": hip_device})
    env.reset(seed=8)
    snap, t0 = env.state.clone(), env.time.clone()
    codes = env.action_type._codes(torch.ones(E, dtype=torch.int64, device=hip_device))
    kc = env.observation_type.fused_cfg()
    env.road.env_step(codes, 15, 1 / 15, kc, env.reward_cfg, env.time, 1.0, None)
    full = env.state.clone()
    env.state.copy_(snap)
    env.time.copy_(t0)
    order = torch.arange(E, dtype=torch.int32, device=hip_device)
    order[5] = -1
    env.road.env_step(codes, 15, 1 / 15, kc, env.reward_cfg, env.time, 1.0, order)
    keep = torch.arange(E, device=hip_device) != 5
    for k in env.state.t:
        assert torch.equal(env.state[k][keep], full[k][keep]), k
        assert torch.equal(env.state[k][5], snap[k][5]), k
