"""Parity at the BASELINE.json sizes: every GPU configuration of SURVEY.md §8(d) stepped on the
MI355X and through the float64 oracle (OpenMP over envs) from the same seeds and actions.

* config 2: 4096 envs x 32 vehicles, Kinematics 15x7
* config 3: 4096 envs x 128 vehicles, OccupancyGrid 7x32x32 (NS = 128: two waves per env)
* config 4: 4096 envs x 64 vehicles, Kinematics 15x7 (the headline; 4 waves/SIMD, all resident)
* config 5: 8192 envs x 64 vehicles, the fused EgoAttention-2h forward's greedy actions fed back

float64 product path: discrete fields (lane, target_lane, crashed, has_impact, speed_index,
observed slot ids, terminated / truncated) exact; continuous state within FULL_TOL relative to
1 + |x| after every policy step -- about 10x the worst values seen on the MI355X (round 5,
profiles/r05/r05a_parity.json: pose, speed, steering <= 9.6e-15, acceleration and impacts
<= 6.3e-14, timers, target speeds and DELTA exact); the Kinematics rows and the OccupancyGrid
bit-identical.  The occupancy, packing and
residency paths these configurations take (16 one-wave workgroups per CU at 64 vehicles, the
two-wave NS = 128 instance, the two-env-per-wave NS = 32 instance) are only exercised here.
"""
import numpy as np
import pytest
import torch

import parity_log
from oracle.oracle import HostState, Oracle
from topotrafficrl_amd import _abi
from topotrafficrl_amd.envs import VecHighwayEnv

pytestmark = pytest.mark.gpu

KIN15 = {"type": "Kinematics", "vehicles_count": 15, "features": ["presence", "x", "y", "vx", "vy", "cos_h", "sin_h"],
         "features_range": {"x": [-100, 100], "y": [-100, 100], "vx": [-20, 20], "vy": [-20, 20]},
         "absolute": False, "order": "sorted"}
GRID7 = {"type": "OccupancyGrid", "features": ["presence", "x", "y", "vx", "vy", "cos_h", "sin_h"],
         "features_range": {"x": [-100, 100], "y": [-100, 100], "vx": [-20, 20], "vy": [-20, 20]},
         "grid_size": [[-32, 32], [-32, 32]], "grid_step": [2, 2], "absolute": False}
# float64 continuous bounds after every fused policy step, relative to 1 + |x|
FULL_TOL = {"x": 1e-13, "y": 1e-13, "heading": 1e-13, "speed": 1e-13, "steer": 1e-13, "acc": 1e-12,
            "impact_x": 1e-12, "impact_y": 1e-12, "target_speed": 0.0, "timer": 0.0, "delta": 0.0}
DISCRETE = ["lane", "target_lane", "speed_index", "kind", "crashed", "has_impact", "lane_change"]
CONTINUOUS = ["x", "y", "heading", "speed", "target_speed", "timer", "delta", "steer", "acc"]


def _compare_state(env, h, where):
    got = env.state.to_numpy()
    for f in DISCRETE:
        bad = np.argwhere(got[f] != h[f])
        assert len(bad) == 0, f"{where}: {f} differs at (env, slot) {bad[:5].tolist()} of {len(bad)}"
    check = parity_log.current_check()
    for f in CONTINUOUS:
        d = parity_log.rel_err(got[f], h[f])
        parity_log.note(check, f, d, f"{parity_log.current_case()} {where}")
        assert float(d.max()) <= FULL_TOL[f], f"{where}: {f} max rel diff {float(d.max()):.3g} at {np.unravel_index(d.argmax(), d.shape)}"
    for f in ("impact_x", "impact_y"):  # meaningful only while has_impact is set
        m = h["has_impact"] != 0
        if m.any():
            d = parity_log.rel_err(got[f][m], h[f][m])
            parity_log.note(check, f, d, f"{parity_log.current_case()} {where}")
            assert float(d.max()) <= FULL_TOL[f], f"{where}: {f}"


def _make(E, N, obs, seed):
    env = VecHighwayEnv({"num_envs": E, "vehicles_count": N, "observation": obs, "device": "cuda:0", "dtype": "f64"})
    obs0, _ = env.reset(seed=seed)
    o = Oracle(env.network.table, env.params)
    h = HostState(E, N)
    o.reset_highway(h, env.reset_cfg, [seed + e for e in range(E)])
    return env, obs0, o, h


def _rollout(E, N, obs_cfg, seed, steps, actions_fn=None):
    env, obs, o, h = _make(E, N, obs_cfg, seed)
    _compare_state(env, h, "reset")
    kin = _abi.kin_cfg(**{k: v for k, v in obs_cfg.items() if k != "type"}) if obs_cfg["type"] == "Kinematics" else None
    grid = None if kin is not None else _abi.grid_cfg(**{k: v for k, v in obs_cfg.items() if k != "type"})
    rng = np.random.default_rng(seed)
    crashed = 0
    for t in range(1, steps + 1):
        a = rng.integers(0, 5, size=E) if actions_fn is None else actions_fn(obs, h, kin)
        obs, rew, term, trunc, info = env.step(torch.from_numpy(np.asarray(a)).to(env.device))
        o.simulate(h, np.asarray(a, dtype=np.int32), 15, 1 / 15)
        _compare_state(env, h, f"step {t}")
        if kin is not None:
            ref, ids = o.observe_kinematics(h, kin)
            err = parity_log.note(parity_log.current_check(), "obs", np.abs(obs.cpu().numpy() - ref),
                                  f"{parity_log.current_case()} step {t}")
            assert err == 0.0, f"step {t}: Kinematics rows differ by {err:.3g}"
            assert np.array_equal(env.observation_type.observed_ids.cpu().numpy(), ids), f"step {t}: observed ids"
        else:
            ref = o.observe_grid(h, grid)
            got = obs.cpu().numpy()
            bad = np.argwhere(got != ref)
            assert len(bad) == 0, f"step {t}: grid differs in {len(bad)} cells, first {bad[:3].tolist()}"
        r_ref, te_ref, tr_ref = o.rewards(h, env.reward_cfg, float(t))
        assert np.array_equal(rew.cpu().numpy(), r_ref), f"step {t}: rewards"
        assert np.array_equal(term.cpu().numpy(), te_ref) and np.array_equal(trunc.cpu().numpy(), tr_ref)
        crashed = int((h["crashed"] != 0).sum())
    return env, h, crashed


@pytest.mark.parametrize("E,N,seed", [(4096, 32, 101), (4096, 64, 202), (8192, 32, 505)],
                         ids=["config2_4096x32", "config4_4096x64", "8192x32_4wave"])
def test_full_size_kinematics_vs_oracle(E, N, seed, hip_device):
    """4096 x 32 runs the two-env-per-wave instance's 2-wave twin (2048 waves, all resident at 2 per
    SIMD); 8192 x 32 (4096 waves) its 4-wave original."""
    env, h, crashed = _rollout(E, N, KIN15, seed, steps=3)
    assert crashed > 0  # the batch is big enough to hold crashes, impacts and their SAT pairs
    assert (h["lane"] != h["target_lane"]).any() or (h["lane"][:, 1:] != 0).any()


def test_full_size_occupancy_grid_vs_oracle(hip_device):
    """config 3: 4096 x 128, OccupancyGrid 7x32x32 of the two-wave NS = 128 instance."""
    _rollout(4096, 128, GRID7, 303, steps=2)


def test_full_size_policy_in_the_loop_vs_oracle(hip_device):
    """config 5: 8192 x 64, acting through the launch the bench times: EgoAttentionPolicy.act with
    int32 actions (ttrl::ego_attention_act: forward, argmax and the epsilon-greedy draw in one
    launch) at epsilon 0 picks each env's action from the GPU observation; it equals the argmax of
    the same network's fused Q; the oracle steps with the same actions, and the float32 torch
    forward of the oracle's own observation picks the same action wherever its top-two Q margin is
    clear."""
    from topotrafficrl_amd.agent import EgoAttentionPolicy
    pol = EgoAttentionPolicy(hip_device, seed=0)
    cpu_net = EgoAttentionPolicy("cpu", seed=0, fused=False).value_net
    env, obs, o, h = _make(8192, 64, KIN15, 404)
    kin = _abi.kin_cfg(**{k: v for k, v in KIN15.items() if k != "type"})
    greedy = torch.zeros((), dtype=torch.float32, device=hip_device)  # epsilon 0 as a device scalar
    for t in range(1, 4):
        act = pol.act(obs, t, epsilon=greedy, dtype=torch.int32)
        assert act.dtype == torch.int32 and act.shape == (8192,)
        q = pol.value_net.fused_q(obs)
        assert torch.equal(act.long(), q.argmax(1)), f"step {t}: the fused acting launch's greedy actions"
        a = act.cpu().numpy()
        ref_obs, _ = o.observe_kinematics(h, kin)
        with torch.no_grad():
            q_ref = cpu_net(torch.from_numpy(ref_obs)).numpy()
        srt = np.sort(q_ref, axis=1)
        clear = (srt[:, -1] - srt[:, -2]) > 1e-4
        assert (a[clear] == q_ref.argmax(1)[clear]).all(), f"step {t}: greedy actions"
        assert np.allclose(q.cpu().numpy(), q_ref, rtol=1e-4, atol=1e-5)
        obs, rew, term, trunc, info = env.step(act)
        o.simulate(h, a.astype(np.int32), 15, 1 / 15)
        _compare_state(env, h, f"step {t}")
        ref_obs, ids = o.observe_kinematics(h, kin)
        assert np.array_equal(obs.cpu().numpy(), ref_obs), f"step {t}: Kinematics rows"
        assert np.array_equal(env.observation_type.observed_ids.cpu().numpy(), ids)


def test_config4_split_equals_one_batch(hip_device):
    """config 4's real split: two 4096-env shards, global ids [0, 4096) and
    [4096, 8192) (env_id_offset), equal one 8192-env batch bit for bit over 3 env.steps -- state,
    observation, observed ids, reward and flags -- with the actions drawn by the fused epsilon-greedy
    policy (epsilon 0.5) keyed on global env ids, so each shard's policy draws the big batch's rows."""
    from topotrafficrl_amd.agent import EgoAttentionPolicy
    E, N = 4096, 64

    def make(n, off):
        env = VecHighwayEnv({"num_envs": n, "vehicles_count": N, "observation": KIN15, "device": hip_device,
                             "dtype": "f64", "env_id_offset": off})
        return env, env.reset(seed=77)[0], EgoAttentionPolicy(hip_device, seed=3, env_id_offset=off)

    big, ob, pb = make(2 * E, 0)
    shards = [make(E, r * E) for r in range(2)]
    half = torch.zeros((), dtype=torch.float32, device=hip_device) + 0.5
    assert torch.equal(ob, torch.cat([s[1] for s in shards]))
    for t in range(3):
        ab = pb.act(ob, t, epsilon=half, dtype=torch.int32)
        acts = [p.act(o, t, epsilon=half, dtype=torch.int32) for _, o, p in shards]
        assert torch.equal(ab, torch.cat(acts)), f"step {t}: actions"
        ob, rb, tb, trb, _ = big.step(ab)
        outs = [env.step(a) for (env, _, _), a in zip(shards, acts)]
        shards = [(env, out[0], p) for (env, _, p), out in zip(shards, outs)]
        for i, x in enumerate((ob, rb, tb, trb)):
            assert torch.equal(x, torch.cat([out[i] for out in outs])), (t, i)
        ids = [env.observation_type.observed_ids for env, _, _ in shards]
        assert torch.equal(big.observation_type.observed_ids, torch.cat(ids)), t
    for k in big.state.t:
        assert torch.equal(big.state[k], torch.cat([env.state[k] for env, _, _ in shards])), k
