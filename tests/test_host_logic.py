"""Host-side logic on CPU: constants and config builders mirror the reference, and
property tests of the float64 oracle (hypothesis) that the HIP path is also held to."""
import numpy as np
import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

from conftest import golden_files, load_golden
from oracle.oracle import HostState, Oracle
from topotrafficrl_amd import _abi
from topotrafficrl_amd.action import BatchedDiscreteMetaAction, action_factory
from topotrafficrl_amd.envs import VecHighwayEnv


def test_params_are_the_reference_class_constants():
    p = _abi.default_params()
    # behavior.py:21-46, controller.py:24-33, kinematics.py:21-29, objects.py:62, controller.py:259
    assert (p.acc_max, p.comfort_acc_max, p.comfort_acc_min) == (6.0, 3.0, -5.0)
    assert (p.distance_wanted, p.time_wanted, p.politeness) == (10.0, 1.5, 0.0)
    assert (p.lane_change_min_acc_gain, p.lane_change_max_braking, p.lane_change_delay) == (0.2, 2.0, 1.0)
    assert p.tau_pursuit == 0.5 * 0.2 and p.kp_a == 1 / 0.6 and p.kp_heading == 1 / 0.2 and p.kp_lateral == 1 / 0.6
    assert p.max_steering == np.pi / 3 and p.diagonal == np.sqrt(5.0 ** 2 + 2.0 ** 2)
    assert p.gap_denom == 2 * np.sqrt(15.0)
    assert list(p.target_speeds[:p.n_target_speeds]) == [20.0, 25.0, 30.0]
    with pytest.raises(KeyError):
        _abi.default_params(not_a_constant=1.0)


def test_lane_table_matches_reference_network():
    d = load_golden(golden_files("highway_n8_s0*")[0])
    t = _abi.straight_lane_table(4)
    g = _abi.lane_table_from_arrays(d["lane_table"])
    for f in ("start_x", "start_y", "dir_x", "dir_y", "length", "width", "heading", "speed_limit"):
        assert list(getattr(t, f)[:4]) == list(getattr(g, f)[:4]), f
    rot = _abi.straight_lane_table(3, angle=0.3)
    assert abs(rot.heading[0] + 0.3) < 1e-15 and rot.n_lanes == 3  # road.py:306 rotates by -angle


def test_observation_config_builders():
    k = _abi.kin_cfg()  # observation.py:213-225 default ranges
    assert (k.range_lo[1], k.range_hi[1]) == (-200.0, 200.0) and (k.range_lo[2], k.range_hi[2]) == (-16, 16)
    assert not k.has_range[0] and k.vehicles_count == 5 and k.n_features == 5
    with pytest.raises(ValueError):
        _abi.kin_cfg(order="random")
    with pytest.raises(ValueError):
        _abi.kin_cfg(features=["presence", "bogus"])
    g = _abi.grid_cfg(grid_size=[[-32, 32], [-32, 32]], grid_step=[2, 2])
    assert (g.shape_x, g.shape_y) == (32, 32)
    g = _abi.grid_cfg()  # observation.py:282-283 defaults: 55 m / 5 m -> 11 cells
    assert (g.shape_x, g.shape_y) == (11, 11) and g.has_range[3] and g.has_range[4]
    with pytest.raises(NotImplementedError):
        _abi.grid_cfg(absolute=True)


def test_pcg64_state_export_matches_numpy():
    for seed in (0, 1, 12345, 2 ** 40 + 3):
        st_ = np.random.PCG64(seed).state["state"]
        w = _abi.pcg64_states([seed])[0]
        assert (int(w[0]) << 64 | int(w[1])) == st_["state"] and (int(w[2]) << 64 | int(w[3])) == st_["inc"]


def test_action_tables():
    class _Env:
        pass
    a = BatchedDiscreteMetaAction(_Env(), longitudinal=True, lateral=False)
    assert a.actions == {0: "SLOWER", 1: "IDLE", 2: "FASTER"} and a.space().n == 3
    a = BatchedDiscreteMetaAction(_Env())
    assert a.actions == {0: "LANE_LEFT", 1: "IDLE", 2: "LANE_RIGHT", 3: "FASTER", 4: "SLOWER"}
    with pytest.raises(ValueError):
        BatchedDiscreteMetaAction(_Env(), longitudinal=False, lateral=False)
    with pytest.raises(NotImplementedError):
        action_factory(_Env(), {"type": "ContinuousAction"})
    with pytest.raises(ValueError):
        action_factory(_Env(), {"type": "Nope"})


def test_env_default_config_keeps_reference_keys():
    c = VecHighwayEnv.default_config()
    for k in ("observation", "action", "simulation_frequency", "policy_frequency", "other_vehicles_type",
              "duration", "collision_reward", "high_speed_reward", "reward_speed_range", "normalize_reward",
              "offroad_terminal", "manual_control"):
        assert k in c, k
    assert c["simulation_frequency"] // c["policy_frequency"] == 15


LANES = _abi.straight_lane_table(4)
PAR = _abi.default_params()


def _scene(n, seeds):
    o = Oracle(LANES, PAR)
    h = HostState(len(seeds), n)
    o.reset_highway(h, _abi.reset_cfg(n, LANES), seeds)
    return o, h


@settings(max_examples=25, deadline=None)
@given(n=st.integers(2, 80), seed=st.integers(0, 2 ** 31))
def test_scene_invariants(n, seed):
    """create_random: x strictly increasing, speeds in [21, 24), DELTA in [3.5, 4.5), timer in [0, 1)."""
    _, h = _scene(n, [seed])
    x = h["x"][0]
    assert np.all(np.diff(x) > 0)
    assert np.all((h["speed"][0, 1:] >= 21.0) & (h["speed"][0, 1:] < 24.0))
    assert np.all((h["delta"][0, 1:] >= 3.5) & (h["delta"][0, 1:] < 4.5))
    assert np.all((h["timer"][0, 1:] >= 0) & (h["timer"][0, 1:] < 1))
    assert h["kind"][0, 0] == _abi.MDP and np.all(h["kind"][0, 1:] == _abi.IDM)


@settings(max_examples=15, deadline=None)
@given(n=st.integers(2, 48), pad=st.integers(1, 40), seed=st.integers(0, 2 ** 31),
       action=st.integers(0, 4))
def test_absent_slots_are_invisible(n, pad, seed, action):
    o, h = _scene(n, [seed])
    wide = HostState(1, n + pad)
    per_env = ("reg_steps", "rng")
    for k, v in h.a.items():
        if k in per_env:
            wide.a[k][:] = v
        else:
            wide.a[k][:, :n] = v
    o.simulate(h, [action], 15, 1 / 15)
    o.simulate(wide, [action], 15, 1 / 15)
    for k, v in h.a.items():
        assert np.array_equal(wide.a[k] if k in per_env else wide.a[k][:, :n], v), k


@settings(max_examples=10, deadline=None)
@given(seeds=st.lists(st.integers(0, 2 ** 31), min_size=2, max_size=5), n=st.integers(2, 40))
def test_envs_are_independent(seeds, n):
    o, batch = _scene(n, seeds)
    acts = np.arange(len(seeds), dtype=np.int32) % 5
    o.simulate(batch, acts, 15, 1 / 15)
    for e, s in enumerate(seeds):
        _, one = _scene(n, [s])
        o.simulate(one, acts[e:e + 1], 15, 1 / 15)
        for k in one.a:
            assert np.array_equal(batch.a[k][e], one.a[k][0]), k


@settings(max_examples=10, deadline=None)
@given(seed=st.integers(0, 2 ** 31))
def test_impacts_only_from_close_pairs(seed):
    """A vehicle carries an impact only if some other vehicle is within the SAT prefilter range."""
    o, h = _scene(40, [seed])
    h.a["x"][0, 5] = h.a["x"][0, 4] + 1.0  # force an overlap
    h.a["y"][0, 5] = h.a["y"][0, 4]
    o.road_step(h)
    imp = np.flatnonzero(h["has_impact"][0])
    assert 4 in imp and 5 in imp
    for i in imp:
        d = np.hypot(h["x"][0] - h["x"][0, i], h["y"][0] - h["y"][0, i])
        d[i] = np.inf
        assert d.min() < PAR.diagonal + 45.0 / 15 + 1


def test_rewards_template():
    o, h = _scene(10, [3])
    cfg = _abi.reward_cfg()
    r, term, trunc = o.rewards(h, cfg, 0.0)
    assert not term[0] and not trunc[0]
    assert abs(r[0] - 0.4 * 0.5) < 1e-7  # speed 25 in [20, 30] -> 0.5, on road, not crashed
    h.a["crashed"][0, 0] = 1
    r, term, _ = o.rewards(h, cfg, 40.0)
    assert term[0] and abs(r[0] - (-1.0 + 0.2)) < 1e-7


def _reward_from_terms(cfg, c):
    """IntersectionEnv._agent_reward (intersection_env.py:78-93) from the _agent_rewards dict."""
    r = cfg.collision_reward * c[0] + cfg.high_speed_reward * c[1] + cfg.arrived_reward * c[2]
    r = cfg.arrived_reward if c[2] else r
    r *= c[3]
    if cfg.normalize_reward:
        r = (r - cfg.collision_reward) / (cfg.arrived_reward - cfg.collision_reward)
    return r


def test_reward_terms_rebuild_the_reward():
    """info["rewards"] terms: 0/1 flags and the clipped speed term; _agent_reward recombines them."""
    o, h = _scene(10, [3, 4, 5])
    h.a["crashed"][1, 0] = 1
    h.a["y"][2, 0] = 50.0  # off road
    for norm in (False, True):
        cfg = _abi.reward_cfg(normalize_reward=norm)
        r, term, _, comp = o.rewards(h, cfg, 0.0, components=True)
        assert comp.shape == (3, 4)
        assert comp[1, 0] == 1 and comp[0, 0] == 0 and comp[2, 3] == 0 and comp[0, 3] == 1
        assert np.all((comp[:, 1] >= 0) & (comp[:, 1] <= 1))
        for e in range(3):
            assert abs(r[e] - _reward_from_terms(cfg, comp[e])) < 1e-6
