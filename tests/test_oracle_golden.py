"""The float64 oracle (oracle/ttrl_oracle.c) against golden vectors captured from the
unmodified reference (oracle/gen_golden.py).  CPU only.

Pinned here: Road.act/Road.step per frame (positions/speeds/headings to 1e-12, every
discrete field exact), the fused 15-frame policy step, Road.neighbour_vehicles,
Kinematics (5x5 default, 15x7 env.json) and OccupancyGrid (7x32x32 dense, 4x11x11 on_road)
observations bit-identical, TimeToCollision exact and Lidar to float32 rounding, and the
numpy-PCG64 scene generator bit-identical.
"""
import numpy as np
import pytest

from conftest import golden_files, load_golden, scene_files
from oracle.oracle import HostState, Oracle
from topotrafficrl_amd import _abi

P = _abi.default_params()
KD = _abi.kin_cfg()
K15 = _abi.kin_cfg(features=["presence", "x", "y", "vx", "vy", "cos_h", "sin_h"], vehicles_count=15,
                   features_range={"x": [-100, 100], "y": [-100, 100], "vx": [-20, 20], "vy": [-20, 20]})
G7 = _abi.grid_cfg(features=["presence", "x", "y", "vx", "vy", "cos_h", "sin_h"],
                   features_range={"x": [-100, 100], "y": [-100, 100], "vx": [-20, 20], "vy": [-20, 20]},
                   grid_size=[[-32, 32], [-32, 32]], grid_step=[2, 2])
GR = _abi.grid_cfg()
CONT = ["x", "y", "heading", "speed", "timer", "target_speed", "steer", "acc"]
DISC = ["lane", "target_lane", "crashed", "has_impact", "speed_index"]
IDS = lambda p: p.split("/")[-1][:-4]  # noqa: E731


def check(h: HostState, g: HostState, tol: float):
    for k in CONT:
        err = np.max(np.abs(h[k] - g[k]) / (1 + np.abs(g[k])))
        assert err <= tol, (k, err)
    imp = g["has_impact"].astype(bool)
    for k in ("impact_x", "impact_y"):
        assert np.max(np.abs(h[k][imp] - g[k][imp]), initial=0.0) <= tol, k
    for k in DISC:
        assert np.array_equal(h[k], g[k]), k


@pytest.fixture(scope="module")
def cases():
    return {IDS(p): load_golden(p) for p in golden_files()}


@pytest.mark.parametrize("name", [IDS(p) for p in golden_files()])
def test_every_frame(name, cases):
    d = cases[name]
    o = Oracle(_abi.lane_table_from_arrays(d["lane_table"]), P)
    for f in range(d["x"].shape[0] - 1):
        h = HostState.from_golden(d, f)
        if f % 15 == 0:
            o.meta_action(h, [int(d["actions"][f // 15])])
        o.road_act(h)
        check(h, HostState.from_golden(d, f, prefix="act_"), 1e-12)
        o.road_step(h)
        check(h, HostState.from_golden(d, f + 1), 1e-12)


@pytest.mark.parametrize("name", [IDS(p) for p in golden_files()])
def test_frame_margins_leave_the_frame_unchanged(name, cases):
    """oracle_frame_margins (the float32 flip classifier) steps the frame exactly as Road.act +
    Road.step do, and reports a finite margin for every vehicle that decides anything."""
    d = cases[name]
    o = Oracle(_abi.lane_table_from_arrays(d["lane_table"]), P)
    tiny = 0
    for f in range(d["x"].shape[0] - 1):
        h = HostState.from_golden(d, f)
        act = [int(d["actions"][f // 15])] if f % 15 == 0 else None
        m = o.frame_margins(h, act)
        check(h, HostState.from_golden(d, f + 1), 1e-12)
        assert np.all(m >= 0) and np.all(np.isfinite(m))
        tiny += int((m < 1e-5).sum())
    assert tiny < 0.5 * m.size * (d["x"].shape[0] - 1)  # small margins are the exception (pile-ups: contacts)


@pytest.mark.parametrize("name", [IDS(p) for p in golden_files()])
def test_frame_links_are_local_and_leave_the_frame_unchanged(name, cases):
    """oracle_frame_links (the causal links of the float32 flip classifier) steps the frame
    exactly as oracle_frame_margins does, never overflows its rows, and links a vehicle only to
    vehicles of its own env near it: an earlier vehicle within the abort's desired gap
    (d0 + v T + v dv / (2 sqrt(a b)) < 200 m at these speeds) or a collision partner."""
    d = cases[name]
    o = Oracle(_abi.lane_table_from_arrays(d["lane_table"]), P)
    n_links = 0
    for f in range(d["x"].shape[0] - 1):
        h = HostState.from_golden(d, f)
        h0 = h.copy()
        act = [int(d["actions"][f // 15])] if f % 15 == 0 else None
        m1, lk = o.frame_margins(h, act, links=True)
        g = h0.copy()
        m0 = o.frame_margins(g, act)
        assert np.array_equal(m0, m1)
        for k in h.a:
            assert np.array_equal(h.a[k], g.a[k], equal_nan=True), k
        assert not np.any(lk == -2) and np.all(lk < h.N)
        for e, i, q in zip(*np.nonzero(lk >= 0)):
            j = lk[e, i, q]
            assert j != i and h0["kind"][e, j] != 0
            assert abs(h0["x"][e, j] - h0["x"][e, i]) < 200.0
        n_links += int((lk >= 0).sum())
    assert n_links > 0 or not name.startswith("dense")  # the pile-up scenes always have partners


@pytest.mark.parametrize("name", [IDS(p) for p in golden_files()])
def test_policy_step_rollout(name, cases):
    d = cases[name]
    o = Oracle(_abi.lane_table_from_arrays(d["lane_table"]), P)
    h = HostState.from_golden(d, 0)
    for p in range(int(d["meta"][2])):
        o.simulate(h, [int(d["actions"][p])], 15, 1 / 15)
        check(h, HostState.from_golden(d, 15 * (p + 1)), 1e-10)


@pytest.mark.parametrize("name", [IDS(p) for p in golden_files()])
def test_neighbour_vehicles(name, cases):
    d = cases[name]
    o = Oracle(_abi.lane_table_from_arrays(d["lane_table"]), P)
    for f in range(d["x"].shape[0] - 1):
        h = HostState.from_golden(d, f, prefix="act_")
        fr, rr = o.neighbours(h)
        assert np.array_equal(fr[0], d["nbr"][f][0]) and np.array_equal(rr[0], d["nbr"][f][1])
        fr, rr = o.neighbours(h, h["target_lane"])
        assert np.array_equal(fr[0], d["nbr"][f][2]) and np.array_equal(rr[0], d["nbr"][f][3])


@pytest.mark.parametrize("name", [IDS(p) for p in golden_files()])
def test_observations(name, cases):
    d = cases[name]
    o = Oracle(_abi.lane_table_from_arrays(d["lane_table"]), P)
    for p in range(int(d["meta"][2]) + 1):
        h = HostState.from_golden(d, 15 * p)
        obs, ids = o.observe_kinematics(h, _abi.kin_cfg(lanes_on_road=int(d["meta"][4])))
        assert np.array_equal(obs[0], d["kin5"][p]) and np.array_equal(ids[0], d["kin5_ids"][p])
        obs, ids = o.observe_kinematics(h, K15)
        assert np.array_equal(obs[0], d["kin15"][p]) and np.array_equal(ids[0], d["kin15_ids"][p])
        assert np.array_equal(o.observe_grid(h, G7)[0], d["grid7"][p])
        assert np.array_equal(o.observe_grid(h, GR)[0], d["grid_onroad"][p])


@pytest.mark.parametrize("name", [IDS(p) for p in golden_files()])
def test_observation_fixtures_equal_the_reference_observers(name, cases):
    """The observation fixtures above (gen_golden.py restates the observers' pandas assembly) equal,
    bit for bit, what the reference's own KinematicObservation / OccupancyGridObservation /
    TimeToCollisionObservation / LidarObservation.observe return on the same scenes
    (oracle/gen_golden_obs.py, observation.py:126-151, 233-275, 353-483, 694-768)."""
    d = cases[name]
    ref = load_golden(golden_files(f"obsref_{name}.npz")[0])
    for k in ("kin5", "kin15", "grid7", "grid_onroad", "ttc", "lidar"):
        assert ref[k].shape == d[k].shape, k
        assert np.array_equal(ref[k].astype(d[k].dtype), d[k]), k


@pytest.mark.parametrize("seed", range(6))
def test_intersection_observation_fixtures_equal_the_reference_observer(seed):
    """The intersection episodes' observations (absolute Kinematics 15x7, order "shuffled" drawing
    env.np_random.shuffle(obs[1:])) equal the reference KinematicObservation's on the same episode,
    including the generator draws (oracle/gen_golden_obs.py::ix_episode)."""
    d = load_golden(golden_files(f"ix_s{seed}.npz")[0])
    ref = load_golden(golden_files(f"obsref_ix_s{seed}.npz")[0])
    assert np.array_equal(ref["obs0"], d["obs0"]) and np.array_equal(ref["obs"], d["obs"])


@pytest.mark.parametrize("name", [IDS(p) for p in golden_files()])
def test_ttc_and_lidar_observations(name, cases):
    """TimeToCollision (the reference's own compute_ttc_grid, finite_mdp.py:104-167) exact;
    Lidar (LidarObservation.trace over utils.rect_corners / distance_to_rect) to float32."""
    d = cases[name]
    o = Oracle(_abi.lane_table_from_arrays(d["lane_table"]), P)
    for p in range(int(d["meta"][2]) + 1):
        h = HostState.from_golden(d, 15 * p)
        assert np.array_equal(o.observe_ttc(h, _abi.ttc_cfg())[0], d["ttc"][p])
        lid = o.observe_lidar(h, _abi.lidar_cfg())[0]
        assert np.max(np.abs(lid - d["lidar"][p])) <= 1e-6 * (1 + np.max(np.abs(d["lidar"][p])))


@pytest.mark.parametrize("name", [IDS(p) for p in scene_files()])
def test_scene_generation_matches_reference_rng(name, cases):
    d = cases[name]
    n, seed = int(d["meta"][0]), int(d["meta"][1])
    lanes = _abi.lane_table_from_arrays(d["lane_table"])
    o = Oracle(lanes, P)
    h = HostState(1, n)
    o.reset_highway(h, _abi.reset_cfg(n, lanes), [seed])
    g = HostState.from_golden(d, 0)
    for k in ["x", "y", "heading", "speed", "target_speed", "timer", "delta"]:
        assert np.array_equal(h[k], g[k]), k
    for k in ["lane", "target_lane", "kind", "speed_index", "lane_change"]:
        assert np.array_equal(h[k], g[k]), k


def test_golden_covers_the_hard_cases(cases):
    """The fixtures must exercise MOBIL lane changes, aborts, impacts and crashes."""
    changes = aborts = impacts = crashes = 0
    for d in cases.values():
        before, after, lane = d["target_lane"][:-1], d["act_target_lane"], d["lane"][:-1]
        changes += int(np.sum((after != before) & (after != lane)))
        aborts += int(np.sum((after != before) & (after == lane)))
        impacts += int(np.isfinite(d["impact_x"]).sum())
        crashes += int(d["crashed"][-1].sum())
    assert changes > 50 and aborts > 0 and impacts > 100 and crashes > 50, (changes, aborts, impacts, crashes)


@pytest.mark.parametrize("name", [IDS(p) for p in golden_files()])
def test_observation_margins_leave_the_observations_unchanged(name, cases):
    """The observation margins (the float32 observation classifier) come with outputs equal to the
    plain observers', and are small in few cells: a cell is excused only near a floor / range /
    nearest-hit decision."""
    d = cases[name]
    lanes = _abi.lane_table_from_arrays(d["lane_table"])
    o = Oracle(lanes, P)
    h = HostState.from_golden(d, 15)
    grid = _abi.grid_cfg(["presence", "x", "y", "vx", "vy", "cos_h", "sin_h"], [[-32, 32], [-32, 32]], [2, 2],
                         {"x": [-100, 100], "y": [-100, 100], "vx": [-20, 20], "vy": [-20, 20]})
    for obs, cfg in ((o.observe_grid, grid), (o.observe_ttc, _abi.ttc_cfg()), (o.observe_lidar, _abi.lidar_cfg())):
        a = obs(h, cfg)
        b, m = obs(h, cfg, margins=True)
        assert np.array_equal(a, b) and m.shape[:2] == a.shape[:2]
        assert np.all(m >= 0) and np.mean(m < 1e-5) < 0.02, (cfg, np.mean(m < 1e-5))
