"""The intersection scenario on the MI355X (simulate kernel, NET_GRAPH instance) against the
golden episodes of the reference (oracle/gen_golden_ix.py) and the float64 oracle.

Against the reference's goldens, continuous fields relative to 1 + |x| within about 10x the worst
values seen on the MI355X (round 5, profiles/r05/r05a_parity.json): one frame IX_FRAME_TOL, a
15-frame fused step IX_STEP_TOL.  The steering command is the loosest field: a vehicle at
0.15 m/s (ix_s3 step 5) carries the difference between numpy's float64 transcendentals and the
device's (or glibc's: the oracle lands on the same value) through the steering law's 1 / v^2
gain, 4.5e-10 in one frame and 8.1e-9 after fifteen; its pose then moves by 2.7e-11.  Against
the float64 oracle itself (the crowded-lane cases) the highway's F64_TOL.  Every discrete field
exact, including routes (popped in place by follow_road), RegulatedRoad yields and the
regulation frame counter."""
import numpy as np
import pytest
import torch

import parity_log
from conftest import golden_files, load_golden
from oracle.oracle import HostState
from test_gpu_parity import F64_TOL, to_dev
from test_ix_oracle import LONGI, P_IX, ix_lanes
from topotrafficrl_amd.road import BatchedRoad, RoadNetwork

pytestmark = pytest.mark.gpu

CONT = ["x", "y", "heading", "speed", "target_speed", "timer", "steer", "acc"]
DISC = ["lane", "target_lane", "crashed", "has_impact", "speed_index", "kind", "yielding", "route_n",
        "route_road", "route_lane"]
IDS = lambda p: p.split("/")[-1][:-4]  # noqa: E731
IX_FRAME_TOL = {"x": 1e-13, "y": 1e-13, "heading": 1e-13, "speed": 1e-13, "steer": 5e-9, "acc": 1e-12,
                "target_speed": 0.0, "timer": 0.0, "impact_x": 1e-13, "impact_y": 1e-13}
IX_STEP_TOL = {"x": 1e-10, "y": 1e-10, "heading": 1e-10, "speed": 1e-12, "steer": 1e-7, "acc": 1e-11,
               "target_speed": 0.0, "timer": 0.0, "impact_x": 1e-13, "impact_y": 1e-13}


def compare(dev, g: HostState, tol: float, n: int):
    d = dev.to_numpy()
    check, where = parity_log.current_check(), parity_log.current_case()
    for k in CONT:
        a, b = d[k][:, :n].astype(np.float64), g[k][:, :n]
        err = parity_log.note(check, k, parity_log.rel_err(a, b), where)
        t = tol[k] if isinstance(tol, dict) else tol
        assert err <= t, (k, err, t)
    imp = g["has_impact"][:, :n].astype(bool)
    for k in ("impact_x", "impact_y"):
        err = parity_log.note(check, k, np.abs(d[k][:, :n][imp] - g[k][:, :n][imp]), where)
        assert err <= (tol[k] if isinstance(tol, dict) else tol), k
    for k in DISC:
        assert np.array_equal(d[k][:, :n], g[k][:, :n]), (k, d[k][:, :n], g[k][:, :n])
    assert np.array_equal(d["reg_steps"], g["reg_steps"])


@pytest.mark.parametrize("pad", [32, 64])
@pytest.mark.parametrize("path", golden_files("ix_*"), ids=IDS)
def test_ix_frames_vs_golden(path, pad, hip_device):
    d = load_golden(path)
    road = None
    for p in range(int(d["meta"][1])):
        n = int((d["pre_kind"][p] > 0).sum())
        dev = to_dev(HostState.from_ix(d, "pre", p), hip_device, pad_to=pad)
        road = BatchedRoad(RoadNetwork(ix_lanes(d)), dev, P_IX)
        road.meta_action(torch.tensor([LONGI[int(d["actions"][p])]]))
        for f in range(15):
            if f > 0:
                dev.load_numpy(to_dev(HostState.from_ix(d, "frame", (p, f - 1)), hip_device, pad_to=pad).to_numpy())
            road.act()
            compare(dev, HostState.from_ix(d, "act", (p, f)), IX_FRAME_TOL, n)
            road.step(1 / 15)
            compare(dev, HostState.from_ix(d, "frame", (p, f)), IX_FRAME_TOL, n)


@pytest.mark.parametrize("path", golden_files("ix_*"), ids=IDS)
def test_ix_fused_steps_vs_golden(path, hip_device):
    d = load_golden(path)
    for p in range(int(d["meta"][1])):
        n = int((d["pre_kind"][p] > 0).sum())
        dev = to_dev(HostState.from_ix(d, "pre", p), hip_device, pad_to=32)
        road = BatchedRoad(RoadNetwork(ix_lanes(d)), dev, P_IX)
        road.simulate(torch.tensor([LONGI[int(d["actions"][p])]]), 15, 1 / 15)
        compare(dev, HostState.from_ix(d, "frame", (p, 14)), IX_STEP_TOL, n)


def test_ix_batch_of_episodes(hip_device):
    """Every (episode, step) of the fixtures as one batch of envs: blocks hold envs whose
    regulation counters differ, so enforcement runs for some envs of a block and not others."""
    ds = [load_golden(pth) for pth in golden_files("ix_*")]
    cases = [(d, p) for d in ds for p in range(int(d["meta"][1]))]
    d0 = cases[0][0]
    hs = [HostState.from_ix(d, "pre", p, pad_to=32) for d, p in cases]
    E = len(hs)
    big = HostState(E, 32)
    for e, h in enumerate(hs):
        for k in big.a:
            big.a[k][e] = h.a[k][0]
    dev = to_dev(big, hip_device)
    road = BatchedRoad(RoadNetwork(ix_lanes(d0)), dev, P_IX)
    road.simulate(torch.tensor([LONGI[int(d["actions"][p])] for d, p in cases]), 15, 1 / 15)
    out = dev.to_numpy()
    for e, (d, p) in enumerate(cases):
        g = HostState.from_ix(d, "frame", (p, 14), pad_to=32)
        n = int((d["pre_kind"][p] > 0).sum())
        for k in DISC:
            assert np.array_equal(out[k][e, :n], g[k][0, :n]), (e, k)
        assert out["reg_steps"][e] == g["reg_steps"][0]
        assert np.max(np.abs(out["x"][e, :n] - g["x"][0, :n])) < 1e-5


def crowded_lane_state(n_extra: int = 22):
    """A golden intersection scene with n_extra copies of an IDM vehicle spread along its straight
    inbound lane (5.2 m apart, same route and speed): the lane's list then holds more vehicles than
    the road-network instance's list rows (GRAPH_LIST_CAP = 14)."""
    d = load_golden(golden_files("ix_*")[0])
    h = HostState.from_ix(d, "pre", 0, pad_to=32)
    t = ix_lanes(d)
    n = int((h["kind"][0] > 0).sum())
    j = next(q for q in range(n) if h["kind"][0, q] == 2 and t.type[h["lane"][0, q]] == 0)
    l = int(h["lane"][0, j])
    s0 = (h["x"][0, j] - t.start_x[l]) * t.dir_x[l] + (h["y"][0, j] - t.start_y[l]) * t.dir_y[l]
    ss = [s for s in s0 + 5.2 * np.arange(-20, 20) if 1.0 <= s <= t.length[l] - 1.0 and abs(s - s0) > 1][:n_extra]
    assert n + len(ss) <= 32
    for q, s in enumerate(ss):
        r = n + q
        for k in h.a:
            if h.a[k].ndim >= 2 and h.a[k].shape[1] == 32:
                h.a[k][0, r] = h.a[k][0, j]
        h["x"][0, r] = t.start_x[l] + s * t.dir_x[l]
        h["y"][0, r] = t.start_y[l] + s * t.dir_y[l]
        h["crashed"][0, r] = 0
        h["has_impact"][0, r] = 0
    return d, h, l, n + len(ss)


def test_crowded_lane_beyond_list_capacity(hip_device):
    """More vehicles on one lane than a list row holds: the neighbour and MOBIL scans continue from
    the lane's on-lane mask (s recomputed, list order kept); frames and a fused step equal the oracle."""
    from oracle.oracle import Oracle
    d, h, l, n = crowded_lane_state()
    t = ix_lanes(d)
    on = sum(1 for q in range(n) if h["lane"][0, q] == l)
    assert on > 14, on
    o = Oracle(t, P_IX)
    dev = to_dev(h, hip_device)
    road = BatchedRoad(RoadNetwork(t), dev, P_IX)
    g = h.copy()
    for f in range(4):  # frame by frame
        road.act()
        o.road_act(g)
        compare(dev, g, F64_TOL, n)
        road.step(1 / 15)
        o.road_step(g, 1 / 15)
        compare(dev, g, F64_TOL, n)
    road.simulate(torch.tensor([LONGI[1]]), 15, 1 / 15)  # and a fused step
    o.simulate(g, [LONGI[1]], 15, 1 / 15)
    compare(dev, g, F64_TOL, n)


def test_crowded_lane_mobil_on_a_regulated_road(hip_device):
    """A 3-lane road with RegulatedRoad enforcement (so the road-network instance runs it, with its
    capped list rows): 22 vehicles on the middle lane, 8 on the outer lanes whose lane-change timers
    are due, so MOBIL scans the crowded middle lane beyond the row capacity; frames and a fused
    step equal the oracle."""
    from oracle.oracle import Oracle
    from topotrafficrl_amd import _abi
    t = _abi.straight_lane_table(3, length=400.0)
    t.regulation_frequency = 2
    rng = np.random.default_rng(3)
    h = HostState(1, 32)
    lanes = [1] * 23 + [0] * 4 + [2] * 4
    xs = np.concatenate([20 + 8.0 * np.arange(23), 30 + 40.0 * np.arange(4), 50 + 40.0 * np.arange(4)])
    for q, (ln, x) in enumerate(zip(lanes, xs)):
        h["kind"][0, q] = _abi.MDP if q == 0 else _abi.IDM
        h["x"][0, q] = x + rng.uniform(-0.5, 0.5)
        h["y"][0, q] = 4.0 * ln + rng.uniform(-0.2, 0.2)
        h["speed"][0, q] = rng.uniform(18, 26)
        h["target_speed"][0, q] = rng.uniform(22, 30)
        h["lane"][0, q] = h["target_lane"][0, q] = ln
        h["timer"][0, q] = 0.99 if ln != 1 else rng.uniform(0, 1)
        h["lane_change"][0, q] = 0 if q == 0 else 1
    h["speed_index"][0, 0] = 1
    n = len(lanes)
    o = Oracle(t, P_IX)
    dev = to_dev(h, hip_device)
    road = BatchedRoad(RoadNetwork(t), dev, P_IX)
    g = h.copy()
    for f in range(6):
        road.act()
        o.road_act(g)
        compare(dev, g, F64_TOL, n)
        road.step(1 / 15)
        o.road_step(g, 1 / 15)
        compare(dev, g, F64_TOL, n)
    road.simulate(torch.tensor([LONGI[1]]), 15, 1 / 15)
    o.simulate(g, [LONGI[1]], 15, 1 / 15)
    compare(dev, g, F64_TOL, n)


def test_full_turn_arc_keeps_the_projection_bounded(hip_device):
    """A road network whose second lane is a CircularLane sweeping three full turns: its bounding
    box for the projection's pruning is the whole circle (lane_box walks at most four cardinal
    points; an unbounded walk over the arc would hang the launch).  Frames and a fused step with
    vehicles on both lanes equal the oracle."""
    from oracle.oracle import Oracle
    from topotrafficrl_amd import _abi
    from topotrafficrl_amd.intersection import network_from_graph
    straight = [_abi.LANE_STRAIGHT, 0.0, 0.0, 300.0, 0.0, 4.0, 15.0, 0, 0, 0, 0, 0, 0, 0, 0, 0]
    arc = [_abi.LANE_CIRCULAR, 0, 0, 0, 0, 4.0, 15.0, 0, 0, 0, 150.0, 40.0, 30.0, np.pi / 2, np.pi / 2 - 6 * np.pi, 0.0]
    net = network_from_graph({"a": {"b": [(straight, 1), (arc, 1)]}}, regulation_frequency=2)
    t = net.table
    assert t.n_lanes == 2 and t.length[1] > 6 * np.pi * 30 - 1
    h = HostState(1, 32)
    xs = [20.0, 45.0, 70.0, 95.0, 130.0, 160.0, 190.0]
    for q, x in enumerate(xs):
        h["kind"][0, q] = _abi.MDP if q == 0 else _abi.IDM
        h["x"][0, q], h["y"][0, q] = x, 0.3 * (q % 2)
        h["speed"][0, q] = h["target_speed"][0, q] = 8.0 + q
        h["lane"][0, q] = h["target_lane"][0, q] = 0
        h["timer"][0, q] = 0.95
        h["lane_change"][0, q] = 0 if q == 0 else 1
    for q, a in enumerate([0.3, 1.9, 3.5]):  # three vehicles on the (counter-clockwise) arc, heading along it
        r = len(xs) + q
        h["kind"][0, r] = _abi.IDM
        h["x"][0, r], h["y"][0, r] = 150.0 + 30.0 * np.cos(a), 40.0 + 30.0 * np.sin(a)
        h["heading"][0, r] = a - np.pi / 2
        h["speed"][0, r] = h["target_speed"][0, r] = 6.0
        h["lane"][0, r] = h["target_lane"][0, r] = 1
        h["lane_change"][0, r] = 1
    h["speed_index"][0, 0] = 1
    n = len(xs) + 3
    o = Oracle(t, P_IX)
    dev = to_dev(h, hip_device)
    road = BatchedRoad(RoadNetwork(t), dev, P_IX)
    g = h.copy()
    for f in range(3):
        road.act()
        o.road_act(g)
        compare(dev, g, F64_TOL, n)
        road.step(1 / 15)
        o.road_step(g, 1 / 15)
        compare(dev, g, F64_TOL, n)
    road.simulate(torch.tensor([LONGI[1]]), 15, 1 / 15)
    o.simulate(g, [LONGI[1]], 15, 1 / 15)
    compare(dev, g, F64_TOL, n)
