"""HIP path vs the float64 oracle and the reference golden vectors (run on an MI355X).

Tolerances (stated per SURVEY.md §8(d)):
  * f64 kernels, one frame from a golden state and multi-frame rollouts (fused 15-frame steps
    against the goldens and the oracle, every BASELINE batch size): discrete fields exact,
    continuous fields within F64_TOL relative to 1 + |x|.  The bounds are about 10x the worst
    values seen on the MI355X (round 5, profiles/r05/r05a_parity.json: pose, speed and steering
    <= 7.5e-15, acceleration and impacts <= 6.3e-14, timers and target speeds exact), far inside
    SURVEY.md's 1e-9 for the fp64 parity mode.
  * f32 kernels, one frame, against the float64 oracle on the same float32-rounded inputs:
    |d| <= 1e-4 * (1 + |x|) on every continuous field; discrete fields exact except flips at a
    float64 decision margin below 1e-5 (oracle_frame_links; check_f32_flips) -- the vehicle's
    own, or through a causal link (a same-frame read) that of a flipped vehicle -- counted and
    bounded.
  * observations (float32 outputs): f64 path bit-identical; f32 path: Kinematics <= 2e-4; grid
    cells, TTC cells and Lidar rays within 1e-4 except where a float64 observation decision (a
    cell floor, a range test, a time bin, a nearest-hit comparison) sits within 1e-5 relative
    (the oracle's observation margins), with no percentage allowance.
"""
import numpy as np
import pytest
import torch

import parity_log
from conftest import golden_files, load_golden, scene_files
from oracle.oracle import HostState, Oracle
from topotrafficrl_amd import _abi
from topotrafficrl_amd.observation import kinematics, occupancy_grid
from topotrafficrl_amd.road import BatchedRoad, RoadNetwork
from topotrafficrl_amd.state import BatchState

pytestmark = pytest.mark.gpu

P = _abi.default_params()
KD = _abi.kin_cfg()
K15 = _abi.kin_cfg(features=["presence", "x", "y", "vx", "vy", "cos_h", "sin_h"], vehicles_count=15,
                   features_range={"x": [-100, 100], "y": [-100, 100], "vx": [-20, 20], "vy": [-20, 20]})
G7 = _abi.grid_cfg(features=["presence", "x", "y", "vx", "vy", "cos_h", "sin_h"],
                   features_range={"x": [-100, 100], "y": [-100, 100], "vx": [-20, 20], "vy": [-20, 20]},
                   grid_size=[[-32, 32], [-32, 32]], grid_step=[2, 2])
GR = _abi.grid_cfg()
CONT = ["x", "y", "heading", "speed", "timer", "target_speed", "steer", "acc"]
F64_TOL = {"x": 1e-13, "y": 1e-13, "heading": 1e-13, "speed": 1e-13, "steer": 1e-13, "acc": 1e-12,
           "timer": 0.0, "target_speed": 0.0, "impact_x": 1e-12, "impact_y": 1e-12}
DISC = ["lane", "target_lane", "crashed", "has_impact", "speed_index"]


def to_dev(h: HostState, device, dtype="f64", pad_to=None):
    N = pad_to or h.N
    b = BatchState(h.E, N, device=device, dtype=dtype)
    arr = {}
    for k, v in h.a.items():
        if k in ("reg_steps", "rng"):  # per-env fields
            arr[k] = v
            continue
        full = np.zeros((h.E, N) + v.shape[2:], dtype=v.dtype)
        if k in ("speed_index", "route_n") or k in _abi.ROUTE_FIELDS:
            full[:] = -1
        full[:, :h.N] = v
        arr[k] = full
    return b.load_numpy(arr)


def compare(dev: BatchState, h: HostState, tol, disc_exact=True, n=None, where: str = ""):
    """Device state vs the oracle / golden: discrete fields exact (``disc_exact``), every continuous
    field within ``tol`` (a float, or a per-field dict) relative to 1 + |x|; each field's worst
    error goes to parity_log under the calling test's name."""
    d = dev.to_numpy()
    n = n or h.N
    worst = 0.0
    check, where = parity_log.current_check(), where or parity_log.current_case()
    for k in CONT:
        a, b = d[k][:, :n].astype(np.float64), h[k][:, :n]
        err = parity_log.note(check, k, parity_log.rel_err(a, b), where)
        t = tol[k] if isinstance(tol, dict) else tol
        assert err <= t, (k, err, t)
        worst = max(worst, err)
    imp = h["has_impact"][:, :n].astype(bool)
    if imp.any():
        for k in ("impact_x", "impact_y"):
            err = parity_log.note(check, k, np.abs(d[k][:, :n][imp] - h[k][:, :n][imp]), where)
            t = tol[k] if isinstance(tol, dict) else tol
            assert err <= t, (k, err, t)
            worst = max(worst, err)
    mism = {k: int(np.sum(d[k][:, :n] != h[k][:, :n])) for k in DISC}
    if disc_exact:
        assert sum(mism.values()) == 0, mism
    return worst, mism


def roads(d, device, dtype="f64", frame=0, pad_to=None):
    lanes = _abi.lane_table_from_arrays(d["lane_table"])
    h = HostState.from_golden(d, frame)
    dev = to_dev(h, device, dtype, pad_to)
    return Oracle(lanes, P), BatchedRoad(RoadNetwork(lanes), dev, P), h, dev


@pytest.mark.parametrize("path", golden_files(), ids=lambda p: p.split("/")[-1][:-4])
def test_single_frames_f64_vs_golden(path, hip_device):
    d = load_golden(path)
    o, road, h, dev = roads(d, hip_device)
    frames = d["x"].shape[0] - 1
    for f in range(frames):
        g = HostState.from_golden(d, f)
        dev.load_numpy(g.a)
        if f % 15 == 0:
            road.meta_action(torch.tensor([int(d["actions"][f // 15])]))
        road.act()
        torch.cuda.synchronize()
        compare(dev, HostState.from_golden(d, f, prefix="act_"), F64_TOL)
        road.step(1 / 15)
        compare(dev, HostState.from_golden(d, f + 1), F64_TOL)


@pytest.mark.parametrize("path", golden_files(), ids=lambda p: p.split("/")[-1][:-4])
def test_fused_rollout_f64_vs_golden(path, hip_device):
    d = load_golden(path)
    o, road, h, dev = roads(d, hip_device)
    for p in range(int(d["meta"][2])):
        road.simulate(torch.tensor([int(d["actions"][p])]), 15, 1 / 15)
        compare(dev, HostState.from_golden(d, 15 * (p + 1)), F64_TOL)


@pytest.mark.parametrize("path", golden_files("highway_*"), ids=lambda p: p.split("/")[-1][:-4])
def test_padded_slots_are_invisible(path, hip_device):
    """A 50-vehicle scene in 64 or 128 slots must give the same result as unpadded."""
    d = load_golden(path)
    n = d["x"].shape[1]
    pad = 64 if n <= 64 and n != 64 else 128
    if n == 128:
        pytest.skip("no larger slot class than 128 in the suite")
    o, road, h, dev = roads(d, hip_device, pad_to=pad)
    road.simulate(torch.tensor([int(d["actions"][0])]), 15, 1 / 15)
    compare(dev, HostState.from_golden(d, 15), F64_TOL, n=n)


def f32_inputs(h: HostState) -> HostState:
    """The float64 state the float32 kernels actually start from: every real field rounded to
    float32.  The oracle steps this state, so the comparison measures the float32 arithmetic and
    not the representation of the inputs."""
    g = h.copy()
    for k in _abi.REAL_FIELDS:
        g.a[k][...] = g.a[k].astype(np.float32).astype(np.float64)
    return g


F32_TOL = 1e-4     # continuous state, one frame: |d| <= 1e-4 * (1 + |x|)
F32_MARGIN = 1e-5  # a discrete flip must sit at a float64 decision margin below this (relative)


F32_EPS = 2.0 ** -22  # four float32 ulps, relative: the rounding of a position-derived quantity


def f32_cont_tol(h: HostState, k: str, n: int) -> np.ndarray:
    """Per-vehicle float32 tolerance of continuous field k: F32_TOL * (1 + |x|), and for the
    steering command also the steering law's own gain from lateral position to angle
    (controller.py:145-187: hc = asin(-r / (0.6 v)), heading rate 5 (psi_ref - psi),
    beta = asin(2.5 / v * rate), steer = atan(2 tan beta), so d steer / d r ~ 2 * 2.5 * 5 / (0.6 v^2)
    = 42 / v^2) times four float32 ulps of the position: a slow vehicle's command carries its
    position's rounding amplified by 1 / v^2 (v -> not_zero's 0.01 at a standstill)."""
    b = h[k][:, :n]
    tol = F32_TOL * (1 + np.abs(b))
    if k == "steer":
        v = np.maximum(np.abs(h["speed"][:, :n]), 1e-2)
        tol = tol + 42.0 / v ** 2 * F32_EPS * (1 + np.abs(h["x"][:, :n]) + np.abs(h["y"][:, :n]))
    return tol


def check_f32_flips(dev: BatchState, h: HostState, margin: np.ndarray, links: np.ndarray, what: str,
                    disc=None) -> int:
    """float32 result vs the float64 oracle on the same (rounded) inputs.  A vehicle "flips" when a
    discrete field differs or a continuous one exceeds F32_TOL.  Every flip must trace back to a
    decision whose float64 margin (oracle_frame_links) is below F32_MARGIN: the vehicle's own, or,
    transitively, that of a flipped vehicle it is causally linked to in this frame -- one whose
    same-frame result its decisions read (an earlier vehicle's target within the lane-change
    abort's desired gap, a collision partner's post-step pose; oracle_frame_links).  Returns the
    count of flips.  ``disc``: the discrete fields (default DISC).  Continuous tolerances:
    f32_cont_tol."""
    d = dev.to_numpy()
    n = h.N
    assert not np.any(links == -2), f"{what}: a causal-link row overflowed"
    flip = np.zeros((h.E, n), dtype=bool)
    for k in disc or DISC:
        diff = d[k][:, :n] != h[k][:, :n]
        flip |= diff.reshape(h.E, n, -1).any(-1)  # per-vehicle rows (routes) count as one field
    for k in CONT:
        a, b = d[k][:, :n].astype(np.float64), h[k][:, :n]
        flip |= np.abs(a - b) > f32_cont_tol(h, k, n)
    imp = h["has_impact"][:, :n].astype(bool) & (d["has_impact"][:, :n] != 0)
    for k in ("impact_x", "impact_y"):
        flip |= imp & (np.abs(d[k][:, :n] - h[k][:, :n]) > F32_TOL * (1 + np.abs(h[k][:, :n])))
    ok = flip & (margin < F32_MARGIN)
    changed = True
    while changed:  # transitive closure over the causal links to excused flips
        changed = False
        for e, i in zip(*np.nonzero(flip & ~ok)):
            src = links[e, i][links[e, i] >= 0]
            if len(src) and ok[e, src].any():
                ok[e, i] = changed = True
    bad = np.argwhere(flip & ~ok)

    def fields(e, i):  # what differs, as (field, float32 result, float64 oracle)
        out = []
        for k in list(disc or DISC) + CONT:
            a, b = d[k][e, i], h[k][e, i]
            if k in CONT and abs(float(a) - float(b)) > f32_cont_tol(h, k, n)[e, i] or \
                    k not in CONT and np.any(a != b):
                out.append((k, np.asarray(a).tolist(), np.asarray(b).tolist()))
        return out

    assert len(bad) == 0, (f"{what}: float32 flips with no small float64 decision margin at (env, slot) "
                           f"{bad[:5].tolist()}; margins {[float(margin[e, i]) for e, i in bad[:5]]}; "
                           f"links {[links[e, i][links[e, i] >= 0].tolist() for e, i in bad[:5]]}; "
                           f"fields {[fields(e, i) for e, i in bad[:3]]}")
    return int(flip.sum())


@pytest.mark.parametrize("path", golden_files(), ids=lambda p: p.split("/")[-1][:-4])
def test_single_frames_f32(path, hip_device):
    """fp32 fast path, one frame from each golden state, against the float64 oracle on the same
    float32-rounded inputs: continuous fields within 1e-4 * (1 + |x|), discrete fields exact except
    flips at float64 decision margins below 1e-5 (check_f32_flips)."""
    d = load_golden(path)
    o, road, h, dev = roads(d, hip_device, dtype="f32")
    frames = d["x"].shape[0] - 1
    flips = 0
    for f in range(frames):
        g = f32_inputs(HostState.from_golden(d, f))
        dev.load_numpy(g.a)
        act = [int(d["actions"][f // 15])] if f % 15 == 0 else None
        if act is not None:
            road.meta_action(torch.tensor(act))
        road.act()
        road.step(1 / 15)
        m, lk = o.frame_margins(g, act, links=True)
        torch.cuda.synchronize()
        flips += check_f32_flips(dev, g, m, lk, f"frame {f}")
    assert flips <= max(2, frames // 10), flips  # flips are rare, not merely excused


@pytest.mark.parametrize("path", golden_files(), ids=lambda p: p.split("/")[-1][:-4])
def test_neighbours_vs_golden(path, hip_device):
    d = load_golden(path)
    o, road, h, dev = roads(d, hip_device)
    for f in range(0, d["x"].shape[0] - 1, 7):
        ga = HostState.from_golden(d, f, prefix="act_")  # post-act state holds the targets queried
        dev.load_numpy(ga.a)
        fr, rr = road.neighbour_vehicles()
        assert np.array_equal(fr.cpu().numpy()[0], d["nbr"][f][0])
        assert np.array_equal(rr.cpu().numpy()[0], d["nbr"][f][1])
        fr, rr = road.neighbour_vehicles(dev["target_lane"])
        assert np.array_equal(fr.cpu().numpy()[0], d["nbr"][f][2])
        assert np.array_equal(rr.cpu().numpy()[0], d["nbr"][f][3])


@pytest.mark.parametrize("dtype", ["f64", "f32"])
@pytest.mark.parametrize("path", golden_files(), ids=lambda p: p.split("/")[-1][:-4])
def test_observations_vs_golden(path, dtype, hip_device):
    d = load_golden(path)
    lanes = _abi.lane_table_from_arrays(d["lane_table"])
    net = RoadNetwork(lanes)
    tol = 0.0 if dtype == "f64" else 2e-4
    for p in range(int(d["meta"][2]) + 1):
        dev = to_dev(HostState.from_golden(d, 15 * p), hip_device, dtype)
        for cfg, key in ((_abi.kin_cfg(lanes_on_road=int(d["meta"][4])), "kin5"), (K15, "kin15")):
            obs, ids = kinematics(dev, net, P, cfg)
            assert np.max(np.abs(obs.cpu().numpy()[0] - d[key][p])) <= tol
            if dtype == "f64":
                assert np.array_equal(ids.cpu().numpy()[0], d[key + "_ids"][p])
        for cfg, key in ((G7, "grid7"), (GR, "grid_onroad")):
            g = occupancy_grid(dev, net, P, cfg).cpu().numpy()[0]
            if dtype == "f64":
                assert np.array_equal(g, d[key][p])
            else:
                # every cell within F32_TOL, except cells whose content sits at a float64 cell-floor
                # margin below F32_MARGIN (an item within ~1e-5 relative of a cell boundary)
                want, m = Oracle(lanes, P).observe_grid(f32_inputs(HostState.from_golden(d, 15 * p)), cfg,
                                                        margins=True)
                off = np.abs(g - want[0]) > F32_TOL
                assert not np.any(off & ~(m[0] < F32_MARGIN)), (key, p, np.argwhere(off & ~(m[0] < F32_MARGIN))[:5])


@pytest.mark.parametrize("dtype", ["f64", "f32"])
@pytest.mark.parametrize("path", scene_files(), ids=lambda p: p.split("/")[-1][:-4])
def test_reset_matches_reference_scene(path, dtype, hip_device):
    """GPU scene generation reproduces numpy default_rng(seed) draws of create_random.
    Straight lanes: bit-exact.  Curved lanes place vehicles through sin/cos/atan2, which the
    device math library rounds within 1 ulp rather than correctly: continuous fields there are
    held to 1e-11 relative (f64; the lane-change timer is (x + y) * pi mod 1, which scales a
    position's rounding by ~600 on a 200 m arc) and every discrete field stays exact."""
    from topotrafficrl_amd.envs import reset_highway
    d = load_golden(path)
    n, seed = int(d["meta"][0]), int(d["meta"][1])
    lanes = _abi.lane_table_from_arrays(d["lane_table"])
    curved = any(lanes.type[i] != _abi.LANE_STRAIGHT for i in range(lanes.n_lanes))
    dev = BatchState(1, n, device=hip_device, dtype=dtype)
    reset_highway(dev, RoadNetwork(lanes), P, _abi.reset_cfg(n, lanes), [seed])
    g = HostState.from_golden(d, 0)
    got = dev.to_numpy()
    for k in ["x", "y", "heading", "speed", "target_speed", "timer", "delta"]:
        ref = g[k].astype(np.float32) if dtype == "f32" else g[k]
        if curved:
            tol = 1e-11 if dtype == "f64" else 1e-5
            assert np.max(np.abs(got[k] - ref) / (1 + np.abs(ref))) <= tol, k
        else:
            assert np.array_equal(got[k], ref), k
    for k in ["lane", "target_lane", "kind", "speed_index", "lane_change"]:
        assert np.array_equal(got[k], g[k]), k


@pytest.mark.parametrize("n", [24, 50, 64, 100, 128, 200])
def test_random_batch_rollout_vs_oracle(n, hip_device):
    """Many envs with different seeds: fused GPU rollout == sequential oracle (f64)."""
    E = 48
    lanes = _abi.straight_lane_table(4)
    o = Oracle(lanes, P)
    h = HostState(E, n)
    seeds = list(range(100, 100 + E))
    o.reset_highway(h, _abi.reset_cfg(n, lanes), seeds)
    dev = to_dev(h, hip_device)
    road = BatchedRoad(RoadNetwork(lanes), dev, P)
    rng = np.random.default_rng(n)
    for p in range(3):
        acts = rng.integers(0, 5, size=E).astype(np.int32)
        o.simulate(h, acts, 15, 1 / 15)
        road.simulate(torch.from_numpy(acts), 15, 1 / 15)
        compare(dev, h, F64_TOL)


@pytest.mark.parametrize("n", [24, 64, 100, 128])
def test_tied_positions_vs_oracle(n, hip_device):
    """Vehicles sharing x exactly (the ego included, same and different lanes): the sorted-order
    neighbour lookups of the straight instance cannot rank them, so those envs take the slot-order
    scans with the reference's tie rules (front: later slot, rear: earlier slot)."""
    E = 32
    lanes = _abi.straight_lane_table(4)
    o = Oracle(lanes, P)
    h = HostState(E, n)
    o.reset_highway(h, _abi.reset_cfg(n, lanes), list(range(300, 300 + E)))
    rng = np.random.default_rng(5)
    for e in range(E):
        for _ in range(1 + e % 4):
            a, b = rng.choice(n, 2, replace=False)
            h["x"][e, a] = h["x"][e, b]
    h["x"][:, 3] = h["x"][:, 0]  # a tie with the ego in every env
    dev = to_dev(h, hip_device)
    road = BatchedRoad(RoadNetwork(lanes), dev, P)
    acts = rng.integers(0, 5, size=E).astype(np.int32)
    o.simulate(h, acts, 1, 1 / 15)
    road.simulate(torch.from_numpy(acts), 1, 1 / 15)
    compare(dev, h, F64_TOL)
    for _ in range(2):
        acts = rng.integers(0, 5, size=E).astype(np.int32)
        o.simulate(h, acts, 15, 1 / 15)
        road.simulate(torch.from_numpy(acts), 15, 1 / 15)
        compare(dev, h, F64_TOL)


@pytest.mark.parametrize("dtype", ["f64", "f32"])
def test_close_pairs_collisions_vs_oracle(dtype, hip_device):
    """Clusters of vehicles at random close poses (many pairs touching, near-touching or
    sweeping into each other): Road.step's collision pass (crashed, impact) == the oracle's.
    Exercises the SAT separation shortcut and the pair queue at its boundary cases."""
    E, n = 2048, 6
    rng = np.random.default_rng(7)
    h = HostState(E, n)
    spread = rng.uniform(4, 25, (E, 1))  # from pile-ups to near misses
    h["x"][:] = 200 + spread * rng.uniform(-1, 1, (E, n))
    h["y"][:] = rng.uniform(-2, 10, (E, n))
    h["heading"][:] = rng.uniform(-0.7, 0.7, (E, n))
    h["speed"][:] = rng.uniform(0, 35, (E, n))
    h["target_speed"][:] = h["speed"]
    h["steer"][:] = rng.uniform(-0.3, 0.3, (E, n))
    h["acc"][:] = rng.uniform(-5, 5, (E, n))
    h["lane"][:] = np.clip(np.round(h["y"] / 4), 0, 3).astype(np.int32)
    h["target_lane"][:] = h["lane"]
    h["kind"][:] = _abi.IDM
    h["crashed"][:] = rng.random((E, n)) < 0.05
    lanes = _abi.straight_lane_table(4)
    o = Oracle(lanes, P)
    if dtype == "f32":
        h = f32_inputs(h)
    dev = to_dev(h, hip_device, dtype)
    road = BatchedRoad(RoadNetwork(lanes), dev, P)
    flips = 0
    for _ in range(3):
        if dtype == "f32":
            m, lk = o.frame_margins(h, None, 1 / 15, act=False, step=True, links=True)
        else:
            o.road_step(h, 1 / 15)
        road.step(1 / 15)
        torch.cuda.synchronize()
        d = dev.to_numpy()
        assert h["crashed"].sum() > E // 2  # the scene really is collision-heavy
        if dtype == "f64":
            bad = sum(int(np.sum(d[k] != h[k])) for k in ("crashed", "has_impact"))
            assert bad == 0
            imp = h["has_impact"].astype(bool)
            for k in ("impact_x", "impact_y", "x", "y"):
                sel = imp if k.startswith("impact") else slice(None)
                assert np.max(np.abs(d[k][sel] - h[k][sel])) < 1e-9, k
        else:
            flips += check_f32_flips(dev, h, m, lk, "collision step")
            h = f32_inputs(h)
            dev.load_numpy(h.a)  # re-sync on the rounded oracle state so one step's flips do not compound
    assert flips <= E * n * 2e-3, flips


@pytest.mark.parametrize("dtype", ["f64", "f32"])
@pytest.mark.parametrize("path", golden_files(), ids=lambda p: p.split("/")[-1][:-4])
def test_ttc_and_lidar_vs_golden(path, dtype, hip_device):
    """TimeToCollision (reference compute_ttc_grid) and Lidar observations on the GPU."""
    from topotrafficrl_amd.observation import lidar, time_to_collision
    d = load_golden(path)
    lanes = _abi.lane_table_from_arrays(d["lane_table"])
    net = RoadNetwork(lanes)
    for p in range(int(d["meta"][2]) + 1):
        dev = to_dev(HostState.from_golden(d, 15 * p), hip_device, dtype)
        ttc = time_to_collision(dev, net, P, _abi.ttc_cfg()).cpu().numpy()[0]
        lid = lidar(dev, net, P, _abi.lidar_cfg()).cpu().numpy()[0]
        if dtype == "f64":
            assert np.array_equal(ttc, d["ttc"][p])
            assert np.max(np.abs(lid - d["lidar"][p])) <= 1e-6
        else:  # fp32: a cell / ray may differ only at a float64 decision margin below F32_MARGIN
            o = Oracle(lanes, P)
            g = f32_inputs(HostState.from_golden(d, 15 * p))
            want, m = o.observe_ttc(g, _abi.ttc_cfg(), margins=True)
            off = ttc != want[0]
            assert not np.any(off & ~(m[0] < F32_MARGIN)), ("ttc", p, np.argwhere(off & ~(m[0] < F32_MARGIN))[:5])
            want, m = o.observe_lidar(g, _abi.lidar_cfg(), margins=True)
            off = np.any(np.abs(lid - want[0]) > F32_TOL, axis=1)
            assert not np.any(off & ~(m[0] < F32_MARGIN)), ("lidar", p, np.nonzero(off & ~(m[0] < F32_MARGIN)))


@pytest.mark.parametrize("n,pad", [(40, 48), (100, 128), (128, 128), (200, 256)])
def test_grid_random_batch_vs_oracle(n, pad, hip_device):
    """OccupancyGrid over a batch (slots padded, the block sized by the slot count,
    one env without an ego): f64 bit-identical to the oracle."""
    E = 37
    lanes = _abi.straight_lane_table(4)
    o = Oracle(lanes, P)
    h = HostState(E, n)
    o.reset_highway(h, _abi.reset_cfg(n, lanes), list(range(500, 500 + E)))
    o.simulate(h, np.random.default_rng(n).integers(0, 5, E).astype(np.int32), 15, 1 / 15)
    h["kind"][5, 0] = _abi.IDM  # env 5 has no controlled vehicle: an all-zero grid
    dev = to_dev(h, hip_device, pad_to=pad)
    net = RoadNetwork(lanes)
    for cfg in (G7, GR):
        got = occupancy_grid(dev, net, P, cfg).cpu().numpy()
        want = o.observe_grid(h, cfg)
        assert np.array_equal(got, want)
        assert not got[5].any()


def test_ttc_and_lidar_random_batch_vs_oracle(hip_device):
    """Many envs, padded slots, crashes: GPU == oracle (f64)."""
    E, n = 64, 48
    lanes = _abi.straight_lane_table(4)
    o = Oracle(lanes, P)
    h = HostState(E, n)
    o.reset_highway(h, _abi.reset_cfg(40, lanes), list(range(E)))
    o.simulate(h, np.random.default_rng(0).integers(0, 5, E).astype(np.int32), 15, 1 / 15)
    dev = to_dev(h, hip_device)
    net = RoadNetwork(lanes)
    from topotrafficrl_amd.observation import lidar, time_to_collision
    for cells, rng_ in ((16, 60.0), (64, 35.0), (7, 100.0)):
        lc = _abi.lidar_cfg(cells, rng_)
        assert np.max(np.abs(lidar(dev, net, P, lc).cpu().numpy() - o.observe_lidar(h, lc))) <= 1e-6
    for hz, pf in ((10, 1), (5, 2)):
        tc = _abi.ttc_cfg(hz, pf)
        assert np.array_equal(time_to_collision(dev, net, P, tc).cpu().numpy(), o.observe_ttc(h, tc))


@pytest.mark.parametrize("n", [60, 120])
def test_collision_pair_queue_overflow_vs_oracle(n, hip_device):
    """Pile-ups with more close pairs than slots (> NS queued pairs in an env) take the
    per-vehicle sweep fallback; results must still equal the oracle (n = 120: the two-wave
    128-slot instance, whose sorted window feeds the queue)."""
    E = 64
    rng = np.random.default_rng(11)
    h = HostState(E, n)
    h["x"][:] = 500 + rng.uniform(-12, 12, (E, n))
    h["y"][:] = rng.uniform(-2, 14, (E, n))
    h["heading"][:] = rng.uniform(-0.4, 0.4, (E, n))
    h["speed"][:] = rng.uniform(0, 30, (E, n))
    h["target_speed"][:] = h["speed"]
    h["lane"][:] = np.clip(np.round(h["y"] / 4), 0, 3).astype(np.int32)
    h["target_lane"][:] = h["lane"]
    h["kind"][:] = _abi.IDM
    lanes = _abi.straight_lane_table(4)
    o = Oracle(lanes, P)
    dev = to_dev(h, hip_device)
    road = BatchedRoad(RoadNetwork(lanes), dev, P)
    for _ in range(2):
        o.road_step(h, 1 / 15)
        road.step(1 / 15)
        torch.cuda.synchronize()
        d = dev.to_numpy()
        for k in ("crashed", "has_impact"):
            assert np.array_equal(d[k], h[k]), k
        imp = h["has_impact"].astype(bool)
        for k in ("impact_x", "impact_y"):
            assert np.max(np.abs(d[k][imp] - h[k][imp])) < 1e-9, k


def test_empty_batch_and_largest_slot_class(hip_device):
    """n_envs = 0 is a no-op for every entry point; n_veh = 256 (the largest slot class) runs
    the fused rollout equal to the oracle."""
    lanes = _abi.straight_lane_table(4)
    empty = BatchState(0, 64, device=hip_device)
    road = BatchedRoad(RoadNetwork(lanes), empty, P)
    road.simulate(torch.zeros(0, dtype=torch.int32), 15, 1 / 15)
    road.act()
    road.step(1 / 15)
    from topotrafficrl_amd.observation import kinematics, occupancy_grid
    out, _ = kinematics(empty, RoadNetwork(lanes), P, _abi.kin_cfg())
    assert out.shape[0] == 0
    assert occupancy_grid(empty, RoadNetwork(lanes), P, _abi.grid_cfg()).shape[0] == 0
    torch.cuda.synchronize()
    E, n = 4, 256
    o = Oracle(lanes, P)
    h = HostState(E, n)
    o.reset_highway(h, _abi.reset_cfg(n, lanes), [7, 8, 9, 10])
    dev = to_dev(h, hip_device)
    road = BatchedRoad(RoadNetwork(lanes), dev, P)
    acts = np.array([0, 1, 3, 4], dtype=np.int32)
    o.simulate(h, acts, 15, 1 / 15)
    road.simulate(torch.from_numpy(acts), 15, 1 / 15)
    compare(dev, h, F64_TOL)
