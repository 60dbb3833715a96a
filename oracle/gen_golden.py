"""Golden-vector generator — TEST INFRASTRUCTURE, runs only in the build container.

This script imports the *unmodified* reference simulation core from
``/root/reference`` (ttrl_env.road / ttrl_env.vehicle / ttrl_env.utils; no stubs:
the package ``__init__`` that needs gymnasium is bypassed by registering an empty
package module) and records per-frame states of straight
highway scenes into ``tests/golden/*.npz``.  Only the resulting data files are
committed; nothing from the reference travels to the GPU box.

What is pinned by the real reference:
  * scene generation       Vehicle.create_random / randomize_behavior   kinematics.py:50-104, behavior.py:64-69
  * one frame              Road.act + Road.step(1/15)                    road.py:461-478
  * ego meta-actions       MDPVehicle.act(label)                         controller.py:295-315
  * neighbour queries      Road.neighbour_vehicles                       road.py:480-513
  * observation primitives Road.close_objects_to, Vehicle.to_dict, lmap  road.py:418-447, kinematics.py:237-261, utils.py:29-31
What is restated here (observation.py imports gymnasium/pygame, absent from the image):
  * KinematicObservation.observe assembly    observation.py:233-275 (pandas-free, same arithmetic)
  * OccupancyGridObservation.observe assembly observation.py:353-434

Usage:  PYTHONDONTWRITEBYTECODE=1 python oracle/gen_golden.py
"""
from __future__ import annotations

import os
import sys
import types

import numpy as np

REF = "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden")


def _import_reference():
    sys.dont_write_bytecode = True
    pkg = types.ModuleType("ttrl_env")
    pkg.__path__ = [os.path.join(REF, "ttrl_env")]
    sys.modules["ttrl_env"] = pkg
    from ttrl_env import utils
    from ttrl_env.road.lane import CircularLane, SineLane, StraightLane
    from ttrl_env.road.road import Road, RoadNetwork
    from ttrl_env.vehicle.behavior import IDMVehicle
    from ttrl_env.vehicle.controller import MDPVehicle
    from ttrl_env.vehicle.kinematics import Vehicle
    for sub in ("envs", "envs.common"):  # skip the package __init__s (they import gymnasium), as above
        m = types.ModuleType("ttrl_env." + sub)
        m.__path__ = [os.path.join(REF, "ttrl_env", *sub.split("."))]
        sys.modules["ttrl_env." + sub] = m
    from ttrl_env.envs.common import finite_mdp  # the module itself imports only utils and Vehicle
    return types.SimpleNamespace(utils=utils, StraightLane=StraightLane, SineLane=SineLane,
                                 CircularLane=CircularLane, Road=Road,
                                 RoadNetwork=RoadNetwork, IDMVehicle=IDMVehicle,
                                 MDPVehicle=MDPVehicle, Vehicle=Vehicle, finite_mdp=finite_mdp)


R = _import_reference()
ACTIONS_ALL = {0: "LANE_LEFT", 1: "IDLE", 2: "LANE_RIGHT", 3: "FASTER", 4: "SLOWER"}  # action.py:204
FIELDS_F = ["x", "y", "heading", "speed", "target_speed", "timer", "delta",
            "steer", "acc", "impact_x", "impact_y"]
FIELDS_I = ["lane", "target_lane", "crashed", "speed_index"]


def reset_idm_constants():
    """intersection_env.py:258-261 mutates these globally; we never import it, but be explicit."""
    R.IDMVehicle.DISTANCE_WANTED = 5.0 + R.Vehicle.LENGTH
    R.IDMVehicle.COMFORT_ACC_MAX = 3.0
    R.IDMVehicle.COMFORT_ACC_MIN = -5.0


def make_highway(n: int, seed: int, lanes: int = 4):
    """Synthetic straight highway of SURVEY.md §3.C: ego MDPVehicle lane 1, x=50, v=25,
    then n-1 IDMVehicle.create_random(spacing=1) + randomize_behavior()."""
    reset_idm_constants()
    net = R.RoadNetwork.straight_road_network(lanes, length=10000, speed_limit=30)
    road = R.Road(network=net, np_random=np.random.default_rng(seed))
    lane = net.get_lane(("0", "1", 1))
    ego = R.MDPVehicle(road, lane.position(50.0, 0.0), lane.heading_at(50.0), 25.0)
    road.vehicles.append(ego)
    for _ in range(n - 1):
        v = R.IDMVehicle.create_random(road, spacing=1)
        v.randomize_behavior()
        road.vehicles.append(v)
    return road


def make_curved(kind: str, n: int, seed: int, lanes: int = 3):
    """The highway scene of make_highway on a single-edge road of curved lanes: parallel
    SineLanes (amplitude 5 m, wavelength 200 m) or concentric CircularLanes (radius 200 + 4 i m,
    a clockwise half circle) -- lane.py:235-350, built with the reference constructors."""
    reset_idm_constants()
    net = R.RoadNetwork()
    for i in range(lanes):
        if kind == "sine":
            lane = R.SineLane([0.0, 4.0 * i], [10000.0, 4.0 * i], amplitude=5.0, pulsation=2 * np.pi / 200,
                              phase=0.0, speed_limit=30)
        else:
            lane = R.CircularLane([0.0, 0.0], 200.0 + 4.0 * i, -np.pi / 2, np.pi / 2, clockwise=True, speed_limit=30)
        net.add_lane("0", "1", lane)
    road = R.Road(network=net, np_random=np.random.default_rng(seed))
    lane = net.get_lane(("0", "1", 1))
    ego = R.MDPVehicle(road, lane.position(50.0, 0.0), lane.heading_at(50.0), 25.0)
    road.vehicles.append(ego)
    for _ in range(n - 1):
        v = R.IDMVehicle.create_random(road, spacing=1)
        v.randomize_behavior()
        road.vehicles.append(v)
    return road


def lane_geometry(road):
    """[L, 16] rows: type, start_x, start_y, end_x, end_y, width, speed_limit, amplitude, pulsation,
    phase, center_x, center_y, radius, start_phase, end_phase, clockwise (_abi.lane_table_from_arrays)."""
    rows = []
    for ln in road.network.lanes_list():
        if isinstance(ln, R.CircularLane):
            rows.append([2, 0, 0, 0, 0, ln.width, ln.speed_limit, 0, 0, 0, ln.center[0], ln.center[1], ln.radius,
                         ln.start_phase, ln.end_phase, 1.0 if ln.clockwise else 0.0])
        elif isinstance(ln, R.SineLane):
            rows.append([1, ln.start[0], ln.start[1], ln.end[0], ln.end[1], ln.width, ln.speed_limit, ln.amplitude,
                         ln.pulsation, ln.phase, 0, 0, 0, 0, 0, 0])
        else:
            rows.append([0, ln.start[0], ln.start[1], ln.end[0], ln.end[1], ln.width, ln.speed_limit,
                         0, 0, 0, 0, 0, 0, 0, 0, 0])
    return np.array(rows, dtype=np.float64)


def make_dense(n: int, seed: int, lanes: int = 4):
    """Stress scene: vehicles packed into ~6 m/vehicle with random headings, speeds and
    in-progress lane changes, so SAT collisions, impacts, lane-change aborts and MOBIL
    all fire within a few frames.  Built with the reference constructors directly."""
    reset_idm_constants()
    net = R.RoadNetwork.straight_road_network(lanes, length=10000, speed_limit=30)
    rng = np.random.default_rng(1000 + seed)
    road = R.Road(network=net, np_random=np.random.default_rng(seed))
    lane = net.get_lane(("0", "1", 1))
    ego = R.MDPVehicle(road, lane.position(30.0, 0.0), lane.heading_at(30.0), 27.0)
    road.vehicles.append(ego)
    span = max(60.0, 6.5 * n / lanes * 1.3)
    for i in range(n - 1):
        lid = int(rng.integers(lanes))
        x = float(rng.uniform(0.0, span))
        y = lid * 4.0 + float(rng.normal(0.0, 0.6))
        h = float(rng.normal(0.0, 0.05))
        spd = float(rng.uniform(12.0, 32.0))
        tgt = lid
        if rng.random() < 0.3:
            tgt = int(np.clip(lid + rng.choice([-1, 1]), 0, lanes - 1))
        timer = float(rng.uniform(0.0, 1.2))
        v = R.IDMVehicle(road, [x, y], h, spd, target_lane_index=("0", "1", tgt),
                         target_speed=float(rng.uniform(18.0, 32.0)), timer=timer)
        v.randomize_behavior()
        road.vehicles.append(v)
    return road


def snapshot(road):
    vs = road.vehicles
    n = len(vs)
    s = {k: np.zeros(n) for k in FIELDS_F}
    s.update({k: np.zeros(n, dtype=np.int32) for k in FIELDS_I})
    for i, v in enumerate(vs):
        s["x"][i], s["y"][i] = v.position
        s["heading"][i] = v.heading
        s["speed"][i] = v.speed
        s["target_speed"][i] = v.target_speed
        s["timer"][i] = getattr(v, "timer", 0.0)
        s["delta"][i] = getattr(v, "DELTA", R.IDMVehicle.DELTA)
        s["steer"][i] = v.action["steering"]
        s["acc"][i] = v.action["acceleration"]
        if v.impact is None:
            s["impact_x"][i] = s["impact_y"][i] = np.nan
        else:
            s["impact_x"][i], s["impact_y"][i] = v.impact
        s["lane"][i] = v.lane_index[2]
        s["target_lane"][i] = v.target_lane_index[2]
        s["crashed"][i] = int(bool(v.crashed))
        s["speed_index"][i] = int(getattr(v, "speed_index", -1))
    return s


def neighbours(road):
    """Road.neighbour_vehicles on own lane and on target lane (road.py:480-513), as indices."""
    vs = road.vehicles
    idx = {id(v): i for i, v in enumerate(vs)}
    n = len(vs)
    out = np.full((4, n), -1, dtype=np.int32)
    for i, v in enumerate(vs):
        f, r = road.neighbour_vehicles(v, v.lane_index)
        out[0, i] = idx[id(f)] if f is not None else -1
        out[1, i] = idx[id(r)] if r is not None else -1
        f, r = road.neighbour_vehicles(v, v.target_lane_index)
        out[2, i] = idx[id(f)] if f is not None else -1
        out[3, i] = idx[id(r)] if r is not None else -1
    return out


# ---------------------------------------------------------------- observations
KIN_DEFAULT = dict(features=["presence", "x", "y", "vx", "vy"], vehicles_count=5,
                   features_range=None, absolute=False, see_behind=False, clip=True)
KIN_ENVJSON = dict(features=["presence", "x", "y", "vx", "vy", "cos_h", "sin_h"], vehicles_count=15,
                   features_range={"x": [-100, 100], "y": [-100, 100], "vx": [-20, 20], "vy": [-20, 20]},
                   absolute=False, see_behind=False, clip=True)
GRID_DENSE = dict(features=["presence", "x", "y", "vx", "vy", "cos_h", "sin_h"],
                  features_range={"x": [-100, 100], "y": [-100, 100], "vx": [-20, 20], "vy": [-20, 20]},
                  grid_size=[[-32, 32], [-32, 32]], grid_step=[2, 2], clip=True)
GRID_ONROAD = dict(features=["presence", "vx", "vy", "on_road"], features_range=None,
                   grid_size=[[-27.5, 27.5], [-27.5, 27.5]], grid_step=[5, 5], clip=True)


def kinematics_obs(road, cfg):
    """KinematicObservation.observe (observation.py:233-275), order='sorted'."""
    ego = road.vehicles[0]
    feats = cfg["features"]
    V = cfg["vehicles_count"]
    rows = [ego.to_dict()]
    close = road.close_objects_to(ego, 5.0 * R.Vehicle.MAX_SPEED, count=V - 1,
                                  see_behind=cfg["see_behind"], sort=True, vehicles_only=False)
    origin = ego if not cfg["absolute"] else None
    ids = []
    idx = {id(v): i for i, v in enumerate(road.vehicles)}
    for v in close[-V + 1:]:
        rows.append(v.to_dict(origin, observe_intentions=False))
        ids.append(idx[id(v)])
    fr = cfg["features_range"]
    if not fr:  # observation.py:213-225
        nl = len(road.network.all_side_lanes(ego.lane_index))
        fr = {"x": [-5.0 * R.Vehicle.MAX_SPEED, 5.0 * R.Vehicle.MAX_SPEED],
              "y": [-4.0 * nl, 4.0 * nl],
              "vx": [-2 * R.Vehicle.MAX_SPEED, 2 * R.Vehicle.MAX_SPEED],
              "vy": [-2 * R.Vehicle.MAX_SPEED, 2 * R.Vehicle.MAX_SPEED]}
    obs = np.zeros((V, len(feats)))
    for r, d in enumerate(rows):
        for c, f in enumerate(feats):
            val = float(d[f])
            if f in fr:
                val = R.utils.lmap(val, [fr[f][0], fr[f][1]], [-1, 1])
                if cfg["clip"]:
                    val = float(np.clip(val, -1, 1))
            obs[r, c] = val
    ids = ids + [-1] * (V - 1 - len(ids))
    return obs.astype(np.float32), np.array(ids, dtype=np.int32)


def grid_obs(road, cfg):
    """OccupancyGridObservation.observe (observation.py:353-434), absolute=False,
    align_to_vehicle_axes=False; on_road via fill_road_layer_by_lanes (:453-483)."""
    ego = road.vehicles[0]
    feats = cfg["features"]
    gsize = np.array(cfg["grid_size"], dtype=np.float64)
    gstep = np.array(cfg["grid_step"], dtype=np.float64)
    shape = np.asarray(np.floor((gsize[:, 1] - gsize[:, 0]) / gstep), dtype=np.uint8)
    grid = np.full((len(feats), *shape), np.nan)
    fr = cfg["features_range"] or {"vx": [-2 * R.Vehicle.MAX_SPEED, 2 * R.Vehicle.MAX_SPEED],
                                   "vy": [-2 * R.Vehicle.MAX_SPEED, 2 * R.Vehicle.MAX_SPEED]}
    recs = [v.to_dict(ego) for v in road.vehicles]
    for d in recs:  # normalize (no clip), observation.py:336-351
        for f, rng_ in fr.items():
            if f in d:
                d[f] = R.utils.lmap(d[f], [rng_[0], rng_[1]], [-1, 1])

    def pos_to_index(px, py):
        return (int(np.floor((px - gsize[0, 0]) / gstep[0])),
                int(np.floor((py - gsize[1, 0]) / gstep[1])))

    for layer, f in enumerate(feats):
        if f in recs[0]:
            for d in recs[::-1]:
                x, y = d["x"], d["y"]
                if "x" in fr:
                    x = R.utils.lmap(x, [-1, 1], [fr["x"][0], fr["x"][1]])
                if "y" in fr:
                    y = R.utils.lmap(y, [-1, 1], [fr["y"][0], fr["y"][1]])
                c = pos_to_index(x, y)
                if 0 <= c[0] < grid.shape[-2] and 0 <= c[1] < grid.shape[-1]:
                    grid[layer, c[0], c[1]] = d[f]
        elif f == "on_road":
            spacing = np.amin(gstep)
            for lane in road.network.lanes_list():
                origin, _ = lane.local_coordinates(ego.position)
                wps = np.arange(origin - 100, origin + 100, spacing).clip(0, lane.length)
                for wp in wps:
                    p = lane.position(wp, 0) - ego.position
                    c = pos_to_index(p[0], p[1])
                    if 0 <= c[0] < grid.shape[-2] and 0 <= c[1] < grid.shape[-1]:
                        grid[layer, c[0], c[1]] = 1
    grid = np.clip(grid, -1, 1)
    return np.nan_to_num(grid).astype(np.float32)


def ttc_obs(road, horizon=10, policy_frequency=1):
    """TimeToCollisionObservation.observe (observation.py:126-151) around the reference's own
    compute_ttc_grid (finite_mdp.py:104-167)."""
    ego = road.vehicles[0]
    env = types.SimpleNamespace(vehicle=ego, road=road, config={"policy_frequency": policy_frequency})
    grid = R.finite_mdp.compute_ttc_grid(env, vehicle=ego, time_quantization=1 / policy_frequency,
                                         horizon=horizon)
    padding = np.ones(np.shape(grid))
    padded_grid = np.concatenate([padding, grid, padding], axis=1)
    obs_lanes = 3
    l0 = grid.shape[1] + ego.lane_index[2] - obs_lanes // 2
    lf = grid.shape[1] + ego.lane_index[2] + obs_lanes // 2
    clamped_grid = padded_grid[:, l0: lf + 1, :]
    repeats = np.ones(clamped_grid.shape[0])
    repeats[np.array([0, -1])] += clamped_grid.shape[0]
    padded_grid = np.repeat(clamped_grid, repeats.astype(int), axis=0)
    obs_speeds = 3
    v0 = grid.shape[0] + ego.speed_index - obs_speeds // 2
    vf = grid.shape[0] + ego.speed_index + obs_speeds // 2
    clamped_grid = padded_grid[v0: vf + 1, :, :]
    return clamped_grid.astype(np.float32)


def lidar_obs(road, cells=16, maximum_range=60.0, normalize=True):
    """LidarObservation.observe / trace (observation.py:694-768) with the reference's
    utils.rect_corners and utils.distance_to_rect."""
    ego = road.vehicles[0]
    angle = 2 * np.pi / cells
    origin, origin_velocity = ego.position.copy(), ego.velocity
    grid = np.ones((cells, 2)) * maximum_range

    def position_to_angle(position):
        return np.arctan2(position[1] - origin[1], position[0] - origin[0]) + angle / 2

    def angle_to_index(a):
        return int(np.floor(a / angle)) % cells

    def index_to_direction(index):
        return np.array([np.cos(index * angle), np.sin(index * angle)])

    for obstacle in road.vehicles + road.objects:
        if obstacle is ego or not obstacle.solid:
            continue
        center_distance = np.linalg.norm(obstacle.position - origin)
        if center_distance > maximum_range:
            continue
        center_index = angle_to_index(position_to_angle(obstacle.position))
        distance = center_distance - obstacle.WIDTH / 2
        if distance <= grid[center_index, 0]:
            direction = index_to_direction(center_index)
            velocity = (obstacle.velocity - origin_velocity).dot(direction)
            grid[center_index, :] = [distance, velocity]
        corners = R.utils.rect_corners(obstacle.position, obstacle.LENGTH, obstacle.WIDTH, obstacle.heading)
        angles = [position_to_angle(corner) for corner in corners]
        min_angle, max_angle = min(angles), max(angles)
        if min_angle < -np.pi / 2 < np.pi / 2 < max_angle:
            min_angle, max_angle = max_angle, min_angle + 2 * np.pi
        start, end = angle_to_index(min_angle), angle_to_index(max_angle)
        if start < end:
            indexes = np.arange(start, end + 1)
        else:
            indexes = np.hstack([np.arange(start, cells), np.arange(0, end + 1)])
        for index in indexes:
            direction = index_to_direction(index)
            ray = [origin, origin + maximum_range * direction]
            distance = R.utils.distance_to_rect(ray, corners)
            if distance <= grid[index, 0]:
                velocity = (obstacle.velocity - origin_velocity).dot(direction)
                grid[index, :] = [distance, velocity]
    obs = grid.copy()
    if normalize:
        obs /= maximum_range
    return obs


# ---------------------------------------------------------------- rollout
def rollout(road, policy_steps: int, seed: int, frames_per_step: int = 15, obs=True):
    """AbstractEnv._simulate (abstract.py:252-282): frame 0 of each policy step applies the
    ego meta-action (DiscreteMetaAction.act, action.py:259-260), then Road.act, Road.step(1/15)."""
    dt = 1 / 15
    rng = np.random.default_rng(7777 + seed)
    actions = rng.integers(0, 5, size=policy_steps).astype(np.int32)
    states = [snapshot(road)]
    acts, nbrs = [], []
    kin5, kin15, kid5, kid15, grid, grid2, ttc, lidar = [], [], [], [], [], [], [], []

    def observe():
        o, i = kinematics_obs(road, KIN_DEFAULT); kin5.append(o); kid5.append(i)
        o, i = kinematics_obs(road, KIN_ENVJSON); kin15.append(o); kid15.append(i)
        grid.append(grid_obs(road, GRID_DENSE))
        grid2.append(grid_obs(road, GRID_ONROAD))
        ttc.append(ttc_obs(road))
        lidar.append(lidar_obs(road))

    if obs:
        observe()
    for p in range(policy_steps):
        for f in range(frames_per_step):
            if f == 0:
                road.vehicles[0].act(ACTIONS_ALL[int(actions[p])])
            road.act()
            acts.append(snapshot(road))           # post-act, pre-step
            nbrs.append(neighbours(road))
            road.step(dt)
            states.append(snapshot(road))
        if obs:
            observe()
    out = {}
    for k in FIELDS_F + FIELDS_I:
        out[k] = np.stack([s[k] for s in states])
        out["act_" + k] = np.stack([s[k] for s in acts])
    out["nbr"] = np.stack(nbrs)
    out["actions"] = actions
    if obs:
        out["kin5"] = np.stack(kin5); out["kin5_ids"] = np.stack(kid5)
        out["kin15"] = np.stack(kin15); out["kin15_ids"] = np.stack(kid15)
        out["grid7"] = np.stack(grid); out["grid_onroad"] = np.stack(grid2)
        out["ttc"] = np.stack(ttc); out["lidar"] = np.stack(lidar)
    return out


def stats(name, d):
    lane_changes = int(((d["act_target_lane"] != d["target_lane"][:-1])).sum())
    crashes = int(d["crashed"][-1].sum())
    impacts = int(np.isfinite(d["impact_x"]).sum())
    changing = int((d["lane"] != d["target_lane"]).sum())
    print(f"{name}: target changes={lane_changes} changing-state={changing} crashed={crashes} impacts={impacts}")


def main():
    os.makedirs(OUT, exist_ok=True)
    cases = []
    for n in (8, 32, 64, 128):
        for seed in (0, 1, 2):
            steps = 4 if n <= 64 else 2
            cases.append(("highway", n, seed, steps))
    for n in (16, 64):
        for seed in (0, 1):
            cases.append(("dense", n, seed, 2))
    for kind in ("sine", "arc"):
        for seed in (0, 1):
            cases.append((kind, 32, seed, 4))
    for kind, n, seed, steps in cases:
        if kind == "highway":
            road = make_highway(n, seed)
        elif kind == "dense":
            road = make_dense(n, seed)
        else:
            road = make_curved(kind, n, seed)
        d = rollout(road, steps, seed)
        d["meta"] = np.array([n, seed, steps, 15, len(road.network.lanes_list())], dtype=np.int64)
        if kind in ("highway", "dense"):
            d["lane_table"] = np.array([[l.start[0], l.start[1], l.end[0], l.end[1], l.width, l.speed_limit]
                                        for l in road.network.lanes_list()])
        else:
            d["lane_table"] = lane_geometry(road)
        name = f"{kind}_n{n}_s{seed}"
        stats(name, d)
        np.savez_compressed(os.path.join(OUT, name + ".npz"), **d)


if __name__ == "__main__":
    main()
