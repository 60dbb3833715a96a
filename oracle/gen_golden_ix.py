"""Golden vectors of the intersection scenario — TEST INFRASTRUCTURE, build container only.

The reference's actual training scenario (scripts/example.py:17, configs/IntersectionEnv/env.json)
is intersection-v0.  Its simulation core is imported unmodified from ``/root/reference`` through
``gen_golden`` (RoadNetwork, StraightLane / CircularLane, RegulatedRoad, IDMVehicle, MDPVehicle);
``intersection_env.py`` itself imports gymnasium (absent), so the env-level code is restated here,
line for line, on top of those reference objects:
  * _make_road            intersection_env.py:141-249
  * _make_vehicles        intersection_env.py:251-318
  * _spawn_vehicle        intersection_env.py:320-348
  * _clear_vehicles       intersection_env.py:350-362
  * has_arrived           intersection_env.py:364-369
  * _agent_reward / _is_terminated / _is_truncated  intersection_env.py:78-119
  * AbstractEnv.reset / step / _simulate           abstract.py:188-282
  * KinematicObservation.observe (absolute, order "shuffled" from env.json) observation.py:233-275
Each episode draws from one ``np.random.default_rng(seed)`` shared by the road and the env,
as gymnasium's ``seeding.np_random`` does, so spawn draws and the observation shuffle interleave
exactly as in the reference.

Usage:  PYTHONDONTWRITEBYTECODE=1 python oracle/gen_golden_ix.py
"""
from __future__ import annotations

import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import gen_golden as G  # noqa: E402  (imports the reference sim core)

R = G.R
from ttrl_env.road.lane import AbstractLane, LineType  # noqa: E402
from ttrl_env.road.regulation import RegulatedRoad  # noqa: E402

OUT = G.OUT
ACTIONS_LONGI = {0: "SLOWER", 1: "IDLE", 2: "FASTER"}  # action.py:207
TARGET_SPEEDS = [0, 4.5, 9]
KIN_IX = dict(features=["presence", "x", "y", "vx", "vy", "cos_h", "sin_h"], vehicles_count=15,
              features_range={"x": [-100, 100], "y": [-100, 100], "vx": [-20, 20], "vy": [-20, 20]},
              absolute=True, see_behind=False, clip=True)
CONFIG = {"duration": 13, "destination": "o1", "initial_vehicle_count": 10, "spawn_probability": 0.6,
          "collision_reward": -5, "high_speed_reward": 1, "arrived_reward": 1, "reward_speed_range": [7.0, 9.0],
          "normalize_reward": False, "offroad_terminal": False, "simulation_frequency": 15, "policy_frequency": 1}
FIELDS_F = G.FIELDS_F
ROUTE_MAX = 4


class IxEnv:
    """IntersectionEnv restated over the reference's road / vehicle classes."""

    def __init__(self, seed: int, order: str = "shuffled"):
        self.np_random = np.random.default_rng(seed)
        self.order = order
        self.config = dict(CONFIG)
        self.time = self.steps = 0
        self._make_road()
        self._make_vehicles(self.config["initial_vehicle_count"])

    # intersection_env.py:141-249
    def _make_road(self):
        lane_width = AbstractLane.DEFAULT_WIDTH
        right_turn_radius = lane_width + 5
        left_turn_radius = right_turn_radius + lane_width
        outer_distance = right_turn_radius + lane_width / 2
        access_length = 50 + 50
        net = R.RoadNetwork()
        n, c, s = LineType.NONE, LineType.CONTINUOUS, LineType.STRIPED
        for corner in range(4):
            angle = np.radians(90 * corner)
            is_horizontal = corner % 2
            priority = 3 if is_horizontal else 1
            rotation = np.array([[np.cos(angle), -np.sin(angle)], [np.sin(angle), np.cos(angle)]])
            start = rotation @ np.array([lane_width / 2, access_length + outer_distance])
            end = rotation @ np.array([lane_width / 2, outer_distance])
            net.add_lane("o" + str(corner), "ir" + str(corner),
                         R.StraightLane(start, end, line_types=[s, c], priority=priority, speed_limit=10))
            r_center = rotation @ (np.array([outer_distance, outer_distance]))
            net.add_lane("ir" + str(corner), "il" + str((corner - 1) % 4),
                         R.CircularLane(r_center, right_turn_radius, angle + np.radians(180), angle + np.radians(270),
                                        line_types=[n, c], priority=priority, speed_limit=10))
            l_center = rotation @ (np.array([-left_turn_radius + lane_width / 2, left_turn_radius - lane_width / 2]))
            net.add_lane("ir" + str(corner), "il" + str((corner + 1) % 4),
                         R.CircularLane(l_center, left_turn_radius, angle + np.radians(0), angle + np.radians(-90),
                                        clockwise=False, line_types=[n, n], priority=priority - 1, speed_limit=10))
            start = rotation @ np.array([lane_width / 2, outer_distance])
            end = rotation @ np.array([lane_width / 2, -outer_distance])
            net.add_lane("ir" + str(corner), "il" + str((corner + 2) % 4),
                         R.StraightLane(start, end, line_types=[s, n], priority=priority, speed_limit=10))
            start = rotation @ np.flip([lane_width / 2, access_length + outer_distance], axis=0)
            end = rotation @ np.flip([lane_width / 2, outer_distance], axis=0)
            net.add_lane("il" + str((corner - 1) % 4), "o" + str((corner - 1) % 4),
                         R.StraightLane(end, start, line_types=[n, c], priority=priority, speed_limit=10))
        self.road = RegulatedRoad(network=net, np_random=self.np_random, record_history=False)

    # intersection_env.py:251-318
    def _make_vehicles(self, n_vehicles=10):
        R.IDMVehicle.DISTANCE_WANTED = 7
        R.IDMVehicle.COMFORT_ACC_MAX = 6
        R.IDMVehicle.COMFORT_ACC_MIN = -3
        simulation_steps = 3
        for t in range(n_vehicles - 1):
            self._spawn_vehicle(np.linspace(0, 80, n_vehicles)[t])
        for _ in range(simulation_steps):
            [(self.road.act(), self.road.step(1 / self.config["simulation_frequency"]))
             for _ in range(self.config["simulation_frequency"])]
        self._spawn_vehicle(60, spawn_probability=1, go_straight=True, position_deviation=0.1, speed_deviation=0)
        self.controlled_vehicles = []
        ego_lane = self.road.network.get_lane(("o0", "ir0", 0))
        destination = self.config["destination"]
        ego = R.MDPVehicle(self.road, ego_lane.position(60 + 5 * self.np_random.normal(1), 0),
                           speed=ego_lane.speed_limit, heading=ego_lane.heading_at(60), target_speeds=TARGET_SPEEDS)
        ego.plan_route_to(destination)
        ego.speed_index = ego.speed_to_index(ego_lane.speed_limit)
        ego.target_speed = ego.index_to_speed(ego.speed_index)
        self.road.vehicles.append(ego)
        self.controlled_vehicles.append(ego)
        for v in self.road.vehicles:  # Prevent early collisions (removal while iterating, as the reference)
            if v is not ego and np.linalg.norm(v.position - ego.position) < 20:
                self.road.vehicles.remove(v)
        self.vehicle = ego

    # intersection_env.py:320-348
    def _spawn_vehicle(self, longitudinal=0, position_deviation=1.0, speed_deviation=1.0, spawn_probability=0.6,
                       go_straight=False):
        if self.np_random.uniform() > spawn_probability:
            return
        route = self.np_random.choice(range(4), size=2, replace=False)
        route[1] = (route[0] + 2) % 4 if go_straight else route[1]
        vehicle = R.IDMVehicle.make_on_lane(self.road, ("o" + str(route[0]), "ir" + str(route[0]), 0),
                                            longitudinal=(longitudinal + 5 + self.np_random.normal() * position_deviation),
                                            speed=8 + self.np_random.normal() * speed_deviation)
        for v in self.road.vehicles:
            if np.linalg.norm(v.position - vehicle.position) < 15:
                return
        vehicle.plan_route_to("o" + str(route[1]))
        vehicle.randomize_behavior()
        self.road.vehicles.append(vehicle)
        return vehicle

    # intersection_env.py:350-362
    def _clear_vehicles(self):
        def is_leaving(vehicle):
            return ("il" in vehicle.lane_index[0] and "o" in vehicle.lane_index[1]
                    and vehicle.lane.local_coordinates(vehicle.position)[0] >= vehicle.lane.length - 4 * vehicle.LENGTH)
        self.road.vehicles = [v for v in self.road.vehicles
                              if v in self.controlled_vehicles or not (is_leaving(v) or v.route is None)]

    def has_arrived(self, vehicle, exit_distance=25):
        return ("il" in vehicle.lane_index[0] and "o" in vehicle.lane_index[1]
                and vehicle.lane.local_coordinates(vehicle.position)[0] >= exit_distance)

    # intersection_env.py:78-119
    def reward(self):
        v = self.vehicle
        scaled = R.utils.lmap(v.speed, self.config["reward_speed_range"], [0, 1])
        rewards = {"collision_reward": v.crashed, "high_speed_reward": np.clip(scaled, 0, 1),
                   "arrived_reward": self.has_arrived(v), "on_road_reward": v.on_road}
        reward = sum(self.config.get(name, 0) * r for name, r in rewards.items())
        reward = self.config["arrived_reward"] if rewards["arrived_reward"] else reward
        reward *= rewards["on_road_reward"]
        return float(reward)

    def terminated(self):
        v = self.vehicle
        return bool(v.crashed or self.has_arrived(v) or (self.config["offroad_terminal"] and not v.on_road))

    def truncated(self):
        return bool(self.time >= self.config["duration"])

    # observation.py:233-275 (absolute; sorted or shuffled with the env generator)
    def observe(self):
        ego = self.vehicle
        cfg = KIN_IX
        feats, V = cfg["features"], cfg["vehicles_count"]
        rows = [ego.to_dict()]
        close = self.road.close_objects_to(ego, 5.0 * R.Vehicle.MAX_SPEED, count=V - 1, see_behind=cfg["see_behind"],
                                           sort=self.order == "sorted", vehicles_only=False)
        for v in close[-V + 1:]:
            rows.append(v.to_dict(None, observe_intentions=False))
        fr = cfg["features_range"]
        obs = np.zeros((V, len(feats)))
        for r, d in enumerate(rows):
            for c, f in enumerate(feats):
                val = float(d[f])
                if f in fr:
                    val = R.utils.lmap(val, [fr[f][0], fr[f][1]], [-1, 1])
                    val = float(np.clip(val, -1, 1))
                obs[r, c] = val
        if self.order == "shuffled":
            self.np_random.shuffle(obs[1:])
        return obs.astype(np.float32)

    # abstract.py:228-282 + intersection_env.py:135-139
    def step(self, action: int, record=None):
        self.time += 1 / self.config["policy_frequency"]
        frames = int(self.config["simulation_frequency"] // self.config["policy_frequency"])
        for frame in range(frames):
            if self.steps % frames == 0:
                self.vehicle.act(ACTIONS_LONGI[int(action)])
            self.road.act()
            if record is not None:
                record["act"].append(snapshot(self))
            self.road.step(1 / self.config["simulation_frequency"])
            self.steps += 1
            if record is not None:
                record["frames"].append(snapshot(self))
        obs = self.observe()
        rew, term, trunc = self.reward(), self.terminated(), self.truncated()
        self._clear_vehicles()
        self._spawn_vehicle(spawn_probability=self.config["spawn_probability"])
        return obs, rew, term, trunc


# ------------------------------------------------------------------ network table
def network_tables(road):
    """Flat lane tables in lanes_list order: geometry rows for _abi.lane_table_from_arrays and
    [L, 6] int rows (road id, from node, to node, priority, exit flag, lane id within road);
    roads and nodes are numbered in graph order (RoadNetwork.graph insertion order)."""
    graph = road.network.graph
    nodes, roads = [], []
    for fr, tos in graph.items():
        if fr not in nodes:
            nodes.append(fr)
        for to in tos:
            if to not in nodes:
                nodes.append(to)
            roads.append((fr, to))
    geom = G.lane_geometry(road)
    net = []
    for r, (fr, to) in enumerate(roads):
        for i, ln in enumerate(graph[fr][to]):
            exit_ = int("il" in fr and "o" in to)
            net.append([r, nodes.index(fr), nodes.index(to), ln.priority, exit_, i])
    return geom, np.array(net, dtype=np.int32), nodes, roads


def lane_flat(road, index):
    k = 0
    for fr, tos in road.network.graph.items():
        for to, lanes in tos.items():
            if (fr, to) == tuple(index[:2]):
                return k + index[2]
            k += len(lanes)
    raise KeyError(index)


def road_id(road, fr, to):
    k = 0
    for f, tos in road.network.graph.items():
        for t in tos:
            if (f, t) == (fr, to):
                return k
            k += 1
    raise KeyError((fr, to))


def snapshot(env):
    road = env.road
    vs = road.vehicles
    n = len(vs)
    s = {k: np.zeros(n) for k in FIELDS_F}
    for k in ("lane", "target_lane", "crashed", "speed_index", "kind", "yielding", "route_n"):
        s[k] = np.zeros(n, dtype=np.int32)
    s["route_road"] = np.full((n, ROUTE_MAX), -1, dtype=np.int32)
    s["route_lane"] = np.full((n, ROUTE_MAX), -1, dtype=np.int32)
    for i, v in enumerate(vs):
        s["x"][i], s["y"][i] = v.position
        s["heading"][i], s["speed"][i], s["target_speed"][i] = v.heading, v.speed, v.target_speed
        s["timer"][i] = getattr(v, "timer", 0.0)
        s["delta"][i] = getattr(v, "DELTA", R.IDMVehicle.DELTA)
        s["steer"][i], s["acc"][i] = v.action["steering"], v.action["acceleration"]
        if v.impact is None:
            s["impact_x"][i] = s["impact_y"][i] = np.nan
        else:
            s["impact_x"][i], s["impact_y"][i] = v.impact
        s["lane"][i] = lane_flat(road, v.lane_index)
        s["target_lane"][i] = lane_flat(road, v.target_lane_index)
        s["crashed"][i] = int(bool(v.crashed))
        s["speed_index"][i] = int(getattr(v, "speed_index", -1))
        s["kind"][i] = 1 if isinstance(v, R.MDPVehicle) else 2
        s["yielding"][i] = int(bool(getattr(v, "is_yielding", False)))
        if v.route is None:
            s["route_n"][i] = -1
        else:
            assert len(v.route) <= ROUTE_MAX
            s["route_n"][i] = len(v.route)
            for k, (fr, to, lid) in enumerate(v.route):
                s["route_road"][i, k] = road_id(road, fr, to)
                s["route_lane"][i, k] = -1 if lid is None else int(lid)
    s["reg_steps"] = np.int32(road.steps)
    return s


def stack(snaps, nmax):
    """[len(snaps), nmax] arrays, padded with absent vehicles (kind 0)."""
    out = {}
    for k in snaps[0]:
        if k == "reg_steps":
            out[k] = np.array([s[k] for s in snaps], dtype=np.int32)
            continue
        a0 = snaps[0][k]
        shape = (len(snaps), nmax) + a0.shape[1:]
        fill = np.nan if k in ("impact_x", "impact_y") else (-1 if k in ("route_road", "route_lane") else 0)
        arr = np.full(shape, fill, dtype=a0.dtype)
        for t, s in enumerate(snaps):
            arr[t, :len(s[k])] = s[k]
        out[k] = arr
    return out


def episode(seed: int, steps: int, order="shuffled"):
    """One reset + ``steps`` env steps.  Per policy step p: the state entering the step ("pre"),
    the 15 post-act and post-step frame states, the observation / reward / flags after the
    frames, and the state after _clear_vehicles + _spawn_vehicle (= pre of p + 1)."""
    env = IxEnv(seed, order)
    obs0 = env.observe()  # AbstractEnv.reset observes once (abstract.py:210): a shuffle draw
    rng = np.random.default_rng(555 + seed)
    actions = rng.integers(0, 3, size=steps).astype(np.int32)
    pres, frames, acts, posts = [], [], [], []
    obs, rew, term, trunc = [], [], [], []
    for p in range(steps):
        pres.append(snapshot(env))
        rec = {"act": [], "frames": []}
        o, r, te, tr = env.step(int(actions[p]), rec)
        frames.append(rec["frames"]); acts.append(rec["act"])
        obs.append(o); rew.append(r); term.append(te); trunc.append(tr)
        posts.append(snapshot(env))
    allsnaps = pres + posts + [s for f in frames for s in f] + [s for a in acts for s in a]
    nmax = max(len(s["x"]) for s in allsnaps)
    d = {}
    for name, snaps in (("pre", pres), ("post", posts)):
        for k, v in stack(snaps, nmax).items():
            d[f"{name}_{k}"] = v
    for name, lists in (("frame", frames), ("act", acts)):
        st = stack([s for f in lists for s in f], nmax)
        for k, v in st.items():
            d[f"{name}_{k}"] = v.reshape((steps, 15) + v.shape[1:])
    d["actions"] = actions
    d["obs0"] = obs0
    d["obs"] = np.stack(obs)
    d["reward"] = np.array(rew)
    d["terminated"] = np.array(term, dtype=np.uint8)
    d["truncated"] = np.array(trunc, dtype=np.uint8)
    geom, net, nodes, roads = network_tables(env.road)
    d["lane_table"] = geom
    d["lane_net"] = net
    d["meta"] = np.array([seed, steps, nmax, len(geom), len(roads)], dtype=np.int64)
    return d


def main():
    os.makedirs(OUT, exist_ok=True)
    for seed in range(6):
        d = episode(seed, 13)
        name = f"ix_s{seed}"
        n_alive = (d["pre_kind"] > 0).sum(axis=1)
        print(f"{name}: vehicles per step {n_alive.tolist()} yield-frames {int(d['frame_yielding'].sum())} "
              f"crashed {int(d['post_crashed'].sum())} reward {np.round(d['reward'], 3).tolist()} "
              f"term {d['terminated'].tolist()}")
        np.savez_compressed(os.path.join(OUT, name + ".npz"), **d)


if __name__ == "__main__":
    main()
