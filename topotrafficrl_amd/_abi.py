"""ctypes mirror of include/ttrl_mi355x.h and the host-side builders of its structs.

The derived lane geometry and behaviour constants are computed here with the
same float64 expressions the reference evaluates (StraightLane.__init__
lane.py:162-194, IDMVehicle/ControlledVehicle class constants behavior.py:20-46,
controller.py:24-33), so the kernels receive bit-identical constants.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

MAX_LANES = 32
MAX_ROADS = 32
MAX_NODES = 32
ROUTE_MAX = 4
RNG_WORDS = 5
IX_MAX_INIT = 16
N_FEATURES = 14
F32, F64 = 0, 1
ABSENT, MDP, IDM = 0, 1, 2
LANE_LEFT, IDLE, LANE_RIGHT, FASTER, SLOWER = 0, 1, 2, 3, 4
ACTIONS_ALL = {0: "LANE_LEFT", 1: "IDLE", 2: "LANE_RIGHT", 3: "FASTER", 4: "SLOWER"}  # action.py:204

FEATURES = ["presence", "x", "y", "vx", "vy", "heading", "cos_h", "sin_h", "cos_d", "sin_d",
            "long_off", "lat_off", "ang_off", "on_road"]
FEATURE_CODE = {f: i for i, f in enumerate(FEATURES)}

REAL_FIELDS = ["x", "y", "heading", "speed", "target_speed", "timer", "delta",
               "steer", "acc", "impact_x", "impact_y"]
I32_FIELDS = ["lane", "target_lane", "speed_index"]
U8_FIELDS = ["kind", "crashed", "has_impact", "lane_change"]
# network / regulation fields: shapes [E, N, ROUTE_MAX], [E, N], [E]
ROUTE_FIELDS = ["route_road", "route_lane"]
NET_FIELDS = ROUTE_FIELDS + ["route_n", "yielding", "reg_steps"]
# AbstractEnv.np_random per env: [E, RNG_WORDS] uint64 numpy Generator(PCG64) state
ALL_FIELDS = REAL_FIELDS + I32_FIELDS + U8_FIELDS + NET_FIELDS + ["rng"]

ERRORS = {-1: "TTRL_E_ARG (bad argument)", -2: "TTRL_E_LAUNCH (HIP error)", -3: "TTRL_E_UNSUPPORTED"}


class LaneTable(C.Structure):
    _fields_ = [("n_lanes", C.c_int32), ("n_roads", C.c_int32),
                ("start_x", C.c_double * MAX_LANES), ("start_y", C.c_double * MAX_LANES),
                ("dir_x", C.c_double * MAX_LANES), ("dir_y", C.c_double * MAX_LANES),
                ("length", C.c_double * MAX_LANES), ("width", C.c_double * MAX_LANES),
                ("heading", C.c_double * MAX_LANES), ("speed_limit", C.c_double * MAX_LANES),
                ("forbidden", C.c_int32 * MAX_LANES), ("type", C.c_int32 * MAX_LANES),
                ("amplitude", C.c_double * MAX_LANES), ("pulsation", C.c_double * MAX_LANES),
                ("phase", C.c_double * MAX_LANES), ("center_x", C.c_double * MAX_LANES),
                ("center_y", C.c_double * MAX_LANES), ("radius", C.c_double * MAX_LANES),
                ("start_phase", C.c_double * MAX_LANES), ("direction", C.c_double * MAX_LANES),
                ("road", C.c_int32 * MAX_LANES), ("lane_id", C.c_int32 * MAX_LANES),
                ("priority", C.c_int32 * MAX_LANES), ("exit_lane", C.c_int32 * MAX_LANES),
                ("road_from", C.c_int32 * MAX_ROADS), ("road_to", C.c_int32 * MAX_ROADS),
                ("road_first", C.c_int32 * MAX_ROADS), ("road_n", C.c_int32 * MAX_ROADS),
                ("regulation_frequency", C.c_int32), ("_pad2", C.c_int32)]


LANE_STRAIGHT, LANE_SINE, LANE_CIRCULAR = 0, 1, 2


class Params(C.Structure):
    _fields_ = [(n, C.c_double) for n in (
        "acc_max", "comfort_acc_max", "comfort_acc_min", "distance_wanted", "time_wanted",
        "gap_denom", "politeness", "lane_change_min_acc_gain", "lane_change_max_braking",
        "lane_change_delay", "tau_pursuit", "kp_a", "kp_heading", "kp_lateral", "max_steering",
        "length", "width", "diagonal", "max_speed", "min_speed", "lane_vehicle_length")] + [
        ("target_speeds", C.c_double * 8), ("n_target_speeds", C.c_int32), ("_pad", C.c_int32)]


class State(C.Structure):
    _fields_ = ([("n_envs", C.c_int32), ("n_veh", C.c_int32), ("dtype", C.c_int32), ("_pad", C.c_int32)]
                + [(n, C.c_void_p) for n in ALL_FIELDS])


class KinCfg(C.Structure):
    _fields_ = [("vehicles_count", C.c_int32), ("n_features", C.c_int32),
                ("features", C.c_int32 * N_FEATURES),
                ("absolute", C.c_int32), ("normalize", C.c_int32), ("clip", C.c_int32),
                ("see_behind", C.c_int32), ("order_shuffled", C.c_int32), ("_pad", C.c_int32),
                ("range_lo", C.c_double * N_FEATURES), ("range_hi", C.c_double * N_FEATURES),
                ("has_range", C.c_int32 * N_FEATURES), ("perception_distance", C.c_double),
                ("shuffle_seed", C.c_uint64), ("shuffle_offset", C.c_uint64)]


class GridCfg(C.Structure):
    _fields_ = [("n_features", C.c_int32), ("features", C.c_int32 * N_FEATURES),
                ("shape_x", C.c_int32), ("shape_y", C.c_int32), ("clip", C.c_int32),
                ("grid_min_x", C.c_double), ("grid_min_y", C.c_double),
                ("step_x", C.c_double), ("step_y", C.c_double),
                ("range_lo", C.c_double * N_FEATURES), ("range_hi", C.c_double * N_FEATURES),
                ("has_range", C.c_int32 * N_FEATURES), ("lane_perception_distance", C.c_double)]


class ResetCfg(C.Structure):
    _fields_ = [("n_vehicles", C.c_int32), ("ego_lane", C.c_int32),
                ("ego_x", C.c_double), ("ego_speed", C.c_double),
                ("speed_lo", C.c_double), ("speed_hi", C.c_double), ("spacing", C.c_double),
                ("density_factor", C.c_double), ("delta_lo", C.c_double), ("delta_hi", C.c_double),
                ("lane_change", C.c_int32), ("_pad", C.c_int32)]


class RewardCfg(C.Structure):
    _fields_ = [("collision_reward", C.c_double), ("high_speed_reward", C.c_double),
                ("speed_lo", C.c_double), ("speed_hi", C.c_double),
                ("normalize_reward", C.c_int32), ("offroad_terminal", C.c_int32),
                ("duration", C.c_double), ("arrived_reward", C.c_double), ("exit_distance", C.c_double)]


class IxCfg(C.Structure):
    _fields_ = [("initial_vehicle_count", C.c_int32), ("warmup_frames", C.c_int32), ("warmup_dt", C.c_double),
                ("init_longitudinal", C.c_double * IX_MAX_INIT), ("spawn_probability", C.c_double),
                ("spawn_offset", C.c_double), ("spawn_speed", C.c_double), ("spawn_clear_distance", C.c_double),
                ("challenger_longitudinal", C.c_double), ("challenger_position_deviation", C.c_double),
                ("challenger_speed_deviation", C.c_double), ("delta_lo", C.c_double), ("delta_hi", C.c_double),
                ("n_corners", C.c_int32), ("entry_lane", C.c_int32 * 4), ("exit_node", C.c_int32 * 4),
                ("ego_lane", C.c_int32), ("ego_destination", C.c_int32),
                ("ego_longitudinal", C.c_double), ("ego_deviation", C.c_double), ("ego_heading_s", C.c_double),
                ("ego_speed", C.c_double), ("ego_clear_distance", C.c_double), ("leave_margin", C.c_double),
                ("path_road", ((C.c_int8 * (ROUTE_MAX - 1)) * 4) * MAX_NODES),
                ("path_len", (C.c_int8 * 4) * MAX_NODES)]


class TtcCfg(C.Structure):
    _fields_ = [("horizon_bins", C.c_int32), ("obs_lanes", C.c_int32), ("obs_speeds", C.c_int32),
                ("_pad", C.c_int32), ("time_quantization", C.c_double)]


class LidarCfg(C.Structure):
    _fields_ = [("cells", C.c_int32), ("normalize", C.c_int32), ("maximum_range", C.c_double)]


# ----------------------------------------------------------------------------- builders
def _single_road(t: "LaneTable") -> "LaneTable":
    """Topology of one road "0" -> "1" holding every lane (road 0, lane_id = l)."""
    t.n_roads = 1
    for i in range(t.n_lanes):
        t.road[i], t.lane_id[i] = 0, i
    t.road_from[0], t.road_to[0], t.road_first[0], t.road_n[0] = 0, 1, 0, t.n_lanes
    return t


def set_network(t: "LaneTable", net: np.ndarray, regulation_frequency: int = 0) -> "LaneTable":
    """Topology rows [L, 6] (road, from node, to node, priority, exit flag, lane id) in
    lanes_list order, as dumped by oracle/gen_golden_ix.network_tables."""
    net = np.asarray(net, dtype=np.int64)
    if len(net) != t.n_lanes:
        raise ValueError("one topology row per lane")
    n_roads = int(net[:, 0].max()) + 1
    if n_roads > MAX_ROADS:
        raise ValueError(f"at most {MAX_ROADS} roads")
    t.n_roads = n_roads
    for i, (rd, fr, to, prio, ex, lid) in enumerate(net):
        t.road[i], t.lane_id[i], t.priority[i], t.exit_lane[i] = int(rd), int(lid), int(prio), int(ex)
        if lid == 0:
            t.road_from[rd], t.road_to[rd], t.road_first[rd] = int(fr), int(to), i
        t.road_n[rd] += 1
    for i in range(t.n_lanes):  # lanes of a road are contiguous, in id order (lanes_list order)
        if t.road_first[t.road[i]] + t.lane_id[i] != i:
            raise ValueError("the lanes of a road must be contiguous and in id order")
    t.regulation_frequency = int(regulation_frequency)
    return t

def straight_lane_table(lanes: int = 4, start: float = 0.0, length: float = 10000.0, angle: float = 0.0,
                        speed_limit: float = 30.0, width: float = 4.0, forbidden=None) -> LaneTable:
    """RoadNetwork.straight_road_network (road.py:291-321) + StraightLane.__init__ (lane.py:162-194)."""
    if not 1 <= lanes <= MAX_LANES:
        raise ValueError(f"lanes must be in [1, {MAX_LANES}]")
    t = LaneTable()
    t.n_lanes = lanes
    rot = np.array([[np.cos(angle), np.sin(angle)], [-np.sin(angle), np.cos(angle)]])
    for i in range(lanes):
        o = rot @ np.array([start, i * 4.0])      # StraightLane.DEFAULT_WIDTH spacing
        e = rot @ np.array([start + length, i * 4.0])
        ln = np.linalg.norm(e - o)
        d = (e - o) / ln
        t.start_x[i], t.start_y[i] = float(o[0]), float(o[1])
        t.dir_x[i], t.dir_y[i] = float(d[0]), float(d[1])
        t.length[i] = float(ln)
        t.width[i] = float(width)
        t.heading[i] = float(np.arctan2(e[1] - o[1], e[0] - o[0]))
        t.speed_limit[i] = float(speed_limit)
        t.forbidden[i] = int(bool(forbidden[i])) if forbidden is not None else 0
    return _single_road(t)


def _set_straight(t: LaneTable, i: int, start, end, width, speed_limit):
    """StraightLane.__init__ lane.py:162-194 (float64, the reference's own expressions)."""
    s, e = np.asarray(start, dtype=np.float64), np.asarray(end, dtype=np.float64)
    ln = np.linalg.norm(e - s)
    d = (e - s) / ln
    t.start_x[i], t.start_y[i], t.dir_x[i], t.dir_y[i] = s[0], s[1], d[0], d[1]
    t.length[i], t.width[i], t.speed_limit[i] = ln, width, speed_limit
    t.heading[i] = np.arctan2(e[1] - s[1], e[0] - s[0])


def lane_table_from_arrays(table: np.ndarray) -> LaneTable:
    """[L, 6] straight rows (start_x, start_y, end_x, end_y, width, speed_limit), or [L, 16]
    geometry rows (type, those 6, amplitude, pulsation, phase, center_x, center_y, radius,
    start_phase, end_phase, clockwise), as dumped by gen_golden."""
    table = np.asarray(table, dtype=np.float64)
    t = LaneTable()
    t.n_lanes = len(table)
    for i, row in enumerate(table):
        if len(row) == 6:
            row = np.concatenate([[LANE_STRAIGHT], row, np.zeros(9)])
        typ, sx, sy, ex, ey, w, lim, amp, puls, ph, cx, cy, rad, sph, eph, cw = row
        t.type[i] = int(typ)
        if int(typ) == LANE_CIRCULAR:  # CircularLane.__init__ lane.py:296-315
            d = 1.0 if cw else -1.0
            t.center_x[i], t.center_y[i], t.radius[i], t.start_phase[i], t.direction[i] = cx, cy, rad, sph, d
            t.length[i] = rad * (eph - sph) * d
            t.width[i], t.speed_limit[i] = w, lim
        else:
            _set_straight(t, i, (sx, sy), (ex, ey), w, lim)
            t.amplitude[i], t.pulsation[i], t.phase[i] = amp, puls, ph
    return _single_road(t)


def sine_lane_table(lanes: int = 4, length: float = 10000.0, amplitude: float = 5.0,
                    pulsation: float = 2 * np.pi / 200, phase: float = 0.0, speed_limit: float = 30.0,
                    width: float = 4.0) -> LaneTable:
    """``lanes`` parallel SineLanes (lane.py:235-290) from (0, 4i) to (length, 4i)."""
    rows = [[LANE_SINE, 0.0, 4.0 * i, length, 4.0 * i, width, speed_limit, amplitude, pulsation, phase,
             0, 0, 0, 0, 0, 0] for i in range(lanes)]
    return lane_table_from_arrays(np.array(rows))


def circular_lane_table(lanes: int = 3, center=(0.0, 0.0), radius: float = 200.0, start_phase: float = -np.pi / 2,
                        end_phase: float = np.pi / 2, clockwise: bool = True, speed_limit: float = 30.0,
                        width: float = 4.0) -> LaneTable:
    """``lanes`` concentric CircularLanes (lane.py:293-350), radius + 4 i."""
    rows = [[LANE_CIRCULAR, 0, 0, 0, 0, width, speed_limit, 0, 0, 0, center[0], center[1], radius + 4.0 * i,
             start_phase, end_phase, 1.0 if clockwise else 0.0] for i in range(lanes)]
    return lane_table_from_arrays(np.array(rows))


def default_params(target_speeds=None, **overrides) -> Params:
    """Reference class constants (behavior.py:20-46, controller.py:24-33, kinematics.py:21-29)."""
    p = Params()
    p.acc_max = 6.0
    p.comfort_acc_max = 3.0
    p.comfort_acc_min = -5.0
    p.distance_wanted = 5.0 + 5.0
    p.time_wanted = 1.5
    p.politeness = 0.0
    p.lane_change_min_acc_gain = 0.2
    p.lane_change_max_braking = 2.0
    p.lane_change_delay = 1.0
    tau_heading = 0.2
    p.tau_pursuit = 0.5 * tau_heading
    p.kp_a = 1 / 0.6
    p.kp_heading = 1 / tau_heading
    p.kp_lateral = 1 / 0.6
    p.max_steering = np.pi / 3
    p.length = 5.0
    p.width = 2.0
    p.max_speed = 40.0
    p.min_speed = -40.0
    p.lane_vehicle_length = 5.0
    for k, v in overrides.items():
        if not hasattr(p, k):
            raise KeyError(k)
        setattr(p, k, v)
    p.gap_denom = float(2 * np.sqrt(-p.comfort_acc_max * p.comfort_acc_min))
    p.diagonal = float(np.sqrt(p.length ** 2 + p.width ** 2))
    ts = np.linspace(20, 30, 3) if target_speeds is None else np.asarray(target_speeds, dtype=np.float64)
    if not 1 <= len(ts) <= 8:
        raise ValueError("1..8 target speeds supported")
    for i, v in enumerate(ts):
        p.target_speeds[i] = float(v)
    p.n_target_speeds = len(ts)
    return p


def _ranges(cfg_ranges, code_arrays):
    lo, hi, has = code_arrays
    for name, (a, b) in (cfg_ranges or {}).items():
        if name in FEATURE_CODE:
            c = FEATURE_CODE[name]
            lo[c], hi[c], has[c] = float(a), float(b), 1


def kin_cfg(features=("presence", "x", "y", "vx", "vy"), vehicles_count=5, features_range=None,
            absolute=False, order="sorted", normalize=True, clip=True, see_behind=False,
            lanes_on_road=4, perception_distance=200.0, shuffle_seed=0, shuffle_offset=0,
            observe_intentions=False, include_obstacles=True, shuffle_rng="philox", **_ignored) -> KinCfg:
    """KinematicObservation.__init__ (observation.py:159-196); default ranges observation.py:213-225.
    ``shuffle_rng``: "philox" (counter-based, seed + offset) or "np_random" (the env's numpy
    Generator in state.rng, exactly as np_random.shuffle(obs[1:]) draws, observation.py:272-273)."""
    if order not in ("sorted", "shuffled"):
        raise ValueError(f"unknown order {order!r}")
    c = KinCfg()
    c.vehicles_count = int(vehicles_count)
    c.n_features = len(features)
    if not 1 <= c.n_features <= N_FEATURES or c.vehicles_count < 1:
        raise ValueError("bad Kinematics observation shape")
    for i, f in enumerate(features):
        if f not in FEATURE_CODE or f == "on_road":
            raise ValueError(f"unsupported Kinematics feature {f!r}")
        c.features[i] = FEATURE_CODE[f]
    c.absolute, c.normalize, c.clip, c.see_behind = int(absolute), int(normalize), int(clip), int(see_behind)
    if shuffle_rng not in ("philox", "np_random"):
        raise ValueError(f"unknown shuffle_rng {shuffle_rng!r}")
    c.order_shuffled = 0 if order == "sorted" else (2 if shuffle_rng == "np_random" else 1)
    if not features_range:
        features_range = {"x": [-5.0 * 40.0, 5.0 * 40.0], "y": [-4 * lanes_on_road, 4 * lanes_on_road],
                          "vx": [-2 * 40.0, 2 * 40.0], "vy": [-2 * 40.0, 2 * 40.0]}
    _ranges(features_range, (c.range_lo, c.range_hi, c.has_range))
    c.perception_distance = float(perception_distance)
    c.shuffle_seed, c.shuffle_offset = int(shuffle_seed), int(shuffle_offset)
    return c


def grid_cfg(features=("presence", "vx", "vy", "on_road"), grid_size=((-27.5, 27.5), (-27.5, 27.5)),
             grid_step=(5, 5), features_range=None, absolute=False, align_to_vehicle_axes=False,
             clip=True, as_image=False, **_ignored) -> GridCfg:
    """OccupancyGridObservation.__init__ (observation.py:285-326); default ranges :343-347."""
    if absolute:
        raise NotImplementedError("OccupancyGrid absolute=True (observation.py:357-358)")
    if align_to_vehicle_axes or as_image:
        raise NotImplementedError("align_to_vehicle_axes / as_image are not on the hot path")
    g = GridCfg()
    g.n_features = len(features)
    for i, f in enumerate(features):
        if f not in FEATURE_CODE:
            raise ValueError(f"unsupported OccupancyGrid feature {f!r}")
        g.features[i] = FEATURE_CODE[f]
    size = np.array(grid_size, dtype=np.float64)
    step = np.array(grid_step, dtype=np.float64)
    shape = np.asarray(np.floor((size[:, 1] - size[:, 0]) / step), dtype=np.uint8)
    g.shape_x, g.shape_y = int(shape[0]), int(shape[1])
    g.grid_min_x, g.grid_min_y = float(size[0, 0]), float(size[1, 0])
    g.step_x, g.step_y = float(step[0]), float(step[1])
    g.clip = int(clip)
    if not features_range:
        features_range = {"vx": [-2 * 40.0, 2 * 40.0], "vy": [-2 * 40.0, 2 * 40.0]}
    _ranges(features_range, (g.range_lo, g.range_hi, g.has_range))
    g.lane_perception_distance = 100.0
    return g


def reset_cfg(n_vehicles, lanes: LaneTable, ego_lane=1, ego_x=50.0, ego_speed=25.0, spacing=1.0,
              lane_change=True) -> ResetCfg:
    """Highway scene parameters, float64 constants as create_random evaluates them."""
    r = ResetCfg()
    r.n_vehicles = int(n_vehicles)
    r.ego_lane = int(ego_lane)
    r.ego_x, r.ego_speed = float(ego_x), float(ego_speed)
    lim = lanes.speed_limit[0]
    r.speed_lo, r.speed_hi = float(0.7 * lim), float(0.8 * lim)
    r.spacing = float(spacing)
    r.density_factor = float(np.exp(-5 / 40 * lanes.n_lanes))
    r.delta_lo, r.delta_hi = 3.5, 4.5
    r.lane_change = int(lane_change)
    return r


def reward_cfg(collision_reward=-1.0, high_speed_reward=0.4, reward_speed_range=(20.0, 30.0),
               normalize_reward=False, offroad_terminal=False, duration=40.0, arrived_reward=None,
               exit_distance=25.0) -> RewardCfg:
    """IntersectionEnv._agent_reward config (intersection_env.py:78-104); arrived_reward None =
    high_speed_reward (the highway template, which has no exit lanes, normalises to it)."""
    c = RewardCfg()
    c.arrived_reward = float(high_speed_reward if arrived_reward is None else arrived_reward)
    c.exit_distance = float(exit_distance)
    c.collision_reward, c.high_speed_reward = float(collision_reward), float(high_speed_reward)
    c.speed_lo, c.speed_hi = float(reward_speed_range[0]), float(reward_speed_range[1])
    c.normalize_reward, c.offroad_terminal = int(normalize_reward), int(offroad_terminal)
    c.duration = float(duration)
    return c


def ttc_cfg(horizon: float = 10, policy_frequency: float = 1, raw: bool = False, **_ignored) -> TtcCfg:
    """TimeToCollisionObservation(horizon) (observation.py:114-151) at the env's policy frequency;
    ``raw``: the whole compute_ttc_grid (finite_mdp.py:104-167) instead of the 3x3 window."""
    c = TtcCfg()
    c.horizon_bins = int(horizon * policy_frequency)
    c.obs_lanes, c.obs_speeds = (0, 0) if raw else (3, 3)
    c.time_quantization = 1.0 / float(policy_frequency)
    if not 1 <= c.horizon_bins <= 64:
        raise ValueError("TTC horizon * policy_frequency must be in [1, 64]")
    return c


def lidar_cfg(cells: int = 16, maximum_range: float = 60.0, normalize: bool = True, **_ignored) -> LidarCfg:
    """LidarObservation(cells, maximum_range, normalize) (observation.py:681-698)."""
    c = LidarCfg()
    c.cells, c.maximum_range, c.normalize = int(cells), float(maximum_range), int(bool(normalize))
    if not 1 <= c.cells <= 64:
        raise ValueError("Lidar cells must be in [1, 64]")
    return c


def pcg64_states(seeds) -> np.ndarray:
    """Initial numpy PCG64 state per env, [E, 4] uint64 {state_hi, state_lo, inc_hi, inc_lo}.
    np.random.default_rng(seed) == Generator(PCG64(SeedSequence(seed)))."""
    out = np.zeros((len(seeds), 4), dtype=np.uint64)
    m = (1 << 64) - 1
    for i, s in enumerate(seeds):  # an int seed or a list of entropy ints (SeedSequence semantics)
        st = np.random.PCG64(np.random.SeedSequence([int(v) for v in s] if isinstance(s, (list, tuple, np.ndarray))
                                                    else int(s))).state["state"]
        out[i] = [(st["state"] >> 64) & m, st["state"] & m, (st["inc"] >> 64) & m, st["inc"] & m]
    return out


def rng_states(seeds) -> np.ndarray:
    """[E, RNG_WORDS] uint64 np_random states of ``np.random.default_rng(seed)`` per env
    (a seed may be an int or a list of entropy ints), has_uint32 clear."""
    out = np.zeros((len(seeds), RNG_WORDS), dtype=np.uint64)
    out[:, :4] = pcg64_states(seeds)
    return out


def rng_from_generator(g: np.random.Generator) -> np.ndarray:
    """The RNG_WORDS words of a live numpy Generator(PCG64) (test helper)."""
    st = g.bit_generator.state
    m = (1 << 64) - 1
    s, inc = st["state"]["state"], st["state"]["inc"]
    return np.array([(s >> 64) & m, s & m, (inc >> 64) & m, inc & m,
                     (int(st["has_uint32"]) << 32) | int(st["uinteger"])], dtype=np.uint64)


def state_struct(ptrs: dict, n_envs: int, n_veh: int, dtype: int) -> State:
    s = State()
    s.n_envs, s.n_veh, s.dtype = int(n_envs), int(n_veh), int(dtype)
    for f in ALL_FIELDS:
        setattr(s, f, ptrs.get(f))
    return s
