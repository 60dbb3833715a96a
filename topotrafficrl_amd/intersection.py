"""The intersection scenario (intersection-v0, the reference's training scenario) batched on the GPU.

Mirrors ttrl_env/envs/intersection_env.py:
  * ``intersection_network()``  <- IntersectionEnv._make_road :141-249 (20 lanes, 12 nodes,
                                   RegulatedRoad priorities), restated with the same numpy
                                   float64 expressions so the lane table is bit-identical
  * ``shortest_path()``         <- RoadNetwork.bfs_paths / shortest_path road.py:159-188
  * ``ix_cfg()``                <- the scene constants of _make_vehicles :251-318 and
                                   _spawn_vehicle :320-348
  * ``VecIntersectionEnv``      <- IntersectionEnv (default_config :17-55, step :135-139,
                                   _reset :131-133, rewards :60-119) over AbstractEnv
                                   (abstract.py:188-282), ``num_envs`` envs in lockstep.

Every env keeps its own ``np_random`` (numpy Generator(PCG64)) in HBM: the device kernels draw
spawns and the observation shuffle from it in the reference's order, so an env seeded ``s``
replays ``IntersectionEnv.reset(seed=s)`` and its steps (tests/test_ix_env.py).
"""
from __future__ import annotations

import copy

import numpy as np
import torch

from . import _abi, ops
from .action import action_factory
from .envs import _keep_tail, _reward_terms, rewards_and_dones
from .observation import BatchedKinematicObservation, observation_factory
from .road import BatchedRoad, RoadNetwork
from .state import BatchState

LANE_WIDTH = 4.0  # AbstractLane.DEFAULT_WIDTH lane.py:20


class _Graph:
    """RoadNetwork.graph insertion order: {from: {to: [lane rows]}} (road.py:21-48)."""

    def __init__(self):
        self.graph: dict = {}

    def add_lane(self, fr: str, to: str, row, priority: int):
        self.graph.setdefault(fr, {}).setdefault(to, []).append((list(row), int(priority)))


def intersection_network(regulation_frequency: int = 2, speed_limit: float = 10.0) -> RoadNetwork:
    """IntersectionEnv._make_road (intersection_env.py:141-249): the 4-way crossing, horizontal
    road with right of way; lanes_list() order, node ids in graph order."""
    lane_width = LANE_WIDTH
    right_turn_radius = lane_width + 5
    left_turn_radius = right_turn_radius + lane_width
    outer_distance = right_turn_radius + lane_width / 2
    access_length = 50 + 50
    g = _Graph()
    straight = lambda s, e: [_abi.LANE_STRAIGHT, s[0], s[1], e[0], e[1], lane_width, speed_limit,  # noqa: E731
                             0, 0, 0, 0, 0, 0, 0, 0, 0]
    circular = lambda c, r, a0, a1, cw: [_abi.LANE_CIRCULAR, 0, 0, 0, 0, lane_width, speed_limit,  # noqa: E731
                                         0, 0, 0, c[0], c[1], r, a0, a1, 1.0 if cw else 0.0]
    for corner in range(4):
        angle = np.radians(90 * corner)
        is_horizontal = corner % 2
        priority = 3 if is_horizontal else 1
        rotation = np.array([[np.cos(angle), -np.sin(angle)], [np.sin(angle), np.cos(angle)]])
        start = rotation @ np.array([lane_width / 2, access_length + outer_distance])
        end = rotation @ np.array([lane_width / 2, outer_distance])
        g.add_lane("o" + str(corner), "ir" + str(corner), straight(start, end), priority)
        r_center = rotation @ (np.array([outer_distance, outer_distance]))
        g.add_lane("ir" + str(corner), "il" + str((corner - 1) % 4),
                   circular(r_center, right_turn_radius, angle + np.radians(180), angle + np.radians(270), True),
                   priority)
        l_center = rotation @ (np.array([-left_turn_radius + lane_width / 2, left_turn_radius - lane_width / 2]))
        g.add_lane("ir" + str(corner), "il" + str((corner + 1) % 4),
                   circular(l_center, left_turn_radius, angle + np.radians(0), angle + np.radians(-90), False),
                   priority - 1)
        start = rotation @ np.array([lane_width / 2, outer_distance])
        end = rotation @ np.array([lane_width / 2, -outer_distance])
        g.add_lane("ir" + str(corner), "il" + str((corner + 2) % 4), straight(start, end), priority)
        start = rotation @ np.flip([lane_width / 2, access_length + outer_distance], axis=0)
        end = rotation @ np.flip([lane_width / 2, outer_distance], axis=0)
        g.add_lane("il" + str((corner - 1) % 4), "o" + str((corner - 1) % 4), straight(end, start), priority)
    return network_from_graph(g.graph, regulation_frequency)


def network_from_graph(graph: dict, regulation_frequency: int = 0) -> RoadNetwork:
    """Flatten a {from: {to: [(geometry row, priority)]}} graph into a lane table with topology."""
    nodes, roads, rows, net = [], [], [], []
    for fr, tos in graph.items():
        if fr not in nodes:
            nodes.append(fr)
        for to, lanes in tos.items():
            if to not in nodes:
                nodes.append(to)
            r = len(roads)
            roads.append((fr, to))
            for i, (row, prio) in enumerate(lanes):
                rows.append(row)
                net.append([r, nodes.index(fr), nodes.index(to), prio, int("il" in fr and "o" in to), i])
    if len(nodes) > _abi.MAX_NODES:
        raise ValueError(f"at most {_abi.MAX_NODES} nodes")
    table = _abi.set_network(_abi.lane_table_from_arrays(np.array(rows, dtype=np.float64)),
                             np.array(net), regulation_frequency=regulation_frequency)
    network = RoadNetwork(table)
    network.nodes, network.roads = nodes, roads
    network.graph = {fr: {to: [k for k, (f, t) in enumerate(roads) if (f, t) == (fr, to)] for to in tos}
                     for fr, tos in graph.items()}
    network.lane_rows = np.array(rows, dtype=np.float64)
    network.lane_net = np.array(net, dtype=np.int32)
    return network


def shortest_path(network: RoadNetwork, start: str, goal: str) -> list:
    """RoadNetwork.shortest_path = next(bfs_paths(start, goal), []) (road.py:159-188)."""
    graph = network.graph
    queue = [(start, [start])]
    while queue:
        node, path = queue.pop(0)
        if node not in graph:
            return []
        for nxt in sorted([k for k in graph[node].keys() if k not in path]):
            if nxt == goal:
                return path + [nxt]
            if nxt in graph:
                queue.append((nxt, path + [nxt]))
    return []


def ix_cfg(network: RoadNetwork, config: dict, params: _abi.Params) -> _abi.IxCfg:
    """Scene constants of IntersectionEnv._make_vehicles / _spawn_vehicle for the device."""
    c = _abi.IxCfg()
    n = int(config["initial_vehicle_count"])
    if not 1 <= n <= _abi.IX_MAX_INIT:
        raise ValueError(f"initial_vehicle_count must be in [1, {_abi.IX_MAX_INIT}]")
    c.initial_vehicle_count = n
    freq = int(config["simulation_frequency"])
    c.warmup_frames = 3 * freq                      # simulation_steps = 3 (intersection_env.py:264)
    c.warmup_dt = 1 / freq
    for t, v in enumerate(np.linspace(0, 80, n)):
        c.init_longitudinal[t] = float(v)
    c.spawn_probability = float(config["spawn_probability"])
    c.spawn_offset, c.spawn_speed, c.spawn_clear_distance = 5.0, 8.0, 15.0
    c.challenger_longitudinal, c.challenger_position_deviation, c.challenger_speed_deviation = 60.0, 0.1, 0.0
    c.delta_lo, c.delta_hi = 3.5, 4.5               # IDMVehicle.DELTA_RANGE behavior.py:39
    c.n_corners = 4
    nodes, roads = network.nodes, network.roads
    lane_of = {}
    for l in range(network.table.n_lanes):
        fr, to = roads[network.table.road[l]]
        lane_of[(fr, to, network.table.lane_id[l])] = l
    for k in range(4):
        c.entry_lane[k] = lane_of[(f"o{k}", f"ir{k}", 0)]
        c.exit_node[k] = nodes.index(f"o{k}")
    c.ego_lane = lane_of[("o0", "ir0", 0)]          # controlled_vehicles = 1: ego_id 0
    dest = config["destination"]
    c.ego_destination = -1 if not dest else int(str(dest)[1:])
    c.ego_longitudinal, c.ego_deviation, c.ego_heading_s = 60.0, 5.0, 60.0
    c.ego_speed = float(network.table.speed_limit[c.ego_lane])
    c.ego_clear_distance = 20.0
    c.leave_margin = 4 * params.length
    # routes the scene can plan: a spawn at corner r0 heads for another corner (choice without
    # replacement), the ego from its lane to the destination; a longer BFS path (a U-turn, 4
    # roads) would not fit ROUTE_MAX and is marked -1
    for i, node in enumerate(nodes):
        for k in range(4):
            path = shortest_path(network, node, f"o{k}")
            rds = [roads.index((path[q], path[q + 1])) for q in range(len(path) - 1)]
            fits = len(rds) <= _abi.ROUTE_MAX - 1
            c.path_len[i][k] = len(rds) if fits else -1
            for q in range(_abi.ROUTE_MAX - 1):
                c.path_road[i][k][q] = rds[q] if fits and q < len(rds) else -1
    ego_node = nodes.index(roads[network.table.road[c.ego_lane]][1])
    for k in ([c.ego_destination] if c.ego_destination >= 0 else [1, 2, 3]):
        if c.path_len[ego_node][k] < 0:
            raise ValueError(f"destination o{k}: the route exceeds ROUTE_MAX = {_abi.ROUTE_MAX}")
    return c


def _device_only(state: BatchState) -> None:
    if state.device.type != "cuda":
        raise RuntimeError("the intersection env runs on a HIP device only (no CPU fallback)")


def ix_reset(state: BatchState, network: RoadNetwork, params: _abi.Params, cfg: _abi.IxCfg,
             entropy: torch.Tensor, mask: torch.Tensor | None = None) -> None:
    """IntersectionEnv.reset on the device: env e replays ``default_rng(list(entropy[e]))``."""
    if entropy.dim() != 2 or entropy.shape[0] != state.n_envs or entropy.dtype != torch.int32:
        raise ValueError("entropy must be an int32 [n_envs, n_words] tensor of uint32 words")
    _device_only(state)
    ops.T.ix_reset_(state.tensors(), ops.st(network.table), ops.st(params), ops.st(cfg),
                    entropy.to(state.device), mask)


def ix_clear_spawn(state: BatchState, network: RoadNetwork, params: _abi.Params, cfg: _abi.IxCfg,
                   mask: torch.Tensor | None = None) -> None:
    """IntersectionEnv.step tail: _clear_vehicles then _spawn_vehicle, on the device."""
    _device_only(state)
    ops.T.ix_clear_spawn_(state.tensors(), ops.st(network.table), ops.st(params), ops.st(cfg), mask)


def copy_envs(dst: BatchState, src: BatchState, mask: torch.Tensor) -> None:
    """Copy the whole rows of the masked envs from ``src`` into ``dst`` (same shape and dtype)."""
    _device_only(dst)
    ops.T.copy_envs_(dst.tensors(), src.tensors(), mask)


def seed_words(seeds) -> np.ndarray:
    """SeedSequence entropy words of int seeds (numpy splits an int into uint32 words, low first)."""
    out = []
    for s in seeds:
        s = int(s)
        if s < 0:
            raise ValueError("seeds must be non-negative")
        w = []
        while True:
            w.append(s & 0xFFFFFFFF)
            s >>= 32
            if s == 0:
                break
        out.append(w)
    width = max(len(w) for w in out)
    if any(len(w) != width for w in out):
        raise ValueError("all seeds of a batch must have the same number of 32-bit words")
    return np.array(out, dtype=np.uint32)


class VecIntersectionEnv:
    """``num_envs`` intersection-v0 envs; the controlled vehicle of each env is its MDPVehicle."""

    metadata = {"render_modes": []}
    PERCEPTION_DISTANCE = 5.0 * 40.0  # abstract.py:41
    SHUFFLE_RNG = "np_random"         # order="shuffled" draws from each env's np_random
    ACTIONS = {0: "SLOWER", 1: "IDLE", 2: "FASTER"}

    def __init__(self, config: dict | None = None, render_mode: str | None = None) -> None:
        if render_mode is not None:
            raise NotImplementedError("rendering is out of scope (SURVEY.md §2)")
        self.config = self.default_config()
        self.configure(config)
        self.road = None
        self.observation_type = self.action_type = None
        self.time = None
        self.steps = 0
        self.done = False
        self._build()
        self.reset()

    @classmethod
    def default_config(cls) -> dict:
        """AbstractEnv.default_config (abstract.py:86-109) + IntersectionEnv.default_config
        (intersection_env.py:17-55) + batching keys."""
        return {
            "observation": {"type": "Kinematics", "vehicles_count": 15,
                            "features": ["presence", "x", "y", "vx", "vy", "cos_h", "sin_h"],
                            "features_range": {"x": [-100, 100], "y": [-100, 100], "vx": [-20, 20], "vy": [-20, 20]},
                            "absolute": True, "flatten": False, "observe_intentions": False},
            "action": {"type": "DiscreteMetaAction", "longitudinal": True, "lateral": False,
                       "target_speeds": [0, 4.5, 9]},
            "simulation_frequency": 15,
            "policy_frequency": 1,
            "other_vehicles_type": "ttrl_env.vehicle.behavior.IDMVehicle",
            "duration": 13,
            "destination": "o1",
            "controlled_vehicles": 1,
            "initial_vehicle_count": 10,
            "spawn_probability": 0.6,
            "collision_reward": -5,
            "high_speed_reward": 1,
            "arrived_reward": 1,
            "reward_speed_range": [7.0, 9.0],
            "normalize_reward": False,
            "offroad_terminal": False,
            "manual_control": False,
            # batching
            "num_envs": 1,
            "vehicle_slots": 32,       # padded row width; the scene holds ~10-20 vehicles
            "env_id_offset": 0,
            "device": "cuda",
            "dtype": "f64",
            "auto_reset": False,
            # auto-reset from scenes reset ahead of time on a side HIP stream (double buffer): a
            # finished env swaps in its next episode's scene, whose 45 warm-up frames ran
            # overlapped with earlier steps, and the following one is prepared in the background
            "overlap_resets": True,
            # the spare resets' 45 warm-up frames in chunks of this many frames, one chunk per step
            # (every step's chunks of the resets in flight in one launch on one side stream); 0: the
            # whole warm-up at once, on side streams in rotation
            "reset_chunk_frames": 15,
            "reset_streams": 2,  # side streams the whole-warm-up resets rotate over (chunks: one)
            # the envs that go on run _clear_vehicles / _spawn_vehicle inside the step launch
            # (ttrl_ix_env_step; Kinematics observations, <= 64 slots), the finished ones swap in
            # their spare scenes in ix_step_tail_ -- bit for bit the two-launch step
            "fuse_tail": True,
        }

    def configure(self, config: dict | None) -> None:
        if config:
            self.config.update(config)

    def _build(self):
        c = self.config
        if c["other_vehicles_type"] != "ttrl_env.vehicle.behavior.IDMVehicle":
            raise NotImplementedError("only IDMVehicle traffic is on the hot path (SURVEY.md §2)")
        if int(c["controlled_vehicles"]) != 1:
            raise NotImplementedError("MultiAgentIntersectionEnv (controlled_vehicles > 1) is out of scope")
        self.num_envs = int(c["num_envs"])
        self.device = torch.device(c["device"])
        self.network = intersection_network()
        # _make_vehicles mutates the IDM class constants (intersection_env.py:258-261)
        self.params = _abi.default_params(target_speeds=c["action"].get("target_speeds", [0, 4.5, 9]),
                                          distance_wanted=7.0, comfort_acc_max=6.0, comfort_acc_min=-3.0)
        self.state = BatchState(self.num_envs, int(c["vehicle_slots"]), device=self.device, dtype=c["dtype"])
        self.road = BatchedRoad(self.network, self.state, self.params)
        self.ix = ix_cfg(self.network, c, self.params)
        self.reward_cfg = _abi.reward_cfg(c["collision_reward"], c["high_speed_reward"], c["reward_speed_range"],
                                          c["normalize_reward"], c["offroad_terminal"], c["duration"],
                                          arrived_reward=c["arrived_reward"])
        self.time = torch.zeros(self.num_envs, dtype=torch.float64, device=self.device)
        self._reward = torch.zeros(self.num_envs, dtype=torch.float32, device=self.device)
        self._term = torch.zeros(self.num_envs, dtype=torch.uint8, device=self.device)
        self._trunc = torch.zeros(self.num_envs, dtype=torch.uint8, device=self.device)
        self._components = torch.zeros((self.num_envs, 4), dtype=torch.float32, device=self.device)
        self._entropy = None  # [E, words + 1]: seed words, then the auto-reset episode counter
        # overlap_resets: every env's next two episodes are prepared ahead of time on side streams,
        # in two spare scenes per env (rows [0, E) and [E, 2E) of self._spare).  An env finishing
        # takes its scene from slot _spare_par[e], which was prepared at least two steps earlier
        # (the slots alternate), so the step waits only for the side-stream work launched two steps
        # back (_spare_prev).  A step's spare resets (45 warm-up frames for a few hundred envs:
        # a latency chain of about one step) go to the two side streams in turn, so the chains of
        # consecutive steps overlap instead of queueing behind each other.
        #
        # reset_chunk_frames (default): a reset's warm-up instead runs 15 frames per step, so its
        # waves last ~a third as long and mostly finish inside the step launch they start behind
        # (a warm-up wave resident when a step launch starts holds one of the workgroup slots the
        # launch needs, pushing a workgroup into a second round).  A scene consumed at step t is
        # begun and warmed 15 frames after step t's tail, warmed 15 more after t+1's and t+2's
        # (side stream A: one call per step, begin + the chunk of every reset in flight), and
        # finished after t+3's tail on side stream B -- at the start of a step, so that B's
        # latency-bound finish has ended before the next tail instead of running beside it.  Each
        # env then owns C + 1 = 4 spare scenes (C chunks), so a slot is taken again 4 finishes
        # later; the tail waits for the previous step's finishes (_wait_ev).
        self._spare = None
        # optional int64 device scalar: each overlapped step's tail adds the vehicles present after
        # it (the next step's live vehicles) -- a live vehicle-step count with no launch of its own
        self.live_counter: torch.Tensor | None = None
        if c["auto_reset"] and c["overlap_resets"]:
            E = self.num_envs
            chunk, wf = int(c["reset_chunk_frames"]), int(self.ix.warmup_frames)
            # chunks must divide the warm-up, and the tail kernel rotates over at most 16 slots
            self._chunk = chunk if 0 < chunk < wf and wf % chunk == 0 and wf // chunk + 2 <= 16 else 0
            self._n_chunks = wf // self._chunk if self._chunk else 1
            # fuse_tail (ttrl_ix_env_step): the step launch itself takes the finished envs' spare
            # scenes, so a chunked reset must be finished one step earlier than the two-launch step
            # needs it (the launch waits for the finishes of two steps back, not the previous step's,
            # which run beside it): one more spare scene per env.  The whole-warm-up rotation already
            # waits for two steps back.
            self._fuse = (bool(c["fuse_tail"]) and c["observation"].get("type", "Kinematics") == "Kinematics"
                          and int(c["vehicle_slots"]) <= 64)
            self._slots = self._n_chunks + (2 if self._fuse else 1) if self._chunk else 2  # spare scenes per env
            self._cohorts = []  # the consumed-row masks of the resets still warming up, oldest first
            self._spare = BatchState(self._slots * E, int(c["vehicle_slots"]), device=self.device, dtype=c["dtype"])
            self._spare_par = torch.zeros(E, dtype=torch.uint8, device=self.device)
            # the step launch's dispatch order (ix_step_tail_ rewrites it after every step: workgroups
            # heaviest first, see ix_order_kernel) and its scratch; any permutation is valid
            self._order = torch.cat([torch.arange(E, dtype=torch.int32, device=self.device),
                                     torch.zeros(E, dtype=torch.int32, device=self.device)])
            n_sides = 2 if self._chunk else max(1, int(c["reset_streams"]))  # chunks: A (begin, warm), B (finish)
            self._sides = tuple(torch.cuda.Stream(self.device) for _ in range(n_sides))
            self._side_i = 0
            self._spare_ready = self._spare_prev = self._wait_ev = self._warm_ev = torch.cuda.Event()
            self._fin_evs = [self._wait_ev, self._wait_ev]  # chunked: side stream B after each of the last two steps
            self._to_finish = None  # chunked: the cohort whose last chunk ran in the previous step
            # [slots * E, words + 1]: each spare scene's seed words and episode counter (the last
            # word); ix_step_tail_ advances the counter of a consumed row by the number of slots
            self._spare_ent = None
        self.define_spaces()

    @property
    def GRAPH_AUTO_RESET(self) -> bool:
        """graph.StepGraph may capture the auto-reset when it runs on the step's own stream (a
        capture cannot leave the side stream's background reset pending across replays)."""
        return self._spare is None

    def define_spaces(self) -> None:
        """abstract.py:123-130"""
        self.observation_type = observation_factory(self, self.config["observation"])
        self.action_type = action_factory(self, self.config["action"])
        self.observation_space = self.observation_type.space()
        self.action_space = self.action_type.space()

    def _seeds(self, seed):
        if seed is None:
            seed = int(np.random.SeedSequence().generate_state(1)[0])
        if isinstance(seed, (list, tuple, np.ndarray, torch.Tensor)):
            s = [int(v) for v in (seed.tolist() if hasattr(seed, "tolist") else seed)]
            if len(s) != self.num_envs:
                raise ValueError("per-env seeds must have num_envs entries")
            return s
        base = int(seed) + int(self.config["env_id_offset"])
        return [base + e for e in range(self.num_envs)]

    def reset(self, *, seed=None, options: dict | None = None):
        """AbstractEnv.reset (abstract.py:188-214) + IntersectionEnv._reset: env e is
        ``IntersectionEnv.reset(seed=seed + env_id_offset + e)``."""
        if self._spare is not None:
            # the side streams may still be resetting the spares (they write _spare and read the
            # spare counters): join every one of them before either buffer is replaced or freed
            # below -- with two or more side streams, _spare_ready covers only the latest
            self._join_sides()
        if options and "config" in options:
            self.configure(options["config"])
            self._build()
        words = seed_words(self._seeds(seed))
        self._entropy = torch.from_numpy(np.concatenate([words, np.zeros((len(words), 1), np.uint32)], 1)
                                         .view(np.int32)).to(self.device)
        self.time.zero_()
        self.steps = 0
        self.done = False
        ix_reset(self.state, self.network, self.params, self.ix, self._entropy[:, :-1])
        if self._spare is not None:  # every env's next episodes (one per spare slot), in the background
            ent, K = self._entropy, self._slots
            self._spare_ent = torch.cat([ent[:, :-1].repeat(K, 1),
                                         torch.cat([ent[:, -1:] + 1 + q for q in range(K)])], 1).contiguous()
            self._spare_par.zero_()
            self._cohorts, self._to_finish = [], None
            self._pinned = []  # the side streams the current spare buffers are recorded on
            self._prepare_spares(None)
            self._spare_prev = self._wait_ev = self._warm_ev = self._spare_ready
            self._fin_evs = [self._spare_ready, self._spare_ready]
        obs = self.observation_type.observe()
        self._rewards_and_dones()  # abstract.py:211 reset's _info evaluates _rewards too
        return obs, self._info(obs, None)

    def _join_sides(self) -> None:
        """Order the main stream after all side-stream work enqueued so far (every spare reset in
        flight, on whichever side stream it runs)."""
        main = torch.cuda.current_stream(self.device)
        for side in self._sides:
            main.wait_stream(side)

    def _prepare_spares(self, mask: torch.Tensor | None) -> None:
        """Reset the spare scenes of ``mask`` ([slots * E]; all: None) on the next side stream,
        after the main stream's work so far (the swap that consumed them) -- whole, or chunked (the
        class comment in _build).  The side stream reads the seed words and episode counters of the
        masked rows only; the main stream writes a row's counter when it consumes that row again,
        after waiting for the side work that finished it (_spare_prev), so the rows in flight are
        never written under it.  The spare buffers are made on the main stream and used on the side
        ones: they are recorded there, so freeing them (a reset, a dropped env) waits for that work."""
        main = torch.cuda.current_stream(self.device)
        for side in self._sides:
            if side not in self._pinned:  # once per side stream and buffer set
                for t in self._spare.tensors() + [self._spare_ent]:
                    t.record_stream(side)
                self._pinned.append(side)
        args = (ops.st(self.network.table), ops.st(self.params), ops.st(self.ix))
        if mask is not None and self._chunk:
            A, B = self._sides
            if self._to_finish is not None:  # B: finish the resets whose last chunk ran in the previous step
                B.wait_stream(main)
                B.wait_event(self._warm_ev)
                fin = self._to_finish
                fin.record_stream(B)
                with torch.cuda.stream(B):
                    ops.T.ix_reset_parts_(self._spare.tensors(), *args, 4, None, None, None, 0, fin)
                    self._wait_ev = torch.cuda.Event()
                    self._wait_ev.record(B)
                self._to_finish = None
            ev = torch.cuda.Event()  # B's position after this step's finishes (if any)
            ev.record(B)
            self._fin_evs = [self._fin_evs[-1], ev]
            A.wait_stream(main)  # A: begin this step's resets, warm every reset in flight one chunk
            self._cohorts.append(mask)
            for m in self._cohorts:  # read on A (a fork's cohorts were cloned on the main stream)
                m.record_stream(A)
            with torch.cuda.stream(A):
                warm = self._cohorts[0]
                for m in self._cohorts[1:]:
                    warm = warm | m
                ops.T.ix_reset_parts_(self._spare.tensors(), *args, 3, self._spare_ent, mask, warm, self._chunk, None)
                self._warm_ev = torch.cuda.Event()
                self._warm_ev.record(A)
            if len(self._cohorts) == self._n_chunks:
                self._to_finish = self._cohorts.pop(0)
            self._spare_prev, self._spare_ready = self._spare_ready, self._warm_ev
            return
        side = self._sides[0] if self._chunk else self._sides[self._side_i]  # the whole reset at once
        self._side_i = (self._side_i + 1) % len(self._sides)
        side.wait_stream(main)
        with torch.cuda.stream(side):
            ix_reset(self._spare, self.network, self.params, self.ix, self._spare_ent, mask)
            ev = torch.cuda.Event()
            ev.record(side)
        if mask is not None:
            mask.record_stream(side)
        self._spare_prev, self._spare_ready = self._spare_ready, ev
        if not self._chunk:
            self._wait_ev = self._spare_prev  # the tail waits for the resets of two steps back

    def step(self, action):
        """IntersectionEnv.step (intersection_env.py:135-139) over AbstractEnv.step (abstract.py:224-250)."""
        if self.road is None:
            raise NotImplementedError("The road and vehicle must be initialized in the environment implementation")
        if self._spare is not None:
            return self._step_overlapped(action)
        self._simulate(action)
        obs = self.observation_type.observe()
        # time += 1 / policy_frequency (abstract.py:239) runs in the rewards launch
        reward, terminated, truncated = self._rewards_and_dones(1 / self.config["policy_frequency"])
        info = self._info(obs, action)
        ix_clear_spawn(self.state, self.network, self.params, self.ix)
        if self.config["auto_reset"]:
            done = terminated | truncated
            info["final_observation"], info["final_mask"] = obs, done
            obs = obs.clone()
            self._auto_reset(done, obs)
        return obs, reward, terminated, truncated, info

    def _step_overlapped(self, action):
        """The auto-reset step with overlapped resets.  fuse_tail (Kinematics, <= 64 slots): one launch,
        ttrl::ix_env_step_ (the fused frames, the observation of the final state, the step tail:
        time += 1 / policy_frequency, rewards, dones, info; clear / spawn for the envs that go on;
        the finished envs swap in their spare scenes and are observed), then the next dispatch order.
        Otherwise two launches: ttrl::env_step_, then ttrl::ix_step_tail_ (clear / spawn, the swap).
        Then the consumed spare rows are reset again on a side stream.  Bit for bit the in-place
        composition (simulate, observe, rewards, clear / spawn, reset, masked observe;
        test_overlapped_resets_equal_in_place_resets, test_fused_tail_equals_the_separate_tail)."""
        ot = self.observation_type
        kin = isinstance(ot, BatchedKinematicObservation)
        frames = int(self.config["simulation_frequency"] // self.config["policy_frequency"])
        idx, lut = None, None
        if action is not None and not self.config["manual_control"]:
            idx, lut = self.action_type._indices(action)  # the launch maps them to meta-action codes
        self.steps += frames
        # the tail launch re-observes a new scene with one slot per lane of a wavefront: wider rows
        # (vehicle_slots > 64) take the masked observation launch instead, which draws the same
        # shuffles from the same generators (test_overlapped_resets_equal_in_place_resets[96])
        fused_obs = kin and self.state.n_veh <= 64
        dt, tinc = 1 / self.config["simulation_frequency"], 1 / self.config["policy_frequency"]
        main = torch.cuda.current_stream(self.device)
        if self._fuse:
            # one launch: the frames, the observation, the step tail, clear / spawn for the envs that go
            # on, the spare scenes of the finished ones (ready: prepared two steps back at the latest)
            main.wait_event(self._fin_evs[0] if self._chunk else self._wait_ev)
            obs, ids, *outs, done, smask, obs2, ids2 = self.road.ix_env_step(
                self.ix, idx, frames, dt, ot.fused_cfg(), self.reward_cfg, self.time, tinc, self._spare,
                self._spare_par, self._entropy, self._spare_ent, self._order, lut, self.live_counter)
            reward, terminated, truncated = _keep_tail(self, outs)
            info = self._info(obs, action)
        else:
            obs, ids, *outs = self.road.env_step(idx, frames, dt, ot.fused_cfg() if kin else None, self.reward_cfg,
                                                 self.time, tinc, self._order, lut)
            reward, terminated, truncated = _keep_tail(self, outs)
            if not kin:
                obs = ot.observe()
            info = self._info(obs, action)
            _device_only(self.state)
            # the slots this step's tail takes were prepared two steps back at the latest (waited for
            # here, after the step launch is queued: the side work gets the launch's time as slack)
            main.wait_event(self._wait_ev)
            done, smask, obs2, ids2 = ops.T.ix_step_tail_(
                self.state.tensors(), ops.st(self.network.table), ops.st(self.params), ops.st(self.ix),
                self._spare.tensors(), terminated, truncated, self._spare_par, self._entropy, self._spare_ent,
                self.time, ops.kin_cfg_tensor(ot.fused_cfg()) if fused_obs else None, obs if fused_obs else None,
                ids if fused_obs else None, self.live_counter, self._order)
        self._prepare_spares(smask)
        info["final_observation"], info["final_mask"] = obs, done
        if fused_obs:
            ot.fused_result(obs2, ids2)
            obs = obs2
        elif kin:
            obs2, ids2 = obs.clone(), ids.clone()
            ot.fused_result(obs2, ids2)
            ot.observe(mask=done.view(torch.uint8), out=obs2)
            obs = obs2
        else:  # the other observers draw nothing: observe the new scenes, keep the others' rows
            new = ot.observe()
            obs = torch.where(done.view(-1, *([1] * (new.dim() - 1))), new, obs)
        return obs, reward, terminated, truncated, info

    def _simulate(self, action=None) -> None:
        frames = int(self.config["simulation_frequency"] // self.config["policy_frequency"])
        codes = None
        if action is not None and not self.config["manual_control"]:
            codes = self.action_type._codes(action)
        self.road.simulate(codes, frames, 1 / self.config["simulation_frequency"])
        self.steps += frames

    REWARD_TERMS = ["collision_reward", "high_speed_reward", "arrived_reward", "on_road_reward"]

    def _rewards_and_dones(self, time_inc: float = 0.0):
        """reward, terminated, truncated [E]; the per-objective terms (_agent_rewards,
        intersection_env.py:95-104) go to self._components [E, 4] for info["rewards"]."""
        return rewards_and_dones(self, time_inc)

    def _info(self, obs, action) -> dict:
        """IntersectionEnv._info (intersection_env.py:120-128) over abstract.py:169-186, batched: device
        tensors [E].  One controlled vehicle per env, so agents_rewards / agents_terminated are
        1-tuples: its _agent_reward and crashed-or-arrived."""
        c = self._components
        # _agent_is_terminal = crashed or arrived, which is _is_terminated itself unless
        # offroad_terminal adds the off-road term (intersection_env.py:106-116); the step's reward
        # and flag tensors are fresh per step, so sharing them costs no copy
        at = self._term if not self.config["offroad_terminal"] else (c[:, 0] != 0) | (c[:, 2] != 0)
        return {"speed": self._ego_speed, "crashed": self._ego_crashed, "action": action,
                "rewards": _reward_terms(self.REWARD_TERMS, c),
                "agents_rewards": (self._reward,), "agents_terminated": (at,)}

    def _auto_reset(self, done: torch.Tensor, obs: torch.Tensor) -> None:
        """In-place auto-reset (overlap_resets off): finished envs restart on the device with
        default_rng([seed words..., episode]) and their first observation is written into
        ``obs``; the others are untouched.  (With overlap_resets, _step_overlapped swaps in scenes
        reset ahead of time instead, bit-identical.)"""
        d = done.view(torch.uint8)  # bool storage is one byte per env: the uint8 mask, no launch
        self._entropy[:, -1] += d
        ix_reset(self.state, self.network, self.params, self.ix, self._entropy, d)
        self.time.masked_fill_(done, 0.0)
        if isinstance(self.observation_type, BatchedKinematicObservation):
            self.observation_type.observe(mask=d, out=obs)
        else:  # the other observers draw nothing: observe all, keep the others' rows
            new = self.observation_type.observe()
            obs.copy_(torch.where(done.view(-1, *([1] * (new.dim() - 1))), new, obs))

    @property
    def vehicle(self):
        """The controlled vehicles (abstract.py:76-79): each env's MDP slot, field -> [E]."""
        return {k: self.state.ego(k) for k in _abi.REAL_FIELDS + _abi.I32_FIELDS + _abi.U8_FIELDS}

    def get_available_actions(self):
        return self.action_type.get_available_actions()

    def close(self) -> None:
        self.done = True

    def render(self):
        raise NotImplementedError("rendering is out of scope (SURVEY.md §2)")

    def __deepcopy__(self, memo):
        new = copy.copy(self)
        new.state = self.state.clone()
        new.road = BatchedRoad(self.network, new.state, self.params)
        new.time = self.time.clone()
        if self._entropy is not None:
            new._entropy = self._entropy.clone()
        if self._spare is not None:  # its own spare scenes, side streams and events
            self._join_sides()  # every in-flight spare reset (not only the latest) lands before the clone
            new._spare = self._spare.clone()
            new._cohorts = [m.clone() for m in self._cohorts]
            new._to_finish = None if self._to_finish is None else self._to_finish.clone()
            new._pinned = []
            new._spare_ent = self._spare_ent.clone()
            new._spare_par = self._spare_par.clone()
            new._order = self._order.clone()
            new._sides = tuple(torch.cuda.Stream(self.device) for _ in self._sides)
            new._side_i = 0
            new._spare_ready = torch.cuda.Event()
            new._spare_ready.record(torch.cuda.current_stream(self.device))
            new._spare_prev = new._wait_ev = new._warm_ev = new._spare_ready
            new._fin_evs = [new._spare_ready, new._spare_ready]
        new.define_spaces()
        return new
