#!/usr/bin/env python3
"""Benchmark of the batched env.step() hot path (BASELINE.json north star).

A "step" is one batched env.step(): the fused 15-frame AbstractEnv._simulate
(meta-action + 15 x {Road.act, Road.step}) of every env on the GPU, then the
Kinematics observation and the rewards.  value = vehicle-steps/s over ALL ranks,
where one vehicle-step = one vehicle through one simulation frame.

Default workload (config 4, per GPU): 4096 envs x 64 vehicles, Kinematics 15x7
(env.json ranges, absolute=false, sorted), synthetic straight 4-lane highway,
random-seeded scenes and uniformly random ego actions (pre-drawn on the device).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--dtype f64|f32] [--config 1..6] [--auto-reset] [--strong]
  python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N

--gpus N > 1 without a torch.distributed.run environment: this process touches no GPU, starts
``python -m torch.distributed.run --nproc-per-node N ... bench.py`` as a CHILD process (one rank
per GPU), relays rank 0's JSON line and exits non-zero unless it reports n_gpus == N.
--strong: a fixed global batch (default 8 x the config's per-GPU envs: 32,768 at config 4) split
over the ranks by sharding.shard, instead of the default weak scaling (the config's envs per GPU).
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
KIN15 = {"type": "Kinematics", "vehicles_count": 15,
         "features": ["presence", "x", "y", "vx", "vy", "cos_h", "sin_h"],
         "features_range": {"x": [-100, 100], "y": [-100, 100], "vx": [-20, 20], "vy": [-20, 20]},
         "absolute": False, "order": "sorted"}
GRID7 = {"type": "OccupancyGrid", "features": ["presence", "x", "y", "vx", "vy", "cos_h", "sin_h"],
         "features_range": {"x": [-100, 100], "y": [-100, 100], "vx": [-20, 20], "vy": [-20, 20]},
         "grid_size": [[-32, 32], [-32, 32]], "grid_step": [2, 2], "absolute": False}
KIN5 = {"type": "Kinematics"}  # KinematicObservation defaults: 5 x 5, sorted, relative (observation.py:159-196)
CONFIGS = {
    # the reference's plumbing case (scripts/example.py scale): one env, 50 vehicles; the GPU line is
    # launch-latency bound by construction, the CPU line is the oracle on one core
    1: dict(num_envs=1, vehicles=50, obs=KIN5, name="1 env x 50 vehicles, Kinematics 5x5 defaults"),
    2: dict(num_envs=4096, vehicles=32, obs=KIN15, name="4096 envs x 32 vehicles, Kinematics 15x7"),
    3: dict(num_envs=4096, vehicles=128, obs=GRID7, name="4096 envs x 128 vehicles, OccupancyGrid 7x32x32"),
    4: dict(num_envs=4096, vehicles=64, obs=KIN15, name="4096 envs x 64 vehicles per GPU, Kinematics 15x7"),
    5: dict(num_envs=8192, vehicles=64, obs=KIN15, name="8192 envs x 64 vehicles, EgoAttention-2h policy in the loop"),
    # the reference's training scenario (scripts/configs/IntersectionEnv/env.json): spawns and
    # clears keep ~10-20 live vehicles in 32 slots; vehicle-steps count live vehicles only
    6: dict(num_envs=4096, vehicles=32, obs=dict(KIN15, absolute=True, order="shuffled"),
            name="4096 intersection-v0 envs (env.json: Kinematics 15x7 absolute, shuffled), 32 slots"),
}


def state_bytes(dtype: str) -> tuple[int, int]:
    """Algorithmic HBM bytes per vehicle for one fused launch: (read, written).
    read: 11 real fields + lane, target_lane, speed_index (i32) + kind, crashed, has_impact, lane_change (u8)
    written: 10 real fields (all but delta) + 3 x i32 + crashed, has_impact (u8)."""
    r = 8 if dtype == "f64" else 4
    return 11 * r + 3 * 4 + 4, 10 * r + 3 * 4 + 2


def launch_bytes(E: int, N: int, dtype: str, obs_cfg: dict | None, graph: bool, grid_cells: int = 0,
                 ix_tail: bool = False) -> int:
    """Algorithmic HBM bytes of one env.step launch (ttrl_env_step): every slot's state read and
    written once (state_bytes); on a road network also its route rows (road, lane: 4 + 4 int8),
    route length and yield flag, read and written; per env the step tail (time read + written,
    reward, terminated, truncated, the 4 reward terms, the info's ego speed / crashed), the action
    read, and on a road network the regulation counter and np_random's 5 words (the shuffled
    observation draws from it), read and written, and the dispatch order read; the Kinematics
    observation and its ids written once; an OccupancyGrid written by the launch (ttrl_env_step_grid):
    its ``grid_cells`` float32 cells per env written once.  ``ix_tail`` (ttrl_ix_env_step, round 6):
    also the next step's observation and ids (a second copy), the done flag, the two spare-mask
    bytes and the live count per env; the spare rows the finished envs swap in (~8 % of the envs
    per step at config 6) are data-dependent and not counted."""
    rd, wr = state_bytes(dtype)
    r = 8 if dtype == "f64" else 4
    per_slot = rd + wr + (2 * (4 + 4 + 1 + 1) if graph else 0)
    per_env = 2 * 8 + 4 + 1 + 1 + 4 * 4 + r + 1 + 4 + ((2 * 4 + 2 * 40 + 4) if graph else 0)
    if obs_cfg is not None and obs_cfg["type"] == "Kinematics":
        V = obs_cfg.get("vehicles_count", 5)
        F = len(obs_cfg.get("features", ["presence", "x", "y", "vx", "vy"]))
        per_env += (2 if ix_tail else 1) * (V * F * 4 + (V - 1) * 4)
    if ix_tail:
        per_env += 1 + 2 + 4
    per_env += 4 * grid_cells
    return E * (N * per_slot + per_env)


def host_threads() -> int:
    """The host cores the CPU baseline uses: the granted CPU share when the job is given one
    (OMP_NUM_THREADS: 16 on the GPU box, whose os.cpu_count() reports the whole machine), else
    every core os.cpu_count() reports."""
    return int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)


def cpu_baseline(vehicles: int, obs_cfg: dict, seconds_target: float = 10.0, envs: int = 4096,
                 threads: int | None = None) -> dict:
    """The float64 C restatement (oracle/) on host cores, bounded sample of the same workload."""
    threads = threads or host_threads()
    os.environ["OMP_NUM_THREADS"] = str(threads)
    from oracle.oracle import HostState, Oracle
    from topotrafficrl_amd import _abi
    lanes = _abi.straight_lane_table(4)
    o = Oracle(lanes, _abi.default_params())
    kin = _abi.kin_cfg(**{k: v for k, v in obs_cfg.items() if k != "type"}) if obs_cfg["type"] == "Kinematics" else None
    grid = _abi.grid_cfg(**{k: v for k, v in obs_cfg.items() if k != "type"}) if kin is None else None
    E = envs  # the same batch as the GPU workload
    h = HostState(E, vehicles)
    o.reset_highway(h, _abi.reset_cfg(vehicles, lanes), list(range(E)))
    rng = np.random.default_rng(0)
    steps, t0 = 0, time.perf_counter()
    while True:
        o.simulate(h, rng.integers(0, 5, size=E).astype(np.int32), 15, 1 / 15)
        if kin is not None:
            o.observe_kinematics(h, kin)
        else:
            o.observe_grid(h, grid)
        steps += 1
        el = time.perf_counter() - t0
        if el >= seconds_target or steps >= (200 if E > 1 else 20000):
            break
    return {"value": E * vehicles * 15 * steps / el, "unit": "vehicle-steps/s", "cores": threads, "kind": "port",
            "host_cpus": os.cpu_count(),
            "sample": f"{E} envs x {vehicles} vehicles x {steps} env.step (15 frames + obs), float64 C restatement "
                      f"of the reference loop order (oracle/ttrl_oracle.c), OpenMP over envs, {el:.1f} s"}


def reference_equiv(vehicles: int, seconds_target: float = 10.0, processes: int | None = None) -> dict:
    """the reference's own loop structure on the host cores -- oracle/objsim.py,
    the per-vehicle-object NumPy restatement (it reproduces the goldens, tests/test_objsim.py), one
    process per core as the reference's Pool design (evaluation.py:234-235), each on its own scenes
    of the synthetic highway for about ``seconds_target``.  Calibrated in the build container
    against the reference's Road.act / Road.step on the same scenes and one core
    (oracle/time_reference.py): ``reference_estimate`` = value / ratio is the reference itself."""
    from oracle import objsim
    processes = processes or host_threads()
    r = objsim.throughput(n=vehicles, seconds=seconds_target, processes=processes)
    ratio = objsim.REFERENCE_RATIO
    return {"value": r["value"], "unit": "vehicle-steps/s", "cores": processes, "kind": "reference-equivalent",
            "per_core": r["per_core"], "calibration_ratio": ratio,
            "reference_estimate": r["value"] / ratio if ratio else None,
            "calibration": "oracle/time_reference.py, profiles/r05/reference_equiv_calibration.txt",
            "sample": f"{processes} processes x 5 env.steps (15 frames) per {vehicles}-vehicle highway scene, "
                      f"Road.act + Road.step over per-vehicle numpy objects (oracle/objsim.py; the observation "
                      f"is not timed: ~2 % of the reference's step), {r['wall_s']:.1f} s wall"}


# live vehicle-steps/s of cpu_baseline_ix over the reference IntersectionEnv's own loop, one core each
# (oracle/time_reference_ix.py, 160 s in alternating rounds; profiles/r06/reference_ix_calibration.txt)
REFERENCE_RATIO_IX = 371.1


def cpu_baseline_ix(seconds_target: float = 10.0) -> dict:
    """The intersection episodes on the float64 C restatement (oracle/), OpenMP over envs: env.step
    = fused frames + shuffled Kinematics + rewards + clear/spawn, with resets (and their 45
    warm-up frames) where episodes end, as the GPU run does."""
    from oracle.oracle import HostState, Oracle
    from topotrafficrl_amd import _abi
    from topotrafficrl_amd.intersection import VecIntersectionEnv, intersection_network, ix_cfg
    threads = host_threads()
    os.environ["OMP_NUM_THREADS"] = str(threads)
    cfg = VecIntersectionEnv.default_config()
    net = intersection_network()
    P = _abi.default_params(target_speeds=[0, 4.5, 9], distance_wanted=7.0, comfort_acc_max=6.0, comfort_acc_min=-3.0)
    o = Oracle(net.table, P)
    ix = ix_cfg(net, cfg, P)
    kin = _abi.kin_cfg(**{k: v for k, v in CONFIGS[6]["obs"].items() if k != "type"}, shuffle_rng="np_random")
    rew = _abi.reward_cfg(-5, 1, [7.0, 9.0], False, False, 13, arrived_reward=1)
    E = 1024
    h = HostState(E, 32)
    o.ix_reset(h, ix, list(range(E)))
    o.observe_kinematics(h, kin)
    t = np.zeros(E)
    episode = np.zeros(E, dtype=np.int64)
    rng = np.random.default_rng(0)
    codes = np.array([_abi.SLOWER, _abi.IDLE, _abi.FASTER], dtype=np.int32)
    steps, live, t0 = 0, 0, time.perf_counter()
    while True:
        live += int((h["kind"] > 0).sum())
        t += 1
        o.simulate(h, codes[rng.integers(0, 3, size=E)], 15, 1 / 15)
        o.observe_kinematics(h, kin)
        _, term, trunc = o.rewards(h, rew, t)
        o.ix_clear_spawn(h, ix)
        done = term | trunc
        if done.any():
            episode += done
            m = done.astype(np.uint8)
            seeds = [[int(e), int(episode[e])] if done[e] else [int(e), 0] for e in range(E)]
            o.ix_reset(h, ix, seeds, mask=m)
            o.observe_kinematics(h, kin, mask=m)
            t[done] = 0
        steps += 1
        el = time.perf_counter() - t0
        if el >= seconds_target or steps >= 2000:
            break
    return {"value": live * 15 / el, "unit": "vehicle-steps/s (live vehicles)", "cores": threads, "kind": "port",
            "host_cpus": os.cpu_count(),
            "sample": f"{E} intersection envs x {steps} env.step (15 frames + shuffled Kinematics + rewards + "
                      f"clear/spawn + auto-resets), float64 C restatement (oracle/ttrl_oracle.c), OpenMP over "
                      f"envs, {el:.1f} s"}


def lib_sha16() -> str:
    import hashlib
    p = os.path.join(ROOT, "topotrafficrl_amd", "lib", "libttrl_mi355x.so")
    return hashlib.sha256(open(p, "rb").read()).hexdigest()[:16]


def read_pmc(dtype: str, cfg_id: int) -> tuple[dict | None, str]:
    """The committed PMC profile of this configuration's kernels (profiles/pmc_traffic.json), used
    only if it was measured on this very build of the kernel library (its sha256 prefix)."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(p):
        return None, "no profiles/pmc_traffic.json"
    try:
        d = json.load(open(p))
    except ValueError:
        return None, "unreadable profiles/pmc_traffic.json"
    e = d.get(f"config{cfg_id}_{dtype}")
    if e is None:
        return None, f"no PMC profile for config {cfg_id} {dtype}"
    if e.get("so_sha16") != lib_sha16():
        return None, f"PMC profile {e.get('profile', '?')} was measured on another build of libttrl_mi355x.so"
    return e, f"profiles/pmc_traffic.json ({e.get('profile', '?')}, libttrl_mi355x.so {e['so_sha16']})"


def launch_ranks(n: int, argv: list) -> int:
    """``bench.py --gpus n`` outside torch.distributed.run: run the ranks as a child
    ``torch.distributed.run`` job on 127.0.0.1 (a subprocess, never an exec: this process has not
    touched the GPU and does not), relay rank 0's JSON line with a ``launcher`` note, and return
    non-zero if the child fails or its line does not report n_gpus == n."""
    with socket.socket() as s_:
        s_.bind(("127.0.0.1", 0))
        port = s_.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__), *argv]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # RCCL on this host needs dmabuf IPC
    p = subprocess.run(cmd, stdout=subprocess.PIPE, text=True, env=env)
    lines = []
    for line in p.stdout.splitlines():
        if line.startswith("{"):
            lines.append(line)
        else:
            print(line, file=sys.stderr)
    if p.returncode != 0:
        print(f"bench.py: the {n}-rank child job failed (exit {p.returncode})", file=sys.stderr)
        return p.returncode
    if len(lines) != 1:
        print(f"bench.py: expected one JSON line from rank 0, got {len(lines)}", file=sys.stderr)
        return 1
    out = json.loads(lines[0])
    if out.get("ranks", out.get("n_gpus")) != n:
        print(f"bench.py: --gpus {n} but the job reports {out.get('ranks')} ranks", file=sys.stderr)
        return 3
    if out.get("n_gpus") != n and not out.get("shared_gpu"):
        print(f"bench.py: --gpus {n} but the ranks report n_gpus = {out.get('n_gpus')}", file=sys.stderr)
        return 3
    if out.get("shared_gpu"):  # a rehearsal of the N-rank logic, never an N-GPU measurement
        print(f"bench.py: {n} ranks shared one GPU (TTRL_BENCH_SHARED_GPU=1): n_gpus = 1, not a scaling point",
              file=sys.stderr)
    out["launcher"] = {"ranks": n, "cmd": "python -m torch.distributed.run --nnodes=1 --nproc-per-node "
                       f"{n} --master-addr 127.0.0.1 bench.py ...", "parent_imported_torch": "torch" in sys.modules}
    print(json.dumps(out), flush=True)
    return 0


def dry_run(args, rank: int, world: int) -> None:
    """The rank logic without a GPU (tests/test_bench.py): gloo process group, the shard of every
    rank, the max-over-ranks reduction; rank 0 prints the line's rank fields."""
    import torch.distributed as dist
    from topotrafficrl_amd import sharding
    if world > 1:
        dist.init_process_group("gloo")
    offset, count, g = shard_of(args, rank, world)
    shards = [(offset, count)]
    if world > 1:
        shards = [None] * world
        dist.all_gather_object(shards, (offset, count))
    elapsed = sharding.max_over_ranks(0.001 * (rank + 1))
    if rank == 0:
        print(json.dumps({"dry_run": True, "n_gpus": world, "ranks": world, "scaling": "strong" if args.strong else "weak",
                          "global_envs": g, "shards": shards, "max_elapsed": elapsed}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def shard_of(args, rank: int, world: int) -> tuple:
    """(global env offset, envs on this rank, global envs) for weak or strong scaling."""
    from topotrafficrl_amd import sharding
    E = CONFIGS[args.config]["num_envs"]
    if args.strong:
        g = args.global_envs or 8 * E
        off, cnt = sharding.shard(g, rank, world)
        return off, cnt, g
    off, cnt = sharding.weak_shard(E, rank)
    return off, cnt, world * E


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--strong", action="store_true",
                    help="strong scaling: --global-envs (default 8 x the config's envs) split over the ranks")
    ap.add_argument("--global-envs", type=int, default=None)
    ap.add_argument("--dry-run", action="store_true", help="the rank / shard logic only, no GPU (tests)")
    ap.add_argument("--steps", type=int, default=None, help="default 20 (config 6: 100)")
    ap.add_argument("--warmup", type=int, default=None, help="default 3 (config 6: 10)")
    ap.add_argument("--dtype", default="f64", choices=["f64", "f32"])
    ap.add_argument("--config", type=int, default=4, choices=[1, 2, 3, 4, 5, 6])
    ap.add_argument("--auto-reset", action="store_true",
                    help="highway envs restart on termination inside env.step (the RL rollout mode)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--graph", action="store_true",
                    help="replay each step as one captured HIP graph (policy + env.step for config 5)")
    args = ap.parse_args()
    # intersection steps are short (~2 ms) and their background resets settle over a few steps:
    # a longer timed window keeps the number stable from run to run
    if args.steps is None:
        args.steps = 100 if args.config in (1, 6) else 20
    if args.warmup is None:
        args.warmup = 10 if args.config == 6 else 3
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")

    from topotrafficrl_amd import sharding
    rank, local, world = sharding.world()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        sys.exit(2)
    if args.dry_run:
        dry_run(args, rank, world)
        return

    import torch
    import torch.distributed as dist
    from topotrafficrl_amd.envs import VecHighwayEnv

    # TTRL_BENCH_SHARED_GPU=1 (rehearsal on a one-GPU box): every rank on cuda:0, gloo for the
    # barrier and the max-over-ranks reduction; the real multi-GPU run uses one GPU per rank + RCCL
    shared = os.environ.get("TTRL_BENCH_SHARED_GPU") == "1"
    if shared:
        local = 0
    if world > 1:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        torch.cuda.set_device(local)
        if shared:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    C = CONFIGS[args.config]
    N = C["vehicles"]
    # weak scaling: the config's envs per GPU, global ids [rank*E, (rank+1)*E); strong: the rank's
    # contiguous block of the global batch (sharding.shard)
    offset, E, global_envs = shard_of(args, rank, world)
    ix = args.config == 6
    if ix:
        from topotrafficrl_amd.intersection import VecIntersectionEnv
        env = VecIntersectionEnv({"num_envs": E, "vehicle_slots": N, "observation": C["obs"], "device": str(dev),
                                  "dtype": args.dtype, "env_id_offset": offset, "auto_reset": True,
                                  # A/B only: TTRL_IX_FUSE_TAIL=0 runs the two-launch step (same results)
                                  "fuse_tail": os.environ.get("TTRL_IX_FUSE_TAIL", "1") != "0"})
    else:
        env = VecHighwayEnv({"num_envs": E, "vehicles_count": N, "observation": C["obs"], "device": str(dev),
                             "dtype": args.dtype, "env_id_offset": offset, "auto_reset": bool(args.auto_reset),
                             # A/B only: TTRL_FUSE_GRID=0 writes config 3's grid with its own kernel
                             "fuse_grid": os.environ.get("TTRL_FUSE_GRID", "1") != "0"})
    policy = None
    if args.config == 5:
        from topotrafficrl_amd.agent import EgoAttentionPolicy
        policy = EgoAttentionPolicy(device=dev, seed=0, env_id_offset=offset)  # draws keyed on global env ids
    obs, _ = env.reset(seed=12345)
    g = torch.Generator(device=dev)
    g.manual_seed(1000 + rank)
    n_act = env.action_space.n
    acts = torch.randint(0, n_act, (args.warmup + args.steps, E), device=dev, generator=g, dtype=torch.int32)
    # config 6 counts live vehicles, not slots: every step's tail launch (ttrl_ix_step_tail) adds the
    # vehicles present after it -- the next step's live vehicles -- to this counter, so the timed
    # steps' count is (live at the first timed step) + counter - (live after the last one)
    live = torch.zeros((), dtype=torch.int64, device=dev)
    if ix:
        env.live_counter = live

    sg = None
    if args.graph:
        from topotrafficrl_amd.graph import StepGraph
        sg = StepGraph(env, obs, policy)

    def one_step(t):
        nonlocal obs
        if sg is not None:
            if policy is None:
                sg.set_actions(acts[t])
            sg.replay()
            return
        a = policy.act(obs, t, dtype=torch.int32) if policy is not None else acts[t]
        obs, rew, term, trunc, info = env.step(a)

    kern_warm = []
    if sg is not None:  # graph replays cannot carry timing events: time the fused kernel on untimed launches
        road = env.road
        for _ in range(3):
            snap = env.state.clone()
            s_, e_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s_.record()
            road.simulate(env.action_type._codes(acts[0]), 15, 1 / 15)
            e_.record()
            torch.cuda.synchronize()
            kern_warm.append(s_.elapsed_time(e_))
            env.state.copy_(snap)
    for t in range(args.warmup):
        one_step(t)
    torch.cuda.synchronize()
    live0 = int((env.state["kind"] != 0).sum()) if ix else 0  # the first timed step's live vehicles
    live.zero_()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    # The launch time for the roofline: HIP events bracket the fused simulate launch
    # (BatchedRoad.simulate, or the one-launch env.step BatchedRoad.env_step / ix_env_step) on the
    # stream it is enqueued on, for every one of the N_EV steps that follow the timed ones (after
    # N_SETTLE bare steps: the sync that ends the timed region leaves the intersection's side streams
    # idle); a step's simulate time is the span from its first launch's start to its last one's end.
    # The events stay out of the timed loop: two markers around every launch cost ~8 us per step
    # there (tools/gap_ab.py, profiles/r06/r06l_event_markers.txt), and bracketing only every 4th
    # timed launch overstated the launch by 6 % against rocprofv3's trace of the same process
    # (profiles/r06/r06o_trace_agreement.txt: the marker before a bracketed launch behind a bare one
    # also times the dispatch behind it).
    N_EV, N_SETTLE = min(args.steps, 20), 3
    from topotrafficrl_amd.road import BatchedRoad
    orig_sim, orig_env_step, orig_ix_step = BatchedRoad.simulate, BatchedRoad.env_step, BatchedRoad.ix_env_step
    launches = []
    sample = [False]

    def timed(fn):
        def wrapper(self_road, *a, **kw):
            if not sample[0]:
                return fn(self_road, *a, **kw)
            st_ = torch.cuda.current_stream(dev)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record(st_)
            r = fn(self_road, *a, **kw)
            e.record(st_)
            launches[-1].append((s, e))
            return r
        return wrapper

    BatchedRoad.simulate, BatchedRoad.env_step = timed(orig_sim), timed(orig_env_step)
    BatchedRoad.ix_env_step = timed(orig_ix_step)
    # config 3: the OccupancyGrid launch (the path's HBM-bound kernel) timed the same way
    from topotrafficrl_amd.observation import BatchedOccupancyGridObservation
    orig_grid = BatchedOccupancyGridObservation.observe
    grid_launches = []

    def timed_grid(self_obs):
        if not sample[0]:
            return orig_grid(self_obs)
        st_ = torch.cuda.current_stream(dev)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record(st_)
        r = orig_grid(self_obs)
        e.record(st_)
        grid_launches.append((s, e))
        return r

    BatchedOccupancyGridObservation.observe = timed_grid
    t0 = time.perf_counter()
    for t in range(args.warmup, args.warmup + args.steps):
        one_step(t)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if ix:  # the counter holds the tails of the timed steps: the last one counts the step after them
        live_steps = live0 + int(live.item()) - int((env.state["kind"] != 0).sum())
    if sg is None:  # untimed: the launch-time steps (actions reused from the start of the table)
        for u in range(N_SETTLE + N_EV):
            sample[0] = u >= N_SETTLE
            if sample[0]:
                launches.append([])
            one_step(u % (args.warmup + args.steps))
        torch.cuda.synchronize()
        sample[0] = False
    BatchedRoad.simulate, BatchedRoad.env_step, BatchedRoad.ix_env_step = orig_sim, orig_env_step, orig_ix_step
    BatchedOccupancyGridObservation.observe = orig_grid

    def span(recs):
        s0 = recs[0][0]
        return max(s0.elapsed_time(e) for _, e in recs) - min(s0.elapsed_time(s) for s, _ in recs)

    kern_ms = float(np.mean(kern_warm)) if sg is not None else float(np.mean([span(r) for r in launches if r]))
    elapsed = sharding.max_over_ranks(elapsed, device=None if shared else dev)

    veh_steps = global_envs * N * 15 * args.steps
    if ix:  # live vehicles, not slots, summed over the ranks
        veh_steps = int(sharding.sum_over_ranks(float(live_steps), device=None if shared else dev)) * 15
    value = veh_steps / elapsed
    rd, wr = state_bytes(args.dtype)
    # per env.step launch: the state, the step tail and (Kinematics) the observation (launch_bytes)
    # config 3: the launch writes the OccupancyGrid too (ttrl_env_step_grid) unless the A/B switch
    # TTRL_FUSE_GRID=0 left it to the grid kernel (roofline_obs)
    fused_grid = C["obs"]["type"] == "OccupancyGrid" and not grid_launches
    cells = int(np.prod(env.observation_space.shape)) if fused_grid else 0
    alg_bytes = launch_bytes(E, N, args.dtype, C["obs"], graph=ix, grid_cells=cells,
                             ix_tail=ix and getattr(env, "_fuse", False))
    kernel = "simulate_kernel (fused 15-frame Road.act+Road.step + step tail)"
    if C["obs"]["type"] == "Kinematics":  # the launch also writes the observation (ttrl_env_step)
        kernel = "simulate_kernel (fused 15-frame Road.act+Road.step + Kinematics observation + step tail)"
    if fused_grid:
        kernel = "simulate_grid_kernel (fused 15-frame Road.act+Road.step + OccupancyGrid + step tail)"
    if ix and getattr(env, "_fuse", False):  # ttrl_ix_env_step: + _clear_vehicles / _spawn_vehicle, the swap
        kernel = ("simulate_ix_kernel (fused 15-frame Road.act+Road.step + Kinematics observation + step tail "
                  "+ _clear_vehicles / _spawn_vehicle + the finished envs' spare scenes)")
    achieved = alg_bytes / (kern_ms * 1e-3) / 1e9
    pmc, pmc_source = read_pmc(args.dtype, args.config)
    hbm = {"achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
           "traffic": (pmc or {}).get("hbm_bytes_per_launch"), "traffic_source": pmc_source}
    out = {
        "metric": "vehicle-steps/sec at 4096 envs×64 vehicles; 1/2/4/8 GPUs; HBM GB/s achieved",
        "value": value,
        "unit": "vehicle-steps/s",
        # the physical devices: a shared-GPU rehearsal (TTRL_BENCH_SHARED_GPU=1) runs every rank on
        # cuda:0, so it is one GPU however many ranks it has (``ranks``, ``shared_gpu``)
        "n_gpus": 1 if shared else world,
        "ranks": world,
        "shared_gpu": shared,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong" if args.strong else "weak",
        "vs_baseline": None,
        "dtype": args.dtype,
        "data": "synthetic",
        "config": {"workload": C["name"], "envs_per_gpu": E, "global_envs": global_envs, "vehicles_per_env": N,
                   "frames_per_step": 15,
                   "observation": C["obs"]["type"], "parallelism": f"env-sharded x{world}, no collective on the step",
                   "hip_graph": bool(args.graph), "auto_reset": bool(args.auto_reset or ix)},
        # the HBM roofline of the fused launch: algorithmic bytes (state read + written once, the
        # observation written once) over the launch time measured here with HIP events
        "roofline": dict(bound="hbm", **hbm, kernel=kernel, kernel_ms=kern_ms, alg_bytes_per_launch=alg_bytes,
                         alg_bytes_per_vehicle_step=alg_bytes / (E * N * 15.0)),
        "env_steps_per_s": global_envs * args.steps / elapsed,
    }
    if pmc and pmc.get("valu_active_cycles_per_wave") and pmc.get("sq_waves"):
        # The roofline that binds: the fused kernel is VALU-issue / latency bound,
        # not HBM bound.  From the PMC profile of this build of the kernel (hash-checked):
        # SQ_ACTIVE_INST_VALU (quad-cycles, x4) over the launch's waves against every SIMD's cycles in
        # the kernel time measured here (1024 SIMDs x the GRBM clock) -- the VALU-busy fraction.
        # The bound is the larger of the two fractions; the HBM view stays in roofline["hbm"].
        waves = pmc["sq_waves"]
        clk = pmc.get("effective_clock_ghz") or 2.4
        simd_cycles_per_s = 1024 * clk * 1e9
        active = pmc["valu_active_cycles_per_wave"] * waves
        busy = active / (simd_cycles_per_s * kern_ms * 1e-3)
        if busy > hbm["frac"]:
            out["roofline"] = dict(bound="valu", achieved=active / (kern_ms * 1e-3), peak=simd_cycles_per_s,
                                   unit="VALU-busy SIMD cycles/s", frac=busy, traffic=hbm["traffic"],
                                   kernel=kernel, kernel_ms=kern_ms, alg_bytes_per_launch=alg_bytes,
                                   alg_bytes_per_vehicle_step=alg_bytes / (E * N * 15.0), hbm=hbm,
                                   valu_insts_per_launch=pmc["valu_insts_per_wave"] * waves,
                                   counters=pmc_source + ": SQ_ACTIVE_INST_VALU, SQ_INSTS_VALU, SQ_WAVES, "
                                                         "GRBM_GUI_ACTIVE")
    if grid_launches and C["obs"]["type"] == "OccupancyGrid":
        # the grid kernel: algorithmic bytes = each vehicle's x, y, heading, speed, lane, kind read
        # once + the [E, F, W, H] float32 grid written once
        g_ms = float(np.mean([s_.elapsed_time(e_) for s_, e_ in grid_launches]))
        r_ = 8 if args.dtype == "f64" else 4
        cells = len(C["obs"]["features"]) * int(np.prod(env.observation_space.shape[1:]))
        g_bytes = E * (N * (4 * r_ + 4 + 1) + cells * 4)
        g_ach = g_bytes / (g_ms * 1e-3) / 1e9
        out["roofline_obs"] = {"bound": "hbm", "achieved": g_ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                               "frac": g_ach / HBM_PEAK_GBS, "traffic": (pmc or {}).get("grid_hbm_bytes_per_launch"),
                               "kernel": "grid_obs_kernel (OccupancyGridObservation.observe)", "kernel_ms": g_ms,
                               "alg_bytes_per_launch": g_bytes}
    if ix:
        out["config"]["live_vehicles_per_env"] = veh_steps / (global_envs * 15 * args.steps)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = (cpu_baseline_ix(args.cpu_seconds) if ix else
                               cpu_baseline(N, C["obs"] if C["obs"]["type"] == "Kinematics" else GRID7,
                                            args.cpu_seconds, envs=E, threads=1 if E == 1 else None))
        # beside the C port: the reference's own per-object loop structure (straight highways only;
        # the intersection's network lanes are not in oracle/objsim.py) ...
        out["cpu_baseline"]["reference_equiv"] = (
            None if ix else reference_equiv(N, args.cpu_seconds, processes=1 if E == 1 else None))
        if ix:  # ... and for the intersection, the port's speed over its calibrated ratio to the reference
            cb = out["cpu_baseline"]
            cb["reference_estimate"] = cb["value"] / REFERENCE_RATIO_IX
            cb["reference_calibration"] = {
                "ratio_port_to_reference": REFERENCE_RATIO_IX, "cores": cb["cores"],
                "source": "oracle/time_reference_ix.py, profiles/r06/reference_ix_calibration.txt: the unmodified "
                          "reference IntersectionEnv (reset + step, shuffled Kinematics) against cpu_baseline_ix, "
                          "one core each in the build container; the estimate assumes the reference's per-env "
                          "loop would scale over these cores as the port's OpenMP envs do (one process per core)"}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
