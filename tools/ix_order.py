"""Experiment (timing only): does the config-6 step launch get faster when its workgroups take the
envs in descending order of live vehicles (the heavy pairs dispatched first, the cheap ones last --
the ones a resident warm-up wave displaces into a second round)?

On in-loop config-6 scenes, the env_step launch (ttrl_env_step's dispatch order) alone and with
spare-scene resets resident on a side stream (as in the bench loop), in several orders; the results
must not depend on the order.  (Round 4 measured this with an experiment build first:
profiles/r04/r04m_ix_order*.txt; ix_order_kernel now writes "pairs_by_sum" every step.)

  python tools/ix_order.py [steps]
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(steps=30):
    from bench import CONFIGS
    from topotrafficrl_amd.intersection import VecIntersectionEnv, ix_reset
    C6 = CONFIGS[6]
    dev = torch.device("cuda:0")
    E, N = C6["num_envs"], C6["vehicles"]
    env = VecIntersectionEnv({"num_envs": E, "vehicle_slots": N, "observation": C6["obs"], "device": str(dev),
                              "dtype": os.environ.get("DT", "f64"), "auto_reset": True})
    env.reset(seed=12345)
    g = torch.Generator(device=dev).manual_seed(1000)
    for _ in range(steps):
        env.step(torch.randint(0, 3, (E,), device=dev, generator=g, dtype=torch.int32))
    env._join_sides()
    torch.cuda.synchronize()
    snap = env.state.clone()
    codes = env.action_type._codes(torch.randint(0, 3, (E,), device=dev, generator=g, dtype=torch.int32))
    live = (snap["kind"] != 0).sum(1)
    orders = {"natural": None,
              "sorted": torch.argsort(live, descending=True, stable=True).to(torch.int32)}
    # natural pairs (2j, 2j + 1), dispatched heaviest pair first (by the pair's max / sum of live)
    pm, ps = live.view(-1, 2).max(1).values, live.view(-1, 2).sum(1)
    base2 = torch.arange(E, device=dev).view(-1, 2)
    orders["pairs_by_sum"] = base2[torch.argsort(ps * 64 + pm, descending=True, stable=True)].flatten().to(torch.int32)
    # heavy with light (rank r with rank E-1-r), pairs dispatched by their max
    srt = torch.argsort(live, descending=True, stable=True)
    bal = torch.stack([srt[:E // 2], srt[E // 2:].flip(0)], 1)
    orders["balanced"] = bal[torch.argsort(live[bal].max(1).values, descending=True, stable=True)].flatten().to(
        torch.int32)
    orders["tail_kernel"] = env._order[:E].clone()  # what ix_step_tail_ wrote after the last step
    kc = env.observation_type.fused_cfg()
    t0 = env.time.clone()
    # E_SUB: the step launch over the first E_SUB envs only (fewer workgroups than the chip's slots)
    sub = int(os.environ.get("E_SUB", E))
    road, tm, cd = env.road, env.time, codes
    if sub < E:
        from topotrafficrl_amd.road import BatchedRoad
        road, tm, cd = BatchedRoad(env.network, env.state.rows(0, sub), env.params), env.time[:sub], codes[:sub]
        ls = live[:sub]
        orders = {"natural": None,
                  "sorted": torch.argsort(ls, descending=True, stable=True).to(torch.int32),
                  "pairs_by_sum": torch.arange(sub, device=dev).view(-1, 2)[torch.argsort(
                      ls.view(-1, 2).sum(1), descending=True, stable=True)].flatten().to(torch.int32)}
    main_s = torch.cuda.current_stream(dev)
    side = torch.cuda.Stream(dev)
    sp = env._spare
    rows = torch.zeros(2 * E, dtype=torch.uint8, device=dev)
    n_res = int(os.environ.get("RESETS", "330"))
    if os.environ.get("PAIRED") == "1":  # the resets packed two to a warm-up workgroup (rows 2j, 2j + 1)
        pairs = torch.randperm(E, generator=torch.Generator().manual_seed(3))[:n_res // 2]
        rows[torch.stack([2 * pairs, 2 * pairs + 1], 1).flatten().to(dev)] = 1
    else:
        rows[torch.randperm(2 * E, generator=torch.Generator().manual_seed(3))[:n_res].to(dev)] = 1
    print(f"resets on the side stream: {int(rows.sum())} rows in {int(rows.view(-1, 2).any(1).sum())} workgroups")
    occ_lib, n_occ = None, int(os.environ.get("OCCUPY", "0"))
    sink = torch.zeros(max(n_occ, 1), dtype=torch.int32, device=dev)
    if n_occ:
        import ctypes
        occ_lib = ctypes.CDLL(os.path.join(ROOT, "tools", "_ab", "occupy.so"))
        occ_lib.occupy.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_longlong, ctypes.c_void_p, ctypes.c_void_p]
        print(f"instead: {n_occ} idle one-wave workgroups on the side stream")

    def launch(order, busy):
        env.state.copy_(snap)
        env.time.copy_(t0)
        torch.cuda.synchronize()
        if busy and occ_lib is not None:  # OCCUPY idle one-wave workgroups (20 KB LDS) for 1.5 ms instead
            assert occ_lib.occupy(n_occ, 20080, 150000, sink.data_ptr(), side.cuda_stream) == 0
        elif busy:  # spare resets (ix_begin, 45 warm-up frames, ix_finish) resident when the step launches
            with torch.cuda.stream(side):
                ix_reset(sp, env.network, env.params, env.ix, env._spare_ent, rows)
            torch.cuda._sleep(int(os.environ.get("SLEEP", "400000")))
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record(main_s)
        road.env_step(cd, 15, 1 / 15, kc, env.reward_cfg, tm, 1.0, order)
        e.record(main_s)
        torch.cuda.synchronize()
        return s.elapsed_time(e), {k: env.state[k].clone() for k in env.state.t}

    lv = live.cpu().numpy()
    print(f"in-loop after {steps} steps: live per env mean {lv.mean():.2f} max {lv.max()}; pair max-sum natural "
          f"{np.maximum(lv[0::2], lv[1::2]).sum()} sorted {np.sort(lv)[::-1][0::2].sum()}", flush=True)
    # which order is the oracle's? (the envs whose results depend on the order, replayed on it)
    _, nat = launch(None, False)
    _, srt = launch(orders["sorted"], False)
    diff = torch.zeros(E, dtype=torch.bool, device=dev)
    for k in nat:
        a, b = nat[k], srt[k]
        diff |= (a != b).reshape(E, -1).any(1) if a.shape[0] == E else torch.zeros_like(diff)
    bad = torch.nonzero(diff).flatten().cpu().numpy()
    print(f"envs whose result depends on the order: {len(bad)} {bad[:16].tolist()}", flush=True)
    if len(bad) and os.environ.get("ORACLE", "1") == "1":
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        from oracle import HostState, Oracle
        pick = bad[:32]
        h = HostState(len(pick), N)
        sn = snap.to_numpy()
        for k in h.a:
            h.a[k][...] = sn[k][pick]
        Oracle(env.network.table, env.params).simulate(h, codes.cpu().numpy()[pick], 15, 1 / 15)
        for name, res in (("natural", nat), ("sorted", srt)):
            ok = [all(np.array_equal(res[k].cpu().numpy()[e], h.a[k][i], equal_nan=True) for k in h.a if k in res and k != "rng")
                  for i, e in enumerate(pick)]
            print(f"  {name}: {sum(ok)}/{len(pick)} of those envs equal the oracle", flush=True)
            for i, e in enumerate(pick[:3]):
                for k in h.a:
                    if k in res and k != "rng":
                        a = res[k].cpu().numpy()[e]
                        if not np.array_equal(a, h.a[k][i], equal_nan=True):
                            j = np.nonzero(np.atleast_1d(a != h.a[k][i]))[0]
                            print(f"    env {e} field {k}: slots {j.tolist()[:6]} device {np.atleast_1d(a)[j][:3]} "
                                  f"oracle {np.atleast_1d(h.a[k][i])[j][:3]}")
        for i, e in enumerate(pick[:4]):
            for k in ("x", "lane", "kind", "crashed"):
                a, b = nat[k].cpu().numpy()[e], srt[k].cpu().numpy()[e]
                if not np.array_equal(a, b):
                    j = np.nonzero(a != b)[0]
                    print(f"  env {e} {k} slots {j.tolist()[:8]} natural {a[j][:4]} sorted {b[j][:4]} "
                          f"oracle {h.a[k][i][j][:4]}")
    ref = None
    for busy in (False, True):
        for name, order in orders.items():
            ts = []
            for r in range(6):
                t, out = launch(order, busy)
                ts.append(t)
                if ref is None:
                    ref = out
                for k in out:
                    if not torch.equal(out[k], ref[k]):
                        print(f"  !! order {name} changes field {k}")
                        break
            print(f"{'with resets' if busy else 'alone':12s} {name:10s} median {np.median(ts[1:]):.3f} ms "
                  f"min {np.min(ts[1:]):.3f}", flush=True)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 30)
