"""Per-phase cycle breakdown of the fused simulate kernel (diagnostic build with
-DTTRL_PHASE_TIMING, see tools/variants.py 'timing'): mid-episode 4096x64 state; with --ix the
intersection's in-loop scenes (each launch times the frames of one real env.step on a copy of its state)."""
import ctypes as C
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from topotrafficrl_amd import _lib  # noqa: E402
from topotrafficrl_amd.envs import VecHighwayEnv  # noqa: E402

NAMES = ["meta", "act-setup", "scan", "mobil-bar+verdict", "abort", "steer/acc+bar", "kinematics", "project+bar",
         "candidates+bar", "sat+bar", "fold", "project-init", "idm-free(pow)", "mobil-queue+bar", "mobil-items",
         "hbm-load+stage", "store", "regulation-pairs", "regulation-predict", "follow_road"]


def main(dtype="f64", steps=30, frames=15, ix=False, E=4096):
    dev = torch.device("cuda:0")
    if ix:  # the intersection scenario (NET_GRAPH instance), 32 slots
        from topotrafficrl_amd.intersection import VecIntersectionEnv
        env = VecIntersectionEnv({"num_envs": 4096, "device": "cuda:0", "dtype": dtype})
    else:
        env = VecHighwayEnv({"num_envs": E, "vehicles_count": 64, "device": "cuda:0", "dtype": dtype})
    env.reset(seed=12345)
    n_act = env.action_space.n
    g = torch.Generator(device=dev).manual_seed(1000)
    lib = _lib.load(os.path.join(ROOT, "tools", "_ab", os.environ.get("TIMING_LIB", "lib_timing.so")))
    sim = lib.ttrl_simulate
    sim.argtypes = [C.c_void_p] * 4 + [C.c_int32, C.c_double, C.c_void_p]
    rd = lib.ttrl_diag_phase_read
    rd.argtypes = [C.c_void_p]
    stream = torch.cuda.current_stream(dev).cuda_stream
    buf = np.zeros(32, dtype=np.uint64)  # 20 phases, project_items' 5 steps, the regulation's 5 steps, 2 counts
    tot = np.zeros(32)
    work = env.state.clone() if ix else env.state
    for t in range(steps):
        a_idx = torch.randint(0, n_act, (E,), device=dev, generator=g)
        a = env.action_type._codes(a_idx)
        if ix:
            # the scenes of a real episode: the product's env.step (clears, spawns, resets) advances the
            # batch, and the timing build runs the same step's frames on a copy of its start state
            work.copy_(env.state)
            env.step(a_idx)
            torch.cuda.synchronize()
        rd(buf.ctypes.data)
        sim(C.byref(work.struct()), C.byref(env.network.table), C.byref(env.params), a.data_ptr(), frames, 1 / 15,
            stream)
        torch.cuda.synchronize()
        rd(buf.ctypes.data)
        if t >= 10:
            tot += buf.astype(np.float64)
    waves = (E if not ix else 2048) * (steps - 10)  # ix: two envs per 64-lane workgroup
    per, pp, rg = tot[:20] / waves, tot[20:25] / waves, tot[25:30] / waves
    print(f"[{dtype}] E={E} cycles per wave per {frames}-frame launch (mean over {steps - 10} launches), total {per.sum():.0f}")
    for n, c in zip(NAMES, per):
        print(f"  {n:16s} {c:10.0f}  {100 * c / per.sum():5.1f}%  ({c / frames:8.0f} per frame)")
    if pp.any():
        print("  project_items steps, cycles per wave per frame: " + ", ".join(
            f"{n} {c / frames:.0f}" for n, c in zip(["A boxes", "B projections", "C minimum", "D lists",
                                                    "counts"], pp)))
    if rg.any():
        print("  regulation steps, cycles per wave per frame: " + ", ".join(
            f"{n} {c / frames:.0f}" for n, c in zip(["P reach+pairs", "A items", "B exact", "C priorities",
                                                    "serial fallback"], rg)))
        print(f"  regulation fallbacks per wave per launch: more pairs than RQ_PAIRS {tot[30] / waves:.3f}, "
              f"more items than the queue {tot[31] / waves:.3f}")
    # the last launch, wave by wave: start / end spread and the per-SIMD finish (load balance)
    nw = E if not ix else 2048
    tr = np.zeros((nw, 3), dtype=np.uint64)
    lib.ttrl_diag_wave_read.argtypes = [C.c_void_p, C.c_int]
    lib.ttrl_diag_wave_read(tr.ctypes.data, nw)
    hw = tr[:, 2]
    xcc = (hw >> np.uint64(32)).astype(np.int64)
    t0, t1 = tr[:, 0].astype(np.int64), tr[:, 1].astype(np.int64)
    for x in np.unique(xcc):  # each XCD has its own shader clock: times relative to its first wave
        b = t0[xcc == x].min()
        t0[xcc == x] -= b
        t1[xcc == x] -= b
    base = 0
    dur = t1 - t0
    simd = (hw >> np.uint64(32)) * np.uint64(1 << 16) + ((hw & np.uint64(0xffff)) >> np.uint64(4))
    print(f"waves {nw}: duration mean {dur.mean():.0f} min {dur.min()} max {dur.max()} p90 {np.percentile(dur, 90):.0f}; "
          f"start spread {t0.max() - base}, last end {t1.max() - base}")
    keys, inv = np.unique(simd, return_inverse=True)
    lo = np.full(len(keys), np.iinfo(np.int64).max); hi = np.zeros(len(keys), dtype=np.int64)
    np.minimum.at(lo, inv, t0); np.maximum.at(hi, inv, t1)
    span = hi - lo
    cnt = np.bincount(inv)
    print(f"SIMDs used {len(keys)}, waves per SIMD {dict(zip(*np.unique(cnt, return_counts=True)))}; per-SIMD span "
          f"(last end - first start, one clock) mean {span.mean():.0f} p10 {np.percentile(span, 10):.0f} "
          f"p50 {np.percentile(span, 50):.0f} p90 {np.percentile(span, 90):.0f} max {span.max()}")
    st = t0 - lo[inv]
    print(f"wave start offset within its SIMD: mean {st.mean():.0f} max {st.max()}")
    if os.environ.get("TIMING_LIB", "lib_timing.so").endswith("lib_timing.so"):  # per-wave phase cycles
        wp = np.zeros((nw, 32), dtype=np.uint32)
        lib.ttrl_diag_wave_phases.argtypes = [C.c_void_p, C.c_int]
        lib.ttrl_diag_wave_phases(wp.ctypes.data, nw)
        tot = wp[:, :20].sum(1).astype(np.float64)
        slow = tot >= np.percentile(tot, 95)
        mid = (tot >= np.percentile(tot, 40)) & (tot <= np.percentile(tot, 60))
        print(f"the slowest 5% of waves (phase sum {tot[slow].mean():.0f}) vs the median ones ({tot[mid].mean():.0f}), "
              f"cycles per launch:")
        names = NAMES + [f"project {n}" for n in ["A", "B", "C", "D", "counts"]] + [
            f"regulation {n}" for n in ["P", "A", "B", "C", "serial"]] + ["#pairs>cap", "#items>cap"]
        for k in np.argsort(-(wp[slow].mean(0) - wp[mid].mean(0)))[:14]:
            print(f"  {names[k]:16s} slow {wp[slow, k].mean():9.0f}  median {wp[mid, k].mean():9.0f}")
        if wp[:, 29].any():
            print(f"waves taking the serial regulation fallback: {(wp[:, 29] > 2000).sum()} of {nw}")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "f64", frames=int(sys.argv[2]) if len(sys.argv) > 2 else 15,
         ix="--ix" in sys.argv, E=int(os.environ.get("ENVS", "4096")))
