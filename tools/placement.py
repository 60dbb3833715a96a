"""Where the hardware puts a launch's waves (diagnostic; the -DTTRL_WAVE_TRACE build, tools/variants.py
'wtrace'): for the headline's simulate launch (4096 x 64, one env per wave) and the intersection's
(4096 envs, two per wave), every wave's start / end shader clock with its HW_ID and XCC_ID, saved raw
(gpurun_out/placement_*.npy) and summarised per CU and SIMD: how many waves each got, and the
durations of a SIMD's waves by their dispatch rank (the SIMD's arbiter issues the oldest first).

  python tools/placement.py [out_dir]
"""
import ctypes as C
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from topotrafficrl_amd import _lib  # noqa: E402
from topotrafficrl_amd.envs import VecHighwayEnv  # noqa: E402


def decode(tr):
    """HW_ID (gfx9 layout): wave 3:0, simd 5:4, pipe 7:6, cu 11:8, sh 12, se 15:13; XCC_ID 3:0."""
    hw = (tr[:, 2] & np.uint64(0xffffffff)).astype(np.int64)
    xcc = ((tr[:, 2] >> np.uint64(32)) & np.uint64(0xf)).astype(np.int64)
    return dict(t0=tr[:, 0].astype(np.int64), t1=tr[:, 1].astype(np.int64), xcc=xcc, se=(hw >> 13) & 7,
                sh=(hw >> 12) & 1, cu=(hw >> 8) & 15, simd=(hw >> 4) & 3)


def summary(tag, tr):
    """Per wave: duration (start / end read on one CU's clock: the clocks of different CUs are not
    aligned, so only same-CU differences mean anything).  Per SIMD: its waves by dispatch rank (the
    order of their block ids) and the SIMD's span (first start to last end)."""
    d = decode(tr)
    t0, t1 = d["t0"], d["t1"]
    dur = t1 - t0
    cu_key = ((d["xcc"] * 8 + d["se"]) * 2 + d["sh"]) * 16 + d["cu"]
    simd_key = cu_key * 4 + d["simd"]
    _, cu_cnt = np.unique(cu_key, return_counts=True)
    keys, inv, simd_cnt = np.unique(simd_key, return_inverse=True, return_counts=True)
    print(f"[{tag}] waves {len(t0)}: duration mean {dur.mean():.0f} p50 {np.median(dur):.0f} "
          f"p90 {np.percentile(dur, 90):.0f} max {dur.max()}")
    print(f"  CUs {len(cu_cnt)}: waves per CU {dict(zip(*[a.tolist() for a in np.unique(cu_cnt, return_counts=True)]))}; "
          f"SIMDs {len(simd_cnt)}: waves per SIMD {dict(zip(*[a.tolist() for a in np.unique(simd_cnt, return_counts=True)]))}")
    per = int(simd_cnt.max())
    ranks = np.full((len(keys), per), np.nan)
    span = np.zeros(len(keys))
    for s_ in range(len(keys)):
        bs = np.sort(np.nonzero(inv == s_)[0])  # block ids = dispatch order
        ranks[s_, :len(bs)] = dur[bs]
        span[s_] = t1[bs].max() - t0[bs].min()
    print(f"  mean duration by dispatch rank on its SIMD {np.nanmean(ranks, 0).astype(int).tolist()}; "
          f"SIMD span mean {span.mean():.0f} max {span.max():.0f}")


def main(out):
    os.makedirs(out, exist_ok=True)
    dev = torch.device("cuda:0")
    lib = _lib.load(os.path.join(ROOT, "tools", "_ab", "lib_wtrace.so"))
    sim = lib.ttrl_simulate
    sim.argtypes = [C.c_void_p] * 4 + [C.c_int32, C.c_double, C.c_void_p]
    lib.ttrl_diag_wave_read.argtypes = [C.c_void_p, C.c_int]
    stream = torch.cuda.current_stream(dev).cuda_stream
    for tag in ("highway", "ix"):
        if tag == "ix":
            from topotrafficrl_amd.intersection import VecIntersectionEnv
            env = VecIntersectionEnv({"num_envs": 4096, "device": "cuda:0", "dtype": "f64", "auto_reset": True})
            nw = 2048
        else:
            env = VecHighwayEnv({"num_envs": 4096, "vehicles_count": 64, "device": "cuda:0", "dtype": "f64"})
            nw = 4096
        env.reset(seed=12345)
        g = torch.Generator(device=dev).manual_seed(1000)
        for t in range(8):
            a_idx = torch.randint(0, env.action_space.n, (4096,), device=dev, generator=g)
            work = env.state.clone()
            env.step(a_idx)
            torch.cuda.synchronize()
            a = env.action_type._codes(a_idx)
            assert sim(C.byref(work.struct()), C.byref(env.network.table), C.byref(env.params), a.data_ptr(), 15,
                       1 / 15, stream) == 0
            torch.cuda.synchronize()
            tr = np.zeros((nw, 3), dtype=np.uint64)
            lib.ttrl_diag_wave_read(tr.ctypes.data, nw)
            np.save(os.path.join(out, f"placement_{tag}_{t}.npy"), tr)
            if t >= 6:
                summary(f"{tag} launch {t}", tr)
        sys.stdout.flush()


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "placement"))
