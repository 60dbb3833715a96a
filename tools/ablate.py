"""Phase ablation of the fused simulate kernel (diagnostic; interleaved rounds in one process)."""
import ctypes as C
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from topotrafficrl_amd import _abi, _lib  # noqa: E402
from topotrafficrl_amd.envs import reset_highway  # noqa: E402
from topotrafficrl_amd.road import RoadNetwork  # noqa: E402
from topotrafficrl_amd.state import BatchState  # noqa: E402

VARIANTS = {"full": 0, "no_coll": 1, "no_mobil": 2, "no_abort": 4, "no_scan": 8, "no_steer": 16,
            "no_kin": 32, "no_lane": 64, "no_idm": 128, "no_sat": 256, "no_pref": 512, "none": 255}


def main(E=4096, N=64, rounds=5):
    # the ablation bits are compiled in only with -DTTRL_DIAG_ABLATE (tools/variants.py build)
    lib = _lib.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "_ab", "lib_ablate.so"))
    fn = lib.ttrl_diag_simulate
    fn.argtypes = [C.c_void_p] * 4 + [C.c_int32, C.c_double, C.c_int32, C.c_void_p]
    fn.restype = C.c_int
    dev = torch.device("cuda:0")
    net = RoadNetwork.straight_road_network(4)
    P = _abi.default_params()
    for dtype in sys.argv[1:] or ["f64", "f32"]:
        base = BatchState(E, N, device=dev, dtype=dtype)
        reset_highway(base, net, P, _abi.reset_cfg(N, net.table), list(range(E)))
        work = base.clone()
        acts = torch.randint(0, 5, (E,), device=dev, dtype=torch.int32)
        stream = torch.cuda.current_stream(dev).cuda_stream
        times = {k: [] for k in VARIANTS}
        for r in range(rounds):
            for name, ab in VARIANTS.items():
                work.copy_(base)
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                rc = fn(C.byref(work.struct()), C.byref(net.table), C.byref(P), acts.data_ptr(), 15, 1 / 15, ab, stream)
                e.record()
                torch.cuda.synchronize()
                assert rc == 0
                times[name].append(s.elapsed_time(e))
        full = np.median(times["full"][1:])
        print(f"[{dtype}] E={E} N={N}")
        for k, v in times.items():
            m = np.median(v[1:])
            print(f"  {k:10s} {m:8.3f} ms  (saves {full - m:+.3f} ms, {100 * (full - m) / full:5.1f}%)")


if __name__ == "__main__":
    main()
