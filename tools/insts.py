"""Per-phase VALU work of the fused simulate kernel (diagnostic; run under rocprofv3 --pmc).

One-frame launches from the same mid-episode 4096 x 64 state, each with one phase ablated
(ttrl_diag_simulate's ablation bits); SQ_INSTS_VALU / SQ_ACTIVE_INST_VALU of a launch minus the
full launch's is that phase's share of the frame (within one frame the ablation barely changes the
work of the later phases: vehicles already changing lane keep changing, and so on).

  python3 tools/variants.py build    # here: tools/_ab/lib_ablate.so (-DTTRL_DIAG_ABLATE)
  rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_SALU --output-format csv \
      -d gpurun_out/insts -o insts -- python3 tools/insts.py
  python3 tools/insts.py --report gpurun_out/insts/insts_counter_collection.csv
"""
import csv
import ctypes as C
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
VARIANTS = {"full": 0, "no_coll": 1, "no_mobil": 2, "no_abort": 4, "no_scan": 8, "no_steer": 16,
            "no_kin": 32, "no_lane": 64, "no_idm": 128, "no_sat": 256, "no_pref": 512}
REPEAT = 3


def run(E=4096, N=64, frames=1):
    import torch
    from topotrafficrl_amd import _abi, _lib
    from topotrafficrl_amd.envs import reset_highway
    from topotrafficrl_amd.road import RoadNetwork
    from topotrafficrl_amd.state import BatchState
    # the ablation bits are compiled in only with -DTTRL_DIAG_ABLATE (tools/variants.py build)
    lib = _lib.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "_ab", "lib_ablate.so"))
    fn = lib.ttrl_diag_simulate
    fn.argtypes = [C.c_void_p] * 4 + [C.c_int32, C.c_double, C.c_int32, C.c_void_p]
    dev = torch.device("cuda:0")
    net = RoadNetwork.straight_road_network(4)
    P = _abi.default_params()
    base = BatchState(E, N, device=dev, dtype="f64")
    reset_highway(base, net, P, _abi.reset_cfg(N, net.table), list(range(E)))
    stream = torch.cuda.current_stream(dev).cuda_stream
    g = torch.Generator(device=dev).manual_seed(1)
    for _ in range(20):  # a mid-episode state
        a = torch.randint(0, 5, (E,), device=dev, dtype=torch.int32, generator=g)
        assert fn(C.byref(base.struct()), C.byref(net.table), C.byref(P), a.data_ptr(), 15, 1 / 15, 0, stream) == 0
    acts = torch.randint(0, 5, (E,), device=dev, dtype=torch.int32, generator=g)
    work = base.clone()
    for name, ab in VARIANTS.items():
        for _ in range(REPEAT):
            work.copy_(base)
            assert fn(C.byref(work.struct()), C.byref(net.table), C.byref(P), acts.data_ptr(), frames, 1 / 15, ab,
                      stream) == 0
    torch.cuda.synchronize()


def report(path):
    rows = [r for r in csv.DictReader(open(path)) if "simulate_kernel" in r["Kernel_Name"]]
    per = defaultdict(dict)
    for r in rows:
        per[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
    disp = [per[k] for k in sorted(per)][-len(VARIANTS) * REPEAT:]
    res = {}
    for n, name in enumerate(VARIANTS):
        ds = disp[n * REPEAT:(n + 1) * REPEAT]
        res[name] = {c: sum(d[c] for d in ds) / REPEAT / ds[0]["SQ_WAVES"] for c in ds[0] if c != "SQ_WAVES"}
    full = res["full"]
    print("per wave, one frame: " + ", ".join(f"{c} {v:.0f}" for c, v in full.items()))
    for name, r in res.items():
        print(f"  {name:10s} " + "  ".join(f"{c.replace('SQ_', '')} {full[c] - v:+8.0f}" for c, v in r.items()))


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--report":
        report(sys.argv[2])
    else:
        run()
