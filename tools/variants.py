"""Build (here) and time (on the GPU) compile-time variants of the fused kernel, interleaved in one process.

  python tools/variants.py build          # cross-compile variants into tools/_ab/
  python tools/variants.py run [f64 f32]  # on the GPU box
"""
import ctypes as C
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
OUT = os.path.join(ROOT, "tools", "_ab")  # scratch: git-ignored, travels to the box; remove after use
VARIANTS = {"head": [], "cur": []}  # committed kernel vs working tree, tuned defaults
# built, not timed: tools/phases.py (timing, wtrace); tools/ablate.py, insts.py, evolve.py (ablate: the
# phase-ablation bits of ttrl_diag_simulate exist only in -DTTRL_DIAG_ABLATE builds)
TIMING = {"timing": ["-DTTRL_PHASE_TIMING"], "wtrace": ["-DTTRL_WAVE_TRACE"], "ablate": ["-DTTRL_DIAG_ABLATE"]}
if os.environ.get("WAVE_VARIANTS"):
    VARIANTS.update({f"w{w}": [f"-DTTRL_SIM_WAVES={w}"] for w in (2, 3, 4, 5, 6)})
# variants built from an edited copy of the working-tree source (measured experiments that need no
# flag in the product source): name -> [(old, new)], each old text present exactly once
SOURCE_EDITS = {
    # 32-slot straight envs one per wave (32 lanes of 64 live, 4096 waves at config 2) on the sorted view
    "ns32x1": [("case 32: return launch_sim<T, 32, 2>", "case 32: return launch_sim<T, 32, 1>"),
               ("(NS * EPW == 64 || (NS == 128 && EPW == 1))", "(NS * EPW == 64 || NS == 32 || (NS == 128 && EPW == 1))")],
}
for name in os.environ.get("EDIT_VARIANTS", "").split(","):
    if name.strip():
        VARIANTS[name.strip()] = []
# variants built from an earlier commit's kernel source (its include/ and csrc/ as they were),
# e.g. REV_VARIANTS="r04=ec952d4;r05=5e3157c": the same fused launch (ttrl_simulate, unchanged since
# round 1) timed against that round's build in one process, on one box
REV = {}
for arg in os.environ.get("REV_VARIANTS", "").split(";"):
    if arg.strip():
        name, rev = arg.split("=", 1)
        REV[name.strip()] = rev.strip()
        VARIANTS[name.strip()] = []
for arg in os.environ.get("EXTRA_VARIANTS", "").split(";"):
    if arg.strip():
        name, flags = arg.split("=", 1)
        VARIANTS[name] = flags.split()


def build():
    os.makedirs(OUT, exist_ok=True)
    src = os.path.join(ROOT, "topotrafficrl_amd", "csrc", "ttrl_mi355x.hip")
    procs = []
    head = os.path.join(OUT, "head.hip")  # variants named head* build the committed kernel source
    with open(head, "w") as f:
        f.write(subprocess.run(["git", "-C", ROOT, "show", "HEAD:topotrafficrl_amd/csrc/ttrl_mi355x.hip"],
                               check=True, capture_output=True, text=True).stdout)
    for name in VARIANTS:
        if name in SOURCE_EDITS:
            text = open(src).read()
            for old, new in SOURCE_EDITS[name]:
                assert text.count(old) == 1, (name, old)
                text = text.replace(old, new)
            with open(os.path.join(OUT, f"{name}.hip"), "w") as f:
                f.write(text)
    for name, rev in REV.items():  # that commit's sources, extracted whole
        d = os.path.join(OUT, f"src_{name}")
        os.makedirs(d, exist_ok=True)
        tar = subprocess.run(["git", "-C", ROOT, "archive", rev, "include", "topotrafficrl_amd/csrc"], check=True,
                             capture_output=True).stdout
        subprocess.run(["tar", "-x", "-C", d], input=tar, check=True)
    only = os.environ.get("ONLY")  # build just these (comma-separated)
    for name, flags in {**VARIANTS, **TIMING}.items():
        if only and name not in only.split(","):
            continue
        base = os.path.join(OUT, f"src_{name}") if name in REV else ROOT
        cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-fPIC",
               "-shared", "-mllvm", "-disable-machine-licm", "-I", os.path.join(base, "include"), "-I",
               os.path.join(base, "topotrafficrl_amd", "csrc"), *flags, "-o", os.path.join(OUT, f"lib_{name}.so"),
               os.path.join(base, "topotrafficrl_amd", "csrc", "ttrl_mi355x.hip") if name in REV else
               head if name.startswith("head") else
               os.path.join(OUT, f"{name}.hip") if name in SOURCE_EDITS else src]
        procs.append(subprocess.Popen(cmd))
    for p in procs:
        assert p.wait() == 0


def run(dtypes, E=4096, N=64, rounds=7):
    import numpy as np
    import torch
    from topotrafficrl_amd import _abi, _lib
    from topotrafficrl_amd.envs import reset_highway
    from topotrafficrl_amd.road import RoadNetwork
    from topotrafficrl_amd.state import BatchState
    dev = torch.device("cuda:0")
    net = RoadNetwork.straight_road_network(4)
    P = _abi.default_params()
    libs = {}
    for name in VARIANTS:
        if not os.path.exists(os.path.join(OUT, f"lib_{name}.so")):
            print(f"  (variant {name} not built: skipped)")
            continue
        lib = _lib.load(os.path.join(OUT, f"lib_{name}.so"), check_abi=name not in REV)
        lib.ttrl_simulate.argtypes = [C.c_void_p] * 4 + [C.c_int32, C.c_double, C.c_void_p]
        libs[name] = lib
    ix = os.environ.get("IX") == "1"  # the intersection scenario (NET_GRAPH instance), 32 slots
    for dtype in dtypes:
        stream = torch.cuda.current_stream(dev).cuda_stream
        if ix:
            from topotrafficrl_amd.intersection import VecIntersectionEnv
            env = VecIntersectionEnv({"num_envs": E, "device": dev, "dtype": dtype})
            env.reset(seed=12345)
            g = torch.Generator(device=dev).manual_seed(1)
            for _ in range(int(os.environ.get("EVOLVE", "6"))):
                env.step(torch.randint(0, 3, (E,), device=dev, generator=g))
            base, net, P, N = env.state, env.network, env.params, env.state.n_veh
            acts = env.action_type._codes(torch.randint(0, 3, (E,), device=dev, generator=g))
        else:
            base = BatchState(E, N, device=dev, dtype=dtype)
            reset_highway(base, net, P, _abi.reset_cfg(N, net.table), list(range(E)))
            torch.cuda.synchronize()
            g = torch.Generator(device=dev).manual_seed(1)
            first = libs[next(iter(libs))]
            for _ in range(int(os.environ.get("EVOLVE", "20"))):  # time a mid-episode state, not the fresh one
                a = torch.randint(0, 5, (E,), device=dev, dtype=torch.int32, generator=g)
                assert first.ttrl_simulate(C.byref(base.struct()), C.byref(net.table), C.byref(P), a.data_ptr(), 15,
                                           1 / 15, stream) == 0
            acts = torch.randint(0, 5, (E,), device=dev, dtype=torch.int32,
                                 generator=torch.Generator(device=dev).manual_seed(0))
        torch.cuda.synchronize()
        ref = None
        work = base.clone()
        times = {k: [] for k in libs}
        for r in range(rounds):
            for name, lib in libs.items():
                work.copy_(base)
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                rc = lib.ttrl_simulate(C.byref(work.struct()), C.byref(net.table), C.byref(P), acts.data_ptr(), 15,
                                       1 / 15, stream)
                e.record()
                torch.cuda.synchronize()
                assert rc == 0
                times[name].append(s.elapsed_time(e))
                out = work["x"].cpu().numpy()
                if ref is None:
                    ref = out
                if not np.array_equal(out, ref):
                    print(f"  !! variant {name} differs from {next(iter(libs))}: max |dx| "
                          f"{np.nanmax(np.abs(out - ref)):.3e}, {int(np.sum(out != ref))} values")
        print(f"[{dtype}] E={E} N={N} fused 15-frame launch, median of {rounds - 1} rounds")
        for k, v in times.items():
            print(f"  {k:10s} {np.median(v[1:]):8.3f} ms  min {np.min(v[1:]):8.3f}")


if __name__ == "__main__":
    if sys.argv[1] == "build":
        build()
    else:
        run(sys.argv[2:] or ["f64", "f32"], E=int(os.environ.get("E", "4096")), N=int(os.environ.get("N", "64")))
