"""The C-ABI boundary on CPU: the HIP library loads, exports every entry point that
include/ttrl_mi355x.h declares, the ctypes mirror matches the C struct layouts, and
argument errors come back as TTRL_E_ARG before any device work.  No GPU needed."""
import ctypes as C
import os
import re
import subprocess

import pytest

from conftest import ROOT
from topotrafficrl_amd import _abi, _lib

HEADER = os.path.join(ROOT, "include", "ttrl_mi355x.h")


def declared():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"^(?:int|int64_t) (ttrl_\w+)\(", txt, re.M)))


def test_library_loads_and_exports_every_declared_symbol():
    lib = _lib.load()
    assert lib.ttrl_abi_version() == 8
    names = declared()
    assert len(names) >= 10
    for n in names:
        assert hasattr(lib, n), n
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r" T (ttrl_\w+)", out))
    assert set(names) <= exported
    assert set(_lib.EXPORTS) == set(names)


def test_ctypes_mirror_matches_c_layout(tmp_path):
    structs = {"ttrl_lane_table_t": _abi.LaneTable, "ttrl_params_t": _abi.Params, "ttrl_state_t": _abi.State,
               "ttrl_kin_cfg_t": _abi.KinCfg, "ttrl_grid_cfg_t": _abi.GridCfg, "ttrl_reset_cfg_t": _abi.ResetCfg,
               "ttrl_reward_cfg_t": _abi.RewardCfg, "ttrl_ttc_cfg_t": _abi.TtcCfg, "ttrl_lidar_cfg_t": _abi.LidarCfg,
               "ttrl_ix_cfg_t": _abi.IxCfg}
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "ttrl_mi355x.h"', "int main(void){"]
    for cname, py in structs.items():
        lines.append(f'printf("{cname} %zu\\n", sizeof({cname}));')
        for fname, _ in py._fields_:
            lines.append(f'printf("{cname}.{fname} %zu\\n", offsetof({cname}, {fname}));')
    lines.append("return 0;}")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    got = dict(line.rsplit(" ", 1) for line in subprocess.run([str(exe)], capture_output=True, text=True,
                                                                  check=True).stdout.split("\n") if line)
    for cname, py in structs.items():
        assert int(got[cname]) == C.sizeof(py), cname
        for fname, _ in py._fields_:
            assert int(got[f"{cname}.{fname}"]) == getattr(py, fname).offset, (cname, fname)


def test_argument_errors_need_no_device():
    lib = _lib.load()
    lanes = _abi.straight_lane_table(4)
    p = _abi.default_params()
    assert lib.ttrl_simulate(None, C.byref(lanes), C.byref(p), None, 15, 1 / 15, None) == -1
    s = _abi.State()  # null buffers
    s.n_envs, s.n_veh, s.dtype = 4, 64, _abi.F64
    assert lib.ttrl_road_act(C.byref(s), C.byref(lanes), C.byref(p), None) == -1
    s.dtype = 7
    assert lib.ttrl_road_step(C.byref(s), C.byref(lanes), C.byref(p), 0.1, None) == -1
    bad = _abi.straight_lane_table(4)
    bad.n_lanes = 99
    s.dtype = _abi.F64
    assert lib.ttrl_neighbours(C.byref(s), C.byref(bad), None, None, None, None) == -1
    # the intersection entry points need the network fields and np_random (state.rng)
    from topotrafficrl_amd.intersection import VecIntersectionEnv, intersection_network, ix_cfg
    net = intersection_network()
    cfg = ix_cfg(net, VecIntersectionEnv.default_config(), p)
    words = (C.c_uint32 * 4)(1, 2, 3, 4)
    assert lib.ttrl_ix_reset(C.byref(s), C.byref(net.table), C.byref(p), C.byref(cfg), words, 1, None, None) == -1
    assert lib.ttrl_ix_clear_spawn(C.byref(s), C.byref(net.table), C.byref(p), C.byref(cfg), None, None) == -1
    kin = _abi.kin_cfg(order="shuffled", shuffle_rng="np_random")
    assert lib.ttrl_observe_kinematics_masked(C.byref(s), C.byref(lanes), C.byref(p), C.byref(kin), None, None,
                                              None, None) == -1


def test_product_refuses_to_run_without_hip_library(tmp_path):
    with pytest.raises(ImportError):
        _lib.load(str(tmp_path / "missing.so"))


def test_product_refuses_cpu_tensors():
    import torch
    from topotrafficrl_amd.road import BatchedRoad, RoadNetwork
    from topotrafficrl_amd.state import BatchState
    st = BatchState(2, 8, device="cpu")
    road = BatchedRoad(RoadNetwork.straight_road_network(4), st)
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        road.act()
    with pytest.raises(RuntimeError):
        road.simulate(torch.zeros(2, dtype=torch.int32))


def test_device_seeding_matches_numpy_seedsequence():
    """ttrl_seed_pcg64 (the SeedSequence -> PCG64 seeding the reset kernel runs on the device)
    equals numpy's np.random.PCG64(SeedSequence(entropy)) state for single and multi-word entropy."""
    import numpy as np
    lib = _lib.load()
    rng = np.random.default_rng(0)
    cases = [[0], [1], [12345], [2 ** 32 - 1], [5, 0, 1], [7, 3, 2], list(rng.integers(0, 2 ** 32, 6))]
    cases += [list(rng.integers(0, 2 ** 32, k)) for k in (1, 2, 3, 4, 5, 9)]
    for ent in cases:
        w = np.asarray(ent, dtype=np.uint32)
        out = np.zeros(4, dtype=np.uint64)
        assert lib.ttrl_seed_pcg64(w.ctypes.data, len(w), out.ctypes.data) == 0
        assert np.array_equal(out, _abi.pcg64_states([[int(v) for v in ent]])[0]), ent
    assert lib.ttrl_seed_pcg64(None, 1, None) == -1


def test_view_budgets_fit_the_residency_they_are_sized_for():
    """LDS bytes per workgroup of the simulate kernel's views (ttrl_diag_view_bytes): the straight
    highway's float64 64-slot env fits 16 workgroups per CU (4 waves per SIMD, 160 KB LDS), the
    intersection's float64 road network (2 envs x 32 slots, 20 lanes; capped list rows and float32
    trajectory prefilters) fits 8 (2 waves per SIMD: a 4096-env batch in one round)."""
    lib = _lib.load()
    f = lib.ttrl_diag_view_bytes
    f.restype = C.c_long
    f.argtypes = [C.c_int32] * 6
    assert f(_abi.F64, 1, 64, 4, 0, 1) * 16 <= 160 * 1024
    assert f(_abi.F64, 2, 32, 20, 1, 0) * 8 <= 160 * 1024
    assert f(_abi.F32, 2, 32, 20, 1, 0) * 8 <= 160 * 1024
