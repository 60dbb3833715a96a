"""oracle/objsim.py -- the per-vehicle-object NumPy restatement behind bench.py's reference-equivalent
CPU baseline -- reproduces the reference's goldens (oracle/gen_golden.py) on
the straight highways and the dense crash scenes: every fused 15-frame policy step from the scene's
first frame, the meta-actions included, continuous fields within 1e-9 relative, discrete fields
exact.  So the CPU baseline times the reference's algorithm, not an approximation of it.  CPU only."""
import numpy as np
import pytest

from conftest import golden_files, load_golden
from oracle import objsim
from oracle.oracle import HostState
from topotrafficrl_amd import _abi

CONT = ["x", "y", "heading", "speed", "target_speed", "timer", "steer", "acc"]
DISC = ["lane", "target_lane", "crashed", "has_impact"]
STRAIGHT = golden_files("highway_*") + golden_files("dense_*")


@pytest.mark.parametrize("path", STRAIGHT, ids=lambda p: p.split("/")[-1][:-4])
def test_objsim_reproduces_the_goldens(path):
    d = load_golden(path)
    table = _abi.lane_table_from_arrays(d["lane_table"])
    p = _abi.default_params()
    road = objsim.road_from_state(HostState.from_golden(d, 0), 0, table, p)
    for step in range(int(d["meta"][2])):
        road.simulate(int(d["actions"][step]), 15, 1 / 15)
        got, want = objsim.state_of(road), HostState.from_golden(d, 15 * (step + 1))
        n = len(road.vehicles)
        for k in CONT:
            err = np.abs(got[k] - want[k][0, :n]) / (1 + np.abs(want[k][0, :n]))
            assert err.max() <= 1e-9, (step, k, err.max())
        for k in DISC:
            assert np.array_equal(got[k].astype(np.int64), want[k][0, :n].astype(np.int64)), (step, k)
        imp = want["has_impact"][0, :n].astype(bool)
        for k in ("impact_x", "impact_y"):
            assert np.max(np.abs(got[k][imp] - want[k][0, :n][imp]), initial=0.0) <= 1e-9, (step, k)


def test_objsim_throughput_reports_per_core():
    r = objsim.throughput(n=16, seconds=0.3)
    assert r["processes"] == 1 and r["value"] > 0 and r["veh_frames"] % (16 * 15) == 0


def test_objsim_pool_runs_one_process_per_core():
    """bench.py's reference_equiv: one spawn-context worker per core, each on its own scenes."""
    r = objsim.throughput(n=16, seconds=0.3, processes=2)
    assert r["processes"] == 2 and r["value"] > r["per_core"] > 0
