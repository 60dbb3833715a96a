"""The intersection scenario on the MI355X (simulate kernel, NET_GRAPH instance) against the
golden episodes of the reference (oracle/gen_golden_ix.py) and the float64 oracle.

Tolerances as tests/test_gpu_parity.py: one frame f64 <= 1e-9 * (1 + |x|), 15-frame fused
steps f64 <= 1e-6 * (1 + |x|); every discrete field exact, including routes (popped in place
by follow_road), RegulatedRoad yields and the regulation frame counter."""
import numpy as np
import pytest
import torch

from conftest import golden_files, load_golden
from oracle.oracle import HostState
from test_gpu_parity import to_dev
from test_ix_oracle import LONGI, P_IX, ix_lanes
from topotrafficrl_amd.road import BatchedRoad, RoadNetwork

pytestmark = pytest.mark.gpu

CONT = ["x", "y", "heading", "speed", "target_speed", "timer", "steer", "acc"]
DISC = ["lane", "target_lane", "crashed", "has_impact", "speed_index", "kind", "yielding", "route_n",
        "route_road", "route_lane"]
IDS = lambda p: p.split("/")[-1][:-4]  # noqa: E731


def compare(dev, g: HostState, tol: float, n: int):
    d = dev.to_numpy()
    for k in CONT:
        a, b = d[k][:, :n].astype(np.float64), g[k][:, :n]
        err = np.max(np.abs(a - b) / (1 + np.abs(b)))
        assert err <= tol, (k, err)
    imp = g["has_impact"][:, :n].astype(bool)
    for k in ("impact_x", "impact_y"):
        assert np.max(np.abs(d[k][:, :n][imp] - g[k][:, :n][imp]), initial=0.0) <= tol, k
    for k in DISC:
        assert np.array_equal(d[k][:, :n], g[k][:, :n]), (k, d[k][:, :n], g[k][:, :n])
    assert np.array_equal(d["reg_steps"], g["reg_steps"])


@pytest.mark.parametrize("pad", [32, 64])
@pytest.mark.parametrize("path", golden_files("ix_*"), ids=IDS)
def test_ix_frames_vs_golden(path, pad, hip_device):
    d = load_golden(path)
    road = None
    for p in range(int(d["meta"][1])):
        n = int((d["pre_kind"][p] > 0).sum())
        dev = to_dev(HostState.from_ix(d, "pre", p), hip_device, pad_to=pad)
        road = BatchedRoad(RoadNetwork(ix_lanes(d)), dev, P_IX)
        road.meta_action(torch.tensor([LONGI[int(d["actions"][p])]]))
        for f in range(15):
            if f > 0:
                dev.load_numpy(to_dev(HostState.from_ix(d, "frame", (p, f - 1)), hip_device, pad_to=pad).to_numpy())
            road.act()
            compare(dev, HostState.from_ix(d, "act", (p, f)), 1e-9, n)
            road.step(1 / 15)
            compare(dev, HostState.from_ix(d, "frame", (p, f)), 1e-9, n)


@pytest.mark.parametrize("path", golden_files("ix_*"), ids=IDS)
def test_ix_fused_steps_vs_golden(path, hip_device):
    d = load_golden(path)
    for p in range(int(d["meta"][1])):
        n = int((d["pre_kind"][p] > 0).sum())
        dev = to_dev(HostState.from_ix(d, "pre", p), hip_device, pad_to=32)
        road = BatchedRoad(RoadNetwork(ix_lanes(d)), dev, P_IX)
        road.simulate(torch.tensor([LONGI[int(d["actions"][p])]]), 15, 1 / 15)
        compare(dev, HostState.from_ix(d, "frame", (p, 14)), 1e-6, n)


def test_ix_batch_of_episodes(hip_device):
    """Every (episode, step) of the fixtures as one batch of envs: blocks hold envs whose
    regulation counters differ, so enforcement runs for some envs of a block and not others."""
    ds = [load_golden(pth) for pth in golden_files("ix_*")]
    cases = [(d, p) for d in ds for p in range(int(d["meta"][1]))]
    d0 = cases[0][0]
    hs = [HostState.from_ix(d, "pre", p, pad_to=32) for d, p in cases]
    E = len(hs)
    big = HostState(E, 32)
    for e, h in enumerate(hs):
        for k in big.a:
            big.a[k][e] = h.a[k][0]
    dev = to_dev(big, hip_device)
    road = BatchedRoad(RoadNetwork(ix_lanes(d0)), dev, P_IX)
    road.simulate(torch.tensor([LONGI[int(d["actions"][p])] for d, p in cases]), 15, 1 / 15)
    out = dev.to_numpy()
    for e, (d, p) in enumerate(cases):
        g = HostState.from_ix(d, "frame", (p, 14), pad_to=32)
        n = int((d["pre_kind"][p] > 0).sum())
        for k in DISC:
            assert np.array_equal(out[k][e, :n], g[k][0, :n]), (e, k)
        assert out["reg_steps"][e] == g["reg_steps"][0]
        assert np.max(np.abs(out["x"][e, :n] - g["x"][0, :n])) < 1e-5
