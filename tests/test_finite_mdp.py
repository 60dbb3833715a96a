"""AbstractEnv.to_finite_mdp batched (topotrafficrl_amd/finite_mdp.py) against the tables of
oracle/gen_golden_mdp.py on highway scenes (the reference's own compute_ttc_grid and
transition_model, plus the restated assembly of finite_mdp.py:51-90): the raw TTC grid from the
oracle and the HIP kernel, the shared transition table, rewards, terminal cells and the ego's
state index — all exact."""
import numpy as np
import pytest
import torch

from conftest import golden_files, load_golden
from oracle.oracle import HostState, Oracle
from topotrafficrl_amd import _abi
from topotrafficrl_amd.finite_mdp import _transition_np

IDS = lambda p: p.split("/")[-1][:-4]  # noqa: E731
FILES = golden_files("mdp_*")


def scene(d, p):
    g = {k: d[k] for k in d if k in ("x", "y", "heading", "speed", "target_speed", "timer", "delta", "steer", "acc",
                                    "impact_x", "impact_y", "lane", "target_lane", "crashed", "speed_index")}
    return HostState.from_golden(g, p)


@pytest.mark.parametrize("path", FILES, ids=IDS)
def test_transition_table_matches_reference(path):
    d = load_golden(path)
    V, L, T = d["grid"].shape[1:]
    for p in range(len(d["state"])):
        assert np.array_equal(_transition_np(V, L, T, 5), d["transition"][p])


@pytest.mark.parametrize("path", FILES, ids=IDS)
def test_oracle_raw_ttc_grid_matches_reference(path):
    d = load_golden(path)
    o = Oracle(_abi.lane_table_from_arrays(d["lane_table"]), _abi.default_params())
    cfg = _abi.ttc_cfg(10, 1, raw=True)
    for p in range(len(d["state"])):
        assert np.array_equal(o.observe_ttc(scene(d, p), cfg)[0], d["grid"][p])


@pytest.mark.gpu
@pytest.mark.parametrize("path", FILES, ids=IDS)
def test_batched_finite_mdp_matches_reference(path, hip_device):
    from test_gpu_parity import to_dev
    from topotrafficrl_amd.envs import VecHighwayEnv
    d = load_golden(path)
    n = d["x"].shape[1]
    c = dict(zip(("collision_reward", "right_lane_reward", "high_speed_reward", "lane_change_reward"), d["config"]))
    steps = len(d["state"])
    env = VecHighwayEnv({"num_envs": steps, "vehicles_count": n, "device": hip_device, **c})
    big = HostState(steps, n)
    for p in range(steps):
        h = scene(d, p)
        for k in big.a:
            big.a[k][p] = h.a[k][0]
    env.state.copy_(to_dev(big, hip_device))
    mdp = env.to_finite_mdp()
    assert np.array_equal(mdp.grid.cpu().numpy(), d["grid"])
    assert np.array_equal(mdp.transition.cpu().numpy(), d["transition"][0])
    assert np.array_equal(mdp.terminal.cpu().numpy(), d["terminal"])
    assert np.array_equal(mdp.state.cpu().numpy(), d["state"])
    assert np.max(np.abs(mdp.reward.cpu().numpy() - d["reward"])) <= 1e-12
    q = mdp.value_iteration(gamma=0.9, iterations=30)
    assert q.shape == mdp.reward.shape and bool(torch.isfinite(q).all())
