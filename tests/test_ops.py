"""torch.ops.ttrl: the HIP entry points registered as PyTorch operators (topotrafficrl_amd/ops.py).
CPU: schemas (which arguments an op mutates) and Meta shapes.  GPU: each op equals the env
classes' direct binding bit for bit."""
import numpy as np
import pytest
import torch

from topotrafficrl_amd import _abi, ops
from topotrafficrl_amd.state import BatchState

LANES = ops.struct_tensor(_abi.straight_lane_table(4))
PARAMS = ops.struct_tensor(_abi.default_params())


def test_schemas_declare_mutation():
    s = torch.ops.ttrl.simulate_.default._schema
    assert s.arguments[0].alias_info is not None and s.arguments[0].alias_info.is_write
    assert torch.ops.ttrl.occupancy_grid.default._schema.arguments[0].alias_info is None
    # the np_random-shuffled observation advances state.rng: kinematics_obs mutates the state
    assert torch.ops.ttrl.kinematics_obs.default._schema.arguments[0].alias_info.is_write


def test_meta_shapes():
    st = BatchState(6, 64, device="meta")
    grid = _abi.grid_cfg(["presence", "vx"], [[-32, 32], [-32, 32]], [2, 2])
    g = torch.ops.ttrl.occupancy_grid(st.tensors(), LANES, PARAMS, ops.struct_tensor(grid))
    assert g.shape == (6, 2, 32, 32) and g.device.type == "meta"
    f, r = torch.ops.ttrl.neighbours(st.tensors(), LANES, None)
    assert f.shape == (6, 64) and f.dtype == torch.int32
    rew, te, tr = torch.ops.ttrl.rewards(st.tensors(), LANES, ops.struct_tensor(_abi.reward_cfg()),
                                         torch.zeros(6, dtype=torch.float64, device="meta"))
    assert rew.shape == (6,) and te.dtype == torch.bool


def test_struct_tensors_are_checked():
    with pytest.raises(ValueError):
        ops._as(torch.zeros(3, dtype=torch.uint8), _abi.LaneTable)


@pytest.mark.gpu
def test_ops_equal_the_direct_binding(hip_device):
    from topotrafficrl_amd.envs import VecHighwayEnv
    from topotrafficrl_amd.observation import kinematics
    env = VecHighwayEnv({"num_envs": 64, "vehicles_count": 40, "device": hip_device})
    env.reset(seed=3)
    a = torch.randint(0, 5, (64,), device=hip_device, generator=torch.Generator(device=hip_device).manual_seed(1))
    other = env.state.clone()
    codes = env.action_type._codes(a)
    env.road.simulate(codes, 15, 1 / 15)
    lanes, params = ops.struct_tensor(env.network.table), ops.struct_tensor(env.params)
    torch.ops.ttrl.simulate_(other.tensors(), lanes, params, codes, 15, 1 / 15)
    for k in env.state.t:
        assert torch.equal(env.state[k], other[k]), k
    kin = env.observation_type.cfg
    o1, i1 = kinematics(env.state, env.network, env.params, kin)
    o2, i2 = torch.ops.ttrl.kinematics_obs(other.tensors(), lanes, params, ops.struct_tensor(kin), None)
    assert torch.equal(o1, o2) and torch.equal(i1[:, :14], i2[:, :14])
    t = torch.full((64,), 3.0, dtype=torch.float64, device=hip_device)
    r2, te2, tr2 = torch.ops.ttrl.rewards(other.tensors(), lanes, ops.struct_tensor(env.reward_cfg), t)
    env.time.fill_(3.0)
    r1, te1, tr1 = env._rewards_and_dones()
    assert torch.equal(r1, r2) and torch.equal(te1, te2) and torch.equal(tr1, tr2)


@pytest.mark.gpu
def test_intersection_ops_equal_the_env(hip_device):
    from topotrafficrl_amd.intersection import VecIntersectionEnv, ix_clear_spawn, ix_reset
    env = VecIntersectionEnv({"num_envs": 32, "device": hip_device})
    other = BatchState(32, 32, device=hip_device)
    words = torch.arange(32, dtype=torch.int32, device=hip_device).view(-1, 1)
    ix_reset(env.state, env.network, env.params, env.ix, words)
    lanes, params, cfg = ops.struct_tensor(env.network.table), ops.struct_tensor(env.params), ops.struct_tensor(env.ix)
    torch.ops.ttrl.ix_reset_(other.tensors(), lanes, params, cfg, words, None)
    ix_clear_spawn(env.state, env.network, env.params, env.ix)
    torch.ops.ttrl.ix_clear_spawn_(other.tensors(), lanes, params, cfg, None)
    for k in env.state.t:
        assert torch.equal(env.state[k], other[k]), k
    assert np.all((other["kind"] > 0).sum(1).cpu().numpy() >= 2)
