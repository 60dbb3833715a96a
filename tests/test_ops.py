"""torch.ops.ttrl: the C ABI registered as PyTorch operators from C++ (csrc/ttrl_torch_ops.cpp).
CPU: every entry point is an operator, schemas declare what they mutate, Meta kernels give the
shapes, there is no CPU kernel.  GPU: every operator equals a direct ctypes call of its C ABI
entry point bit for bit."""
import ctypes as C

import numpy as np
import pytest
import torch

from topotrafficrl_amd import _abi, _lib, ops
from topotrafficrl_amd.state import BatchState

LANES = ops.struct_tensor(_abi.straight_lane_table(4))
PARAMS = ops.struct_tensor(_abi.default_params())
MUTATES = {"simulate_", "road_act_", "road_step_", "meta_action_", "env_step_", "kinematics_obs",
           "kinematics_obs_masked_", "reset_highway_", "reset_highway_seeded_", "auto_reset_highway_", "ix_reset_",
           "ix_reset_parts_", "ix_clear_spawn_", "ix_step_tail_", "ix_env_step_", "copy_envs_"}


def test_every_device_entry_point_is_an_operator():
    abi = {n for n in _lib.EXPORTS if n not in ("ttrl_abi_version", "ttrl_seed_pcg64", "ttrl_ego_attention_sizes")}
    covered = {"ttrl_" + {"simulate_": "simulate", "road_act_": "road_act", "road_step_": "road_step",
                          "meta_action_": "meta_action", "env_step_": "env_step", "neighbours": "neighbours",
                          "kinematics_obs": "observe_kinematics", "kinematics_obs_masked_": "observe_kinematics_masked",
                          "occupancy_grid": "observe_grid", "observe_ttc": "observe_ttc",
                          "observe_lidar": "observe_lidar", "reset_highway_": "reset_highway",
                          "reset_highway_seeded_": "reset_highway_seeded",
                          "auto_reset_highway_": "auto_reset_highway", "ix_reset_": "ix_reset",
                          "ix_reset_parts_": "ix_reset_parts",
                          "ix_clear_spawn_": "ix_clear_spawn", "ix_step_tail_": "ix_step_tail",
                          "ix_env_step_": "ix_env_step",
                          "copy_envs_": "copy_envs", "rewards": "rewards",
                          "rewards_ex": "rewards_ex", "rewards_step_": "rewards_step",
                          "ego_attention_q": "ego_attention_q", "ego_attention_act": "ego_attention_act"}[o]
               for o in ops.OPS}
    covered.add("ttrl_env_step_grid")  # env_step_ with a grid_cfg
    assert covered == abi
    for o in ops.OPS:
        assert hasattr(torch.ops.ttrl, o), o


@pytest.mark.parametrize("name", ops.OPS)
def test_schemas_declare_mutation(name):
    s = getattr(torch.ops.ttrl, name).default._schema
    first = s.arguments[0]
    writes = first.alias_info is not None and first.alias_info.is_write
    assert writes == (name in MUTATES), str(s)


def test_time_is_mutated_by_the_step_ops():
    for name in ("env_step_", "rewards_step_", "auto_reset_highway_", "ix_step_tail_", "ix_env_step_"):
        s = getattr(torch.ops.ttrl, name).default._schema
        t = [a for a in s.arguments if a.name == "time"][0]
        assert t.alias_info is not None and t.alias_info.is_write


def test_meta_shapes():
    st = BatchState(6, 64, device="meta")
    grid = _abi.grid_cfg(["presence", "vx"], [[-32, 32], [-32, 32]], [2, 2])
    g = torch.ops.ttrl.occupancy_grid(st.tensors(), LANES, PARAMS, ops.struct_tensor(grid))
    assert g.shape == (6, 2, 32, 32) and g.device.type == "meta"
    f, r = torch.ops.ttrl.neighbours(st.tensors(), LANES, None)
    assert f.shape == (6, 64) and f.dtype == torch.int32
    t = torch.zeros(6, dtype=torch.float64, device="meta")
    rew, te, tr = torch.ops.ttrl.rewards(st.tensors(), LANES, ops.struct_tensor(_abi.reward_cfg()), t)
    assert rew.shape == (6,) and te.dtype == torch.bool
    kin = _abi.kin_cfg(features=["presence", "x", "y", "vx", "vy", "cos_h", "sin_h"], vehicles_count=15)
    outs = torch.ops.ttrl.env_step_(st.tensors(), LANES, PARAMS, None, 15, 1 / 15, ops.struct_tensor(kin),
                                    ops.struct_tensor(_abi.reward_cfg()), t, 1.0)
    assert [tuple(o.shape) for o in outs] == [(6, 15, 7), (6, 14), (6,), (6,), (6,), (6, 4), (6,), (6,)]
    assert outs[6].dtype == torch.float64 and outs[3].dtype == torch.bool
    outs = torch.ops.ttrl.env_step_(st.tensors(), LANES, PARAMS, None, 15, 1 / 15, None,
                                    ops.struct_tensor(_abi.reward_cfg()), t, 1.0, grid_cfg=ops.struct_tensor(grid))
    assert [tuple(o.shape) for o in outs] == [(6, 2, 32, 32), (0,), (6,), (6,), (6,), (6, 4), (6,), (6,)]
    o, i = torch.ops.ttrl.kinematics_obs(st.tensors(), LANES, PARAMS, ops.struct_tensor(kin))
    assert o.shape == (6, 15, 7) and i.shape == (6, 14)
    ttc = torch.ops.ttrl.observe_ttc(st.tensors(), LANES, PARAMS, ops.struct_tensor(_abi.ttc_cfg()))
    assert ttc.shape == (6, 3, 3, 10)
    raw = torch.ops.ttrl.observe_ttc(st.tensors(), LANES, PARAMS, ops.struct_tensor(_abi.ttc_cfg(raw=True)))
    assert raw.shape == (6, 3, 4, 10)
    lid = torch.ops.ttrl.observe_lidar(st.tensors(), LANES, PARAMS, ops.struct_tensor(_abi.lidar_cfg()))
    assert lid.shape == (6, 16, 2)
    q = torch.ops.ttrl.ego_attention_q(torch.zeros(9, 15, 7, device="meta"), torch.zeros(10, device="meta"), 2, 5)
    assert q.shape == (9, 5)
    spare = BatchState(12, 64, device="meta")
    u8 = torch.zeros(6, dtype=torch.uint8, device="meta")
    done, smask, o2, i2 = torch.ops.ttrl.ix_step_tail_(
        st.tensors(), LANES, PARAMS, ops.struct_tensor(_abi.IxCfg()), spare.tensors(), u8.bool(), u8.bool(), u8,
        torch.zeros(6, 3, dtype=torch.int32, device="meta"), torch.zeros(12, 3, dtype=torch.int32, device="meta"), t,
        ops.struct_tensor(kin), o, i)
    assert done.shape == (6,) and done.dtype == torch.bool and smask.shape == (12,)
    assert o2.shape == (6, 15, 7) and i2.shape == (6, 14)


def test_cached_struct_bytes_follow_in_place_changes():
    """ops.st caches a struct's bytes, keyed on the bytes themselves: an in-place change of a field
    (scalar or array element) after the first use reaches the next call."""
    p = _abi.default_params()
    t0 = ops.st(p)
    assert ops.st(p) is t0  # unchanged: the cached tensor
    p.politeness = 0.25
    t1 = ops.st(p)
    assert t1 is not t0 and bytes(t1.numpy()) == bytes(p)
    lanes = _abi.straight_lane_table(4)
    ops.st(lanes)
    lanes.length[2] = 123.0
    assert bytes(ops.st(lanes).numpy()) == bytes(lanes)


def test_struct_tensors_are_checked():
    st = BatchState(2, 8, device="meta")
    with pytest.raises(RuntimeError, match="uint8 CPU tensor"):
        torch.ops.ttrl.neighbours(st.tensors(), torch.zeros(3, dtype=torch.uint8), None)
    with pytest.raises(RuntimeError, match="uint8 CPU tensor"):
        torch.ops.ttrl.occupancy_grid(st.tensors(), LANES, PARAMS, PARAMS)
    with pytest.raises(RuntimeError, match="24 tensors"):
        torch.ops.ttrl.neighbours(st.tensors()[:5], LANES, None)


def test_no_cpu_kernel():
    """The oracle is never dispatched to: on CPU tensors the ops have no kernel and raise."""
    st = BatchState(2, 8, device="cpu")
    with pytest.raises(NotImplementedError):
        torch.ops.ttrl.simulate_(st.tensors(), LANES, PARAMS, None, 1, 1 / 15)


# ---------------------------------------------------------------------------------------- GPU

def _stream():
    return torch.cuda.current_stream().cuda_stream


def _pair(hip_device, E=64, N=40, seed=3, dtype="f64"):
    from topotrafficrl_amd.envs import VecHighwayEnv
    env = VecHighwayEnv({"num_envs": E, "vehicles_count": N, "device": hip_device, "dtype": dtype})
    env.reset(seed=seed)
    rng = np.random.default_rng(seed)
    for _ in range(2):  # a state with lane changes and crashes in flight
        env.step(torch.from_numpy(rng.integers(0, 5, size=E)))
    return env, env.state.clone()


def _equal(a: BatchState, b: BatchState):
    for k in a.t:
        assert torch.equal(a[k], b[k]), k


def _c(st: BatchState):
    return C.byref(st.struct())


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["f64", "f32"])
def test_frame_ops_equal_the_c_abi(dtype, hip_device):
    env, other = _pair(hip_device, dtype=dtype)
    st = env.state
    lib = _lib.load()
    lanes, params = ops.st(env.network.table), ops.st(env.params)
    R, P = C.byref(env.network.table), C.byref(env.params)
    a = torch.randint(0, 5, (64,), device=hip_device, dtype=torch.int32,
                      generator=torch.Generator(device=hip_device).manual_seed(1))
    assert lib.ttrl_meta_action(_c(st), R, P, a.data_ptr(), _stream()) == 0
    torch.ops.ttrl.meta_action_(other.tensors(), lanes, params, a)
    assert lib.ttrl_road_act(_c(st), R, P, _stream()) == 0
    torch.ops.ttrl.road_act_(other.tensors(), lanes, params)
    assert lib.ttrl_road_step(_c(st), R, P, 1 / 15, _stream()) == 0
    torch.ops.ttrl.road_step_(other.tensors(), lanes, params, 1 / 15)
    assert lib.ttrl_simulate(_c(st), R, P, a.data_ptr(), 15, 1 / 15, _stream()) == 0
    torch.ops.ttrl.simulate_(other.tensors(), lanes, params, a, 15, 1 / 15)
    torch.cuda.synchronize()
    _equal(st, other)
    q = torch.randint(0, 4, (64, 40), device=hip_device, dtype=torch.int32)
    f1, r1 = torch.empty_like(q), torch.empty_like(q)
    assert lib.ttrl_neighbours(_c(st), R, q.data_ptr(), f1.data_ptr(), r1.data_ptr(), _stream()) == 0
    f2, r2 = torch.ops.ttrl.neighbours(other.tensors(), lanes, q)
    assert torch.equal(f1, f2) and torch.equal(r1, r2)


@pytest.mark.gpu
def test_env_step_and_rewards_ops_equal_the_c_abi(hip_device):
    env, other = _pair(hip_device)
    st = env.state
    lib = _lib.load()
    lanes, params, rc = ops.st(env.network.table), ops.st(env.params), ops.st(env.reward_cfg)
    R, P, RC = C.byref(env.network.table), C.byref(env.params), C.byref(env.reward_cfg)
    kin = env.observation_type.cfg
    E, V, F = 64, kin.vehicles_count, kin.n_features
    a = torch.randint(0, 5, (E,), device=hip_device, dtype=torch.int32)
    t1 = torch.full((E,), 2.0, dtype=torch.float64, device=hip_device)
    t2 = t1.clone()
    obs = torch.empty((E, V, F), device=hip_device)
    ids = torch.empty((E, V - 1), dtype=torch.int32, device=hip_device)
    rew, comp = torch.empty(E, device=hip_device), torch.empty((E, 4), device=hip_device)
    te, tr, cr = (torch.empty(E, dtype=torch.uint8, device=hip_device) for _ in range(3))
    sp = torch.empty(E, dtype=torch.float64, device=hip_device)
    assert lib.ttrl_env_step(_c(st), R, P, a.data_ptr(), 15, 1 / 15, C.byref(kin), obs.data_ptr(), ids.data_ptr(), RC,
                             t1.data_ptr(), 1.0, rew.data_ptr(), te.data_ptr(), tr.data_ptr(), comp.data_ptr(),
                             sp.data_ptr(), cr.data_ptr(), None, None, 0, _stream()) == 0
    outs = torch.ops.ttrl.env_step_(other.tensors(), lanes, params, a, 15, 1 / 15, ops.struct_tensor(kin), rc, t2, 1.0)
    torch.cuda.synchronize()
    _equal(st, other)
    assert torch.equal(t1, t2)
    for x, y in zip((obs, ids, rew, te, tr, comp, sp, cr), outs):
        assert torch.equal(x.view(torch.uint8) if x.dtype == torch.uint8 else x,
                           y.view(torch.uint8) if y.dtype == torch.bool else y)
    # the step tail alone, the reward variants
    o2 = torch.ops.ttrl.rewards_step_(other.tensors(), lanes, rc, t2, 1.0)
    assert lib.ttrl_rewards_step(_c(st), R, RC, t1.data_ptr(), 1.0, rew.data_ptr(), te.data_ptr(), tr.data_ptr(),
                                 comp.data_ptr(), sp.data_ptr(), cr.data_ptr(), _stream()) == 0
    torch.cuda.synchronize()
    assert torch.equal(t1, t2) and torch.equal(rew, o2[0]) and torch.equal(te, o2[1].view(torch.uint8))
    assert torch.equal(comp, o2[3]) and torch.equal(sp, o2[4]) and torch.equal(cr, o2[5].view(torch.uint8))
    r3, te3, tr3, c3 = torch.ops.ttrl.rewards_ex(other.tensors(), lanes, rc, t2)
    assert lib.ttrl_rewards_ex(_c(st), R, RC, t1.data_ptr(), rew.data_ptr(), te.data_ptr(), tr.data_ptr(),
                               comp.data_ptr(), _stream()) == 0
    r4, te4, tr4 = torch.ops.ttrl.rewards(other.tensors(), lanes, rc, t2)
    torch.cuda.synchronize()
    assert torch.equal(rew, r3) and torch.equal(comp, c3) and torch.equal(r3, r4) and torch.equal(te3, te4)


@pytest.mark.gpu
@pytest.mark.parametrize("N", [100, 40, 20])
def test_env_step_grid_op_equals_the_c_abi(N, hip_device):
    """ttrl::env_step_ with a grid_cfg against a direct ctypes call of ttrl_env_step_grid (100 and 40
    vehicles: the 128- and 64-slot fused launches; 20: the two-launch path of the 32-slot instance),
    and both against ttrl_env_step followed by ttrl_observe_grid."""
    env, other = _pair(hip_device, N=N)
    third = env.state.clone()
    st = env.state
    lib = _lib.load()
    lanes, params, rc = ops.st(env.network.table), ops.st(env.params), ops.st(env.reward_cfg)
    R, P, RC = C.byref(env.network.table), C.byref(env.params), C.byref(env.reward_cfg)
    grid = _abi.grid_cfg(["presence", "x", "y", "vx", "vy", "on_road", "cos_h"], [[-32, 32], [-32, 32]], [2, 2],
                         {"x": [-100, 100], "y": [-100, 100], "vx": [-20, 20], "vy": [-20, 20]})
    E = 64
    a = torch.randint(0, 5, (E,), device=hip_device, dtype=torch.int32,
                      generator=torch.Generator(device=hip_device).manual_seed(5))
    t1 = torch.full((E,), 2.0, dtype=torch.float64, device=hip_device)
    t2, t3 = t1.clone(), t1.clone()
    g1 = torch.empty((E, 7, 32, 32), device=hip_device)
    rew, comp = torch.empty(E, device=hip_device), torch.empty((E, 4), device=hip_device)
    te, tr, cr = (torch.empty(E, dtype=torch.uint8, device=hip_device) for _ in range(3))
    sp = torch.empty(E, dtype=torch.float64, device=hip_device)
    assert lib.ttrl_env_step_grid(_c(st), R, P, a.data_ptr(), 15, 1 / 15, C.byref(grid), g1.data_ptr(), RC,
                                  t1.data_ptr(), 1.0, rew.data_ptr(), te.data_ptr(), tr.data_ptr(), comp.data_ptr(),
                                  sp.data_ptr(), cr.data_ptr(), None, 0, _stream()) == 0
    outs = torch.ops.ttrl.env_step_(other.tensors(), lanes, params, a, 15, 1 / 15, None, rc, t2, 1.0,
                                    grid_cfg=ops.struct_tensor(grid))
    sep = torch.ops.ttrl.env_step_(third.tensors(), lanes, params, a, 15, 1 / 15, None, rc, t3, 1.0)
    g3 = torch.ops.ttrl.occupancy_grid(third.tensors(), lanes, params, ops.struct_tensor(grid))
    torch.cuda.synchronize()
    _equal(st, other)
    _equal(st, third)
    assert torch.equal(t1, t2) and torch.equal(t1, t3)
    assert torch.equal(g1, outs[0]) and torch.equal(g1, g3)
    assert float(g1[:, 5].sum()) > 0  # the on_road layer is drawn
    for x, y, z in zip((rew, te, tr, comp, sp, cr), outs[2:], sep[2:]):
        y = y.view(torch.uint8) if y.dtype == torch.bool else y
        z = z.view(torch.uint8) if z.dtype == torch.bool else z
        assert torch.equal(x, y) and torch.equal(x, z)


@pytest.mark.gpu
def test_observation_ops_equal_the_c_abi(hip_device):
    env, other = _pair(hip_device, N=64)
    st = env.state
    lib = _lib.load()
    lanes, params = ops.st(env.network.table), ops.st(env.params)
    R, P = C.byref(env.network.table), C.byref(env.params)
    kin = _abi.kin_cfg(features=["presence", "x", "y", "vx", "vy", "cos_h", "sin_h"], vehicles_count=15)
    o1 = torch.empty((64, 15, 7), device=hip_device)
    i1 = torch.empty((64, 14), dtype=torch.int32, device=hip_device)
    assert lib.ttrl_observe_kinematics(_c(st), R, P, C.byref(kin), o1.data_ptr(), i1.data_ptr(), _stream()) == 0
    o2, i2 = torch.ops.ttrl.kinematics_obs(other.tensors(), lanes, params, ops.struct_tensor(kin))
    torch.cuda.synchronize()
    assert torch.equal(o1, o2) and torch.equal(i1, i2)
    mask = (torch.arange(64, device=hip_device) % 3 == 0).to(torch.uint8)
    o3, i3 = torch.zeros_like(o1), torch.full_like(i1, -7)
    torch.ops.ttrl.kinematics_obs_masked_(other.tensors(), lanes, params, ops.struct_tensor(kin), mask, o3, i3)
    m = mask.bool()
    assert torch.equal(o3[m], o1[m]) and torch.equal(i3[m], i1[m]) and bool((o3[~m] == 0).all())
    grid = _abi.grid_cfg(["presence", "x", "y", "vx", "vy", "cos_h", "sin_h"], [[-32, 32], [-32, 32]], [2, 2])
    g1 = torch.empty((64, 7, 32, 32), device=hip_device)
    assert lib.ttrl_observe_grid(_c(st), R, P, C.byref(grid), g1.data_ptr(), _stream()) == 0
    g2 = torch.ops.ttrl.occupancy_grid(other.tensors(), lanes, params, ops.struct_tensor(grid))
    tc, lc = _abi.ttc_cfg(), _abi.lidar_cfg()
    t1 = torch.empty((64, 3, 3, 10), device=hip_device)
    assert lib.ttrl_observe_ttc(_c(st), R, P, C.byref(tc), t1.data_ptr(), _stream()) == 0
    t2 = torch.ops.ttrl.observe_ttc(other.tensors(), lanes, params, ops.struct_tensor(tc))
    l1 = torch.empty((64, 16, 2), device=hip_device)
    assert lib.ttrl_observe_lidar(_c(st), R, P, C.byref(lc), l1.data_ptr(), _stream()) == 0
    l2 = torch.ops.ttrl.observe_lidar(other.tensors(), lanes, params, ops.struct_tensor(lc))
    torch.cuda.synchronize()
    assert torch.equal(g1, g2) and torch.equal(t1, t2) and torch.equal(l1, l2)


@pytest.mark.gpu
def test_reset_ops_equal_the_c_abi(hip_device):
    env, other = _pair(hip_device)
    st = env.state
    lib = _lib.load()
    lanes, params, cfg = ops.st(env.network.table), ops.st(env.params), ops.st(env.reset_cfg)
    R, P, RC = C.byref(env.network.table), C.byref(env.params), C.byref(env.reset_cfg)
    pcg = torch.from_numpy(_abi.pcg64_states([2 ** 40 + e for e in range(64)]).view(np.int64)).to(hip_device)
    assert lib.ttrl_reset_highway(_c(st), R, P, RC, pcg.data_ptr(), _stream()) == 0
    torch.ops.ttrl.reset_highway_(other.tensors(), lanes, params, cfg, pcg)
    torch.cuda.synchronize()
    _equal(st, other)
    words = torch.randint(0, 2 ** 31, (64, 3), dtype=torch.int32, device=hip_device)
    mask = (torch.arange(64, device=hip_device) % 2).to(torch.uint8)
    assert lib.ttrl_reset_highway_seeded(_c(st), R, P, RC, words.data_ptr(), 3, mask.data_ptr(), _stream()) == 0
    torch.ops.ttrl.reset_highway_seeded_(other.tensors(), lanes, params, cfg, words, mask)
    torch.cuda.synchronize()
    _equal(st, other)


@pytest.mark.gpu
def test_auto_reset_op_equals_the_c_abi_and_the_seeded_reset(hip_device):
    """ttrl::auto_reset_highway_ == its C ABI call, and == the bookkeeping done by hand (done mask,
    episode word + 1, time 0) followed by ttrl_reset_highway_seeded of the done envs."""
    env, other = _pair(hip_device)
    third = env.state.clone()
    lib = _lib.load()
    lanes, params, cfg = ops.st(env.network.table), ops.st(env.params), ops.st(env.reset_cfg)
    R, P, RC = C.byref(env.network.table), C.byref(env.params), C.byref(env.reset_cfg)
    g = torch.Generator(device=hip_device).manual_seed(5)
    term = torch.rand(64, device=hip_device, generator=g) < 0.2
    trunc = torch.rand(64, device=hip_device, generator=g) < 0.1
    ent = torch.randint(0, 2 ** 31, (64, 3), dtype=torch.int32, device=hip_device, generator=g)
    e1, e2, e3 = ent.clone(), ent.clone(), ent.clone()
    t1 = torch.full((64,), 7.0, dtype=torch.float64, device=hip_device)
    t2, t3 = t1.clone(), t1.clone()
    d1 = torch.empty(64, dtype=torch.uint8, device=hip_device)
    assert lib.ttrl_auto_reset_highway(_c(env.state), R, P, RC, e1.data_ptr(), 3, 2, term.data_ptr(), trunc.data_ptr(),
                                       t1.data_ptr(), d1.data_ptr(), _stream()) == 0
    d2 = torch.ops.ttrl.auto_reset_highway_(other.tensors(), lanes, params, cfg, e2, 2, term, trunc, t2)
    done = term | trunc
    e3[:, 2] += done.to(torch.int32)
    t3.masked_fill_(done, 0.0)
    torch.ops.ttrl.reset_highway_seeded_(third.tensors(), lanes, params, cfg, e3, done.to(torch.uint8))
    torch.cuda.synchronize()
    assert torch.equal(d1.bool(), d2) and torch.equal(d2, done)
    assert torch.equal(e1, e2) and torch.equal(e2, e3) and torch.equal(t1, t2) and torch.equal(t2, t3)
    _equal(env.state, other)
    _equal(other, third)


@pytest.mark.gpu
def test_intersection_ops_equal_the_c_abi(hip_device):
    from topotrafficrl_amd.intersection import VecIntersectionEnv
    env = VecIntersectionEnv({"num_envs": 32, "device": hip_device})
    a, b = BatchState(32, 32, device=hip_device), BatchState(32, 32, device=hip_device)
    lib = _lib.load()
    lanes, params, cfg = ops.st(env.network.table), ops.st(env.params), ops.st(env.ix)
    R, P, IX = C.byref(env.network.table), C.byref(env.params), C.byref(env.ix)
    words = torch.arange(32, dtype=torch.int32, device=hip_device).view(-1, 1)
    assert lib.ttrl_ix_reset(_c(a), R, P, IX, words.data_ptr(), 1, None, _stream()) == 0
    torch.ops.ttrl.ix_reset_(b.tensors(), lanes, params, cfg, words, None)
    assert lib.ttrl_ix_clear_spawn(_c(a), R, P, IX, None, _stream()) == 0
    torch.ops.ttrl.ix_clear_spawn_(b.tensors(), lanes, params, cfg, None)
    torch.cuda.synchronize()
    _equal(a, b)
    assert np.all((b["kind"] > 0).sum(1).cpu().numpy() >= 2)
    c, d = BatchState(32, 32, device=hip_device), BatchState(32, 32, device=hip_device)
    mask = (torch.arange(32, device=hip_device) % 3 == 1).to(torch.uint8)
    assert lib.ttrl_copy_envs(_c(c), _c(a), mask.data_ptr(), _stream()) == 0
    torch.ops.ttrl.copy_envs_(d.tensors(), b.tensors(), mask)
    torch.cuda.synchronize()
    _equal(c, d)
    # the reset in parts: begin, the 45 warm-up frames as 15 + 30, finish, through the C ABI and the
    # operator, equals the whole reset of the same envs (masked: the others keep their rows)
    e, f = a.clone(), a.clone()
    w2 = words + 100
    assert lib.ttrl_ix_reset(_c(e), R, P, IX, w2.data_ptr(), 1, mask.data_ptr(), _stream()) == 0
    assert lib.ttrl_ix_reset_parts(_c(f), R, P, IX, 3, w2.data_ptr(), 1, mask.data_ptr(), mask.data_ptr(), 15, None,
                                   _stream()) == 0
    torch.ops.ttrl.ix_reset_parts_(f.tensors(), lanes, params, cfg, 6, None, None, mask, 30, mask)
    torch.cuda.synchronize()
    _equal(e, f)
    assert lib.ttrl_ix_reset_parts(_c(f), R, P, IX, 8, None, 0, None, None, 0, None, _stream()) == -1


@pytest.mark.gpu
def test_ix_env_step_op_equals_the_c_abi(hip_device):
    """ttrl::ix_env_step_ against a direct ctypes call of ttrl_ix_env_step, on copies of in-loop
    intersection scenes whose clocks put some envs at their last step (those swap in spares)."""
    from topotrafficrl_amd.intersection import VecIntersectionEnv
    env = VecIntersectionEnv({"num_envs": 32, "device": hip_device, "auto_reset": True, "duration": 3})
    env.reset(seed=3)
    g = torch.Generator(device=hip_device).manual_seed(1)
    for _ in range(2):
        env.step(torch.randint(0, 3, (32,), device=hip_device, generator=g))
    env._join_sides()
    torch.cuda.synchronize()
    lib = _lib.load()
    lanes, params, cfg = ops.st(env.network.table), ops.st(env.params), ops.st(env.ix)
    R, P, IX = C.byref(env.network.table), C.byref(env.params), C.byref(env.ix)
    kin = env.observation_type.fused_cfg()
    rc = env.reward_cfg
    act = torch.randint(0, 3, (32,), device=hip_device, generator=g, dtype=torch.int32)
    codes = env.action_type._codes(act).to(torch.int32)
    a, b = env.state.clone(), env.state.clone()
    sa, sb = env._spare.clone(), env._spare.clone()
    ta, tb = env.time.clone(), env.time.clone()
    oa, ob = env._order.clone(), env._order.clone()
    la, lb = torch.zeros((), dtype=torch.int64, device=hip_device), torch.zeros((), dtype=torch.int64, device=hip_device)
    pa, pb = env._spare_par.clone(), env._spare_par.clone()
    ea, eb = env._entropy.clone(), env._entropy.clone()
    fa, fb = env._spare_ent.clone(), env._spare_ent.clone()
    outs = torch.ops.ttrl.ix_env_step_(a.tensors(), lanes, params, cfg, codes, 15, 1 / 15, ops.kin_cfg_tensor(kin),
                                       ops.st(rc), ta, 1.0, sa.tensors(), pa, ea, fa, oa, None, la)
    E, V, F = 32, kin.vehicles_count, kin.n_features
    o = [torch.empty(E, V, F, device=hip_device), torch.empty(E, V - 1, dtype=torch.int32, device=hip_device),
         torch.empty(E, device=hip_device), torch.empty(E, dtype=torch.bool, device=hip_device),
         torch.empty(E, dtype=torch.bool, device=hip_device), torch.empty(E, 4, device=hip_device),
         torch.empty(E, dtype=torch.float64, device=hip_device), torch.empty(E, dtype=torch.bool, device=hip_device),
         torch.empty(E, dtype=torch.bool, device=hip_device), torch.empty(sb.n_envs, dtype=torch.uint8, device=hip_device),
         torch.empty(E, V, F, device=hip_device), torch.empty(E, V - 1, dtype=torch.int32, device=hip_device)]
    assert lib.ttrl_ix_env_step(_c(b), R, P, IX, codes.data_ptr(), 15, 1 / 15, C.byref(kin), o[0].data_ptr(),
                                o[1].data_ptr(), o[10].data_ptr(), o[11].data_ptr(), C.byref(rc), tb.data_ptr(), 1.0,
                                o[2].data_ptr(), o[3].data_ptr(), o[4].data_ptr(), o[5].data_ptr(), o[6].data_ptr(),
                                o[7].data_ptr(), _c(sb), pb.data_ptr(), eb.data_ptr(), fb.data_ptr(), eb.shape[1],
                                o[8].data_ptr(), o[9].data_ptr(), ob.data_ptr(), None, 0, lb.data_ptr(),
                                _stream()) == 0
    torch.cuda.synchronize()
    for x, y in zip(outs, o):
        assert torch.equal(x, y)
    _equal(a, b)
    _equal(sa, sb)
    for x, y in ((ta, tb), (oa, ob), (la, lb), (pa, pb), (ea, eb), (fa, fb)):
        assert torch.equal(x, y)
    assert bool(o[8].any())  # truncations at time 3 (and any crashes): spares swapped in


@pytest.mark.gpu
def test_ego_attention_op_equals_the_c_abi(hip_device):
    from topotrafficrl_amd.agent import EgoAttentionNetwork
    net = EgoAttentionNetwork(5).reset(torch.Generator().manual_seed(0)).to(hip_device)
    x = torch.rand(100, 15, 7, device=hip_device) * 2 - 1
    x[:, :, 0] = (x[:, :, 0] > 0).float()
    w = net.packed_weights()
    lib = _lib.load()
    n_scratch = C.c_int64()
    lib.ttrl_ego_attention_sizes(7, 5, 100, 15, C.byref(n_scratch))
    scratch = torch.empty(int(n_scratch.value), device=hip_device)
    q1 = torch.empty((100, 5), device=hip_device)
    assert lib.ttrl_ego_attention_q(x.data_ptr(), 100, 15, 7, 2, w.data_ptr(), 5, scratch.data_ptr(), q1.data_ptr(),
                                    _stream()) == 0
    q2 = torch.ops.ttrl.ego_attention_q(x, w, 2, 5)
    torch.cuda.synchronize()
    assert torch.equal(q1, q2)
    act1 = torch.empty(100, dtype=torch.int64, device=hip_device)
    act32 = torch.empty(100, dtype=torch.int32, device=hip_device)
    q3 = torch.empty((100, 5), device=hip_device)
    assert lib.ttrl_ego_attention_act(x.data_ptr(), 100, 15, 7, 2, w.data_ptr(), 5, 0.3, None, 77, 5, None, 0,
                                      q3.data_ptr(), act1.data_ptr(), act32.data_ptr(), _stream()) == 0
    assert lib.ttrl_ego_attention_act(x.data_ptr(), 100, 15, 7, 2, w.data_ptr(), 5, 0.3, None, 77, 5, None, 0,
                                      q3.data_ptr(), None, None, _stream()) != 0  # no action output
    assert lib.ttrl_ego_attention_act(x.data_ptr(), 100, 15, 7, 2, w.data_ptr(), 5, 0.3, None, 77, 5, None, -1,
                                      q3.data_ptr(), act1.data_ptr(), None, _stream()) != 0  # negative offset
    act2, q4 = torch.ops.ttrl.ego_attention_act(x, w, 2, 5, 0.3, 77, 5)
    act3, _ = torch.ops.ttrl.ego_attention_act(x, w, 2, 5, 0.3, 77, 5, int32_actions=True)
    torch.cuda.synchronize()
    assert torch.equal(q3, q1) and torch.equal(q4, q1) and torch.equal(act1, act2)
    assert act3.dtype == torch.int32 and torch.equal(act32, act3) and torch.equal(act3.long(), act2)
