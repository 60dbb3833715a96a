"""The HIP entry points as PyTorch operators: ``torch.ops.ttrl.*``.

Registered with ``torch.library`` over the same C ABI the env classes call through ctypes
(include/ttrl_mi355x.h), for callers that compose the simulator with other torch code:
schemas declare which state tensors an op mutates, every op has a shape-only Meta
implementation (torch.compile / FakeTensor tracing), and the HIP implementations enqueue on
the current stream of the tensors' device.  Arguments:

  state   list of the BatchState tensors in _abi.ALL_FIELDS order (``BatchState.tensors()``)
  lanes / params / cfg   the ABI structs as uint8 CPU tensors (``struct_tensor(_abi.LaneTable())``)

The env classes keep the direct ctypes binding: a registered op adds ~7 µs of dispatch per
call (measured), which the 0.5 ms batched step does not need to pay.
"""
from __future__ import annotations

import ctypes as C

import torch

from . import _abi, _lib

_LIB = torch.library.Library("ttrl", "DEF")
_SCHEMAS = {
    "simulate_": "simulate_(Tensor(a!)[] state, Tensor lanes, Tensor params, Tensor? actions, int frames, float dt) -> ()",
    "road_act_": "road_act_(Tensor(a!)[] state, Tensor lanes, Tensor params) -> ()",
    "road_step_": "road_step_(Tensor(a!)[] state, Tensor lanes, Tensor params, float dt) -> ()",
    "meta_action_": "meta_action_(Tensor(a!)[] state, Tensor lanes, Tensor params, Tensor actions) -> ()",
    "neighbours": "neighbours(Tensor[] state, Tensor lanes, Tensor? query_lane) -> (Tensor, Tensor)",
    "kinematics_obs": "kinematics_obs(Tensor(a!)[] state, Tensor lanes, Tensor params, Tensor cfg, Tensor? mask) "
                      "-> (Tensor, Tensor)",
    "occupancy_grid": "occupancy_grid(Tensor[] state, Tensor lanes, Tensor params, Tensor cfg) -> Tensor",
    "rewards": "rewards(Tensor[] state, Tensor lanes, Tensor cfg, Tensor time) -> (Tensor, Tensor, Tensor)",
    "ix_reset_": "ix_reset_(Tensor(a!)[] state, Tensor lanes, Tensor params, Tensor cfg, Tensor entropy, "
                 "Tensor? mask) -> ()",
    "ix_clear_spawn_": "ix_clear_spawn_(Tensor(a!)[] state, Tensor lanes, Tensor params, Tensor cfg, Tensor? mask) -> ()",
}
for _s in _SCHEMAS.values():
    _LIB.define(_s)


def struct_tensor(s: C.Structure) -> torch.Tensor:
    """An ABI struct as a uint8 CPU tensor (its exact bytes)."""
    return torch.frombuffer(bytearray(bytes(s)), dtype=torch.uint8)


def _as(t: torch.Tensor, cls):
    if t.device.type != "cpu" or t.dtype != torch.uint8 or t.numel() != C.sizeof(cls):
        raise ValueError(f"expected a {C.sizeof(cls)}-byte uint8 CPU tensor holding a {cls.__name__}")
    return cls.from_buffer_copy(t.numpy().tobytes())


def _state(ts: list) -> _abi.State:
    if len(ts) != len(_abi.ALL_FIELDS):
        raise ValueError(f"state: {len(_abi.ALL_FIELDS)} tensors in _abi.ALL_FIELDS order")
    x = ts[0]
    if x.device.type != "cuda":
        raise RuntimeError("ttrl ops run on a HIP device only (no CPU fallback)")
    dtype = {torch.float64: _abi.F64, torch.float32: _abi.F32}[x.dtype]
    return _abi.state_struct({f: t.data_ptr() for f, t in zip(_abi.ALL_FIELDS, ts)}, x.shape[0], x.shape[1], dtype)


def _stream(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


def _i32(t, n, dev):
    if t is None:
        return None
    t = t.to(device=dev, dtype=torch.int32).contiguous()
    if t.numel() != n:
        raise ValueError(f"expected {n} entries")
    return t


def _u8(t, n, dev):
    if t is None:
        return None
    t = t.to(device=dev, dtype=torch.uint8).contiguous()
    if t.numel() != n:
        raise ValueError(f"expected {n} entries")
    return t


def _simulate(state, lanes, params, actions, frames, dt):
    s, a = _state(state), _i32(actions, state[0].shape[0], state[0].device)
    _lib.call("ttrl_simulate", C.byref(s), C.byref(_as(lanes, _abi.LaneTable)), C.byref(_as(params, _abi.Params)),
              None if a is None else a.data_ptr(), int(frames), float(dt), _stream(state[0]))


def _road_act(state, lanes, params):
    _lib.call("ttrl_road_act", C.byref(_state(state)), C.byref(_as(lanes, _abi.LaneTable)),
              C.byref(_as(params, _abi.Params)), _stream(state[0]))


def _road_step(state, lanes, params, dt):
    _lib.call("ttrl_road_step", C.byref(_state(state)), C.byref(_as(lanes, _abi.LaneTable)),
              C.byref(_as(params, _abi.Params)), float(dt), _stream(state[0]))


def _meta_action(state, lanes, params, actions):
    a = _i32(actions, state[0].shape[0], state[0].device)
    _lib.call("ttrl_meta_action", C.byref(_state(state)), C.byref(_as(lanes, _abi.LaneTable)),
              C.byref(_as(params, _abi.Params)), a.data_ptr(), _stream(state[0]))


def _neighbours(state, lanes, query_lane):
    E, N = state[0].shape
    q = _i32(query_lane, E * N, state[0].device)
    f = torch.empty((E, N), dtype=torch.int32, device=state[0].device)
    r = torch.empty_like(f)
    _lib.call("ttrl_neighbours", C.byref(_state(state)), C.byref(_as(lanes, _abi.LaneTable)),
              None if q is None else q.data_ptr(), f.data_ptr(), r.data_ptr(), _stream(state[0]))
    return f, r


def _kin_shapes(state, cfg):
    c = _as(cfg, _abi.KinCfg)
    E = state[0].shape[0]
    return c, (E, c.vehicles_count, c.n_features), (E, max(c.vehicles_count - 1, 1))


def _kinematics_obs(state, lanes, params, cfg, mask):
    c, so, si = _kin_shapes(state, cfg)
    out = torch.zeros(so, dtype=torch.float32, device=state[0].device)
    ids = torch.full(si, -1, dtype=torch.int32, device=state[0].device)
    m = _u8(mask, so[0], state[0].device)
    _lib.call("ttrl_observe_kinematics_masked", C.byref(_state(state)), C.byref(_as(lanes, _abi.LaneTable)),
              C.byref(_as(params, _abi.Params)), C.byref(c), None if m is None else m.data_ptr(), out.data_ptr(),
              ids.data_ptr(), _stream(state[0]))
    return out, ids


def _grid_shape(state, cfg):
    c = _as(cfg, _abi.GridCfg)
    return c, (state[0].shape[0], c.n_features, c.shape_x, c.shape_y)


def _occupancy_grid(state, lanes, params, cfg):
    c, shape = _grid_shape(state, cfg)
    out = torch.empty(shape, dtype=torch.float32, device=state[0].device)
    _lib.call("ttrl_observe_grid", C.byref(_state(state)), C.byref(_as(lanes, _abi.LaneTable)),
              C.byref(_as(params, _abi.Params)), C.byref(c), out.data_ptr(), _stream(state[0]))
    return out


def _rewards(state, lanes, cfg, time):
    E, dev = state[0].shape[0], state[0].device
    t = time.to(device=dev, dtype=torch.float64).contiguous()
    rew = torch.empty(E, dtype=torch.float32, device=dev)
    term = torch.empty(E, dtype=torch.uint8, device=dev)
    trunc = torch.empty(E, dtype=torch.uint8, device=dev)
    _lib.call("ttrl_rewards", C.byref(_state(state)), C.byref(_as(lanes, _abi.LaneTable)),
              C.byref(_as(cfg, _abi.RewardCfg)), t.data_ptr(), rew.data_ptr(), term.data_ptr(), trunc.data_ptr(),
              _stream(state[0]))
    return rew, term.bool(), trunc.bool()


def _ix_reset(state, lanes, params, cfg, entropy, mask):
    E, dev = state[0].shape[0], state[0].device
    w = entropy.to(device=dev, dtype=torch.int32).contiguous()
    if w.dim() != 2 or w.shape[0] != E:
        raise ValueError("entropy must be [n_envs, n_words] uint32 words (int32)")
    m = _u8(mask, E, dev)
    _lib.call("ttrl_ix_reset", C.byref(_state(state)), C.byref(_as(lanes, _abi.LaneTable)),
              C.byref(_as(params, _abi.Params)), C.byref(_as(cfg, _abi.IxCfg)), w.data_ptr(), int(w.shape[1]),
              None if m is None else m.data_ptr(), _stream(state[0]))


def _ix_clear_spawn(state, lanes, params, cfg, mask):
    m = _u8(mask, state[0].shape[0], state[0].device)
    _lib.call("ttrl_ix_clear_spawn", C.byref(_state(state)), C.byref(_as(lanes, _abi.LaneTable)),
              C.byref(_as(params, _abi.Params)), C.byref(_as(cfg, _abi.IxCfg)), None if m is None else m.data_ptr(),
              _stream(state[0]))


_IMPLS = {"simulate_": _simulate, "road_act_": _road_act, "road_step_": _road_step, "meta_action_": _meta_action,
          "neighbours": _neighbours, "kinematics_obs": _kinematics_obs, "occupancy_grid": _occupancy_grid,
          "rewards": _rewards, "ix_reset_": _ix_reset, "ix_clear_spawn_": _ix_clear_spawn}
for _name, _fn in _IMPLS.items():
    _LIB.impl(_name, _fn, "CUDA")  # the HIP device of ROCm PyTorch


# Meta (shape-only) implementations for FakeTensor tracing
def _meta_none(*args):
    return None


def _meta_neighbours(state, lanes, query_lane):
    E, N = state[0].shape
    f = state[0].new_empty((E, N), dtype=torch.int32)
    return f, torch.empty_like(f)


def _meta_kin(state, lanes, params, cfg, mask):
    _, so, si = _kin_shapes(state, cfg)
    return state[0].new_empty(so, dtype=torch.float32), state[0].new_empty(si, dtype=torch.int32)


def _meta_grid(state, lanes, params, cfg):
    return state[0].new_empty(_grid_shape(state, cfg)[1], dtype=torch.float32)


def _meta_rewards(state, lanes, cfg, time):
    E = state[0].shape[0]
    return (state[0].new_empty(E, dtype=torch.float32), state[0].new_empty(E, dtype=torch.bool),
            state[0].new_empty(E, dtype=torch.bool))


for _name in ("simulate_", "road_act_", "road_step_", "meta_action_", "ix_reset_", "ix_clear_spawn_"):
    _LIB.impl(_name, _meta_none, "Meta")
_LIB.impl("neighbours", _meta_neighbours, "Meta")
_LIB.impl("kinematics_obs", _meta_kin, "Meta")
_LIB.impl("occupancy_grid", _meta_grid, "Meta")
_LIB.impl("rewards", _meta_rewards, "Meta")
