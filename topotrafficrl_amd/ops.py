"""The HIP entry points as PyTorch operators: ``torch.ops.ttrl.*`` (SURVEY.md §8(b) "Native ops").

The operators are registered from C++ (``csrc/ttrl_torch_ops.cpp``: ``TORCH_LIBRARY(ttrl, m)``,
``TORCH_LIBRARY_IMPL(ttrl, CUDA, m)`` and shape-only ``Meta`` kernels), built by
``__graft_entry__.build()`` into ``lib/libttrl_torch.so`` over the C ABI library
``lib/libttrl_mi355x.so``.  Every product path of the package (``VecHighwayEnv``,
``BatchedRoad``, the observation types, the intersection env, the fused policy forward) calls
these operators; there is no CPU kernel and no fallback.  Arguments:

  state   list of the BatchState tensors in _abi.ALL_FIELDS order (``BatchState.tensors()``)
  lanes / params / cfg   the ABI structs as uint8 CPU tensors (``struct_tensor(_abi.LaneTable())``)

Schemas declare which tensors an op mutates (``Tensor(a!)``); the ops enqueue on the current
HIP stream of the state's device and allocate their outputs from the caching allocator.
"""
from __future__ import annotations

import ctypes as C
import os

import torch

from . import _lib

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib", "libttrl_torch.so")
OPS = ["simulate_", "road_act_", "road_step_", "meta_action_", "env_step_", "neighbours", "kinematics_obs",
       "kinematics_obs_masked_", "occupancy_grid", "observe_ttc", "observe_lidar", "reset_highway_",
       "reset_highway_seeded_", "auto_reset_highway_", "ix_reset_", "ix_reset_parts_", "ix_clear_spawn_", "ix_step_tail_", "ix_env_step_", "copy_envs_", "rewards", "rewards_ex",
       "rewards_step_", "ego_attention_q", "ego_attention_act"]

_loaded = False


def load() -> None:
    """Register torch.ops.ttrl (once).  Raises if the operator library is not built."""
    global _loaded
    if _loaded:
        return
    _lib.load()  # the C ABI library it links against, with its ABI-version check
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"operator library not built: {LIB_PATH} (run __graft_entry__.build())")
    torch.ops.load_library(LIB_PATH)
    _loaded = True


def struct_tensor(s: C.Structure) -> torch.Tensor:
    """An ABI struct as a uint8 CPU tensor (its exact bytes)."""
    return torch.frombuffer(bytearray(bytes(s)), dtype=torch.uint8)


def st(s: C.Structure) -> torch.Tensor:
    """``struct_tensor(s)`` cached on the struct (lane tables, params, reward / reset / grid /
    intersection configs are passed on every step).  The cache is keyed on the struct's current
    bytes, so a field changed in place after the first use (``params.politeness = ...``,
    ``cfg.init_longitudinal[3] = ...``) reaches the next call: a snapshot and a compare of a few
    KB, no tensor rebuilt unless the bytes moved."""
    b = bytes(s)
    cached = getattr(s, "_ttrl_bytes", None)
    if cached is None or cached[0] != b:
        cached = (b, torch.frombuffer(bytearray(b), dtype=torch.uint8))
        s._ttrl_bytes = cached
    return cached[1]


def kin_cfg_tensor(cfg) -> torch.Tensor:
    """A Kinematics cfg: the Philox-shuffled order (order_shuffled 1) moves its shuffle words on
    every call, so it is serialised per call; the others are cached."""
    return struct_tensor(cfg) if cfg.order_shuffled == 1 else st(cfg)


load()
T = torch.ops.ttrl
