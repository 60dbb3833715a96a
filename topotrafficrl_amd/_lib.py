"""ctypes loader of the in-tree C ABI library (topotrafficrl_amd/lib/libttrl_mi355x.so).

The product calls the library through the PyTorch operators of ops.py (lib/libttrl_torch.so,
linked against it); this loader checks the ABI version and the exported symbols, and serves the
ABI tests and the kernel-timing tools.  There is no fallback: if the library is missing or fails
to load, every product entry point raises.  Build it with ``python -c "import __graft_entry__ as g; g.build()"``
or ``python -m topotrafficrl_amd.build``.
"""
from __future__ import annotations

import ctypes as C
import os

from . import _abi

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "lib", "libttrl_mi355x.so")

_P = C.c_void_p
_SIGS = {
    "ttrl_abi_version": ([], C.c_int),
    "ttrl_meta_action": ([_P, _P, _P, _P, _P], C.c_int),
    "ttrl_road_act": ([_P, _P, _P, _P], C.c_int),
    "ttrl_road_step": ([_P, _P, _P, C.c_double, _P], C.c_int),
    "ttrl_simulate": ([_P, _P, _P, _P, C.c_int32, C.c_double, _P], C.c_int),
    "ttrl_env_step": ([_P, _P, _P, _P, C.c_int32, C.c_double, _P, _P, _P, _P, _P, C.c_double, _P, _P, _P, _P, _P,
                       _P, _P, _P, C.c_int32, _P], C.c_int),
    "ttrl_env_step_grid": ([_P, _P, _P, _P, C.c_int32, C.c_double, _P, _P, _P, _P, C.c_double, _P, _P, _P, _P, _P, _P,
                            _P, C.c_int32, _P], C.c_int),
    "ttrl_neighbours": ([_P, _P, _P, _P, _P, _P], C.c_int),
    "ttrl_observe_kinematics": ([_P, _P, _P, _P, _P, _P, _P], C.c_int),
    "ttrl_observe_kinematics_masked": ([_P, _P, _P, _P, _P, _P, _P, _P], C.c_int),
    "ttrl_observe_grid": ([_P, _P, _P, _P, _P, _P], C.c_int),
    "ttrl_observe_ttc": ([_P, _P, _P, _P, _P, _P], C.c_int),
    "ttrl_observe_lidar": ([_P, _P, _P, _P, _P, _P], C.c_int),
    "ttrl_reset_highway": ([_P, _P, _P, _P, _P, _P], C.c_int),
    "ttrl_reset_highway_seeded": ([_P, _P, _P, _P, _P, C.c_int32, _P, _P], C.c_int),
    "ttrl_auto_reset_highway": ([_P, _P, _P, _P, _P, C.c_int32, C.c_int32, _P, _P, _P, _P, _P], C.c_int),
    "ttrl_seed_pcg64": ([_P, C.c_int32, _P], C.c_int),
    "ttrl_rewards": ([_P, _P, _P, _P, _P, _P, _P, _P], C.c_int),
    "ttrl_rewards_ex": ([_P, _P, _P, _P, _P, _P, _P, _P, _P], C.c_int),
    "ttrl_rewards_step": ([_P, _P, _P, _P, C.c_double, _P, _P, _P, _P, _P, _P, _P], C.c_int),
    "ttrl_ix_reset": ([_P, _P, _P, _P, _P, C.c_int32, _P, _P], C.c_int),
    "ttrl_ix_reset_parts": ([_P, _P, _P, _P, C.c_int32, _P, C.c_int32, _P, _P, C.c_int32, _P, _P], C.c_int),
    "ttrl_ix_clear_spawn": ([_P, _P, _P, _P, _P, _P], C.c_int),
    "ttrl_ix_step_tail": ([_P, _P, _P, _P, _P, _P, _P, _P, _P, _P, C.c_int32, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P,
                           _P],
                          C.c_int),
    "ttrl_ix_env_step": ([_P, _P, _P, _P, _P, C.c_int32, C.c_double, _P, _P, _P, _P, _P, _P, _P, C.c_double, _P, _P,
                          _P, _P, _P, _P, _P, _P, _P, _P, C.c_int32, _P, _P, _P, _P, C.c_int32, _P, _P], C.c_int),
    "ttrl_copy_envs": ([_P, _P, _P, _P], C.c_int),
    "ttrl_ego_attention_sizes": ([C.c_int32, C.c_int32, C.c_int32, C.c_int32, _P], C.c_int64),
    "ttrl_ego_attention_q": ([_P, C.c_int32, C.c_int32, C.c_int32, C.c_int32, _P, C.c_int32, _P, _P, _P], C.c_int),
    "ttrl_ego_attention_act": ([_P, C.c_int32, C.c_int32, C.c_int32, C.c_int32, _P, C.c_int32, C.c_float, _P,
                                C.c_uint64, C.c_int64, _P, C.c_int64, _P, _P, _P, _P], C.c_int),
}
EXPORTS = [k for k in _SIGS]

_lib = None


class TTRLError(RuntimeError):
    pass


def load(path: str | None = None, check_abi: bool = True) -> C.CDLL:
    """Load (once) and return the HIP library; raises if it is not built.  ``check_abi`` False:
    an earlier round's build loaded by path for an A/B timing of entry points whose signature
    did not change (tools/variants.py REV_VARIANTS; ttrl_simulate only)."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    # `path`: an alternative build of the same library, for the A/B timing tools only (tools/);
    # the product always runs lib/libttrl_mi355x.so, which the operator library links by rpath
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise ImportError(f"HIP library not built: {p} (run __graft_entry__.build())")
    lib = C.CDLL(p)
    for name, (args, res) in _SIGS.items():
        fn = getattr(lib, name, None)
        if fn is None:
            if path is None:
                raise ImportError(f"{p} lacks {name}: rebuild it")
            continue  # an older build loaded for comparison (tools/variants.py)
        fn.argtypes = args
        fn.restype = res
    if (check_abi or path is None) and lib.ttrl_abi_version() != 8:  # include/ttrl_mi355x.h TTRL_ABI_VERSION
        raise ImportError("ABI version mismatch with include/ttrl_mi355x.h")
    if path is None:
        _lib = lib
    return lib


def call(name: str, *args) -> None:
    rc = getattr(load(), name)(*args)
    if rc != 0:
        raise TTRLError(f"{name} failed: {rc} {_abi.ERRORS.get(rc, '')}")
