"""Diagnostic: per-step drift of the device intersection episodes against the golden ones."""
import sys
import os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np
import torch
from conftest import golden_files, load_golden
from oracle.oracle import HostState
from test_gpu_ix_env import ENV_JSON, GOLD
from topotrafficrl_amd.intersection import VecIntersectionEnv

env = VecIntersectionEnv({**ENV_JSON, "num_envs": len(GOLD), "device": "cuda"})
env.reset(seed=0)
acts = np.stack([d["actions"] for d in GOLD], 1)
for p in range(acts.shape[0]):
    obs, rew, term, trunc, info = env.step(torch.from_numpy(acts[p]).cuda())
    st = env.state.to_numpy()
    for e, d in enumerate(GOLD):
        g = HostState.from_ix(d, "post", p, pad_to=32)
        n = int((g["kind"] > 0).sum())
        errs = {k: float(np.max(np.abs(st[k][e, :n] - g[k][0, :n]), initial=0)) for k in ("x", "y", "heading", "speed", "steer")}
        disc = all(np.array_equal(st[k][e, :n], g[k][0, :n]) for k in ("lane", "kind", "crashed", "route_n", "yielding"))
        oerr = float(np.max(np.abs(obs[e].cpu().numpy() - d["obs"][p])))
        slow = g["speed"][0, :n]
        print(p, e, "obs %.2e" % oerr, " ".join("%s %.1e" % kv for kv in errs.items()), "disc", disc,
              "minv %.3f" % np.min(np.abs(slow)))
