"""Diagnostic (timing only): how much of a masked per-env launch (ix_begin / the warm-up frames /
ix_finish over the spare rows) is the dispatch of its masked-out workgroups?  The same ~330 resets
timed inside spare states of 4096, 8192 and 16384 rows (alone on the GPU).

  python tools/ix_dispatch.py
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(active=330):
    from topotrafficrl_amd import ops
    from topotrafficrl_amd.intersection import VecIntersectionEnv
    from topotrafficrl_amd.state import BatchState
    dev = torch.device("cuda:0")
    env = VecIntersectionEnv({"num_envs": 16, "device": str(dev)})
    args = (ops.st(env.network.table), ops.st(env.params), ops.st(env.ix))

    def timed(fn):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda._sleep(100000)
        s.record()
        fn()
        e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) * 1e3

    for rows in (4096, 8192, 16384):
        st = BatchState(rows, 32, device=dev)
        ent = torch.randint(0, 2 ** 31 - 1, (rows, 3), dtype=torch.int32, device=dev)
        mask = torch.zeros(rows, dtype=torch.uint8, device=dev)
        mask[torch.randperm(rows, generator=torch.Generator().manual_seed(1))[:active].to(dev)] = 1
        res = {"begin": [], "warm15": [], "finish": []}
        for _ in range(4):
            res["begin"].append(timed(lambda: ops.T.ix_reset_parts_(st.tensors(), *args, 1, ent, mask, None, 0, None)))
            res["warm15"].append(timed(lambda: ops.T.ix_reset_parts_(st.tensors(), *args, 2, None, None, mask, 15, None)))
            ops.T.ix_reset_parts_(st.tensors(), *args, 2, None, None, mask, 30, None)
            res["finish"].append(timed(lambda: ops.T.ix_reset_parts_(st.tensors(), *args, 4, None, None, None, 0, mask)))
        print(f"{rows:6d} rows, {active} resets: " + ", ".join(f"{k} {np.median(v[1:]):.1f} us" for k, v in res.items()),
              flush=True)


if __name__ == "__main__":
    main()
