"""Shared test helpers (no tests here)."""
import numpy as np

from oracle.oracle import HostState


def batch_of_ix_states(golds, key="pre", pad_to=32) -> HostState:
    """Every step state of the golden intersection episodes as one batch of envs."""
    cases = [(d, p) for d in golds for p in range(int(d["meta"][1]))]
    big = HostState(len(cases), pad_to)
    for e, (d, p) in enumerate(cases):
        h = HostState.from_ix(d, key, p, pad_to=pad_to)
        for k in big.a:
            big.a[k][e] = h.a[k][0]
    return big
