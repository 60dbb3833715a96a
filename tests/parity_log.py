"""The worst parity error each check observed, per field, over a test session.

The float64 multi-frame bounds in tests/ are set from these numbers (about 10x the worst value
seen on the MI355X), so every run reports them: ``conftest.pytest_terminal_summary``
prints the table, and with ``TTRL_PARITY_LOG=<path>`` it is also written there as JSON.
"""
from __future__ import annotations

import os

import numpy as np

WORST: dict = {}  # (check, field) -> [worst error, where, samples]
COUNTS: dict = {}  # (check, what) -> count


def rel_err(got, want) -> np.ndarray:
    """|got - want| / (1 + |want|), float64."""
    got = np.asarray(got, dtype=np.float64)
    want = np.asarray(want, dtype=np.float64)
    return np.abs(got - want) / (1 + np.abs(want))


def note(check: str, field: str, err, where: str = "") -> float:
    """Record the largest value of ``err`` for (check, field); returns it."""
    e = np.asarray(err, dtype=np.float64)
    w = float(e.max()) if e.size else 0.0
    cur = WORST.get((check, field))
    if cur is None:
        WORST[(check, field)] = [w, where, 1]
    else:
        cur[2] += 1
        if w > cur[0]:
            cur[0], cur[1] = w, where
    return w


def current_check() -> str:
    """The running test function's name (parametrisations grouped together)."""
    t = os.environ.get("PYTEST_CURRENT_TEST", "?").split(" ")[0]
    return t.split("::")[-1].split("[")[0]


def current_case() -> str:
    t = os.environ.get("PYTEST_CURRENT_TEST", "?").split(" ")[0]
    return t.split("[", 1)[1][:-1] if "[" in t else ""


def count(check: str, what: str, n: int = 1) -> None:
    COUNTS[(check, what)] = COUNTS.get((check, what), 0) + int(n)


def rows() -> list:
    return [{"check": c, "field": f, "worst": v[0], "where": v[1], "samples": v[2]}
            for (c, f), v in sorted(WORST.items())] + \
        [{"check": c, "count": what, "n": n} for (c, what), n in sorted(COUNTS.items())]
