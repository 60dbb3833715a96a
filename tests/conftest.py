import glob
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def golden_files(pattern="*.npz"):
    """Road-frame fixtures of gen_golden.py; the intersection episodes (ix_*, gen_golden_ix.py) and
    the finite-MDP tables (mdp_*, gen_golden_mdp.py) have their own layouts and are only returned
    when asked for by name."""
    files = sorted(glob.glob(os.path.join(GOLDEN, pattern)))
    if pattern == "*.npz":
        files = [f for f in files if not os.path.basename(f).startswith(("ix_", "mdp_", "policy_", "dqn_", "obsref_", "envref_"))]
    return files


def scene_files():
    """Scenes built by the highway scene generator (create_random): the straight highways and
    the curved-lane roads (SineLane, CircularLane); the dense scenes are hand-placed."""
    return sorted(golden_files("highway_*") + golden_files("sine_*") + golden_files("arc_*"))


def load_golden(path):
    with np.load(path) as d:
        return {k: d[k] for k in d.files}


def pytest_terminal_summary(terminalreporter, exitstatus, config):
    """The worst parity errors the checks observed (tests/parity_log.py), and TTRL_PARITY_LOG."""
    import parity_log
    rows = parity_log.rows()
    if not rows:
        return
    tr = terminalreporter
    tr.write_sep("-", "worst observed parity errors (check, field: worst [where] samples)")
    for r in rows:
        if "worst" in r:
            tr.write_line(f"{r['check']:48s} {r['field']:16s} {r['worst']:.3e}  [{r['where']}]  n={r['samples']}")
        else:
            tr.write_line(f"{r['check']:48s} {r['count']:16s} {r['n']}")
    path = os.environ.get("TTRL_PARITY_LOG")
    if path:
        import json
        with open(path, "w") as f:
            json.dump(rows, f, indent=1)


@pytest.fixture(scope="session")
def hip_device():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test selected but no HIP device is visible")
    return torch.device("cuda:0")
