"""Per-kernel durations and the main stream's timeline of a rocprofv3 kernel trace (diagnostic).

  python tools/trace_durations.py <kernel_trace.csv> [main_kernel_substring]

Prints, per (kernel, grid size): calls, median and max duration in us.  With a main kernel name
(e.g. simulate_ix_kernel), also the median time between the starts of consecutive launches of it
(the step period) and the median gaps of the main stream around it: every kernel dispatched on the
same queue between two main launches, with its median start offset and duration.
"""
import csv
import re
import sys
from collections import defaultdict

import numpy as np


def short(name: str) -> str:
    m = re.search(r"(\w+_kernel\w*?)(?:<|I[dfi]|$)", name)
    if "vectorized_elementwise" in name or "elementwise_kernel" in name:
        return "torch_elementwise"
    return m.group(1) if m else name[:40]


def main(path: str, main_k: str | None = None) -> None:
    rows = list(csv.DictReader(open(path)))
    for r in rows:
        r["t0"], r["t1"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        r["k"] = short(r["Kernel_Name"])
        r["grid"] = int(r["Grid_Size_X"])
    d = defaultdict(list)
    for r in rows:
        d[(r["k"], r["grid"])].append((r["t1"] - r["t0"]) / 1e3)
    for (k, g), v in sorted(d.items()):
        print(f"  {k:28s} grid {g:8d}  calls {len(v):4d}  median {np.median(v):8.1f}  max {np.max(v):8.1f}")
    if not main_k:
        return
    rows.sort(key=lambda r: r["t0"])
    mains = [r for r in rows if main_k in r["Kernel_Name"]]
    q = mains[0]["Queue_Id"]
    starts = [r["t0"] for r in mains]
    print(f"step period ({main_k} start to start): median {np.median(np.diff(starts)) / 1e3:.1f} us "
          f"over {len(starts) - 1} steps")
    follow = defaultdict(list)  # kernels on the main queue between two main launches: offset, duration
    for a, b in zip(mains[:-1], mains[1:]):
        for r in rows:
            if r["Queue_Id"] == q and a["t0"] < r["t0"] < b["t0"]:
                follow[r["k"]].append(((r["t0"] - a["t1"]) / 1e3, (r["t1"] - r["t0"]) / 1e3))
        follow["(next main launch)"].append(((b["t0"] - a["t1"]) / 1e3, 0.0))
    print(f"main queue after each {main_k} (median start after its end, median duration, us):")
    for k, v in follow.items():
        a = np.array(v)
        print(f"  {k:28s} start +{np.median(a[:, 0]):7.1f}  dur {np.median(a[:, 1]):7.1f}  (n {len(v)})")
    other = defaultdict(list)  # side-queue kernels overlapping a main launch
    for a in mains:
        for r in rows:
            if r["Queue_Id"] != q and r["t0"] < a["t1"] and r["t1"] > a["t0"]:
                other[r["k"]].append((min(r["t1"], a["t1"]) - max(r["t0"], a["t0"])) / 1e3)
    print(f"side-queue kernels overlapping a {main_k} (median overlap, us; per main launch count):")
    for k, v in other.items():
        print(f"  {k:28s} overlap {np.median(v):7.1f}  count {len(v) / len(mains):.2f}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
