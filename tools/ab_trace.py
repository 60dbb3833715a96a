"""Per-variant kernel durations and PMC counters of a `tools/variants.py run` under rocprofv3
(diagnostic).  variants.py launches the fused kernel EVOLVE times with its first variant, then
rounds of one launch per variant in a fixed order; this maps the dispatches of the kernel back to
the variants by that order.

  python tools/ab_trace.py <kernel_trace.csv | counter_collection.csv> <kernel substring> <evolve> <v1,v2,...>
"""
import csv
import sys
from collections import defaultdict

import numpy as np


def main(path, sub, evolve, names):
    rows = [r for r in csv.DictReader(open(path)) if sub in r["Kernel_Name"]]
    if "Counter_Name" in (rows[0] if rows else {}):
        per = defaultdict(dict)  # dispatch -> counter -> value
        for r in rows:
            d = int(r["Dispatch_Id"])
            per[d][r["Counter_Name"]] = per[d].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        disp = sorted(per)[evolve:]
        out = defaultdict(lambda: defaultdict(list))
        for j, d in enumerate(disp):
            for c, v in per[d].items():
                out[names[j % len(names)]][c].append(v)
        counters = sorted({c for v in out.values() for c in v})
        print(f"{'variant':8s} " + " ".join(f"{c:>22s}" for c in counters) + "   (median per launch)")
        for n in names:
            print(f"{n:8s} " + " ".join(f"{np.median(out[n][c]):22.0f}" for c in counters))
        return
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    rows = rows[evolve:]
    out = defaultdict(list)
    for j, r in enumerate(rows):
        out[names[j % len(names)]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for n in names:
        v = out[n][1:]  # the first round is a warm-up (as variants.py's own medians)
        print(f"{n:8s} launches {len(v):3d}  median {np.median(v):8.1f} us  min {np.min(v):8.1f}  max {np.max(v):8.1f}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4].split(","))
