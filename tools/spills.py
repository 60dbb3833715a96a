"""Static scratch (spill) sites of one kernel instance with their source lines (line tables):
  FILTER=simulate_kernelIdLi64ELi1ELi0 python tools/spills.py [extra hipcc flags...]"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
out = "/tmp/ttrl_spills.s"
subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-mllvm",
                "-disable-machine-licm", "-gline-tables-only", "--cuda-device-only", "-S", "-I",
                os.path.join(ROOT, "include"), "-o", out, *sys.argv[1:],
                os.path.join(ROOT, "topotrafficrl_amd", "csrc", "ttrl_mi355x.hip")], check=True,
               stderr=subprocess.DEVNULL)
lines = open(out).read().split("\n")
starts = [(i, l.split(":")[0]) for i, l in enumerate(lines) if re.match(r"^_Z\S+:\s*(;.*)?$", l)]
filt = os.environ.get("FILTER", "simulate_kernelIdLi64ELi1ELi0")
for n, (i, name) in enumerate(starts):
    if filt not in name:
        continue
    body = lines[i:starts[n + 1][0] if n + 1 < len(starts) else len(lines)]
    loc, depth = None, 0
    for j, l in enumerate(body):
        m = re.match(r"\s*\.loc\s+\d+\s+(\d+)\s+(\d+)", l)
        if m:
            loc = (int(m.group(1)), int(m.group(2)))
        m = re.search(r"Depth=(\d+)", l)
        if l.startswith(".LBB") or l.startswith("; %bb"):
            depth = int(m.group(1)) if m else 0
        if "scratch_" in l:
            print(f"{j:6d} line {loc[0] if loc else '?':>5} depth {depth} {l.strip()[:70]}")
    break
