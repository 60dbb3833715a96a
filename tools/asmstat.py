"""Static instruction statistics of the simulate kernels (device assembly, no GPU needed).

  python tools/asmstat.py [extra hipcc flags...]    # e.g. -DTTRL_DEV_ONE for a quick build
Prints per simulate_kernel instance: instruction count, SGPR-spill (v_writelane / v_readlane),
scratch traffic, calls, and the VGPR / SGPR / scratch / occupancy of the resource report."""
import collections
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main(flags):
    out = "/tmp/ttrl_asmstat.s"
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-mllvm",
           "-disable-machine-licm", "-I",
           os.path.join(ROOT, "include"), "--cuda-device-only", "-S", "-o", out, *flags,
           os.path.join(ROOT, "topotrafficrl_amd", "csrc", "ttrl_mi355x.hip")]
    subprocess.run(cmd, check=True, stderr=subprocess.DEVNULL)
    lines = open(out).read().split("\n")
    starts = [(i, l.split(":")[0]) for i, l in enumerate(lines) if re.match(r"^_Z\S+:\s*(;.*)?$", l)]
    filt = os.environ.get("FILTER", "simulate_kernel")
    for n, (i, name) in enumerate(starts):
        if filt not in name:
            continue
        end = starts[n + 1][0] if n + 1 < len(starts) else len(lines)
        body = lines[i:end]
        ins = [b.strip().split()[0] for b in body if b.startswith("\t") and not b.startswith("\t.")
               and not b.startswith("\t;") and b.strip()]
        c = collections.Counter(ins)
        meta = {}
        for b in lines[end:end + 80]:
            m = re.match(r"\s*;\s*(NumVgprs|NumSgprs|ScratchSize|Occupancy|codeLenInByte):\s*(\d+)", b)
            if m and m.group(1) not in meta:
                meta[m.group(1)] = int(m.group(2))
        short = re.sub(r"_ZN12_GLOBAL__N_1\d+", "", name)[:48]
        print(f"{short:48s} insts {len(ins):5d} valu {sum(v for k, v in c.items() if k.startswith('v_')):5d} "
              f"salu {sum(v for k, v in c.items() if k.startswith('s_')):5d} lds {sum(v for k, v in c.items() if k.startswith('ds_')):4d} "
              f"wlane {c['v_writelane_b32']:3d} rlane {c['v_readlane_b32']:3d} "
              f"scratch_ops {sum(v for k, v in c.items() if k.startswith('scratch_')):3d} calls {c['s_swappc_b64']} "
              f"{meta}")


if __name__ == "__main__":
    main(sys.argv[1:])
