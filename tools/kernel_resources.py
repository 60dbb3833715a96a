"""Registers, scratch and occupancy of every simulate_kernel instance, from the compiler's
kernel-resource-usage remarks (device-only compile of the product source, here on the CPU).

  python tools/kernel_resources.py [log]   # log: an existing remarks log instead of compiling
"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def remarks():
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-fPIC",
           "-mllvm", "-disable-machine-licm", "-I", os.path.join(ROOT, "include"),
           "-I", os.path.join(ROOT, "topotrafficrl_amd", "csrc"), "--cuda-device-only", "-c",
           "-Rpass-analysis=kernel-resource-usage", os.path.join(ROOT, "topotrafficrl_amd", "csrc", "ttrl_mi355x.hip"),
           "-o", "/tmp/ttrl_kres.o"]
    return subprocess.run(cmd, capture_output=True, text=True, check=True).stderr


def main():
    text = open(sys.argv[1]).read() if len(sys.argv) > 1 else remarks()
    rows, cur = [], None
    for line in text.splitlines():
        m = re.search(r"remark: (.*?) \[-Rpass", line)
        if not m:
            continue
        t = m.group(1).strip()
        if t.startswith("Function Name:"):
            cur = {"name": t.split(":", 1)[1].strip()}
            rows.append(cur)
        elif cur is not None and ":" in t:
            k, v = t.split(":", 1)
            cur[k.strip()] = v.strip()
    net = {"0": "straight", "1": "curved", "2": "graph"}
    print(f"{'instance (T, NS, EPW, net, wave budget)':44s} {'VGPRs':>5s} {'scratch B/lane':>14s} {'waves/SIMD':>10s}")
    for r in rows:
        m = re.search(r"simulate_kernelI([df])Li(\d+)ELi(\d+)ELi(\d+)ELi(\d+)E", r["name"])
        if not m:  # the fused step instances: config 3's grid epilogue, config 6's intersection tail
            g = re.search(r"simulate_(grid|ix)_kernelI([df])Li(\d+)E(?:Li(\d+)E)?", r["name"])
            if g:
                kind, t, ns, epw = g.groups()
                name = (f"{'double' if t == 'd' else 'float'}, {ns}, {epw or 1}, "
                        f"{'straight + grid' if kind == 'grid' else 'graph + ix tail'}, default")
                print(f"{name:44s} {r.get('VGPRs', '?'):>5s} {r.get('ScratchSize [bytes/lane]', '?'):>14s} "
                      f"{r.get('Occupancy [waves/SIMD]', '?'):>10s}")
            continue
        t, ns, epw, nt, wb = m.groups()
        name = f"{'double' if t == 'd' else 'float'}, {ns}, {epw}, {net[nt]}, {wb if wb != '0' else 'default'}"
        print(f"{name:44s} {r.get('VGPRs', '?'):>5s} {r.get('ScratchSize [bytes/lane]', '?'):>14s} "
              f"{r.get('Occupancy [waves/SIMD]', '?'):>10s}")


if __name__ == "__main__":
    main()
