"""Summarise a tools/profile_box.sh run into profiles/ (tracked): kernel stats, HBM traffic
per launch from separate FETCH_SIZE / WRITE_SIZE passes (gfx950: FETCH_SIZE counts half of
the bytes of wide streaming reads -> x2; both in KiB -> x1024, MI355X_MICROARCH.md §HBM),
SQ instruction mix, and the effective clock (GRBM_GUI_ACTIVE / 8 XCDs / wall)."""
import csv
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TAG = sys.argv[1] if len(sys.argv) > 1 else "r01"
SRC = os.path.join(ROOT, "gpurun_out", f"prof_{TAG}")
DST = os.path.join(ROOT, "profiles")
os.makedirs(DST, exist_ok=True)
SIM = "simulate_kernel"


def short(name):
    n = name.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
    return n[:90]


def counters(path):
    """{(kernel, counter): [values per dispatch]} and {kernel: [durations ns]}"""
    vals = defaultdict(list)
    dur = defaultdict(list)
    seen = set()
    for r in csv.DictReader(open(path)):
        k = short(r["Kernel_Name"])
        vals[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
        key = (r["Dispatch_Id"], k)
        if key not in seen:
            seen.add(key)
            dur[k].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    return vals, dur


def mean(v):
    return sum(v) / len(v) if v else float("nan")


import hashlib  # noqa: E402
SO_SHA16 = hashlib.sha256(open(os.path.join(ROOT, "topotrafficrl_amd", "lib", "libttrl_mi355x.so"), "rb").read()
                          ).hexdigest()[:16]  # the build the counters were measured on (shipped from this tree)
out_json = {}
md = [f"# Profile {TAG}: `python bench.py` (config 4: 4096 envs x 64 vehicles, Kinematics 15x7), MI355X", ""]
for dt in ("f64", "f32"):
    stats = os.path.join(SRC, f"trace_{dt}_kernel_stats.csv")
    shutil.copy(stats, os.path.join(DST, f"{TAG}_kernel_stats_{dt}.csv"))
    bench = open(os.path.join(SRC, f"bench_trace_{dt}.json")).read().strip().splitlines()[-1]
    shutil.copy(os.path.join(SRC, f"bench_trace_{dt}.json"), os.path.join(DST, f"{TAG}_bench_under_rocprof_{dt}.json"))
    md += [f"## dtype {dt}", "", "| kernel | calls | avg us | share |", "|---|---|---|---|"]
    sim_avg = None
    for r in list(csv.DictReader(open(stats)))[:8]:
        md.append(f"| `{short(r['Name'])}` | {r['Calls']} | {float(r['AverageNs']) / 1e3:.1f} | {float(r['Percentage']):.1f}% |")
        if SIM in r["Name"]:
            sim_avg = float(r["AverageNs"])
    fetch, _ = counters(os.path.join(SRC, f"fetch_{dt}_counter_collection.csv"))
    write, _ = counters(os.path.join(SRC, f"write_{dt}_counter_collection.csv"))
    sq, sq_dur = counters(os.path.join(SRC, f"sq_{dt}_counter_collection.csv"))
    grbm, grbm_dur = counters(os.path.join(SRC, f"grbm_{dt}_counter_collection.csv"))
    simk = [k for (k, c) in fetch if SIM in k][0]
    f_kib = mean(fetch[(simk, "FETCH_SIZE")])
    w_kib = mean(write[(simk, "WRITE_SIZE")])
    hbm = (2 * f_kib + w_kib) * 1024
    e = json.loads(bench)
    alg = e["roofline"]["alg_bytes_per_launch"]
    waves = mean(sq[(simk, "SQ_WAVES")])
    valu = mean(sq[(simk, "SQ_INSTS_VALU")])
    lds = mean(sq[(simk, "SQ_INSTS_LDS")])
    salu = mean(sq[(simk, "SQ_INSTS_SALU")])
    busy = mean(sq[(simk, "SQ_BUSY_CYCLES")])
    wave_cyc = mean(sq[(simk, "SQ_WAVE_CYCLES")])
    wait_inst = mean(sq[(simk, "SQ_WAIT_INST_ANY")])
    act_valu = mean(sq[(simk, "SQ_ACTIVE_INST_VALU")])
    gui = mean(grbm[(simk, "GRBM_GUI_ACTIVE")])
    clk = gui / 8 / (mean(grbm_dur[simk]) * 1e-9) / 1e9
    out_json[f"config4_{dt}"] = {
        "kernel": simk, "fetch_size_kib_raw": f_kib, "write_size_kib": w_kib,
        "hbm_bytes_per_launch": hbm, "alg_bytes_per_launch": alg,
        "note": "hbm = (2*FETCH_SIZE + WRITE_SIZE)*1024; FETCH_SIZE doubled per the gfx950 calibration",
        "sq_waves": waves, "valu_insts_per_wave": valu / waves, "lds_insts_per_wave": lds / waves,
        "salu_insts_per_wave": salu / waves, "effective_clock_ghz": clk,
        # SQ_ACTIVE_INST_VALU counts quad-cycles (4 shader cycles) per wave
        "valu_active_cycles_per_wave": 4 * act_valu / waves,
        "kernel_ns_trace_avg": sim_avg, "profile": TAG, "so_sha16": SO_SHA16}
    md += ["", f"Fused `{simk}`: trace avg {sim_avg / 1e3:.1f} us per 15-frame launch "
               f"(bench line under rocprof: {e['value']:.3e} veh-steps/s).",
           f"* HBM per launch (PMC, separate passes): FETCH_SIZE {f_kib:.0f} KiB (x2 gfx950) + WRITE_SIZE "
           f"{w_kib:.0f} KiB = {hbm / 1e6:.1f} MB vs algorithmic {alg / 1e6:.1f} MB "
           f"(state read + written once per launch).",
           f"* per wave: {valu / waves:.0f} VALU, {lds / waves:.0f} LDS, {salu / waves:.0f} SALU instructions "
           f"({waves:.0f} waves); SQ_BUSY_CYCLES {busy:.3g}, SQ_WAVE_CYCLES {wave_cyc:.3g}, "
           f"WAIT_INST_ANY/WAVE_CYCLES {wait_inst / max(wave_cyc, 1):.2f}, ACTIVE_INST_VALU/WAVE_CYCLES "
           f"{act_valu / max(wave_cyc, 1):.2f}",
           f"* effective clock (GRBM_GUI_ACTIVE/8/wall): {clk:.2f} GHz", ""]
# config 3: the OccupancyGrid kernel (the path's HBM-bound launch) and the NS = 128 simulate launch
c3 = os.path.join(SRC, "trace_c3_kernel_stats.csv")
if os.path.exists(c3):
    shutil.copy(c3, os.path.join(DST, f"{TAG}_kernel_stats_c3.csv"))
    shutil.copy(os.path.join(SRC, "bench_trace_c3.json"), os.path.join(DST, f"{TAG}_bench_under_rocprof_c3.json"))
    fetch, _ = counters(os.path.join(SRC, "fetch_c3_counter_collection.csv"))
    write, _ = counters(os.path.join(SRC, "write_c3_counter_collection.csv"))
    e = json.loads(open(os.path.join(SRC, "bench_trace_c3.json")).read().strip().splitlines()[-1])
    stats = {short(r["Name"]): float(r["AverageNs"]) for r in csv.DictReader(open(c3))}
    entry = {"note": "hbm = (2*FETCH_SIZE + WRITE_SIZE)*1024; FETCH_SIZE doubled per the gfx950 calibration",
             "profile": TAG, "so_sha16": SO_SHA16}
    md += ["## config 3 (4096 x 128, OccupancyGrid 7x32x32), f64", "", "| kernel | avg us | HBM MB per launch | algorithmic MB |",
           "|---|---|---|---|"]
    for tag, pat, alg in (("", SIM, e["roofline"]["alg_bytes_per_launch"]),
                          ("grid_", "grid_obs_kernel", (e.get("roofline_obs") or {}).get("alg_bytes_per_launch"))):
        ks = [k for (k, c) in fetch if pat in k]
        if not ks:
            continue
        k = ks[0]
        hbm = (2 * mean(fetch[(k, "FETCH_SIZE")]) + mean(write[(k, "WRITE_SIZE")])) * 1024
        avg = [v for n, v in stats.items() if pat in n]
        entry.update({tag + "kernel": k, tag + "hbm_bytes_per_launch": hbm, tag + "alg_bytes_per_launch": alg,
                      tag + "kernel_ns_trace_avg": avg[0] if avg else None})
        md.append(f"| `{k}` | {avg[0] / 1e3 if avg else float('nan'):.1f} | {hbm / 1e6:.1f} | "
                  f"{(alg or float('nan')) / 1e6:.1f} |")
    out_json["config3_f64"] = entry
    md.append("")
json.dump(out_json, open(os.path.join(DST, "pmc_traffic.json"), "w"), indent=1)
open(os.path.join(DST, f"{TAG}_summary.md"), "w").write("\n".join(md) + "\n")
print("\n".join(md))
