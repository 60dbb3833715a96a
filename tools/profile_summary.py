"""Summarise a tools/profile_box.sh run into profiles/ (tracked): per bench configuration, the
kernel stats, HBM traffic per launch of the fused simulate kernel from separate FETCH_SIZE /
WRITE_SIZE passes (gfx950: FETCH_SIZE counts half of the bytes of wide streaming reads -> x2; both
in KiB -> x1024, MI355X_MICROARCH.md §HBM), the SQ instruction mix and waits, and the effective
clock (GRBM_GUI_ACTIVE / 8 XCDs / duration).  Writes profiles/pmc_traffic.json, whose entries
bench.py uses only on the build they were measured on (so_sha16).

Config 6 runs the same simulate kernel for the step and, on side streams, for the resets' 45
warm-up frames (ix_reset: ix_begin, simulate, ix_finish): a simulate dispatch that directly
follows an ix_begin dispatch is a warm-up and is left out of the step launch's figures.

  python tools/profile_summary.py TAG"""
import csv
import glob
import hashlib
import json
import os
import re
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TAG = sys.argv[1] if len(sys.argv) > 1 else "r01"
SRC = os.path.join(ROOT, "gpurun_out", f"prof_{TAG}")
DST = os.path.join(ROOT, "profiles")
SIM = "simulate_kernel"
NAMES = {2: "4096 envs x 32 vehicles, Kinematics 15x7", 3: "4096 envs x 128 vehicles, OccupancyGrid 7x32x32",
         4: "4096 envs x 64 vehicles, Kinematics 15x7 (headline)", 5: "8192 x 64 + EgoAttention-2h policy",
         6: "4096 intersection-v0 envs, auto-reset, overlapped resets"}


def short(name):
    n = name.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
    return n[:90]


def step_dispatches(rows, id_key="Dispatch_Id", name_key="Kernel_Name"):
    """Dispatch ids of the step's simulate launches: every simulate dispatch except those directly
    after an ix_begin dispatch (the resets' warm-ups)."""
    order = sorted({(int(r[id_key]), short(r[name_key])) for r in rows})
    # round 6: config 6's step is simulate_ix_kernel (the warm-ups stay simulate_kernel) and config 3's
    # simulate_grid_kernel; when a trace holds one of them, it is the step launch
    for fused in ("simulate_ix_kernel", "simulate_grid_kernel"):
        if any(fused in k for _, k in order):
            return {did for did, k in order if fused in k}
    keep, prev = set(), ""
    for did, k in order:
        if SIM in k and "ix_begin_kernel" not in prev:
            keep.add(did)
        prev = k
    return keep


def counters(path):
    """{counter: [values per step-simulate dispatch]}, the kernel name and the durations (ns)"""
    rows = list(csv.DictReader(open(path)))
    keep = step_dispatches(rows)
    vals = defaultdict(list)
    dur, seen, kern = [], set(), None
    for r in rows:
        did = int(r["Dispatch_Id"])
        if did not in keep:
            continue
        kern = short(r["Kernel_Name"])
        vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
        if did not in seen:
            seen.add(did)
            dur.append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    return vals, kern, dur


def mean(v):
    return sum(v) / len(v) if v else float("nan")


def main():
    so_sha16 = hashlib.sha256(open(os.path.join(ROOT, "topotrafficrl_amd", "lib", "libttrl_mi355x.so"), "rb").read()
                              ).hexdigest()[:16]  # the build the counters were measured on (shipped from this tree)
    out_json, md = {}, [f"# Profile {TAG}: `bench.py` configurations under rocprofv3 (MI355X), libttrl_mi355x.so "
                        f"{so_sha16}", ""]
    runs = sorted({re.match(r"bench_trace_(c\d+_f\d+)\.json", os.path.basename(p)).group(1)
                   for p in glob.glob(os.path.join(SRC, "bench_trace_c*_f*.json"))})
    for n in runs:
        cfg, dt = int(n[1:n.index("_")]), n[n.index("_") + 1:]
        bench = open(os.path.join(SRC, f"bench_trace_{n}.json")).read().strip().splitlines()[-1]
        e = json.loads(bench)
        shutil.copy(os.path.join(SRC, f"bench_trace_{n}.json"), os.path.join(DST, f"{TAG}_bench_under_rocprof_{n}.json"))
        stats = os.path.join(SRC, f"trace_{n}_kernel_stats.csv")
        shutil.copy(stats, os.path.join(DST, f"{TAG}_kernel_stats_{n}.csv"))
        trace = list(csv.DictReader(open(os.path.join(SRC, f"trace_{n}_kernel_trace.csv"))))
        keep = step_dispatches(trace)
        step_ns = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in trace if int(r["Dispatch_Id"]) in keep]
        md += [f"## config {cfg} {dt}: {NAMES.get(cfg, '')}", "",
               f"bench line under rocprof: {e['value']:.3e} vehicle-steps/s, {e['ms_per_step']:.3f} ms per step", "",
               "| kernel | calls | avg us | share |", "|---|---|---|---|"]
        for r in list(csv.DictReader(open(stats)))[:8]:
            md.append(f"| `{short(r['Name'])}` | {r['Calls']} | {float(r['AverageNs']) / 1e3:.1f} | "
                      f"{float(r['Percentage']):.1f}% |")
        fetch, simk, _ = counters(os.path.join(SRC, f"fetch_{n}_counter_collection.csv"))
        write, _, _ = counters(os.path.join(SRC, f"write_{n}_counter_collection.csv"))
        sq, _, _ = counters(os.path.join(SRC, f"sq_{n}_counter_collection.csv"))
        sq2_path = os.path.join(SRC, f"sq2_{n}_counter_collection.csv")
        sq2 = counters(sq2_path)[0] if os.path.exists(sq2_path) else {}
        grbm, _, grbm_dur = counters(os.path.join(SRC, f"grbm_{n}_counter_collection.csv"))
        f_kib, w_kib = mean(fetch["FETCH_SIZE"]), mean(write["WRITE_SIZE"])
        hbm = (2 * f_kib + w_kib) * 1024
        alg = e["roofline"]["alg_bytes_per_launch"]
        waves = mean(sq["SQ_WAVES"])
        per = lambda c: mean(sq[c]) / waves  # noqa: E731
        wave_cyc, wait_inst, act_valu = mean(sq["SQ_WAVE_CYCLES"]), mean(sq["SQ_WAIT_INST_ANY"]), mean(sq["SQ_ACTIVE_INST_VALU"])
        clk = mean(grbm["GRBM_GUI_ACTIVE"]) / 8 / (mean(grbm_dur) * 1e-9) / 1e9
        trace_avg = mean(step_ns)
        entry = {
            "kernel": simk, "fetch_size_kib_raw": f_kib, "write_size_kib": w_kib, "hbm_bytes_per_launch": hbm,
            "alg_bytes_per_launch": alg,
            "note": "hbm = (2*FETCH_SIZE + WRITE_SIZE)*1024; FETCH_SIZE doubled per the gfx950 calibration",
            "sq_waves": waves, "valu_insts_per_wave": per("SQ_INSTS_VALU"), "lds_insts_per_wave": per("SQ_INSTS_LDS"),
            "salu_insts_per_wave": per("SQ_INSTS_SALU"), "effective_clock_ghz": clk,
            # SQ_ACTIVE_INST_VALU counts quad-cycles (4 shader cycles) per wave
            "valu_active_cycles_per_wave": 4 * act_valu / waves,
            "wait_inst_any_per_wave_cycles": wait_inst / max(wave_cyc, 1),
            "kernel_ns_trace_avg": trace_avg, "launches": len(step_ns), "profile": TAG, "so_sha16": so_sha16}
        if sq2:
            entry["lds_bank_conflict_cycles_per_wave"] = mean(sq2["SQ_LDS_BANK_CONFLICT"]) / waves
            entry["wait_any_per_wave_cycles"] = mean(sq2["SQ_WAIT_ANY"]) / max(wave_cyc, 1)
        md += ["", f"Fused `{simk}` (the step's launches{', warm-ups of the resets excluded' if cfg == 6 else ''}): "
                   f"trace avg {trace_avg / 1e3:.1f} us over {len(step_ns)} launches.",
               f"* HBM per launch (PMC, separate passes): FETCH_SIZE {f_kib:.0f} KiB (x2 gfx950) + WRITE_SIZE "
               f"{w_kib:.0f} KiB = {hbm / 1e6:.1f} MB vs algorithmic {alg / 1e6:.1f} MB.",
               f"* per wave: {per('SQ_INSTS_VALU'):.0f} VALU, {per('SQ_INSTS_LDS'):.0f} LDS, "
               f"{per('SQ_INSTS_SALU'):.0f} SALU instructions ({waves:.0f} waves); VALU-active "
               f"{4 * act_valu / waves:.0f} cycles per wave; WAIT_INST_ANY / WAVE_CYCLES "
               f"{wait_inst / max(wave_cyc, 1):.2f}"
               + (f"; LDS bank conflicts {entry['lds_bank_conflict_cycles_per_wave']:.0f} cycles per wave"
                  if sq2 else ""),
               f"* effective clock (GRBM_GUI_ACTIVE/8/duration): {clk:.2f} GHz", ""]
        if cfg == 3 and "roofline_obs" in e:  # the OccupancyGrid launch (the path's HBM-bound kernel)
            rows = list(csv.DictReader(open(os.path.join(SRC, f"fetch_{n}_counter_collection.csv"))))
            gf = [float(r["Counter_Value"]) for r in rows if "grid_obs_kernel" in r["Kernel_Name"]]
            rows = list(csv.DictReader(open(os.path.join(SRC, f"write_{n}_counter_collection.csv"))))
            gw = [float(r["Counter_Value"]) for r in rows if "grid_obs_kernel" in r["Kernel_Name"]]
            if gf and gw:
                entry["grid_hbm_bytes_per_launch"] = (2 * mean(gf) + mean(gw)) * 1024
                entry["grid_alg_bytes_per_launch"] = e["roofline_obs"]["alg_bytes_per_launch"]
                md += [f"* grid_obs_kernel: {entry['grid_hbm_bytes_per_launch'] / 1e6:.1f} MB per launch vs "
                       f"{entry['grid_alg_bytes_per_launch'] / 1e6:.1f} MB algorithmic", ""]
        out_json[f"config{cfg}_{dt}"] = entry
    json.dump(out_json, open(os.path.join(DST, "pmc_traffic.json"), "w"), indent=1)
    open(os.path.join(DST, f"{TAG}_summary.md"), "w").write("\n".join(md) + "\n")
    print("\n".join(md))


if __name__ == "__main__":
    main()
