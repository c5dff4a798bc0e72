"""Fold a tools/prof_round.sh output directory into committed profile files.

usage: python3 tools/pmc_summary.py <gpurun_out/prof_TAG> <TAG> [config_key] [ticks_per_launch]

The profiled runs (tools/lines.py prof) run the bench line's own command with
GGRS_BENCH_PROFILE=1 and write <pass>_meta.json (bench.py write_meta): the profile key,
the kernel-source id and fan-out state the launches ran with, and the kernel's own clock
span of every timed launch.  Those keys override the arguments, and every timed dispatch
of the kernel trace is paired with its clock span ("clock_vs_rocprof": rocprofv3's
duration minus the clock span, the dispatch overhead bench.py adds).

Writes profiles/<TAG>_kernel_stats.csv (rocprofv3 --stats, verbatim) and
profiles/<TAG>_pmc.json: per-kernel average counters per launch, and for the
dominant kernel (steady_kernel, or p2p_kernel for a P2P bench) the HBM bytes per launch and per tick:
    hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024
FETCH_SIZE/WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE counts half the bytes of
a wide coalesced read (MI355X_MICROARCH.md §HBM), hence the factor 2 on the
read side (the raw values are kept too).
"""
import csv
import glob
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def find(d, pattern):
    return sorted(glob.glob(os.path.join(d, "**", pattern), recursive=True))


def counters(d):
    """{kernel_name: {counter: [per-dispatch values]}} from every *counter_collection.csv under d."""
    out = defaultdict(lambda: defaultdict(list))
    for path in find(d, "*counter_collection.csv"):
        per_dispatch = defaultdict(lambda: defaultdict(float))
        names = {}
        with open(path) as f:
            for row in csv.DictReader(f):
                disp = row.get("Dispatch_Id") or row.get("Correlation_Id")
                names[disp] = row["Kernel_Name"]
                per_dispatch[disp][row["Counter_Name"]] += float(row["Counter_Value"])
        for disp, cs in per_dispatch.items():
            for c, v in cs.items():
                out[names[disp]][c].append(v)
    return out


def short(name):
    return name.split("(")[0].replace("void ", "").strip()


def main():
    d, tag = sys.argv[1], sys.argv[2]
    cfg_key = sys.argv[3] if len(sys.argv) > 3 else "ex_game P=2 cd=7 W=8 d=2 S=65536"
    tpl = int(sys.argv[4]) if len(sys.argv) > 4 else 50
    prof = os.environ.get("GGRS_PROFILES_OUT") or os.path.join(ROOT, "profiles")  # (the GPU box: under gpurun_out)
    os.makedirs(prof, exist_ok=True)
    stats = find(os.path.join(d, "stats"), "*kernel_stats.csv")
    summary = {"tag": tag, "config_key": cfg_key, "ticks_per_launch": tpl, "kernels": {}}
    meta_path = os.path.join(d, "stats_meta.json")
    meta = json.load(open(meta_path)) if os.path.exists(meta_path) else {}
    if meta:
        summary["config_key"] = meta["config_key"]
        summary["source_id"] = meta.get("source_id")
        summary["fanout_state"] = meta.get("fanout_state")
        summary["line_kernel_avg_us"] = meta.get("kernel_avg_us")
        summary["bytes_per_launch"] = meta.get("bytes_per_launch")
    if stats:
        shutil.copy(stats[0], os.path.join(prof, f"{tag}_kernel_stats.csv"))
        with open(stats[0]) as f:
            for row in csv.DictReader(f):
                summary["kernels"].setdefault(short(row["Name"]), {}).update(
                    {"calls": int(row["Calls"]), "avg_ns": float(row["AverageNs"]),
                     "total_ns": float(row["TotalDurationNs"])})
    for sub in ("pmc_fetch", "pmc_write", "pmc_sq", "pmc_l2"):
        for k, cs in counters(os.path.join(d, sub)).items():
            ent = summary["kernels"].setdefault(short(k), {})
            for c, vals in cs.items():
                # steady launches of the measured shape: drop the warm-up launch (first)
                v = vals[1:] if len(vals) > 1 else vals
                ent[c] = sum(v) / len(v)
    # the dominant kernel: the fused steady / P2P kernel of the bench line; with the run's meta, among
    # the kernels of its timed launches (the trace's last dispatches, one per clock span)
    steady = [k for k in summary["kernels"] if "steady_kernel" in k or "p2p_kernel" in k or "fanout" in k]
    spans0 = meta.get("clock_spans_us")
    traces0 = find(os.path.join(d, "stats"), "*kernel_trace.csv")
    if spans0 and traces0:
        with open(traces0[0]) as f:
            rows0 = [r for r in csv.DictReader(f) if short(r["Kernel_Name"]) in steady]
        rows0.sort(key=lambda r: int(r["Start_Timestamp"]))
        timed = {short(r["Kernel_Name"]) for r in rows0[-len(spans0):]}
        if timed:
            steady = [k for k in steady if k in timed]
            summary["timed_kernels"] = sorted(timed)
    if steady:
        k = max(steady, key=lambda n: summary["kernels"][n].get("total_ns", 0.0))
        e = summary["kernels"][k]
        summary["dominant_kernel"] = k
        if "FETCH_SIZE" in e and "WRITE_SIZE" in e:
            b = (2 * e["FETCH_SIZE"] + e["WRITE_SIZE"]) * 1024
            summary["hbm_bytes_per_launch"] = b
            summary["hbm_bytes_per_tick"] = b / tpl
            # the speculative fan-out runs one p2p_kernel and one fan-out kernel per tick: a tick's
            # traffic is both dispatches' (whichever of the two takes longer)
            fan = [o for o in steady if "fanout" in o]
            if fan and any("p2p_kernel" in o for o in steady):
                for o in steady:
                    if o != k and ("fanout" in o or "p2p_kernel" in o) and "FETCH_SIZE" in summary["kernels"][o]:
                        eo = summary["kernels"][o]
                        summary["hbm_bytes_per_tick"] += (2 * eo["FETCH_SIZE"] + eo["WRITE_SIZE"]) * 1024 / tpl
                        summary["tick_kernels"] = [k, o]
            summary["hbm_bytes_raw_per_launch"] = (e["FETCH_SIZE"] + e["WRITE_SIZE"]) * 1024
        # Issue side (MI355X_MICROARCH.md: 1,024 SIMDs, a wave64 VALU instruction occupies a SIMD-32
        # for 2 cycles at full rate; SQ_BUSY_CYCLES sums the 32 shader engines' SQs, GRBM_GUI_ACTIVE
        # the 8 XCDs).  valu_issue_frac = SQ_INSTS_VALU * 2 / (1024 * elapsed cycles): the share of
        # VALU issue slots used, a lower bound (f64 and transcendental ops take more than 2 cycles).
        if "SQ_INSTS_VALU" in e and e.get("SQ_BUSY_CYCLES") and e.get("avg_ns"):
            cyc = e["SQ_BUSY_CYCLES"] / 32.0
            summary["issue"] = {
                "valu_insts_per_launch": e["SQ_INSTS_VALU"],
                "valu_insts_per_wave": e["SQ_INSTS_VALU"] / max(1.0, e.get("SQ_WAVES", 1.0)),
                "elapsed_cycles": cyc,
                "clock_GHz_sq": cyc / e["avg_ns"],
                "clock_GHz_grbm": (e["GRBM_GUI_ACTIVE"] / 8.0 / e["avg_ns"]) if e.get("GRBM_GUI_ACTIVE") else None,
                "valu_issue_frac": e["SQ_INSTS_VALU"] * 2.0 / (1024.0 * cyc),
                # every vector and scalar instruction takes a SIMD issue slot (tools/ubench_mix.hip: a
                # scalar op beside the other wave's vector ops still costs ~3 cycles of the SIMD); the
                # SIMD issues about one instruction per quad-cycle at this instruction mix (two-point PMC,
                # profiles/r05_twopoint_pmc.json), so this is the issue limiter's utilisation
                "salu_insts_per_wave": e.get("SQ_INSTS_SALU", 0.0) / max(1.0, e.get("SQ_WAVES", 1.0)),
                "issue_per_quad": (e["SQ_INSTS_VALU"] + e.get("SQ_INSTS_SALU", 0.0)) / (1024.0 * cyc / 4.0),
                "active_inst_valu_frac": e.get("SQ_ACTIVE_INST_VALU", 0.0) * 4.0 / (1024.0 * cyc),
                "issue_stall_frac": e.get("SQ_WAIT_INST_ANY", 0.0) / max(1.0, e.get("SQ_WAVE_CYCLES", 1.0)),
                "waves_dispatched_per_simd": e.get("SQ_WAVES", 0.0) / 1024.0,
                # SQ_WAVE_CYCLES counts quad-cycles (MI355X_MICROARCH.md, s_memtime vs SQ PMC units):
                # the average number of waves resident per SIMD over the kernel
                "waves_per_simd": e.get("SQ_WAVE_CYCLES", 0.0) * 4.0 / (1024.0 * cyc),
                "l2_hit": (e["TCC_HIT_sum"] / (e["TCC_HIT_sum"] + e["TCC_MISS_sum"]))
                if e.get("TCC_HIT_sum") is not None and e.get("TCC_MISS_sum") is not None else None,
            }
    # the timed dispatches' rocprofv3 durations against the kernel's own clock spans (same run)
    spans = meta.get("clock_spans_us")
    traces = find(os.path.join(d, "stats"), "*kernel_trace.csv")
    if spans and traces and summary.get("dominant_kernel"):
        with open(traces[0]) as f:
            rows = [r for r in csv.DictReader(f) if ("p2p_kernel" in r["Kernel_Name"] or "steady_kernel" in r["Kernel_Name"]
                                                     or "fanout_kernel" in r["Kernel_Name"])]
        rows.sort(key=lambda r: int(r["Start_Timestamp"]))
        # timed launches = the trace's last len(spans) dispatches of the kernel(s) the clock covers
        # (the two-launch fan-out alternates p2p_kernel and fanout_kernel)
        cand = rows
        if len(cand) >= len(spans):
            cand = cand[-len(spans):]
            dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in cand]
            diff = sorted(a - b for a, b in zip(dur, spans))
            summary["clock_vs_rocprof"] = {
                "dispatches": len(dur), "rocprof_avg_us": sum(dur) / len(dur), "clock_avg_us": sum(spans) / len(spans),
                "overhead_median_us": diff[len(diff) // 2], "overhead_min_us": diff[0], "overhead_max_us": diff[-1]}
    out = os.path.join(prof, f"{tag}_pmc.json")
    with open(out, "w") as f:
        json.dump(summary, f, indent=1, sort_keys=True)
    print(json.dumps(summary, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
