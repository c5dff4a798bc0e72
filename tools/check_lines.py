"""Recompute every bench line's roofline fraction from its committed rocprofv3 summary (VERDICT r05
"next" 1): algorithmic bytes per timed launch (the line's roofline.algorithmic_bytes_per_launch) over
the AverageNs of the line's dominant kernel in profiles/TAG_NAME_kernel_stats.csv (its every
dispatch is a timed launch of the line's shape: GGRS_BENCH_PROFILE=1 and whole-launch warm-ups),
against the 8 TB/s spec; next to it the line's kernel time as clock span + calibrated dispatch overhead
and the range of (rocprofv3 duration - clock span) over the profiled run's timed dispatches (the same
process as the summary): what is left of a difference is the kernel's run-to-run spread.

    python3 tools/check_lines.py r06 [DIR]     # DIR: where bench_TAG_*.jsonl and the summaries are
"""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    tag = sys.argv[1]
    d = sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "profiles")
    worst = 0.0
    print(f"{'line':22s} {'frac':>7s} {'recomputed':>10s} {'diff':>7s} {'kernel_us':>10s} {'rocprof_us':>10s} "
          f"{'calls':>5s} {'clock+ovh_us':>12s} {'ovh range_us':>13s} {'dram/ceil':>9s} bound")
    for path in sorted(glob.glob(os.path.join(d, f"bench_{tag}_*.jsonl"))):
        name = os.path.basename(path)[len(f"bench_{tag}_"):-len(".jsonl")]
        line = json.loads(open(path).readline())
        r = line["roofline"]
        pmc = os.path.join(d, f"{tag}_{name}_pmc.json")
        if not os.path.exists(pmc):
            print(f"{name:22s} no profile")
            continue
        p = json.load(open(pmc))
        k = p.get("dominant_kernel")
        stats = os.path.join(d, f"{tag}_{name}_kernel_stats.csv")
        avg, calls = None, 0
        for row in csv.DictReader(open(stats)):
            if row["Name"].split("(")[0].replace("void ", "").strip() == k:
                avg, calls = float(row["AverageNs"]), int(row["Calls"])
        per_launch = r["algorithmic_bytes_per_launch"]
        if p.get("tick_kernels") or (len(p.get("timed_kernels", [])) > 1):
            # two kernels per tick: the stats' per-dispatch averages of both, per tick
            tot = 0.0
            for row in csv.DictReader(open(stats)):
                n = row["Name"].split("(")[0].replace("void ", "").strip()
                if n in p.get("timed_kernels", []):
                    tot += float(row["AverageNs"])
            avg = tot
        rec = per_launch / (avg * 1e-9) / 1e9 / 8000.0
        diff = rec / r["frac"] - 1.0
        worst = max(worst, abs(diff))
        dc = r.get("dram_frac_of_ceiling")
        # the profiled run's dispatches paired with their own clock spans (same process: no run-to-run
        # spread): the spread of rocprofv3 duration minus clock span over the timed dispatches
        cv = p.get("clock_vs_rocprof") or {}
        rng = f"{cv.get('overhead_min_us', 0):.2f}-{cv.get('overhead_max_us', 0):.2f}" if cv else "-"
        print(f"{name:22s} {r['frac']:7.3f} {rec:10.3f} {100 * diff:6.1f}% {r['kernel_avg_us']:10.2f} {avg / 1e3:10.2f} "
              f"{calls:5d} {r.get('kernel_clock_us', 0):7.2f}+{r.get('dispatch_overhead_us') or 0:4.2f} {rng:>13s} "
              f"{dc if dc is None else round(dc, 2)!s:>9s} {r['bound']}")
    print(f"worst |diff| {100 * worst:.1f}%")


if __name__ == "__main__":
    main()
