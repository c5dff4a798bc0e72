"""Fold the clock-vs-rocprofv3 pairs of a round's profiles into bench.py's dispatch overhead.

    python3 tools/clock_calib.py r06      # profiles/r06_*_pmc.json -> profiles/r06_clock_calibration.json

Every profiled line (tools/lines.py prof, GGRS_BENCH_PROFILE=1) ran its own command under
rocprofv3 --kernel-trace; tools/pmc_summary.py paired each timed dispatch's rocprofv3 duration
with the kernel's own clock span of the same launch (rb_launch_clock_*: first wave start to last
wave end on the 100 MHz constant clock); the line's overhead is the mean difference.  It
is the dispatch's setup before the first wave plus its end-of-kernel release after the
last: bench.py adds it, per launch, to the clock span of the launches it times (by the line's
configuration, else the median over all lines), so that its kernel time is rocprofv3's.
"""
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    tag = sys.argv[1]
    prof = os.environ.get("GGRS_PROFILES_OUT") or os.path.join(ROOT, "profiles")
    by, rows = {}, []
    for path in sorted(glob.glob(os.path.join(prof, f"{tag}_*_pmc.json"))):
        d = json.load(open(path))
        c = d.get("clock_vs_rocprof")
        if not c:
            continue
        # the mean difference: the line's clock average plus it is then its dispatches' rocprofv3 average
        # (the --stats AverageNs a recomputation starts from)
        by[d["config_key"]] = round(c["rocprof_avg_us"] - c["clock_avg_us"], 3)
        rows.append({"profile": "profiles/" + os.path.basename(path), "config_key": d["config_key"], **c})
    if not rows:
        raise SystemExit("no profile with clock_vs_rocprof")
    med = sorted(by.values())[len(by) // 2]
    out = {"what": "rocprofv3 dispatch duration minus the kernel's own clock span (first wave start to last wave "
                   "end), per timed dispatch of each profiled bench line, the mean per line (by_config; the median "
                   "over lines for a configuration not profiled); bench.py adds it to the clock spans it measures", "dispatch_overhead_us": med, "by_config": by, "lines": rows}
    with open(os.path.join(prof, f"{tag}_clock_calibration.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps({"dispatch_overhead_us": med, "lines": len(rows)}))


if __name__ == "__main__":
    main()
