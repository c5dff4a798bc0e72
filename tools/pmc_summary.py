"""Fold a tools/prof_round.sh output directory into committed profile files.

usage: python3 tools/pmc_summary.py <gpurun_out/prof_TAG> <TAG> [config_key] [ticks_per_launch]

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
    prof = os.path.join(ROOT, "profiles")
    os.makedirs(prof, exist_ok=True)
    stats = find(os.path.join(d, "stats"), "*kernel_stats.csv")
    summary = {"tag": tag, "config_key": cfg_key, "ticks_per_launch": tpl, "kernels": {}}
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
    # the dominant kernel: the fused steady / P2P kernel of the bench line
    steady = [k for k in summary["kernels"] if "steady_kernel" in k or "p2p_kernel" in k]
    if steady:
        k = max(steady, key=lambda n: summary["kernels"][n].get("total_ns", 0.0))
        e = summary["kernels"][k]
        summary["dominant_kernel"] = k
        if "FETCH_SIZE" in e and "WRITE_SIZE" in e:
            b = (2 * e["FETCH_SIZE"] + e["WRITE_SIZE"]) * 1024
            summary["hbm_bytes_per_launch"] = b
            summary["hbm_bytes_per_tick"] = b / tpl
            summary["hbm_bytes_raw_per_launch"] = (e["FETCH_SIZE"] + e["WRITE_SIZE"]) * 1024
    out = os.path.join(prof, f"{tag}_pmc.json")
    with open(out, "w") as f:
        json.dump(summary, f, indent=1, sort_keys=True)
    print(json.dumps(summary, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
