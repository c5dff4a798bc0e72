"""Fold tools/calib_fetch.hip's rocprofv3 PMC passes into the counted/known byte ratios.

    python3 tools/calib_fetch.py gpurun_out/calib_fetch r06   # -> profiles/r06_calib_fetch.json

<dir>/fetch and <dir>/write hold the --pmc FETCH_SIZE and --pmc WRITE_SIZE runs (csv output);
every dispatch of read_kernel<B> / write_kernel<B> touched 4 GiB exactly once, coalesced."""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KNOWN = 4 << 30


def per_kernel(d, counter):
    vals = defaultdict(list)
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        per = defaultdict(float)
        name = {}
        with open(path) as f:
            for r in csv.DictReader(f):
                if r["Counter_Name"] != counter:
                    continue
                k = r.get("Dispatch_Id") or r.get("Correlation_Id")
                per[k] += float(r["Counter_Value"])
                name[k] = r["Kernel_Name"]
        for k, v in sorted(per.items(), key=lambda kv: int(kv[0])):
            m = re.search(r"(read|write)_kernel<(\d+)>", name[k])
            if m:
                vals[f"{m.group(1)}{m.group(2)}"].append(v * 1024 / KNOWN)
    return vals


def main():
    d, tag = sys.argv[1], sys.argv[2]
    out = {"what": "counted bytes / known bytes per dispatch (4 GiB touched once, coalesced, past the 256 MiB "
                   "Infinity Cache): FETCH_SIZE for read_kernel<B>, WRITE_SIZE for write_kernel<B>, B bytes per lane",
           "fetch_ratio": {}, "write_ratio": {}}
    for k, v in per_kernel(os.path.join(d, "fetch"), "FETCH_SIZE").items():
        if k.startswith("read"):
            out["fetch_ratio"][k] = sum(v) / len(v)
    for k, v in per_kernel(os.path.join(d, "write"), "WRITE_SIZE").items():
        if k.startswith("write"):
            out["write_ratio"][k] = sum(v) / len(v)
    with open(os.path.join(ROOT, "profiles", f"{tag}_calib_fetch.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
