"""Summarise tools/pmc_mix.sh: per-wave, per-tick instruction counts of the P2P kernel."""
import csv
import glob
import sys
from collections import defaultdict

out, name, ticks = sys.argv[1], sys.argv[2], int(sys.argv[3])
files = glob.glob(f"{out}/**/*counter_collection.csv", recursive=True)
acc = defaultdict(lambda: defaultdict(list))
for f in files:
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "p2p_kernel" not in k:
            continue
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, c in acc.items():
    avg = {n: sum(v) / len(v) for n, v in c.items()}
    waves = avg.get("SQ_WAVES", 1.0)
    per = {n: avg[n] / waves / ticks for n in avg if n != "SQ_WAVES"}
    print(name, k.split("(")[0][-60:], "dispatches", len(c.get("SQ_WAVES", [])),
          " ".join(f"{n[3:]}={v:.0f}" for n, v in sorted(per.items())))
