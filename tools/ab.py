"""Interleaved A/B of library builds on one GPU box (the method behind every "measured A/B" in
DESIGN.md): each variant is a libggrs_amd.so built by tools/mkvar.sh (ggrs_amd/var/lib_NAME.so;
"cur" = the product library), loaded through GGRS_AMD_LIB; every repetition runs every variant
once, each a fresh bench.py process, so box drift hits all variants alike.

    python3 tools/ab.py --vars cur,prio10 --reps 3 -- --steps 400 --no-cpu-baseline
    python3 tools/ab.py --vars cur,q4 --reps 2 -- --session p2p --sessions-per-gpu 131072 --steps 200

Prints per variant and repetition the bench line's value, wall per step and kernel time per tick
(HIP events), then the medians.  Environment for the bench (e.g. GGRS_BENCH_EVENTS) passes through.
"""
import argparse
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def lib_of(v):
    return os.path.join(ROOT, "ggrs_amd", "libggrs_amd.so") if v == "cur" else \
        os.path.join(ROOT, "ggrs_amd", "var", f"lib_{v}.so")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--vars", required=True)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--timeout", type=int, default=300)
    ap.add_argument("bench_args", nargs=argparse.REMAINDER)
    a = ap.parse_args()
    args = [x for x in a.bench_args if x != "--"]
    vs = a.vars.split(",")
    res = {v: [] for v in vs}
    for rep in range(a.reps):
        for v in vs:
            env = dict(os.environ, GGRS_AMD_LIB=lib_of(v))
            p = subprocess.run(["timeout", "-k", "10", str(a.timeout), sys.executable, "-u", "bench.py"] + args,
                               cwd=ROOT, env=env, capture_output=True, text=True)
            rows = [l for l in p.stdout.splitlines() if l.startswith("{")]
            if p.returncode != 0 or not rows:
                print(f"{v}: failed rc={p.returncode}\n{p.stderr[-2000:]}", flush=True)
                return 1
            d = json.loads(rows[-1])
            r = d["roofline"]
            k = r["kernel_avg_us"] / max(1e-9, r["ticks_per_launch"])
            res[v].append((d["value"], d["ms_per_step"] * 1e3, k))
            print(f"rep {rep} {v:12s} value {d['value']:.4e}  wall/step {d['ms_per_step'] * 1e3:8.2f} us  "
                  f"kernel/tick {k:8.3f} us", flush=True)
    for v in vs:
        val, wall, k = (statistics.median(x[i] for x in res[v]) for i in range(3))
        print(f"median {v:12s} value {val:.4e}  wall/step {wall:8.2f} us  kernel/tick {k:8.3f} us")
    return 0


if __name__ == "__main__":
    sys.exit(main())
