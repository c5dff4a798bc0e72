"""The bench lines of a round and their rocprofv3 evidence, in one table.

    python3 tools/lines.py bench TAG [NAME ...]   # GPU box: every line, fresh process each, with its CPU
                                                  # baseline -> gpurun_out/bench_TAG_NAME.jsonl
    python3 tools/lines.py prof TAG [NAME ...]    # GPU box: the line's own command under rocprofv3
                                                  # --kernel-trace --stats and four --pmc passes
                                                  # (GGRS_BENCH_PROFILE=1) -> gpurun_out/prof_TAG_NAME/
    python3 tools/lines.py fold TAG [NAME ...]    # here: profiles/TAG_NAME_{kernel_stats.csv,pmc.json}
                                                  # (tools/pmc_summary.py), keyed like bench.py's lookup
    python3 tools/lines.py copy TAG [NAME ...]    # here: gpurun_out/bench_TAG_* -> profiles/
    python3 tools/lines.py line TAG [NAME ...]    # GPU box: per line prof, fold (into gpurun_out/prof_TAG),
                                                  # clock calibration, then the bench run

Each line: the bench.py arguments of the bench run, (unused since round 6: the profiled run is
the bench run's own command), bench.py's profile key for it and the ticks per timed launch.
The profiled runs set GGRS_BENCH_PROFILE=1: warm-up ticks one launch each and no live-play
block, so that the dominant kernel's every dispatch in the --stats summary is a timed launch of
the line (its AverageNs is the timed launches' average, the line's frac recomputes from it).  The PMC passes follow MI355X_MICROARCH.md's slot budget: FETCH_SIZE
alone, WRITE_SIZE alone, 8 SQ counters + GRBM, the L2 hit/miss pair; each under its own KILL
timeout (a pass that over-asks for counters hangs instead of failing).
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
X = "ex_game P=2 cd=7 W=8 d=2"
B = "brawler P=2 cd=7 W=8 d=2"
Q = "p2p ex_game P=2 W=8 d=2 rd=2 lag=1,4"
QB = "p2p brawler P=2 W=8 d=2 rd=2 lag=1,4"
Q4 = "p2p ex_game P=4 W=8 d=2 rd=2 lag=1,4"
P2P = "--session p2p"
# name: (bench args, profiled-run args (unused since round 6), profile key, ticks per timed launch).
# P2P warm-ups are whole timed launches (multiples of --ticks-per-launch): the warm-up's dispatches
# of the dominant kernel then have the timed shape too, and the adaptive fan-out sees the same calls
# whether or not the run is profiled.
LINES = {
    "driver": ("--gpus 1 --steps 20 --warmup 5", "--steps 20 --warmup 20 --ticks-per-launch 20", f"{X} S=65536 tpl=20", 20),
    "synctest": ("--steps 400 --warmup 32", "--steps 200 --warmup 50", f"{X} S=65536", 50),
    "synctest1": ("--ticks-per-launch 1 --steps 100 --warmup 32", "--ticks-per-launch 1 --steps 60 --warmup 32",
                  f"{X} S=65536 tpl=1", 1),
    "synctest131k": ("--sessions-per-gpu 131072 --steps 200 --warmup 32", "--sessions-per-gpu 131072 --steps 100 --warmup 50",
                     f"{X} S=131072", 50),
    "synctest1_131k": ("--sessions-per-gpu 131072 --ticks-per-launch 1 --steps 100 --warmup 32",
                       "--sessions-per-gpu 131072 --ticks-per-launch 1 --steps 40 --warmup 32", f"{X} S=131072 tpl=1", 1),
    "synctest1m": ("--sessions-per-gpu 1048576 --steps 20 --warmup 5 --realtime-ticks 32",
                   "--sessions-per-gpu 1048576 --steps 20 --warmup 20 --ticks-per-launch 20", f"{X} S=1048576 tpl=20", 20),
    "synctest1_1m": ("--sessions-per-gpu 1048576 --ticks-per-launch 1 --steps 40 --warmup 16 --realtime-ticks 0",
                     "--sessions-per-gpu 1048576 --ticks-per-launch 1 --steps 20 --warmup 16", f"{X} S=1048576 tpl=1", 1),
    "brawler": ("--game brawler --steps 100 --warmup 32", "--game brawler --steps 100 --warmup 50", f"{B} S=65536", 50),
    "brawler1": ("--game brawler --ticks-per-launch 1 --steps 32 --warmup 8",
                 "--game brawler --ticks-per-launch 1 --steps 16 --warmup 8", f"{B} S=65536 tpl=1", 1),
    "p2p": (f"{P2P} --steps 400 --warmup 50", f"{P2P} --steps 200 --warmup 50", f"{Q} S=65536", 50),
    "p2p131k": (f"{P2P} --sessions-per-gpu 131072 --steps 400 --warmup 50",
                f"{P2P} --sessions-per-gpu 131072 --steps 200 --warmup 50", f"{Q} S=131072", 50),
    "p2p1": (f"{P2P} --ticks-per-launch 1 --steps 400 --warmup 32", f"{P2P} --ticks-per-launch 1 --steps 100 --warmup 32",
             f"{Q} S=65536 tpl=1", 1),
    "p2p1_131k": (f"{P2P} --ticks-per-launch 1 --sessions-per-gpu 131072 --steps 200 --warmup 32",
                  f"{P2P} --ticks-per-launch 1 --sessions-per-gpu 131072 --steps 60 --warmup 32", f"{Q} S=131072 tpl=1", 1),
    "p2p1_1m": (f"{P2P} --ticks-per-launch 1 --sessions-per-gpu 1048576 --steps 50 --warmup 16",
                f"{P2P} --ticks-per-launch 1 --sessions-per-gpu 1048576 --steps 20 --warmup 16", f"{Q} S=1048576 tpl=1", 1),
    "p2p_sparse": (f"{P2P} --sparse-saving --steps 400 --warmup 50", f"{P2P} --sparse-saving --steps 200 --warmup 50",
                   f"{Q} S=65536 sparse", 50),
    "brawler_p2p": (f"--game brawler {P2P} --steps 100 --warmup 50", f"--game brawler {P2P} --steps 100 --warmup 50",
                    f"{QB} S=65536", 50),
    "brawler_p2p_sparse": (f"--game brawler {P2P} --sparse-saving --steps 100 --warmup 50",
                           f"--game brawler {P2P} --sparse-saving --steps 100 --warmup 50", f"{QB} S=65536 sparse", 50),
    # config 4: the default fan-out (per player for ex_game at K = 16), and the one-player form
    "c4": (f"{P2P} --num-players 4 --fanout --steps 100 --warmup 50", f"{P2P} --num-players 4 --fanout --steps 100 --warmup 50",
           f"{Q4} S=65536 fanout per-player", 50),
    "c4_one": (f"{P2P} --num-players 4 --fanout --fanout-mode single --steps 100 --warmup 50",
               f"{P2P} --num-players 4 --fanout --fanout-mode single --steps 100 --warmup 50",
               f"{Q4} S=65536 fanout", 50),
    "c4_k8": (f"{P2P} --num-players 4 --fanout --fanout-k 8 --steps 100 --warmup 50",
              f"{P2P} --num-players 4 --fanout --fanout-k 8 --steps 100 --warmup 50", f"{Q4} S=65536 fanout8", 50),
    "brawler_fan": (f"--game brawler {P2P} --fanout --steps 60 --warmup 100 --ticks-per-launch 20",
                    f"--game brawler {P2P} --fanout --steps 20 --warmup 80", f"{QB} S=65536 fanout tpl=20", 20),
    "wire": (f"{P2P} --wire --steps 200 --warmup 32", f"{P2P} --wire --steps 100 --warmup 16", f"{Q} S=65536 wire tpl=1", 1),
    "wire_replay": (f"{P2P} --wire-replay --steps 400 --warmup 50", f"{P2P} --wire-replay --steps 200 --warmup 50",
                    f"{Q} S=65536 wire-replay", 50),
}
PMC = {
    "pmc_fetch": "FETCH_SIZE",
    "pmc_write": "WRITE_SIZE",
    "pmc_sq": "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY "
              "SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE",
    "pmc_l2": "TCC_HIT_sum TCC_MISS_sum",
}


def run(cmd, log, timeout):
    print(f"=== {' '.join(cmd)[:160]}", flush=True)
    with open(log, "w") as f:
        try:
            rc = subprocess.run(["timeout", "-s", "KILL", str(timeout)] + cmd, stdout=f, stderr=subprocess.STDOUT,
                                cwd=ROOT).returncode
        except OSError as e:
            print(e)
            return 1
    print(f"=== rc={rc}", flush=True)
    return rc


def bench(tag, names):
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    for k in ("GGRS_BENCH_PROFILE", "GGRS_BENCH_META"):
        os.environ.pop(k, None)
    for n in names:
        out = os.path.join(ROOT, "gpurun_out", f"bench_{tag}_{n}")
        rc = run(["python3", "-u", "bench.py"] + LINES[n][0].split(), out + ".log", 900)
        rows = [l for l in open(out + ".log") if l.startswith("{")]
        with open(out + ".jsonl", "w") as f:
            f.writelines(rows)
        for l in rows:
            d = json.loads(l)
            r, c = d["roofline"], d.get("cpu_baseline") or {}
            print(f"  {n}: value {d['value']:.4g} {d['unit']}  ms/step {d['ms_per_step']:.4f}  kernel_us "
                  f"{r.get('kernel_avg_us', 0):.1f}  frac {r['frac']:.3f}  bound {r.get('bound')}  cpu {c.get('value', 0):.3g}",
                  flush=True)
        if rc != 0:
            return rc
    return 0


def prof(tag, names):
    os.environ.setdefault("TMPDIR", "/tmp")
    for n in names:
        d = os.path.join(ROOT, "gpurun_out", f"prof_{tag}_{n}")
        os.makedirs(d, exist_ok=True)
        # the line's own command, timed by the kernel's clock (which rocprofv3 does not perturb), its
        # warm-up one launch per tick (GGRS_BENCH_PROFILE=1)
        os.environ["GGRS_BENCH_PROFILE"] = "1"
        base = ["python3", "-u", "bench.py"] + LINES[n][0].split() + ["--no-cpu-baseline"]
        passes = [("stats", ["--kernel-trace", "--stats"])] + [(k, ["--pmc"] + v.split()) for k, v in PMC.items()]
        for sub, args in passes:
            os.environ["GGRS_BENCH_META"] = os.path.join(d, f"{sub}_meta.json")
            cmd = ["rocprofv3"] + args + ["-d", os.path.join(d, sub), "-o", "run", "--output-format", "csv", "--"] + base
            if run(cmd, os.path.join(d, sub + ".log"), 300) != 0:
                return 1
    return 0


def line(tag, names):
    """GPU box: per line, the profiled runs, their fold into GGRS_PROFILES_OUT (default
    gpurun_out/prof_TAG), the clock calibration over the lines profiled so far, then the bench
    run, which reads that calibration and profile: the line and the profile it is checked
    against come from the same box, minutes apart."""
    out = os.environ.setdefault("GGRS_PROFILES_OUT", os.path.join(ROOT, "gpurun_out", f"prof_{tag}"))
    os.makedirs(out, exist_ok=True)
    for n in names:
        if prof(tag, [n]) != 0:
            return 1
        subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_summary.py"),
                        os.path.join(ROOT, "gpurun_out", f"prof_{tag}_{n}"), f"{tag}_{n}", LINES[n][2], str(LINES[n][3])],
                       check=True, stdout=subprocess.DEVNULL)
        subprocess.run([sys.executable, os.path.join(ROOT, "tools", "clock_calib.py"), tag], check=True)
        if bench(tag, [n]) != 0:
            return 1
    return 0


def fold(tag, names):
    for n in names:
        d = os.path.join(ROOT, "gpurun_out", f"prof_{tag}_{n}")
        if not os.path.isdir(d):
            print(f"skip {n}")
            continue
        subprocess.run(["python3", os.path.join(ROOT, "tools", "pmc_summary.py"), d, f"{tag}_{n}", LINES[n][2],
                        str(LINES[n][3])], check=True, stdout=subprocess.DEVNULL)
        print(f"{tag}_{n} <- {LINES[n][2]}")
    return 0


def copy(tag, names):
    for n in names:
        src = os.path.join(ROOT, "gpurun_out", f"bench_{tag}_{n}.jsonl")
        if os.path.exists(src):
            with open(src) as f, open(os.path.join(ROOT, "profiles", f"bench_{tag}_{n}.jsonl"), "w") as g:
                g.write(f.read())
    return 0


if __name__ == "__main__":
    what, tag = sys.argv[1], sys.argv[2]
    names = sys.argv[3:] or list(LINES)
    bad = [n for n in names if n not in LINES]
    if bad:
        raise SystemExit(f"unknown lines {bad}; known: {list(LINES)}")
    sys.exit({"bench": bench, "prof": prof, "fold": fold, "copy": copy, "line": line}[what](tag, names))
