"""Register and scratch use of every kernel of the product build (the compiler's own report,
-Rpass-analysis=kernel-resource-usage, on the Makefile's flags), one line per kernel.

    python3 tools/resource_report.py > profiles/r06_resource_usage.txt
"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "ggrs_amd", "csrc")
FLAGS = ["-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-ffp-contract=off",
         "-fhip-fp32-correctly-rounded-divide-sqrt", "-DRB_EXPERIMENTS=0"]
TUS = sys.argv[1:] or ["ops_exgame_p2.hip", "ops_exgame_p3.hip", "ops_exgame_p4.hip", "ops_brawler_p2.hip", "ops_stub.hip"]


def main():
    print(f"# {' '.join(FLAGS)} (+ -mllvm -amdgpu-sched-strategy=max-ilp for ops_exgame_p*, as the Makefile)")
    print(f"# {'VGPR':>4s} {'AGPR':>4s} {'SGPR':>4s} {'SGPR spill':>10s} {'VGPR spill':>10s} {'scratch B/lane':>14s} "
          f"{'waves/SIMD':>10s} {'LDS B':>6s}  kernel")
    for tu in TUS:
        extra = ["-mllvm", "-amdgpu-sched-strategy=max-ilp"] if tu.startswith("ops_exgame_p") else []
        with tempfile.TemporaryDirectory() as td:
            p = subprocess.run(["/opt/rocm/bin/hipcc"] + FLAGS + extra + ["--cuda-device-only", "-S", "-o",
                               os.path.join(td, "x.s"), tu, "-Rpass-analysis=kernel-resource-usage"],
                               cwd=CSRC, capture_output=True, text=True)
        rows, cur = [], None
        for line in p.stderr.splitlines():
            m = re.search(r"Function Name: (\S+)", line)
            if m:
                cur = {"name": m.group(1)}
                rows.append(cur)
                continue
            for key, tag in (("VGPRs: ", "v"), ("AGPRs: ", "a"), ("SGPRs: ", "s"), ("SGPRs Spill: ", "ss"),
                             ("VGPRs Spill: ", "vs"), ("ScratchSize [bytes/lane]: ", "sc"),
                             ("Occupancy [waves/SIMD]: ", "o"), ("LDS Size [bytes/block]: ", "l")):
                m = re.search(re.escape(key) + r"(\d+)", line)
                if m and cur is not None:
                    cur[tag] = int(m.group(1))
        print(f"## {tu}")
        for r in rows:
            n = subprocess.run(["c++filt", r["name"]], capture_output=True, text=True).stdout.strip()
            if "kernel" not in n:
                continue
            n = n.replace("void rb::", "").replace("rb::", "")
            n = n.split("(")[0]
            print(f"  {r.get('v', 0):4d} {r.get('a', 0):4d} {r.get('s', 0):4d} {r.get('ss', 0):10d} {r.get('vs', 0):10d} "
                  f"{r.get('sc', 0):14d} {r.get('o', 0):10d} {r.get('l', 0):6d}  {n}")


if __name__ == "__main__":
    main()
