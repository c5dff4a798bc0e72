"""Fold tools/pmc_twopoint.sh's passes into one table per batch size (steady_kernel launches
only): per-launch counter means, and the derived per-SIMD rates that name the limiter.
usage: python3 tools/pmc_twopoint.py TAG [SIZES...] > profiles/<TAG>_twopoint.json"""
import collections
import csv
import glob
import json
import sys

tag = sys.argv[1]
sizes = [int(x) for x in sys.argv[2:]] or [65536, 131072]
KERNEL = "steady_kernel"
SIMDS, CUS = 1024, 256
out = {"tag": tag, "kernel": "rb::steady_kernel<rb::ExGame<2, true>, 7, false> (50-tick launches)", "sizes": {}}
for S in sizes:
    acc = collections.defaultdict(list)
    dur = []
    for path in sorted(glob.glob(f"gpurun_out/pmc2_{tag}_{S}_p*/run_counter_collection.csv")):
        per = collections.defaultdict(dict)
        for r in csv.DictReader(open(path)):
            if KERNEL not in r["Kernel_Name"] or int(r["Grid_Size"]) != S * 2:
                continue
            d = int(r["Dispatch_Id"])
            per[d][r["Counter_Name"]] = per[d].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            per[d]["_ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        # the first steady launch of a run is the warmup's (a different tick count): skip it
        for d in sorted(per)[1:]:
            for k, v in per[d].items():
                acc[k].append(v)
    m = {k: sum(v) / len(v) for k, v in acc.items()}
    if not m:
        continue
    clk = m["GRBM_GUI_ACTIVE"] / 8 / (m["_ns"] * 1e-9) / 1e9  # GHz (8 XCDs summed)
    cyc = m["GRBM_GUI_ACTIVE"] / 8  # elapsed cycles of the launch
    waves = m.get("SQ_WAVES", 0)
    ticks = 50
    r = {"launch_us": m["_ns"] / 1e3, "clock_GHz": clk, "elapsed_cycles": cyc, "waves": waves,
         "waves_per_simd_dispatched": waves / SIMDS,
         "counters_per_launch": {k: v for k, v in sorted(m.items()) if not k.startswith("_")}}
    # SQ_WAVE_CYCLES / WAIT / ACTIVE are in quad-cycles, summed over waves
    wc = m["SQ_WAVE_CYCLES"] * 4
    r["waves_resident_per_simd"] = wc / cyc / SIMDS
    r["wave_time_split"] = {"wait_any (s_waitcnt / dependency on memory)": m["SQ_WAIT_ANY"] * 4 / wc,
                            "wait_inst_any (issue stall: not selected / pipe busy)": m["SQ_WAIT_INST_ANY"] * 4 / wc,
                            "active_inst_any (issuing)": m["SQ_ACTIVE_INST_ANY"] * 4 / wc}
    ni = {k: m.get(k, 0.0) for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_SMEM", "SQ_INSTS_BRANCH",
                                     "SQ_INSTS_VMEM_WR", "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_MUL_F64",
                                     "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_TRANS_F32", "SQ_INSTS_VALU_CVT",
                                     "SQ_INSTS_VALU_INT32", "SQ_INSTS_VALU_FMA_F32", "SQ_INSTS_VALU_MUL_F32",
                                     "SQ_INSTS_VALU_ADD_F32")}
    r["insts_per_wave_tick"] = {k: v / waves / ticks for k, v in ni.items()}
    f64 = ni["SQ_INSTS_VALU_FMA_F64"] + ni["SQ_INSTS_VALU_MUL_F64"] + ni["SQ_INSTS_VALU_ADD_F64"]
    allv = ni["SQ_INSTS_VALU"]
    # per-SIMD issue: every instruction of a wave takes one issue slot; VALU throughput per SIMD
    # 2 cycles per wave64 f32 op (SIMD-32), f64 and transcendental ops 4 (half rate) as a model
    r["per_simd"] = {
        "valu_per_cycle": allv / SIMDS / cyc,
        "all_insts_per_cycle": (allv + ni["SQ_INSTS_SALU"] + ni["SQ_INSTS_SMEM"] + ni["SQ_INSTS_BRANCH"]) / SIMDS / cyc,
        "valu_pipe_busy_model": (2 * (allv - f64 - ni["SQ_INSTS_VALU_TRANS_F32"]) + 4 * (f64 + ni["SQ_INSTS_VALU_TRANS_F32"])) / SIMDS / cyc,
        "active_inst_valu_frac": m["SQ_ACTIVE_INST_VALU"] * 4 / SIMDS / cyc,
        "valu2_dual_issue_quads_frac": m.get("SQ_ACTIVE_INST_VALU2", 0.0) / SIMDS / (cyc / 4),
        "salu_active_frac_per_cu": m.get("SQ_ACTIVE_INST_SCA", 0.0) * 4 / CUS / cyc,
    }
    if "SQC_ICACHE_MISSES" in m:
        r["icache_miss_rate"] = m["SQC_ICACHE_MISSES"] / max(1.0, m["SQC_ICACHE_MISSES"] + m["SQC_ICACHE_HITS"])
    if "TCC_HIT_sum" in m:
        r["l2_hit"] = m["TCC_HIT_sum"] / max(1.0, m["TCC_HIT_sum"] + m["TCC_MISS_sum"])
    r["session_frames_per_s_kernel"] = S * ticks * 8 / (m["_ns"] * 1e-9)
    out["sizes"][str(S)] = r
json.dump(out, sys.stdout, indent=1)
print()
