"""bench.py — session-frames resimulated per second at an 8-frame rollback.

Workload (BASELINE.json configs[1]): 65,536 independent ex_game SyncTest
sessions per GPU, 2 players, check_distance 7 (max_prediction 8), input
delay 2: every step (= one tick) loads frame c-7, resimulates and re-saves 7
frames, saves frame c and advances to c+1 — 8 AdvanceFrames per session.
Synthetic seeded inputs (ggrs_amd.synth), resident in HBM before timing.

N>1: one process per GPU (torch.distributed.run), sessions sharded (weak
scaling: sessions per GPU fixed), no data-path collective; every
--report-interval ticks the per-session desync reports (checksum of the last
settled frame + mismatch flag) are all-gathered over RCCL.

--game brawler runs BASELINE configs[2] instead: the fixed-point 256-entity
brawler (8 KiB of integer state per session, one wavefront per session),
same session count and rollback shape; its snapshot ring (4 GiB at 65,536
sessions) does not fit any cache, so it is the HBM-bound line.

Prints ONE JSON line (rank 0).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "session-frames resimulated/sec (node) at 8-frame rollback; % HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec


def algorithmic_bytes_per_session_tick(P: int, cd: int, nw: int, cs_bytes: int, in_bytes: int) -> int:
    """Bytes one steady-state tick must move per session: SURVEY.md section 8(d)
    B_tick = S_state * (1 load + cd saves) + cd * cs_bytes * 2 (checksum written
    + first-seen checksum read) + (cd + 1) * P * in_bytes (the inputs of every
    AdvanceFrame) + 4 (session status word).  S_state = 4 * nw: the per-session
    frame word is implicit (the batch-uniform cell tag).
    Values the fused kernel carries in registers across ticks still count: the
    figure is the algorithm's, not the implementation's."""
    return 4 * nw * (1 + cd) + cd * cs_bytes * 2 + (cd + 1) * P * in_bytes + 4


def init_dist(dist, dev):
    """RCCL over xGMI (backend "nccl"); GGRS_BENCH_BACKEND=gloo rehearses the
    multi-rank path with several ranks on one GPU (RCCL refuses duplicate GPUs)."""
    backend = os.environ.get("GGRS_BENCH_BACKEND", "nccl")
    if backend == "nccl":
        dist.init_process_group("nccl", device_id=dev)
    else:
        dist.init_process_group(backend)


def cpu_threads():
    """Host cores this process may use: the CPU affinity mask, further bounded by
    a cgroup CPU quota when one is set (cgroup v2 cpu.max).  The north star asks
    for the reference CPU path "across all host cores of the same box"; on a
    shared GPU box that is the CPU share this job is given, not os.cpu_count()
    (reported next to it)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    return max(1, n)


def cpu_info(threads):
    return {"cores": threads, "host_cpus": os.cpu_count()}


def free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n):
    """--gpus N > 1 without an outside launcher: start N rank processes (one per
    GPU, RANK/LOCAL_RANK/WORLD_SIZE set, rendezvous on 127.0.0.1) before this
    process touches the GPU; rank 0's stdout (the JSON line) passes through,
    the other ranks' stdout goes to stderr.  Returns the worst exit code."""
    import subprocess
    port = free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      stdout=None if r == 0 else sys.stderr))
    rcs = [None] * n
    try:
        while any(rc is None for rc in rcs):
            for i, p in enumerate(procs):
                if rcs[i] is None:
                    rcs[i] = p.poll()
                    if rcs[i] not in (None, 0):  # one rank failed: the others would hang in a collective
                        for q in procs:
                            if q.poll() is None:
                                q.terminate()
            time.sleep(0.05)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    return max(abs(rc) for rc in rcs)


def cpu_baseline(args, P):
    """The reference CPU path timed on this box's host cores: the C++
    line-faithful restatement with the reference's allocation pattern (kind
    "port"), and for ex_game next to it the optimized CPU loop SURVEY 8(d)
    asks for ("optimized": oracle/soa_baseline.cpp, same arithmetic and
    checksums, no per-request allocation, cache-blocked sessions)."""
    from oracle import oracle as O
    threads = cpu_threads()
    S, warm, ticks = args.cpu_sessions, 16, args.cpu_ticks
    fn = O.bench_brawler if args.game == "brawler" else O.bench_exgame
    if S is None:
        S = 4096 if args.game == "brawler" else 65536
    if ticks is None:
        ticks = 256 if args.game == "brawler" else 384
    secs, nerr = fn(P, args.check_distance, args.input_delay, args.max_prediction, S, warm, ticks, threads, args.seed)
    sf = S * ticks * (args.check_distance + 1)
    out = {"value": sf / secs, "unit": "session-frames/s", **cpu_info(threads), "kind": "port",
           "sample": f"{S} {args.game} sessions x {ticks} steady-state ticks ({sf} session-frames) of the C++ "
                     f"line-faithful restatement (reference allocation pattern), {threads} host threads "
                     f"(every core this job may use), {secs:.2f} s wall, {nerr} errors"}
    if args.game == "ex_game":
        oticks = 512
        osecs, oerr = O.bench_exgame_soa(P, args.check_distance, args.input_delay, args.max_prediction, S, warm,
                                         oticks, threads, args.seed)
        osf = S * oticks * (args.check_distance + 1)
        out["optimized"] = {
            "value": osf / osecs, "unit": "session-frames/s", **cpu_info(threads), "kind": "optimized",
            "sample": f"{S} ex_game sessions x {oticks} steady-state ticks ({osf} session-frames), same inputs, "
                      f"State::advance arithmetic (glibc sinf/cosf) and fletcher16 as the port; per-session "
                      f"snapshot rings in flat arrays, no per-request allocation, closed-form fletcher16, "
                      f"256-session blocks kept in cache across ticks (oracle/soa_baseline.cpp), {threads} host "
                      f"threads, {osecs:.2f} s wall, {oerr} errors"}
    return out


def measured_copy_gbps(dev, nbytes=1 << 30, iters=10):
    """Device-to-device copy bandwidth (read + write bytes / time) of a 1 GiB
    buffer: the STREAM-copy ceiling SURVEY.md 8(d) asks to report next to the
    8 TB/s spec peak.  Runs outside every timed region."""
    import torch
    a = torch.empty(nbytes // 4, dtype=torch.int32, device=dev)
    b = torch.empty_like(a)
    b.copy_(a)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        b.copy_(a)
    e1.record()
    e1.synchronize()
    gbps = 2 * nbytes * iters / (e0.elapsed_time(e1) / 1e3) / 1e9
    del a, b
    return gbps


P2P_ONLY_SOURCES = ("p2p.hpp", "p2p_engine.hip", "wire.hip")


def source_id(family="p2p"):
    """Identity of the device code a profile describes: a hash of the kernel sources, the
    header and the build flags (ggrs_amd/csrc/*.hip, *.hpp, Makefile, include/*), the same
    for every build of the same sources.  A PMC profile is used only for the sources it was
    taken on.  The SyncTest family ("synctest") leaves out the sources only the P2P batches
    compile into their kernels (P2P_ONLY_SOURCES: p2p_kernel, the fan-out, the wire codec),
    so a P2P change does not orphan the SyncTest profiles."""
    import glob
    import hashlib
    h = hashlib.sha256()
    files = sorted(glob.glob(os.path.join(ROOT, "ggrs_amd", "csrc", "*.hip")) +
                   glob.glob(os.path.join(ROOT, "ggrs_amd", "csrc", "*.hpp")) +
                   [os.path.join(ROOT, "ggrs_amd", "csrc", "Makefile")] +
                   glob.glob(os.path.join(ROOT, "include", "*.h*")))
    if family == "synctest":
        files = [f for f in files if os.path.basename(f) not in P2P_ONLY_SOURCES]
    for f in files:
        h.update(os.path.basename(f).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def pmc_profile(cfg_key, fanout_state=None, family="p2p"):
    """The committed rocprofv3 PMC summary of this exact configuration and launch shape
    (profiles/*pmc*.json, written by tools/pmc_summary.py), taken on the current kernel
    sources (`source_id`) and, for a fan-out line, with the fan-out in the same state
    ("active" / "paused") as in the launches timed here; the newest round's file wins.
    None when there is none: the line is then `unprofiled`.  Its hbm_bytes_per_tick is
    FETCH_SIZE x2 + WRITE_SIZE (MI355X_MICROARCH.md's gfx950 correction, checked for this
    engine's access widths by tools/calib_fetch.hip); its `issue` block holds SQ_INSTS_VALU,
    the clock and the VALU issue-slot fraction."""
    import glob
    src = source_id(family)
    best = None
    paths = sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc*.json")))
    if os.environ.get("GGRS_PROFILES_OUT"):  # (tools/lines.py line: this call's own profiles, folded on the box)
        paths += sorted(glob.glob(os.path.join(os.environ["GGRS_PROFILES_OUT"], "*pmc*.json")))
    for path in paths:
        try:
            d = json.load(open(path))
        except Exception:
            continue
        if (d.get("config_key") == cfg_key and d.get("hbm_bytes_per_tick") and d.get("source_id") == src
                and (fanout_state is None or d.get("fanout_state") == fanout_state)):
            best = dict(d, file="profiles/" + os.path.basename(path))
    return best


CLOCK_CAL_FILE = os.path.join(ROOT, "profiles", "r06_clock_calibration.json")


def dispatch_overhead_us(cfg_key=None):
    """What rocprofv3's dispatch duration adds to the kernel's own clock (first wave start to
    last wave end, rb_launch_clock_*): the dispatch's setup before the first wave and its
    end-of-kernel release after the last, per launch.  Calibrated by running the bench lines
    under rocprofv3 --kernel-trace and pairing every timed dispatch with its clock span
    (tools/clock_calib.py -> profiles/r06_clock_calibration.json): the median of this line's
    configuration when it was profiled, else the median over all lines; (0, None) when absent."""
    path = CLOCK_CAL_FILE
    out = os.environ.get("GGRS_PROFILES_OUT")  # (tools/lines.py line: this call's own calibration)
    if out and os.path.exists(os.path.join(out, os.path.basename(CLOCK_CAL_FILE))):
        path = os.path.join(out, os.path.basename(CLOCK_CAL_FILE))
    try:
        d = json.load(open(path))
        by = d.get("by_config", {})
        v = by[cfg_key] if cfg_key in by else d["dispatch_overhead_us"]
        return float(v), "profiles/" + os.path.basename(path)
    except (OSError, KeyError, ValueError):
        return 0.0, None


def kernel_time(spans_us, units, per_unit_dispatches=1, cfg_key=None):
    """Average kernel time per timed launch (or per tick of a two-kernel tick) from the clock
    spans: the spans plus the calibrated dispatch overhead of every dispatch.  Returns
    (seconds per unit, clock-only seconds per unit, overhead us, calibration file)."""
    ovh, cal = dispatch_overhead_us(cfg_key)
    clock = sum(spans_us) / max(1, units)
    return (clock + ovh * per_unit_dispatches) / 1e6, clock / 1e6, ovh, cal


def write_meta(**kw):
    """GGRS_BENCH_META=path (profiled runs, tools/lines.py prof): what the fold needs to key the
    profile and to pair its dispatches with the clock spans."""
    path = os.environ.get("GGRS_BENCH_META")
    if path:
        with open(path, "w") as f:
            json.dump(kw, f)


STORE_CEILING_FILE = os.path.join(ROOT, "profiles", "r02_calib_write.json")


def store_ceiling_gbps():
    """The calibrated store-only ceiling of the brawler's SaveGameState pattern
    (tools/calib_write.hip, profiles/r02_calib_write.json: 5.9 TB/s), or None."""
    try:
        return float(json.load(open(STORE_CEILING_FILE))["store_only_GBps"])
    except (OSError, KeyError, ValueError):
        return None


def roofline_block(bytes_per_launch, avg_kernel_s, ticks_per_launch, launches, kernel, prof, model, copy_gbps=None):
    """The bench line's roofline object.  `achieved`/`frac` are the contract's:
    algorithmic bytes per launch (`model` says which bytes) over the measured
    average launch time, against the 8 TB/s spec peak (`frac_basis`).  Next to
    them, from the committed PMC profile of the same configuration: the HBM
    bytes the counters saw (`traffic`) and their fraction of peak (`dram_frac`),
    the VALU issue-slot fraction, and `bound` = what actually limits the
    kernel, decided from those counters: "hbm" when the DRAM-side traffic is
    above 0.7 of the measured store ceiling (what DRAM takes in practice,
    profiles/r02_calib_write.json), "valu" when the VALU issue slots are above 0.7 busy,
    "latency" (dependent chains at low occupancy) otherwise; "unprofiled"
    when no PMC profile of this configuration is committed, or when the profile's traffic
    over this kernel time would exceed the fastest rate DRAM was measured to take (the copy
    `copy_gbps` or the calibrated store-only ceiling): counters that describe other launches
    than the ones timed here are refused, not reported."""
    achieved = bytes_per_launch / avg_kernel_s / 1e9
    r = {"bound": "unprofiled", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
         "frac": achieved / HBM_PEAK_GBS, "frac_basis": "algorithmic bytes / kernel time / 8 TB/s HBM spec",
         "traffic": None, "dram_frac": None, "algorithmic_bytes_per_launch": bytes_per_launch, "bytes_model": model,
         "kernel_avg_us": avg_kernel_s * 1e6, "ticks_per_launch": ticks_per_launch, "launches_timed": launches,
         "kernel": kernel}
    # the fastest rate DRAM was measured to take on this engine's patterns: the device-to-device copy
    # (read + write) or the calibrated store-only stream, whichever is higher
    ceiling = max(copy_gbps or 0.0, store_ceiling_gbps() or 0.0) or None
    if prof and ceiling and prof["hbm_bytes_per_tick"] * ticks_per_launch / avg_kernel_s / 1e9 > ceiling:
        r["pmc_refused"] = (f"{prof['file']}: its traffic over this kernel time would be "
                            f"{prof['hbm_bytes_per_tick'] * ticks_per_launch / avg_kernel_s / 1e9:.0f} GB/s, above the "
                            f"{ceiling:.0f} GB/s measured ceiling (copy {copy_gbps or 0:.0f}, store-only "
                            f"{store_ceiling_gbps() or 0:.0f})")
        prof = None
    if prof:
        traffic = prof["hbm_bytes_per_tick"] * ticks_per_launch
        r["traffic"] = traffic
        r["dram_frac"] = r["traffic_frac"] = traffic / avg_kernel_s / 1e9 / HBM_PEAK_GBS
        r["pmc_profile"] = prof["file"]
        r["pmc_source_id"] = prof.get("source_id")
        iss = prof.get("issue")
        if iss:
            r["valu"] = {k: iss[k] for k in ("valu_insts_per_wave", "salu_insts_per_wave", "valu_issue_frac",
                                              "issue_per_quad", "active_inst_valu_frac", "issue_stall_frac",
                                              "waves_per_simd", "waves_dispatched_per_simd", "clock_GHz_sq",
                                              "l2_hit") if k in iss}
            # against what DRAM delivers in practice: the calibrated store ceiling (5.9 TB/s), not the spec
            ceil = store_ceiling_gbps() or HBM_PEAK_GBS
            r["dram_frac_of_ceiling"] = traffic / avg_kernel_s / 1e9 / ceil
            if r["dram_frac_of_ceiling"] > 0.7:
                r["bound"], r["limiter"] = "hbm", (f"hbm bandwidth: {r['dram_frac_of_ceiling']:.2f} of the "
                                                   f"{ceil:.0f} GB/s measured store ceiling")
            elif iss.get("issue_per_quad", 0.0) > 0.8:
                # SIMD instruction issue (profiles/r05_twopoint_pmc.json: doubling the resident waves moves
                # the issue rate from 0.92 to 0.99 instructions per quad-cycle and gains 4%; issue stalls
                # go from 21% to 54% of wave time)
                r["bound"], r["limiter"] = "issue", (
                    f"SIMD instruction issue: {iss['issue_per_quad']:.2f} vector + scalar instructions per "
                    f"quad-cycle per SIMD at {iss['waves_per_simd']:.1f} waves per SIMD (dual issue is rare at "
                    f"this mix); HBM traffic {r['dram_frac']:.2f} of peak")
            elif iss["valu_issue_frac"] > 0.7:
                r["bound"], r["limiter"] = "valu", "valu issue"
            else:
                r["bound"] = "latency"
                r["limiter"] = (f"dependency latency: {iss['waves_per_simd']:.1f} waves resident per SIMD, "
                                f"{iss['valu_issue_frac']:.2f} of VALU issue slots, HBM traffic "
                                f"{r['dram_frac']:.2f} of peak")
    return r


def rehearsal(args):
    """CPU rehearsal of the N-rank path: the self-launcher, the 127.0.0.1
    rendezvous, the report all-gather and the audit compare, with plan-only
    batches (device = -1: the host bookkeeping of every tick, no device work)
    and no GPU.  Each report's checksum is a keyed hash of (global session id,
    frame) — a replica reports what its owner reports, so the compare must
    find nothing — except that --rehearsal-corrupt makes rank 0's first
    replica lie once.  Prints one JSON line with value null."""
    import numpy as np
    import torch
    import torch.distributed as dist

    import ggrs_amd as G
    from ggrs_amd import shard
    from ggrs_amd.synth import splitmix64

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        dist.init_process_group(os.environ.get("GGRS_BENCH_BACKEND", "gloo"))
    P, cd, S = args.num_players, args.check_distance, args.sessions_per_gpu
    A = min(args.audit_sessions, S) if world > 1 else 0
    warm = cd + 1 + args.warmup
    T = warm + args.steps
    lo, hi = shard.shard_range(rank, world, S * world)
    nlo = shard.shard_range((rank + 1) % world, world, S * world)[0]
    inputs = G.synth_inputs(hi - lo, P, T, seed=args.seed, first_session=lo)
    if A:
        inputs = np.concatenate([inputs, G.synth_inputs(A, P, T, seed=args.seed, first_session=nlo)], 2)
    inputs = np.ascontiguousarray(inputs)
    gid = np.concatenate([np.arange(lo, hi), np.arange(nlo, nlo + A)]).astype(np.uint64)
    sess = (G.SessionBuilder(G.Game.EX_GAME, num_sessions=S + A, device=-1).with_num_players(P)
            .with_max_prediction_window(args.max_prediction).with_check_distance(cd)
            .with_input_delay(args.input_delay).start_synctest_session())
    interval = args.report_interval or 10
    gathers = mism = audit_bad = 0
    first_bad = None
    t = 0
    t0 = time.perf_counter()
    while t < T:
        n = min(T - t, interval - sess.current_frame() % interval)
        sess.run_ticks(inputs[t:t + n])
        t += n
        if world > 1 and sess.current_frame() % interval == 0:
            f = sess.current_frame() - 1
            cs = splitmix64((gid << np.uint64(20)) ^ np.uint64(f))
            if os.environ.get("GGRS_REHEARSAL_CORRUPT") and rank == 0 and A and gathers == 0:
                cs[S] ^= np.uint64(1)
            if os.environ.get("GGRS_BENCH_REPORT", "compact") == "compact":  # 4 B per session, as the GPU path
                rep = shard.pack_compact(cs & np.uint64(0xFFFF), f, np.full(S + A, -1, np.int32))
                g = shard.gather_compact(torch.from_numpy(rep.copy()))
                mism += int(shard.count_desynced_compact(g, world, S, A))
                nbad = int(shard.audit_compare_compact(g, world, S, A))
                if first_bad is None and nbad:
                    rows = g.view(world, S + A)
                    bad = (rows[:, S:] != torch.roll(rows[:, :A], shifts=-1, dims=0)).nonzero()[0].tolist()
                    first_bad = [((bad[0] + 1) % world) * S + bad[1], f]
            else:
                rep = shard.pack_reports(np.stack([cs, np.zeros_like(cs)], 1), f, np.full(S + A, -1, np.int32))
                g = shard.gather_reports(torch.from_numpy(rep.view(np.int64).reshape(-1, shard.REPORT_WORDS).copy()))
                mism += int(shard.count_desynced(g, world, S, A))
                nbad, detail = shard.audit_compare(g, world, S, A)
                nbad = int(nbad)
                if first_bad is None and nbad:
                    first_bad = [int(x) for x in detail[0]]
            audit_bad += nbad
            gathers += 1
    elapsed = time.perf_counter() - t0
    if rank == 0:
        print(json.dumps({
            "metric": METRIC, "value": None, "unit": "session-frames/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": elapsed * 1e3 / args.steps, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic", "rehearsal": True,
            "config": {"workload": f"plan-only rehearsal: {S} sessions/rank + {A} audit replicas, no device work",
                       "sessions_per_gpu": S, "total_sessions": S * world,
                       "desync_reports": {"ranks": dist.get_world_size() if world > 1 else 1,
                                          "backend": dist.get_backend() if world > 1 else None,
                                          "gathers": gathers, "mismatch_rows_seen": mism,
                                          "audit_sessions_per_rank": A, "audit_compared": A * world * gathers,
                                          "audit_desynced": audit_bad, "first_desync": first_bad}},
            "roofline": None, "cpu_baseline": None}), flush=True)
    sess.close()
    if world > 1:
        dist.destroy_process_group()


def bench_p2p(args):
    """P2PSession rollback batches: every tick delivers the remote inputs that
    arrived (synthetic lag), adds the local input and advances; sessions whose
    predictions were wrong roll back to their first incorrect frame and
    resimulate.  value = AdvanceFrames the games executed (resimulated + new)
    per second, counted on the device."""
    import numpy as np
    import torch
    import torch.distributed as dist

    import ggrs_amd as G
    from ggrs_amd import shard
    from ggrs_amd.p2p import PlayerType, synth_network

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    local = local % max(1, torch.cuda.device_count())  # one rank per GPU (ranks share a GPU only in rehearsals)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        init_dist(dist, dev)
    P, S, W = args.num_players, args.sessions_per_gpu, args.max_prediction
    lo, hi = (int(x) for x in args.lag.split(","))
    T = args.warmup + args.steps
    mask = 0b1
    brawler = args.game == "brawler"
    imask = args.input_mask if args.input_mask is not None else (0xFF if brawler else 0x0F)
    g0, g1 = shard.shard_range(rank, world, S * world)
    inputs, upto, rin = synth_network(g1 - g0, P, T, mask, args.remote_delay, lo, hi, seed=args.seed, first_session=g0,
                                      mask=imask)
    di, du, dr = (torch.from_numpy(a).to(dev) for a in (inputs, upto, rin))
    K = args.fanout_k
    b = (G.SessionBuilder(G.Game.BRAWLER if brawler else G.Game.EX_GAME, num_sessions=S, device=local)
         .with_num_players(P).with_max_prediction_window(W).with_input_delay(args.input_delay)
         .with_remote_input_delay(args.remote_delay).with_sparse_saving_mode(args.sparse_saving)
         .with_block_size(args.block_size)
         .with_speculative_fanout(args.fanout, K, per_player=None if args.fanout_mode == "auto" else
                                  args.fanout_mode == "per-player"))
    for h in range(P):
        b.add_player(PlayerType.Local if (mask >> h) & 1 else PlayerType.Remote, h)
    per_player_mode = b._per_player_resolved()
    stream = torch.cuda.Stream(device=dev)
    # Timing as the SyncTest path (GGRS_BENCH_EVENTS): the kernel's own clock on every timed launch by
    # default.  The warm-up runs in the timed region's call sizes whether or not the run is profiled:
    # the adaptive fan-out decides by ticks and calls, so a profiled run must take the same decisions
    # (tools/lines.py picks warm-ups that are whole timed launches, so every dispatch of the dominant
    # kernel has the timed shape).
    timing = os.environ.get("GGRS_BENCH_EVENTS", "clock")
    if timing not in ("clock", "launch"):
        raise SystemExit("GGRS_BENCH_EVENTS: clock or launch")

    def new_batch():
        x = b.start_p2p_session()
        x.set_stream(stream)
        return x

    sess = new_batch()
    tpl = args.ticks_per_launch
    import ctypes
    lib = G._lib.load()
    ptr = lambda t: ctypes.c_void_p(t.data_ptr())
    sp = ctypes.c_void_p(stream.cuda_stream)
    F = dr.shape[0]
    lstride = P * S * di.element_size()
    stride = 32
    if args.wire_replay:  # received traffic replayed: every tick's packets encoded ahead (untimed)
        rpk = torch.zeros((T, P, S, stride), dtype=torch.uint8, device=dev)
        rln, rst = (torch.zeros((T, P, S), dtype=torch.int32, device=dev) for _ in range(2))
        rng = np.random.default_rng(args.seed)
        with torch.cuda.stream(stream):
            none = torch.full((S,), -1, dtype=torch.int32, device=dev)
            for t in range(T):
                for h in range(P):
                    if (mask >> h) & 1:
                        continue
                    # the peer knows the receiver had the previous tick's deliveries and re-sends 0-2
                    # frames before them (an un-acked sender), as tests/test_wire.py's schedule
                    prev = du[t - 1, h] if t > 0 else none
                    redo = torch.from_numpy(rng.integers(0, 3, S).astype(np.int32)).to(dev)
                    acked = torch.where(prev < 0, prev, torch.clamp(prev - redo, min=args.remote_delay - 1))
                    acked = torch.where(acked < args.remote_delay, none, acked).contiguous()
                    assert lib.rb_encode_input_packets(local, sp, h, P, S, 1, ptr(dr), F, args.remote_delay,
                                                       ptr(acked), ptr(du[t, h].contiguous()), ptr(rpk[t, h]), stride,
                                                       ptr(rln[t, h]), ptr(rst[t, h])) == 0
            torch.cuda.synchronize()
        assert int((rln < 0).sum()) == 0, "a packet did not fit its row"

    def make_run(batch, one_at_a_time=False):
        """The timed loop of one batch, every native call's arguments built ahead (a compiled
        host's loop): only the C calls run inside it.  one_at_a_time: each call completes
        before the next is issued."""
        settle = torch.cuda.synchronize if one_at_a_time else (lambda: None)
        h_ = batch._h
        if args.wire:  # the remote inputs travel as packets: no delivery tensors on the receiver
            pk = torch.zeros((1, P, S, stride), dtype=torch.uint8, device=dev)
            ln, st = (torch.zeros((1, P, S), dtype=torch.int32, device=dev) for _ in range(2))
            acks = torch.full((P, S), -1, dtype=torch.int32, device=dev)  # the receiver's newest frame per endpoint
            remotes = [h for h in range(P) if not (mask >> h) & 1]
            # per tick, each remote peer's send_pending_output since its last ack (device encode), then
            # one launch that decodes the packets inside the tick's poll and runs the tick
            enc_args = [[(local, sp, h, P, S, 1, ptr(dr), F, args.remote_delay, ptr(acks[h]), ptr(du[t, h]),
                          ptr(pk[0, h]), stride, ptr(ln[0, h]), ptr(st[0, h])) for h in remotes] for t in range(T)]
            tick_args = [(h_, 1, ptr(di[t]), lstride, ptr(pk), stride, ptr(ln), ptr(st), None, ptr(acks))
                         for t in range(T)]
            enc, tick_fn = lib.rb_encode_input_packets, lib.rb_p2p_run_ticks_packets
            keep = (pk, ln, st, acks)

            def run(t0, t1):
                bad = 0
                for t in range(t0, t1):
                    for a in enc_args[t]:
                        bad |= enc(*a)
                    bad |= tick_fn(*tick_args[t])
                    settle()
                if bad:
                    raise SystemExit("wire path: a call failed")
        else:
            if args.wire_replay:
                fn = lib.rb_p2p_run_ticks_packets
                mk = lambda t, n: (h_, n, ptr(di[t]), lstride, ptr(rpk[t]), stride, ptr(rln[t]), ptr(rst[t]), None, None)
            else:
                fn = lib.rb_p2p_run_ticks
                mk = lambda t, n: (h_, n, ptr(di[t]), lstride, ptr(du[t]), ptr(dr), F)
            keep = None
            calls = {}

            def run(t0, t1):
                bad = 0
                for t in range(t0, t1, tpl):
                    n = min(t1, t + tpl) - t
                    a = calls.get((t, n))
                    if a is None:
                        a = calls[(t, n)] = mk(t, n)
                    bad |= fn(*a)
                    settle()
                if bad:
                    raise SystemExit("p2p: a call failed")

            for t in range(args.warmup, T, tpl):  # the timed region's calls, built ahead
                calls[(t, min(T, t + tpl) - t)] = mk(t, min(T, t + tpl) - t)
        run.keep = keep
        return run

    run = make_run(sess)
    n_timed = len(range(args.warmup, T, tpl)) if not args.wire else args.steps  # launches of the timed region
    two_kernel = False  # the two-launch fan-out (fanout_kernel between one-tick P2P launches), set below
    with torch.cuda.stream(stream):
        sess.profile_enable(timing == "launch")  # the warmup takes the timed region's path
        run(0, args.warmup)
        torch.cuda.synchronize()
        sess.profile_take()
        a0 = sess.totals()
        if timing == "clock":  # slots for every launch the timed region can make (two per tick at most)
            sess.launch_clock_arm(2 * args.steps)
            torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        run(args.warmup, T)
        torch.cuda.synchronize()
        if world > 1:  # (at N = 1 there is no barrier between two synchronizes)
            dist.barrier()
            torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
        kernel_ms, launches = sess.profile_take()
        spans = sess.launch_clock_read(2 * args.steps) if timing == "clock" else None
    a1 = sess.totals()
    adv, saves, loads, selects, branch = (a1[i] - a0[i] for i in range(5))
    thr, unexpected, panics = sess.counters()
    tot = torch.tensor([adv, saves, loads, panics, selects, branch], dtype=torch.float64, device=dev)
    el = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(tot)
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    adv, saves, loads, panics, selects, branch = (int(x) for x in tot.tolist())
    elapsed = float(el.item())
    if rank == 0:
        # algorithmic bytes (this rank's launches): cells loaded + saved (40 B state,
        # 2 B checksum, 4 B frame tag per save), the inputs of every AdvanceFrame
        # (P bytes), and per session-tick the local input read + ring write, the
        # delivery watermark and one remote input read + ring write (8 B)
        state = 4 * 256 * 8 if brawler else 4 * 5 * P
        bytes_rank = (adv / world * P + saves / world * (state + 6) + loads / world * state
                      + S * args.steps * 8)
        generic_fan = os.environ.get("RB_FANOUT_GENERIC", "0") not in ("", "0")
        if args.fanout and branch == 0:  # the adaptive fan-out was paused through the timed region: plain ticks
            pass
        elif args.fanout and (generic_fan or brawler):  # fanout_kernel: per branch frame its cell + checksum stored
            # and its inputs; per session-tick the base cell load and K branch states stored; per select the
            # selected cells read back
            bytes_rank += branch / world * (state + 2 + P) + S * args.steps * state * (K + 1) + selects / world * state
        elif args.fanout:  # the in-kernel fan-out (p2p.hpp inlane_fan): only the speculated player's words
            # are branched, so per presimulated branch frame its part of the cell (state / P) is stored (the
            # base frame's excepted: one per branch per session-tick), per session-tick the K final branch
            # parts; per select the selected branch's parts read back (its frames: about the branch depth)
            ps = state // P
            bytes_rank += branch / world * ps + S * args.steps * K * ps + selects / world * ps * 2
        timer = {"timer": "kernel clock + dispatch overhead" if spans is not None else "HIP events (hipExtLaunchKernel)"}
        per_tick = False
        if spans is not None:
            # one clock slot per kernel launch; the two-launch fan-out (fanout_kernel between one-tick P2P
            # launches) has two per tick, and its unit is then the tick (both kernels)
            per_tick = len(spans) > n_timed
            launches = args.steps if per_tick else len(spans)
        fan_state = None
        if args.fanout:  # the state of the adaptive fan-out through the timed launches
            fan_state = "active" if branch > 0 else "paused"
        cfg_key = (f"p2p {args.game} P={P} W={W} d={args.input_delay} rd={args.remote_delay} lag={lo},{hi} S={S}"
                   + (" sparse" if args.sparse_saving else "") + (f" fanout{'' if K == 16 else K}" if args.fanout else "")
                   + (" per-player" if args.fanout and per_player_mode else "")
                   + (" wire" if args.wire else "") + (" wire-replay" if args.wire_replay else ""))
        tl = int(round(args.steps / max(1, launches)))  # the PMC profile of the launch shape timed here
        cfg_key += f" tpl={tl}" if tl != 50 else ""
        if spans is not None:
            avg_kernel_s, clock_s, ovh, cal = kernel_time(spans, launches, 2 if per_tick else 1, cfg_key)
            timer.update({"kernel_clock_us": clock_s * 1e6, "dispatch_overhead_us": ovh, "calibration": cal,
                          "dispatches": len(spans)})
        else:
            avg_kernel_s = kernel_ms / 1e3 / max(1, launches)
        gname = f"Brawler<{P}>" if brawler else f"ExGame<{P},true>"
        roofline = roofline_block(bytes_rank / max(1, launches), avg_kernel_s, args.steps / max(1, launches), launches,
                                  f"p2p_kernel<{gname}>" + ((" + fanout_kernel (per tick)" if generic_fan or brawler
                                                             else " with the in-kernel fan-out (fused P2P ticks)")
                                                            if args.fanout and branch > 0 else
                                                            " (the adaptive fan-out paused: plain P2P ticks)"
                                                            if args.fanout
                                                            else (" (one tick per launch)" if tl == 1 else
                                                                  " (fused P2P ticks)")),
                                  pmc_profile(cfg_key, fan_state), "algorithmic: cells loaded/saved, inputs, deliveries",
                                  measured_copy_gbps(dev))
        roofline.update(timer)
        write_meta(config_key=cfg_key, source_id=source_id(), fanout_state=fan_state, kernel="p2p_kernel",
                   clock_spans_us=spans, dispatch_overhead_us=timer.get("dispatch_overhead_us"),
                   kernel_avg_us=avg_kernel_s * 1e6, bytes_per_launch=bytes_rank / max(1, launches))
        line = {
            "metric": "P2P session-frames simulated/sec (node), rollback to the first mispredicted frame",
            "value": adv / elapsed, "unit": "session-frames/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": elapsed * 1e3 / args.steps, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
            "config": {"workload": f"{args.game} P2PSession x {S} sessions/GPU, {P} players (handle 0 local), "
                                   f"max_prediction {W}, input delay {args.input_delay}, remote delay "
                                   f"{args.remote_delay}, network lag {lo}-{hi} frames"
                                   + (", sparse saving" if args.sparse_saving else "")
                                   + (f", speculative fan-out {K} candidates/frame" if args.fanout else "")
                                   + f", inputs masked 0x{imask:X}"
                                   + (", inputs delivered as packets (per tick: the peers' device encode, then "
                                      "one launch decoding them inside the tick)" if args.wire else "")
                                   + (f", inputs delivered as packets: received traffic replayed ({tpl} ticks per "
                                      "launch, each decoding its packets inside the tick; the peers' packets encoded "
                                      "before the timed region)" if args.wire_replay else ""),
                       "sessions_per_gpu": S, "total_sessions": S * world,
                       "advance_frames_per_session_tick": adv / (S * world * args.steps),
                       "rollbacks_per_session_tick": (loads + selects) / (S * world * args.steps),
                       "speculative": ({"branches": K, "alphabet": 16 if not brawler else 256,
                                        "mode": ("per-player" if per_player_mode else "single") +
                                                (" (auto)" if args.fanout_mode == "auto" else ""),
                                        "candidates": "whole alphabet" if (not brawler and K >= 16) else
                                                      "the K most recently added distinct inputs (the queue's "
                                                      "move-to-front list), then the smallest values",
                                        "selects": selects, "loads": loads,
                                        "select_fraction": selects / max(1, selects + loads),
                                        "branch_frames_per_s": branch / elapsed,
                                        "adaptive": dict(zip(("active_at_end", "window_select_fraction",
                                                              "windows_measured", "turned_off"),
                                                             sess.fanout_state()))}
                                       if args.fanout else None),
                       "prediction_threshold_hits": thr, "panics": panics,
                       "parallelism": f"session-sharded x{world}"},
            "roofline": roofline,
            "cpu_baseline": None,
        }
        if world == 1 and not args.no_cpu_baseline:
            # the reference rollback path (the oracle's P2PSession + ex_game, reference allocation
            # pattern) on the same arrays: same inputs, same delivery schedule, same rollbacks
            from oracle import oracle as O
            threads = cpu_threads()
            cs_ = min(S, 8192) if brawler else S  # the brawler port: a bounded sample of sessions
            secs, cadv, nerr = O.bench_p2p_exgame(P, W, args.input_delay, mask, args.remote_delay,
                                                  np.ascontiguousarray(inputs[:, :, :cs_]),
                                                  np.ascontiguousarray(upto[:, :, :cs_]),
                                                  np.ascontiguousarray(rin[:, :, :cs_]), args.warmup, threads,
                                                  game=O.BRAWLER if brawler else O.EX_GAME)
            line["cpu_baseline"] = {
                "value": cadv / secs, "unit": "session-frames/s", **cpu_info(threads), "kind": "port",
                "sample": f"{cs_} of the {S} sessions x {args.steps} timed ticks ({cadv} AdvanceFrames), same inputs "
                          f"and deliveries, through the C++ restatement of P2PSession rollback (no fan-out: the "
                          f"reference has none), {threads} host threads, {secs:.2f} s wall, {nerr} errors"}
        print(json.dumps(line), flush=True)
    sess.close()
    if world > 1:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--warmup", type=int, default=32)
    ap.add_argument("--sessions-per-gpu", type=int, default=None,
                    help="default: 65,536 at --gpus 1 (BASELINE configs[1]), 131,072 at --gpus N > 1 "
                         "(configs[4]: 1,048,576 sessions over 8 GPUs)")
    ap.add_argument("--num-players", type=int, default=2)
    ap.add_argument("--check-distance", type=int, default=7)
    ap.add_argument("--max-prediction", type=int, default=8)
    ap.add_argument("--input-delay", type=int, default=2)
    ap.add_argument("--seed", type=int, default=0x67677273)
    ap.add_argument("--report-interval", type=int, default=100,
                    help="ticks between RCCL all-gathers of desync reports (N>1); 0 = never")
    ap.add_argument("--ticks-per-launch", type=int, default=50,
                    help="steady-state ticks fused into one steady_kernel launch (rb_run_ticks call)")
    ap.add_argument("--realtime-ticks", type=int, default=64,
                    help="after the timed region, this many ticks of one rb_run_ticks call each (live play, "
                         "inputs arriving per tick): the line's realtime / headroom_60hz fields; 0 = skip")
    ap.add_argument("--game", choices=["ex_game", "brawler"], default="ex_game",
                    help="ex_game = BASELINE configs[1] (default); brawler = configs[2]")
    ap.add_argument("--cpu-sessions", type=int, default=None)
    ap.add_argument("--cpu-ticks", type=int, default=None)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--block-size", type=int, default=0)
    ap.add_argument("--session", choices=["synctest", "p2p"], default="synctest",
                    help="synctest = the headline (BASELINE configs[1]); p2p = P2PSession rollback batches "
                         "(SURVEY 8f row 1): handle 0 local, the others remote, synthetic network lag")
    ap.add_argument("--lag", type=str, default="1,4", help="p2p: min,max network lag in frames")
    ap.add_argument("--remote-delay", type=int, default=2, help="p2p: the remote peers' input delay")
    ap.add_argument("--sparse-saving", action="store_true", help="p2p: with_sparse_saving_mode(true)")
    ap.add_argument("--wire", action="store_true",
                    help="p2p: remote inputs travel as packets each tick: device encode (send_pending_output) + "
                         "decode (on_input) into the delivery tensors, then one P2P tick")
    ap.add_argument("--wire-replay", action="store_true",
                    help="p2p: the remote inputs arrive as the peers' packets, recorded ahead (untimed) and replayed "
                         "--ticks-per-launch ticks per launch, each tick decoding its packets (rb_p2p_run_ticks_packets)")
    ap.add_argument("--fanout", action="store_true",
                    help="p2p: speculative fan-out, --fanout-k candidate inputs per session per tick (BASELINE "
                         "configs[3]; use with --num-players 4)")
    ap.add_argument("--fanout-mode", choices=["auto", "single", "per-player"], default="auto",
                    help="p2p --fanout: speculate the remote player with the oldest unconfirmed input (single) or "
                         "every remote player (per-player, RB_P2P_FLAG_FANOUT_PER_PLAYER; whole alphabet only); "
                         "auto (default) = per-player for ex_game at K = 16, else single")
    ap.add_argument("--fanout-k", type=int, default=16,
                    help="p2p --fanout: candidates per session (1..16): ex_game's whole alphabet at 16, else the "
                         "most likely K")
    ap.add_argument("--input-mask", type=lambda x: int(x, 0), default=None,
                    help="synthetic input bits (default 0x0F ex_game, 0xFF brawler)")
    ap.add_argument("--audit-sessions", type=int, default=64,
                    help="N>1: each rank also simulates this many sessions of the next rank's shard; after every "
                         "report all-gather the owner's checksums are compared with the replica's (DesyncDetected)")
    ap.add_argument("--rehearsal", action="store_true",
                    help="CPU rehearsal of the N-rank path (launcher, rendezvous, report all-gather, audit compare) "
                         "with plan-only batches (host bookkeeping, no device): GGRS_BENCH_BACKEND=gloo, no GPU, "
                         "value null")
    args = ap.parse_args()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return launch_ranks(args.gpus)  # before anything touches the GPU
    if args.sessions_per_gpu is None:  # configs[1] at N=1; configs[4]'s per-GPU shard (1,048,576 / 8) at N>1
        args.sessions_per_gpu = 65536 if args.gpus == 1 else 131072
        if args.rehearsal:
            args.sessions_per_gpu = 256
    if args.rehearsal:
        return rehearsal(args)
    if args.session == "p2p":
        return bench_p2p(args)

    import numpy as np
    import torch
    import torch.distributed as dist

    import ggrs_amd as G
    from ggrs_amd import shard

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    local = local % max(1, torch.cuda.device_count())  # one rank per GPU (ranks share a GPU only in rehearsals)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        init_dist(dist, dev)  # RCCL over xGMI

    P, cd = args.num_players, args.check_distance
    S = args.sessions_per_gpu
    # The first cd+1 ticks are start-up ticks (no rollback yet, sync_test_session.rs:89): they
    # always run untimed, before the W requested warmup ticks, so the timed region is steady state
    # and the warmup has run the fused steady kernel at least once.
    warm = cd + 1 + args.warmup
    RT = args.realtime_ticks  # one-tick-per-call ticks after the timed region (the 60 Hz serving path)
    # Kernel timing (GGRS_BENCH_EVENTS).  "clock" (default): every timed launch records its own first
    # wave start and last wave end on the chip's 100 MHz constant clock (rb_launch_clock_*; two plain
    # stores per wave, nothing on the stream or the host inside the timed region), and the kernel time
    # is that span plus the dispatch overhead rocprofv3 adds to it (dispatch_overhead_us, calibrated
    # against rocprofv3 --kernel-trace of these lines).  A profiler does not perturb that clock, so a
    # line run under rocprofv3 reports the kernel time it would without.  "launch": the timed launches'
    # own HIP events (hipExtLaunchKernel; ~12 us of wall per call, and under rocprofv3 they read 8-40%
    # high, tools/timer_check.py).
    timing = os.environ.get("GGRS_BENCH_EVENTS", "clock")
    if timing not in ("clock", "launch"):
        raise SystemExit("GGRS_BENCH_EVENTS: clock or launch")
    # GGRS_BENCH_PROFILE=1 (tools/lines.py prof, the rocprofv3 runs): the warm-up ticks run one
    # tick_kernel launch each and the live-play block is skipped, so that every dispatch of the
    # dominant kernel in the profile is a timed launch of the line's shape (its rocprofv3 --stats
    # average is then the timed launches' average).
    profiling = os.environ.get("GGRS_BENCH_PROFILE", "0") not in ("", "0")
    if profiling:
        RT = 0
    checked = os.environ.get("GGRS_BENCH_CHECKED", "1") not in ("", "0")
    T = warm + args.steps + RT
    # This rank's shard: global sessions [rank*S, (rank+1)*S); inputs keyed by global id.  With
    # N > 1 the batch also holds A audit replicas: the first A sessions of rank (r+1) % N.
    lo, hi = shard.shard_range(rank, world, S * world)
    A = min(args.audit_sessions, S) if world > 1 else 0
    nlo = shard.shard_range((rank + 1) % world, world, S * world)[0]
    brawler = args.game == "brawler"
    imask = 0xFF if brawler else 0x0F
    inputs = G.synth_inputs(hi - lo, P, T, seed=args.seed, first_session=lo, mask=imask)
    if A:
        inputs = np.concatenate([inputs, G.synth_inputs(A, P, T, seed=args.seed, first_session=nlo, mask=imask)], 2)
    dinputs = torch.from_numpy(np.ascontiguousarray(inputs)).to(dev)  # [T, P, S + A] u8, resident in HBM

    stream = torch.cuda.Stream(device=dev)
    game = G.Game.BRAWLER if brawler else G.Game.EX_GAME

    def new_batch():
        b = (G.SessionBuilder(game, num_sessions=S + A, device=local).with_num_players(P)
             .with_max_prediction_window(args.max_prediction).with_check_distance(cd)
             .with_input_delay(args.input_delay).with_checked_mismatches(checked)
             .with_block_size(args.block_size).start_synctest_session())
        b.set_stream(stream)
        return b

    sess = new_batch()
    # the desync report: 4 B per session (rb_export_compact_report: 16-bit checksum + mismatch flag and
    # delta; both bench games checksum in 16 bits), or the 24 B rb_checksum_report (GGRS_BENCH_REPORT=full)
    compact = os.environ.get("GGRS_BENCH_REPORT", "compact") == "compact"
    report_bytes = 4 if compact else 24
    reports = (torch.zeros((S + A,), dtype=torch.int32, device=dev) if compact else
               torch.zeros((S + A, shard.REPORT_WORDS), dtype=torch.int64, device=dev))
    desyncs = torch.zeros((), dtype=torch.int64, device=dev)  # sessions reporting MismatchedChecksum
    audit_bad = torch.zeros((), dtype=torch.int64, device=dev)  # DesyncDetected: owner vs replica checksums
    gathers = [0]

    def chunks(t0, t1, final_report=False, batch=None):
        """Ticks [t0, t1) as native multi-tick calls of at most --ticks-per-launch
        ticks (one steady_kernel launch each once past the first cd+1 ticks),
        split further at desync-report points: (input slice, steady, report after).
        With N > 1 a report is all-gathered every --report-interval ticks and,
        with final_report, after the last tick (so every timed region runs the
        collective at least once).  SyncTest's current frame after t ticks is
        t, so the split is known up front and the slices are views made before
        the timed region."""
        out, t = [], t0
        every = world > 1 and args.report_interval
        while t < t1:
            n = min(t1 - t, args.ticks_per_launch)
            steady = t > cd
            if not steady:  # start-up ticks: per-tick launches, then align the steady chunks
                n = min(n, cd + 1 - t)
            if every:
                n = min(n, args.report_interval - t % args.report_interval)
            t += n
            report = world > 1 and ((every and t % args.report_interval == 0) or (final_report and t == t1))
            # each call prepared ahead (session.prepare_ticks): inside the loop only the native
            # rb_run_ticks call runs, as in a compiled host
            call, check = (batch or sess).prepare_ticks(dinputs[t - n:t])
            out.append((call, check, steady, report))
        return out

    gather_ev = []  # HIP event pairs around each all-gather (torch's current stream = the batch stream)

    def run(plan):
        steady_launches = 0
        for call, check, steady, report in plan:
            st = call()
            if st:
                check(st)  # raises with the batch's error
            steady_launches += steady
            if report:
                f = sess.current_frame() - 1
                (sess.export_compact_report if compact else sess.export_checksum_report)(f, reports)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                # RCCL all-gather of desync reports
                gathered = (shard.gather_compact if compact else shard.gather_reports)(reports)
                e1.record()
                gather_ev.append((e0, e1))
                if compact:
                    desyncs.add_(shard.count_desynced_compact(gathered, world, S, A))  # mismatch flag
                    audit_bad.add_(shard.audit_compare_compact(gathered, world, S, A))  # owner != replica
                else:
                    desyncs.add_(shard.count_desynced(gathered, world, S, A))  # mismatch_frame != NULL_FRAME
                    audit_bad.add_(shard.audit_compare(gathered, world, S, A, detail=False)[0])  # owner != replica
                # (the count only: the detail list's nonzero() would stall the host inside the timed loop)
                gathers[0] += 1
        return steady_launches

    with torch.cuda.stream(stream):
        timed_plan = chunks(warm, warm + args.steps, final_report=True)
        if profiling:  # every warm-up tick its own tick_kernel launch (see GGRS_BENCH_PROFILE above)
            for t in range(warm):
                for h in range(P):
                    sess.add_local_input(h, dinputs[t, h])
                sess.advance_frame()
        else:
            # the warmup takes the timed region's exact path (with GGRS_BENCH_EVENTS=launch, profiling
            # events around every fused launch), so no first-call cost of that path lands inside it
            sess.profile_enable(timing == "launch")
            run(chunks(0, warm))
        if world > 1:  # one untimed report all-gather: the collective's first-call setup stays out of timing
            (sess.export_compact_report if compact else sess.export_checksum_report)(sess.current_frame() - 1, reports)
            (shard.gather_compact if compact else shard.gather_reports)(reports)
        torch.cuda.synchronize()
        sess.profile_take()
        sess.profile_enable(timing == "launch")
        fused = 1 <= cd <= 16  # fused steady ticks exist for check distances 1..16 (kernels.hpp kMaxFusedCD)
        clocked = timing == "clock" and fused
        if clocked:
            sess.launch_clock_arm(len(timed_plan))  # (clears the slots on the stream: before the sync below)
            torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
            torch.cuda.synchronize()
        trace = os.environ.get("GGRS_BENCH_TRACE")
        if trace:  # (recorded once here: torch creates an event's HIP event at its first record)
            ev_a, ev_b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ev_a.record()
            ev_b.record()
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        if trace:
            ev_a.record()
        launches = run(timed_plan)
        t_call = time.perf_counter()
        if trace:
            ev_b.record()
        torch.cuda.synchronize()
        t_sync = time.perf_counter()
        if world > 1:  # (at N = 1 there is no barrier between two synchronizes)
            dist.barrier()
            torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
        if trace:
            print(f"[trace] calls {1e6 * (t_call - t0):.1f} us, first sync done at {1e6 * (t_sync - t0):.1f} us, "
                  f"elapsed {1e6 * elapsed:.1f} us, GPU marker to marker {1e3 * ev_a.elapsed_time(ev_b):.1f} us",
                  file=sys.stderr, flush=True)
        kernel_ms, timed_ticks = sess.profile_take()  # (GGRS_BENCH_EVENTS=launch, or tick_kernel sampling)
        spans = sess.launch_clock_read(len(timed_plan)) if clocked else None
        sess.profile_enable(False)
        gather_ms = [a.elapsed_time(b) for a, b in gather_ev]
        # The 60 Hz serving path, after (outside) the timed region: inputs arrive one tick at a
        # time (ex_game_synctest.rs:50-61), so each tick is its own call and launch.
        rt = None
        if RT:
            # wall time of RT/2 one-tick calls, then the kernel time of each launch of RT/2 more from
            # the kernel's own clock (as the timed region)
            t_rt = warm + args.steps
            half = RT // 2
            rt_calls = [sess.prepare_ticks(dinputs[t_rt + k:t_rt + k + 1])[0] for k in range(RT)]
            torch.cuda.synchronize()
            r0 = time.perf_counter()
            for k in range(half):
                if rt_calls[k]():
                    raise SystemExit(f"realtime tick {k} failed")
            torch.cuda.synchronize()
            rt_wall = time.perf_counter() - r0
            if fused:
                sess.launch_clock_arm(RT - half)
            else:
                sess.profile_enable(True)
            for k in range(half, RT):
                if rt_calls[k]():
                    raise SystemExit(f"realtime tick {k} failed")
            torch.cuda.synchronize()
            if fused:
                rt_spans = sess.launch_clock_read(RT - half)
                rt_kernel_s = kernel_time(rt_spans, len(rt_spans), 1, f"{args.game} P={P} cd={cd} W={args.max_prediction} "
                                          f"d={args.input_delay} S={S} tpl=1")[0]
            else:
                rt_kernel_ms, rt_ticks = sess.profile_take()
                rt_kernel_s = rt_kernel_ms / 1e3 / max(1, rt_ticks)
            rt = {"ticks": RT, "ticks_per_call": 1, "wall_us_per_tick": rt_wall / half * 1e6,
                  "kernel_us_per_tick": rt_kernel_s * 1e6,
                  "max_ticks_per_s": half / rt_wall, "headroom_60hz": half / rt_wall / 60.0,
                  "tick_latency_us": rt_kernel_s * 1e6,
                  "note": "one tick per rb_run_ticks call (live play, inputs arriving per tick), all sessions of "
                          "this GPU: wall over the first half, kernel time (the kernel's own clock plus the "
                          "calibrated dispatch overhead) over the second; headroom = sustainable ticks/s / 60"}

    nfail = int((sess.mismatches()[:S] != G.NULL_FRAME).sum())  # owned sessions only
    el = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    bad = torch.tensor([nfail], dtype=torch.int64, device=dev)
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
        dist.all_reduce(bad, op=dist.ReduceOp.SUM)
        ranks_seen = dist.get_world_size()
        backend = dist.get_backend()
    elapsed = float(el.item())

    if rank == 0:
        frames_per_tick = cd + 1
        total = S * world * frames_per_tick * args.steps
        value = total / elapsed
        # fused steady ticks exist for check distances 1..16 (kernels.hpp kMaxFusedCD); past that
        # every tick is a tick_kernel launch, timed by events on every 8th one (engine sampling)
        timer = {"timer": "kernel clock + dispatch overhead" if clocked else "HIP events (hipExtLaunchKernel)"}
        if clocked:
            assert len(spans) == launches, (len(spans), launches)
            ticks_per_launch = args.steps / max(1, launches)
            tl = int(round(ticks_per_launch))
            avg_kernel_s, clock_s, ovh, cal = kernel_time(
                spans, launches, 1, f"{args.game} P={P} cd={cd} W={args.max_prediction} d={args.input_delay} S={S}"
                + (f" tpl={tl}" if tl != 50 else ""))
            timer.update({"kernel_clock_us": clock_s * 1e6, "dispatch_overhead_us": ovh, "calibration": cal})
        elif fused:
            assert timed_ticks == args.steps, (timed_ticks, args.steps)
            avg_kernel_s = kernel_ms / 1e3 / max(1, launches)  # per steady_kernel launch
            ticks_per_launch = timed_ticks / max(1, launches)
        else:
            launches = timed_ticks  # the sampled launches
            avg_kernel_s = kernel_ms / 1e3 / max(1, timed_ticks)
            ticks_per_launch = 1
        # device words of one session's state: ex_game 5 f32 per player (frame
        # word implicit); brawler 256 entities x 8 i32
        nw = 256 * 8 if brawler else 5 * P
        bpt = algorithmic_bytes_per_session_tick(P, cd, nw=nw, cs_bytes=2, in_bytes=1)
        tpl = args.ticks_per_launch
        if brawler and tpl > 1:
            # HBM-required bytes: the LoadGameState of a tick re-reads the cell the same lanes
            # saved one tick earlier in the same launch, so only the saves must reach HBM
            bpt -= 4 * nw
            model = ("HBM-required: cd saves x 8 KiB + checksums + inputs (the load re-reads the cell the "
                     "same wave saved one tick earlier in this launch)")
        elif brawler:
            model = ("algorithmic (SURVEY 8d): 1 load + cd saves x 8 KiB, checksums, inputs, status; one tick "
                     "per launch, so the loaded cell (saved a launch and 3.5 GiB of stores earlier) streams "
                     "from DRAM")
        else:
            model = "algorithmic (SURVEY 8d): 1 load + cd saves x 40 B, checksums, inputs, status"
        bytes_per_launch = bpt * (S + A) * ticks_per_launch  # the kernel runs the audit replicas too
        # the PMC profile of exactly the launch shape timed here: ticks per timed launch (the driver's
        # --steps 20 times one 20-tick launch, whatever --ticks-per-launch says)
        tl = int(round(ticks_per_launch))
        cfg_key = f"{args.game} P={P} cd={cd} W={args.max_prediction} d={args.input_delay} S={S}" + (
            f" tpl={tl}" if tl != 50 else "")
        copy_gbps = measured_copy_gbps(dev)
        roofline = roofline_block(bytes_per_launch, avg_kernel_s, ticks_per_launch, launches,
                                  ((f"steady_kernel<Brawler<{P}>,{cd}>" if brawler else
                                    f"steady_kernel<ExGame<{P},true>,{cd}>") +
                                   (" (fused steady-state ticks)" if tpl > 1 else " (one tick per launch)"))
                                  if fused else (f"tick_kernel<{'Brawler' if brawler else 'ExGame'}<{P}>> (one launch "
                                                 f"per tick: no fused kernel past check distance 16)"),
                                  pmc_profile(cfg_key, family="synctest"), model, copy_gbps)
        roofline.update(timer)
        roofline["algorithmic_bytes_per_session_tick"] = bpt
        roofline["measured_copy_GBps"] = copy_gbps
        write_meta(config_key=cfg_key, source_id=source_id("synctest"), fanout_state=None, kernel="steady_kernel",
                   clock_spans_us=spans, dispatch_overhead_us=timer.get("dispatch_overhead_us"),
                   kernel_avg_us=avg_kernel_s * 1e6, bytes_per_launch=bytes_per_launch)
        if brawler:
            ceil = store_ceiling_gbps()
            roofline["store_ceiling_GBps"] = ceil
            roofline["frac_of_store_ceiling"] = roofline["achieved"] / ceil if ceil else None
            if tpl > 1 and ceil and roofline["achieved"] > ceil:
                # a wave keeps its session for all the launch's ticks, and only about 3 waves per SIMD are
                # resident: the ~3k sessions in flight rewrite their 64 KiB rings (~200 MB) inside the 256 MiB
                # Infinity Cache, so more bytes are saved per second than DRAM can take
                roofline["bound"] = "infinity-cache"
                roofline["limiter"] = ("Infinity-Cache assisted (time-skewed sessions): the saves of the sessions "
                                       "in flight are absorbed by the 256 MiB MALL; above the "
                                       f"{ceil:.0f} GB/s DRAM store ceiling, so not an HBM figure")
        line = {
            "metric": METRIC,
            "value": value,
            "unit": "session-frames/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "i32" if brawler else "f32",
            "data": "synthetic",
            "config": {
                "workload": (f"fixed-point 256-entity brawler (8 KiB i32 state) SyncTestSession"
                             if brawler else "ex_game SyncTestSession")
                            + f" x {S} sessions/GPU ({S * world} total), {P} players, "
                            f"check_distance {cd} (8-frame rollback), input delay {args.input_delay}",
                "sessions_per_gpu": S,
                "total_sessions": S * world,
                "num_players": P,
                "max_prediction": args.max_prediction,
                "check_distance": cd,
                "input_delay": args.input_delay,
                "checked_mismatches": checked,
                "session_frames_per_step_per_session": frames_per_tick,
                "parallelism": f"session-sharded x{world}" + (f", RCCL allgather of desync reports every "
                                                              f"{args.report_interval} ticks" if world > 1 else ""),
                "mismatched_sessions": int(bad.item()),
                "desync_reports": ({"ranks": ranks_seen, "backend": backend, "gathers": gathers[0],
                                    "interval_ticks": args.report_interval,
                                    "allgather_ms": gather_ms, "allgather_bytes_per_rank": (S + A) * report_bytes,
                                    "report": "compact 4 B (rb_export_compact_report)" if compact else
                                              "rb_checksum_report 24 B",
                                    "mismatch_rows_seen": int(desyncs.item()),
                                    "audit_sessions_per_rank": A, "audit_compared": A * world * gathers[0],
                                    "audit_desynced": int(audit_bad.item())} if world > 1 else None),
            },
            "roofline": roofline,
            "realtime": rt,
            "headroom_60hz": {"fused": args.steps / elapsed / 60.0,
                              "one_tick_per_call": rt["headroom_60hz"] if rt else None,
                              "note": "sustainable ticks/s of this GPU's sessions / 60: fused = the timed "
                                      "region (inputs known ahead, a SyncTest replay), one_tick_per_call = "
                                      "live play (realtime block)"},
            "cpu_baseline": None,
        }
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(args, P)
        print(json.dumps(line), flush=True)
    sess.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
