#!/usr/bin/env python3
"""Benchmark of the eSLAM per-step particle-filter hot path on MI355X.

Metric (BASELINE.json): M particle-updates/s (predict+weight+resample) @ 1/2/4/8 MI355X.
One step = EmbodiedSlamFilter::update on one batch of synthetic odometry + 4 foot contacts:
project (predict) -> updateWeights (contact model against the MLS map) -> normalizeWeights ->
stratified resample, forced every step (minEffective = N + 1, measurement gate forced).
Workload at N=1: BASELINE configs[2] -- 4M particles, 100 x 100 m MLS map @ 0.1 m.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--particles P]

For N > 1 launch with torch.distributed.run (one process per GPU); each rank holds
P particles of one global filter (weak scaling).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "slam-eslam_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

# algorithmic bytes per particle-update (208 B for the whole step)
BYTES_REFERENCE = 208         # the reference algorithm's passes: predict+weight 96, normalise 8,
                              # resample 104 (scan 8, gather 48, write 48) -- reported, not the roofline
# per kernel as launched: the resample gather is fused into the next step's k_project_weight
BYTES_K1 = 113                # gathered read x, y, th, z, zs, w (48) + write x, y, th, z, zs, w, mprob, flags (57)
                              # + the 4-byte segment mark read and cleared (8)
BYTES_K3 = 29                 # k_normalize_segments: read w, mprob, flags (17), write w (8), segment marks (4)
BYTES_STEP = BYTES_K1 + BYTES_K3   # what the fused step moves per particle-update: the step roofline
BYTES_K1_DELTA = BYTES_K1 + 4  # per-particle maps: + the table name (the lookups of the cells under the
                               # feet -- window centre, slot, page cell -- hit L2)
# k_map_merge, per particle: pose x, y, theta, z, zsigma 40, table name read + written 8,
# sharing class 4, plan need 2, window centre 8, table generation 4, and the fused resample gather's
# w, mprob, flags read + written 34, x..zsigma written 40, marks 8 -> 148
BYTES_MERGE_PARTICLE = 148
BYTES_MERGE_CELL = 16         # per cell write (insert or fuse): the cell read and written
BYTES_MERGE_PAGE = 1024       # per page taken: the tile's 64 cells read (copy on write) and written
# per table copied on write: its S slots read and written (+ the centre)
def merge_table_bytes(slots):
    return 8 * slots + 8


def window_slots(max_sensor_range, scale):
    """eslam_detmath.h dm_lm_half: the per-particle map window's tiles per side, squared."""
    import math
    q = max_sensor_range / (8.0 * scale)
    h = 1 if not q > 1.0 else min(15, math.ceil(q))
    return (2 * h + 1) ** 2
CONFIG3_GLOBAL = 16 * 1024 * 1024  # BASELINE configs[3]: 16M particles over 8 GPUs
CONFIG4_GLOBAL = 64 * 1024 * 1024  # BASELINE configs[4]: 64M particles over 8 GPUs
HBM_PEAK_GBS = 8000.0         # MI355X HBM3E spec (MI355X_MICROARCH.md)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--particles", type=int, default=None,
                    help="particles per GPU (default: configs[2]'s 4M on any number of GPUs -- weak scaling "
                         "keeps the one-GPU line's per-GPU work; configs[3]'s 16M over 8 GPUs is 2097152)")
    ap.add_argument("--map-cells", type=int, default=1000)
    ap.add_argument("--rough", action="store_true", help="rough multi-patch terrain (config 5 map)")
    ap.add_argument("--map-pages", type=int, default=0,
                    help="per-particle maps: page pool per particle (eslam_config.local_map_pages; 0: the default)")
    ap.add_argument("--local-maps", action="store_true",
                    help="configs[4]'s per-particle local maps (useSharedMap = false): rough terrain, unmapped "
                         "beyond x = 0.3 m, one map update (processMap merge) per step; default 8M particles per "
                         "GPU (64M over 8 GPUs with --gpus 8)")
    ap.add_argument("--scan-patches", type=int, default=0,
                    help="with --local-maps: the scan's patch count (0: the 48-patch 0.6 x 0.9 m scan; e.g. 600: "
                         "a 2.5 x 2.4 m MLS ahead at 0.1 m, synthetic.scan_area)")
    ap.add_argument("--match", action="store_true",
                    help="with --local-maps: processMap(scan, match = true, update = true), the match "
                         "weighting (eslam_gpu_map_match) before every merge")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-cpu-aos", action="store_true",
                    help="skip cpu_baseline.aos, the oracle with the reference's 288-byte particle records")
    ap.add_argument("--sharded", action="store_true",
                    help="run the multi-GPU (sharded, RCCL) path even on one rank (measures its overhead)")
    ap.add_argument("--comm", choices=["rccl", "torch"], default=os.environ.get("ESLAM_COMM", "rccl"),
                    help="multi-GPU exchanges: the library's own RCCL communicator, or torch.distributed callbacks")
    ap.add_argument("--cpu-sample", type=int, default=None,
                    help="particles in the CPU baseline sample (default 1M; 256k with --local-maps)")
    ap.add_argument("--cpu-steps", type=int, default=None, help="steps of the CPU baseline (default 48; 24 with --local-maps)")
    ap.add_argument("--cpu-threads", type=int, default=1,
                    help="OpenMP threads of the oracle's per-particle loops (1 = the reference default, "
                         "USE_OPENMP off; results are identical for any count)")
    return ap.parse_args()


PROFILE_SUMMARY = os.path.join(ROOT, "profiles", "r06", "summary.json")
PROFILE_SUMMARIES = {"local-maps": os.path.join(ROOT, "profiles", "r06", "summary_local_maps.json")}


def pmc_traffic(kernel, n, map_cells, workload):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC passes
    (tools/profile.sh -> profiles/<round>/summary.json: FETCH_SIZE x2 + WRITE_SIZE, the
    gfx950 correction of MI355X_MICROARCH.md), when they were taken on this workload."""
    path = PROFILE_SUMMARIES.get(workload, PROFILE_SUMMARY)
    try:
        with open(path) as fh:
            d = json.load(fh)
    except (OSError, ValueError):
        return None
    if d.get("particles") != n or d.get("map_cells") != map_cells or d.get("workload", "flat") != workload:
        return None
    for name, e in d.get("kernels", {}).items():
        if name.startswith(kernel) and "hbm_bytes_per_dispatch" in e:
            out = {"bytes_per_launch": round(e["hbm_bytes_per_dispatch"]), "fetch_bytes": round(e["fetch_size_bytes"]),
                   "write_bytes": round(e["write_size_bytes"]), "source": os.path.relpath(path, ROOT)}
            # what actually bounds the kernel: the VALU (rocprofv3 derived metrics, same run)
            if "valubusy_pct" in e:
                out["valu_busy_pct"] = round(e["valubusy_pct"], 1)
            if "valuutilization_pct" in e:
                out["valu_lane_utilization_pct"] = round(e["valuutilization_pct"], 1)
            return out
    return None


def workload_name(n, world, rough, local_maps=False):
    """the BASELINE.json configuration a run corresponds to (per-GPU size, weak scaling)"""
    if local_maps:
        if n * world == CONFIG4_GLOBAL:
            return "configs[4]"
        return ("configs[4]'s 8M-per-GPU shard (of 64M over 8 GPUs)%s" % (", weak-scaled to %d GPUs" % world if world > 1 else "")) \
            if n == CONFIG4_GLOBAL // 8 else "configs[4]-style per-particle maps"
    if rough:
        return "configs[4]-style terrain"
    if world == 1:
        return {262144: "configs[1]", 4 * 1024 * 1024: "configs[2]"}.get(n, "custom size")
    if n * world == CONFIG3_GLOBAL:
        return "configs[3]"
    if n == CONFIG3_GLOBAL // 8:
        return "configs[3]'s 2M-per-GPU shard, weak-scaled to %d GPUs" % world
    if n == 4 * 1024 * 1024:
        return "configs[2]'s 4M per GPU, weak-scaled to %d GPUs (%dM global)" % (world, 4 * world)
    return "custom size, weak-scaled"


def host_cpu():
    """model name and logical CPU count of this host (the CPU baseline's machine)"""
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return model, os.cpu_count()


def time_oracle(args, grid, flags, scan, steps, aos):
    """Seconds for `steps` steps of the bench workload on a cpu_sample-particle oracle filter
    (first step, the uniform reset, untimed)."""
    import eslam_abi as A
    import oracle_ffi as O
    import synthetic as S
    n = args.cpu_sample
    stream = S.step_stream(steps + 1, tilt=scan is not None)
    cfg = S.bench_config(A.default_config(), n)
    cfg.flags |= flags
    f = O.OracleFilter(cfg, O.SUM_REFERENCE, aos=aos)
    f.set_threads(args.cpu_threads)
    f.set_map(grid)
    f.init_gaussian(n, [0.0, 0.0, 0.0], [0.1, 0.1, 0.1], 0.18, 1.001)
    f.step(stream[0])
    if scan is not None:
        f.map_update(scan)
    t0 = time.perf_counter()
    for st in stream[1:1 + steps]:
        f.step(st)
        if scan is not None:
            f.map_update(scan)
    return time.perf_counter() - t0


def cpu_baseline(args, grid, flags=0, scan=None):
    """The CPU oracle (a restatement of the reference path, reference-order double sums) on
    this host, on a bounded sample of the same workload: one thread by default (the
    reference's build default), --cpu-threads for its OpenMP per-particle loops.  `aos`: the
    same oracle built with the reference's 288-byte particle records (src/PoseParticle.hpp:52-86
    + src/PoseEstimator.hpp:108-117; whole-record copies at resample) on half the steps --
    closer to the reference's memory behaviour than the SoA figure."""
    n, k = args.cpu_sample, args.cpu_steps
    dt = time_oracle(args, grid, flags, scan, k, aos=False)
    model, ncpu = host_cpu()
    what = "rough map, per-particle maps + map update" if scan is not None else "flat map"
    out = {"value": round(n * k / dt / 1e6, 4), "unit": "M particle-updates/s", "cores": args.cpu_threads, "kind": "port",
           "cpu_model": model, "host_logical_cpus": ncpu,
           "sample": f"{n} particles x {k} steps of the same workload ({what}, forced update+resample), "
                     f"oracle/eslam_oracle.c (SoA state) in reference-sum mode, {args.cpu_threads} thread(s), {dt:.1f} s"}
    if not args.no_cpu_aos:
        ka = max(1, k // 2)
        da = time_oracle(args, grid, flags, scan, ka, aos=True)
        out["aos"] = {"value": round(n * ka / da / 1e6, 4), "unit": "M particle-updates/s", "cores": args.cpu_threads,
                      "kind": "port",
                      "sample": f"{n} particles x {ka} steps, the same oracle built -DOR_AOS (288-byte particle "
                                f"records, whole-record resample copies), {da:.1f} s"}
    return out


def visible_gpus():
    """GPUs this process could open, counted without any HIP or torch.cuda call: the KFD
    topology's GPU nodes (simd_count > 0), narrowed by a *_VISIBLE_DEVICES list if one is set.
    The parent of a multi-rank run must not initialise the GPU (it forks the ranks)."""
    import glob
    n = 0
    for prop in glob.glob("/sys/class/kfd/kfd/topology/nodes/*/properties"):
        try:
            with open(prop) as fh:
                kv = dict(line.split()[:2] for line in fh if len(line.split()) >= 2)
        except OSError:
            continue
        if int(kv.get("simd_count", "0")) > 0:
            n += 1
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            n = min(n, len([t for t in v.split(",") if t.strip()]))
    return n


def spawn_ranks(args):
    """`bench.py --gpus N` without a launcher: start N ranks of this script as child processes
    (fresh interpreters, RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* set), forward rank 0's JSON line
    and exit with the worst exit code.  The parent never touches the GPU: it counts devices
    from the KFD topology in /sys (visible_gpus) and execs nothing."""
    import subprocess
    import socket
    visible = visible_gpus()
    if visible < args.gpus:
        sys.stderr.write(f"bench.py: --gpus {args.gpus} but only {visible} GPU(s) visible\n")
        sys.exit(2)
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus), LOCAL_WORLD_SIZE=str(args.gpus),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      stdout=subprocess.PIPE if r == 0 else subprocess.DEVNULL))
    # poll every rank: one that fails (RCCL init, out of memory) would leave the others waiting
    # in a collective forever, so the rest are stopped and the run fails
    import threading
    box = {}
    reader = threading.Thread(target=lambda: box.setdefault("out", procs[0].stdout.read()), daemon=True)
    reader.start()
    deadline = time.monotonic() + 3600
    rcs = [None] * len(procs)
    while any(rc is None for rc in rcs):
        for r, p in enumerate(procs):
            if rcs[r] is None:
                rcs[r] = p.poll()
        failed = [rc for rc in rcs if rc not in (None, 0)]
        if failed or time.monotonic() > deadline:
            for p in procs:
                if p.poll() is None:
                    p.terminate()
            for p in procs:
                try:
                    p.wait(timeout=30)
                except subprocess.TimeoutExpired:
                    p.kill()
            if not failed:
                sys.stderr.write("bench.py: ranks did not finish within the time limit\n")
                sys.exit(124)
            rcs = [p.returncode for p in procs]
            break
        time.sleep(0.2)
    reader.join(timeout=30)
    out = box.get("out", b"")
    sys.stdout.write(out.decode())
    sys.stdout.flush()
    bad = [r for r in rcs if r]
    sys.exit(0 if not bad else (bad[0] if bad[0] > 0 else 128 - bad[0]))


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        spawn_ranks(args)
    if args.local_maps:
        args.rough = True
    if args.cpu_sample is None:
        args.cpu_sample = 262144 if args.local_maps else 1048576
        if args.local_maps and args.scan_patches > 48:      # the same ~10-30 s of CPU work
            args.cpu_sample = max(4096, (262144 * 48 // args.scan_patches) // 1024 * 1024)
    if args.cpu_steps is None:
        args.cpu_steps = 24 if args.local_maps else 48
    if args.particles is None:
        if args.local_maps:
            args.particles = CONFIG4_GLOBAL // 8
        else:
            args.particles = 4 * 1024 * 1024
    # stdout carries exactly one JSON line: native libraries (RCCL prints a version banner
    # when a communicator is created) write to stderr until the result is printed
    sys.stdout.flush()
    json_fd = os.dup(1)
    os.dup2(2, 1)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        sys.stderr.write(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}\n")
        sys.exit(2)
    dist = None
    sharded = world > 1 or args.sharded
    if sharded:
        import torch
        import torch.distributed as tdist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
        torch.cuda.set_device(local_rank)
        tdist.init_process_group("nccl")
        dist = tdist

    import numpy as np
    import eslam_abi as A
    import eslam_amd
    import synthetic as S

    n = args.particles
    grid = S.rough_map(cells=args.map_cells) if args.rough else S.flat_map(cells=args.map_cells)
    scan = None
    if args.local_maps:
        grid = S.unmapped_beyond(grid, 0.3)    # the front feet stand on cells only the scans map
        scan = S.scan_area(args.scan_patches) if args.scan_patches > 0 else S.scan_patches()
    stream = S.step_stream(args.warmup + 2 * args.steps + 1, tilt=args.local_maps)
    cfg = S.bench_config(A.default_config(), n * world)
    if args.match and not args.local_maps:
        raise SystemExit("bench.py: --match needs --local-maps (the match reads per-particle maps)")
    if args.local_maps:
        cfg.flags |= A.FLAG_PARTICLE_MAPS
        cfg.local_map_pages = args.map_pages
    if sharded:
        # the summation chunk sized by the rank's own particles (eslam_config.sum_chunk_rows):
        # every rank's weighting kernel fills the chip whatever the rank count (4M a rank: 13
        # rows, as on one GPU; configs[3]'s 2M a rank: 7 instead of the 16M's 13)
        cfg.sum_chunk_rows = A.chunk_rows(n)
    if sharded:
        # one global filter of n * world particles, sharded over the ranks: RCCL all_gathers
        # of the statistics / totals / counts and an all_to_all_v of the migrating particles
        import eslam_dist
        f = None
        if args.comm == "rccl":
            try:
                f = eslam_dist.RcclShardedGpuFilter(cfg, n * world, rank, world, device=local_rank)
            except Exception as e:       # joining the library's communicator failed (on every rank:
                # ncclCommInitRank is collective): the same exchanges through torch.distributed
                sys.stderr.write(f"bench.py: the library's RCCL communicator failed ({e}); "
                                 "using torch.distributed exchanges\n")
                args.comm = "torch (library RCCL failed)"
        if f is None:
            comm = eslam_dist.TorchComm(device_memory=True, device=local_rank)
            f = eslam_dist.ShardedGpuFilter(cfg, n * world, comm, device=local_rank)
        assert f.n_local == n, (f.n_local, n)
    else:
        f = eslam_amd.GpuFilter(cfg, device=0)
    f.set_map(grid)
    f.init_gaussian(n, [0.0, 0.0, 0.0], [0.1, 0.1, 0.1], 0.18, 1.001)
    if scan is not None:
        step_one = f.step

        def step_and_map(st):                  # EmbodiedSlamFilter::update + processMap(scan, match, update)
            r = step_one(st)
            if args.match:
                f.map_match(scan)
            f.map_update(scan)
            return r
        f_step = step_and_map
    else:
        f_step = f.step

    def barrier():
        f.sync()
        if dist is not None:
            import torch
            torch.cuda.synchronize()
            dist.barrier()

    for st in stream[:args.warmup]:
        f_step(st)
    barrier()
    # timed region: K steps back to back, no per-kernel events (HIP event records between
    # the launches cost ~10 % of a step here)
    t0 = time.perf_counter()
    for st in stream[args.warmup:args.warmup + args.steps]:
        f_step(st)
    t_enq = time.perf_counter()             # the host has queued every launch (nothing waits on the GPU)
    info = f.sync()
    barrier()
    dt = time.perf_counter() - t0
    # kernel breakdown: the next K steps of the same stream with HIP events around every
    # launch, on the context's stream (eslam_gpu_enable_timing)
    f.enable_timing(True)
    barrier()
    t1 = time.perf_counter()
    for st in stream[args.warmup + args.steps:args.warmup + 2 * args.steps]:
        f_step(st)
    f.sync()
    barrier()
    dt_ev = time.perf_counter() - t1
    kt = f.kernel_times()
    f.enable_timing(False)
    if dist is not None:
        import torch
        t = torch.tensor([dt, dt_ev], device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt, dt_ev = float(t[0].item()), float(t[1].item())
    total_updates = n * world * args.steps
    value = total_updates / dt / 1e6
    ms_step = dt / args.steps * 1e3

    # roofline of the dominant kernel (HIP events around every launch of the timed region);
    # per-particle maps: the map merge competes too (its write-back covers the changed stores)
    per_kernel = {"k_project_weight": (kt["project_weight_ms"], (BYTES_K1_DELTA if args.local_maps else BYTES_K1) * n),
                  "k_normalize_segments": (kt["normalize_scan_ms"], BYTES_K3 * n)}
    if args.local_maps:
        slots = window_slots(cfg.max_sensor_range, 0.1)
        per_kernel["k_map_merge"] = (kt["map_merge_ms"], BYTES_MERGE_PARTICLE * n + BYTES_MERGE_CELL * info.map_cells_written
                                     + BYTES_MERGE_PAGE * info.map_pages_taken
                                     + merge_table_bytes(slots) * info.map_stores_copied)
    dom = max(per_kernel, key=lambda k: per_kernel[k][0])
    dom_ms, dom_launch_bytes = per_kernel[dom]
    dom_bytes = dom_launch_bytes / n
    achieved = dom_launch_bytes / (dom_ms * 1e-3) / 1e9 if dom_ms > 0 else 0.0
    workload = "local-maps" if args.local_maps else ("rough" if args.rough else "flat")
    traffic = pmc_traffic(dom, n, args.map_cells, workload) if not sharded else None
    result = {
        "metric": "M particle-updates/s (predict+weight+resample) @ 1/2/4/8 MI355X",
        "value": round(value, 3),
        "unit": "M particle-updates/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "dtype_note": "all particle state, weights, sums and map values' arithmetic in fp64 (map cells stored as "
                      "fp32); the project step's Box-Muller radius and angle are IEEE fp32 (DESIGN.md 2), the "
                      "oracle computing the same fp32 operations",
        "data": "synthetic (%s %gx%g m MLS map @0.1 m; odometry + 4 foot contacts per step%s)"
                % ("rough multi-patch" if args.rough else "flat", args.map_cells / 10, args.map_cells / 10,
                   "; unmapped beyond x = 0.3 m, a %d-patch scan merged into every particle's map per step"
                   % len(scan) if scan is not None else ""),
        "config": {"workload": "%s: %d particles/GPU, 1 MI355X per rank, %sMLS %dx%d @0.1 m, 4 contacts, "
                               "resample forced every step%s" % (workload_name(n, world, args.rough, args.local_maps), n,
                                                                 "rough " if args.rough else "", args.map_cells,
                                                                 args.map_cells,
                                                                 (", per-particle local maps + map %supdate per step"
                                                                  % ("match + " if args.match else ""))
                                                                 if args.local_maps else ""),
                   "particles_per_gpu": n, "global_particles": n * world,
                   "parallelism": "dp%d (particle shards%s)" % (world, (", sharded path, %s exchanges" % args.comm)
                                                                   if sharded else "")},
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": traffic["bytes_per_launch"] if traffic else None, "traffic_detail": traffic,
                     "algorithmic_bytes_per_particle": round(dom_bytes, 2),
                     "avg_launch_ms": round(dom_ms, 5)},
        "kernel_ms": {k: round(v, 5) for k, v in kt.items()},
        "host_enqueue_ms_per_step": round((t_enq - t0) / args.steps * 1e3, 4),
        "kernel_ms_note": "HIP events around every launch on the context stream, over a second pass of "
                          "the same K steps (ms_per_step with events: %.4f); single-GPU update steps fold the finalize "
                          "into k_normalize_segments (block 0), so finalize_ms times an empty region there"
                          % (dt_ev / args.steps * 1e3),
        "step_roofline_frac": round(BYTES_STEP * n * world / (dt / args.steps) / 1e9 / (HBM_PEAK_GBS * world), 4),
        "step_roofline_note": "%d B per particle-update: the fused step's algorithmic bytes (K1 %d + K3 %d); the "
                              "reference algorithm's unfused passes would move %d B (fraction %.4f)"
                              % (BYTES_STEP, BYTES_K1, BYTES_K3, BYTES_REFERENCE,
                                 BYTES_REFERENCE * n * world / (dt / args.steps) / 1e9 / (HBM_PEAK_GBS * world)),
        "last_update": {"effective": info.effective, "resampled": info.resampled},
        **({"map_update": {"patches_dropped": info.map_patches_dropped, "tables_copied": info.map_stores_copied,
                           "maps_changed": info.map_stores_changed, "patches_covered": info.map_patches_covered,
                           "cells_written": info.map_cells_written, "pages_taken": info.map_pages_taken,
                           "tiles_evicted": info.map_tiles_evicted, "scan_patches": len(scan),
                           "pages_free": info.map_pages_free, "patches_total": n * len(scan),
                           "data_particles": info.data_particles, "window_slots": window_slots(cfg.max_sensor_range, 0.1),
                           "note": "the last step's map update: scan patches beyond a particle's window (farther "
                                   "than maxSensorRange), shared tables a change copied on write, maps the merge "
                                   "changed, scan patches on cells the shared grid covers (merged into the particle's copy "
                                   "of the grid's cell, DESIGN.md 5c), cell writes, pages taken from the pool and left free; data_particles: "
                                   "the last update's particles whose feet found patches; kernel_ms.map_* time "
                                   "the update's phases (map_cow_ms: the tables' sharing classes and free list, "
                                   "map_plan_ms: the page plan and any collection, map_merge_ms: the merge)"}}
           if args.local_maps else {}),
        "build_id": eslam_amd.build_id(),
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(args, grid, cfg.flags & A.FLAG_PARTICLE_MAPS, scan)
    sys.stdout.flush()
    os.dup2(json_fd, 1)
    if rank == 0:
        print(json.dumps(result), flush=True)
    f.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
