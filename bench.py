"""Benchmark: Mrays/s of the MI355X wavefront path tracer on BASELINE.json's
headline workload, next to the reference CPU algorithm timed on this host.

    python bench.py [--gpus N --steps K --warmup W] [--workload C3|C2|C4|C5]

Workloads (BASELINE.json configs):
  C3  bundled indoor scene, 1280x720, 256 spp, unbounded bounces + Russian roulette (headline)
  C2  the same scene, 1280x720, 64 spp, at most 8 path segments
  C4  1920x1080, 1024 spp (row-sharded over the GPUs)
  C5  indoor + 648 Suzannes baked into one 10.2M-triangle BLAS, 1280x720, 64 spp

One step = one complete render of the workload: clear the accumulator, render
its spp frames (one sample per pixel each, frame f seeded initSeed(p + 1799 f)
as renderer.cpp:169; step i renders frames [i*spp, (i+1)*spp)), drain the
sample stream until every frame is accumulated.  With N > 1 (torch.distributed
.run, one rank per GPU) each rank renders an interleaved row shard of every
frame (row b -> rank b % N) and, after its drain, its float accumulator is
gathered to rank 0 over RCCL once per render; the total work is fixed, so
scaling is "strong".  Mrays/s = W*H*spp*steps / seconds / 1e6 (main.cpp:431:
camera samples per second).

The CPU baseline (rank 0, N = 1) is the oracle's restatement of the
reference's CPU renderer (oracle/cpu_ref_bench, OpenMP rows like
renderer.cpp:163) on bounded samples of the last timed step's frames, timed
twice: at the environment's thread share over every --cpu-row-step-th row (its
accumulator rows are compared bit for bit with the GPU's: "parity"), and on
every CPU of the affinity mask over all rows (same sample count); the faster
is the reported value, with the cgroup CPU quota recorded.  At N > 1 rank 0
checks the frame assembled from the gather against the oracle the same way.

Prints ONE JSON line (rank 0).
"""
import argparse
import json
import os
import platform
import subprocess
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "surf-path-tracer_amd")
for p in (REPO, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

METRIC = "Mrays/s at 1280×720, 256 spp, indoor scene; 1/2/4/8 MI355X + CPU ref"
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
# Algorithmic HBM bytes per extension ray of k_extend:
# read ray o, d (32 B: origin, direction, tmax, id), write hit t, u, v, inst, prim (20 B).
EXTEND_BYTES_PER_RAY = 52
# C5: the BVH is HBM-resident, so scene bytes join B_alg: 32 B per node fetched + 36 B
# per triangle tested, per extension ray, from the oracle's instrumented traversal
# (profiles/r2_c5/oracle_visits.txt: 108.8 nodes, 51.4 triangles per ray).
C5_SCENE_BYTES_PER_RAY = 32 * 108.8 + 36 * 51.4
# Pipeline bytes per camera sample (SURVEY.md 8d B_alg): path generate, extension ray, shaded hit,
# continuing path, shadow ray, accumulator contribution.
B_EVENT = {"n_ext": 52, "n_hit": 68, "n_cont": 48, "n_shadow": 88, "n_acc": 24}
# rocprofv3 summary of this bench command per workload (tools/profile_round.sh + tools/summarize_profile.py):
# k_extend's average duration (--kernel-trace --stats) and HBM bytes per launch (FETCH_SIZE x2 +
# WRITE_SIZE, separate PMC passes, MI355X_MICROARCH.md HBM/rocprofv3 section).
PMC_SUMMARY = os.path.join(REPO, "profiles", "r{}_{}", "summary.json")
PMC_ROUNDS = (6, 5, 4)   # the newest committed rocprof summary of the workload (tools/round.sh profiles)

WORKLOADS = {
    "C3": dict(scene="indoor", width=1280, height=720, spp=256, max_segments=0, cpu_row_step=5),
    "C2": dict(scene="indoor", width=1280, height=720, spp=64, max_segments=8, cpu_row_step=2),
    "C4": dict(scene="indoor", width=1920, height=1080, spp=1024, max_segments=0, cpu_row_step=20),
    "C5": dict(scene="c5", width=1280, height=720, spp=64, max_segments=0, cpu_row_step=45),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3, help="timed renders")
    ap.add_argument("--warmup", type=int, default=1, help="untimed renders before the timed region")
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="C3")
    ap.add_argument("--width", type=int, default=0, help="override the workload's width")
    ap.add_argument("--height", type=int, default=0, help="override the workload's height")
    ap.add_argument("--spp", type=int, default=0, help="override the workload's samples per pixel (frames per render)")
    ap.add_argument("--row-block", type=int, default=1,
                    help="N > 1: rows per interleaved shard block (1 spreads the long-path-heavy rows over all GPUs)")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0: the lease's CPU share (OMP_NUM_THREADS, else the affinity mask)")
    ap.add_argument("--cpu-row-step", type=int, default=0, help="CPU sample: every n-th row of the last step's frames")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--cpu-full-host", type=int, default=1,
                    help="also time the CPU baseline on every CPU of the affinity mask: 1 (default) unless the cgroup "
                         "CPU quota already equals the lease's threads, 2 always, 0 never")
    ap.add_argument("--profile-pass", type=int, default=1,
                    help="renders re-run with per-kernel HIP events for the roofline (0 = none)")
    ap.add_argument("--tail", type=str, default="", help="tuning: drain policy 'threshold,lanes_per_wave,stage_segments'")
    ap.add_argument("--tail-coop", type=int, default=-1, help="tuning: cooperative drain when <= N paths remain")
    ap.add_argument("--pool", type=int, default=0, help="tuning: paths in flight (0: the library default, 5 frames)")
    return ap.parse_args()


def host_cpu_info():
    """What the CPU baseline ran on: the model, sockets and hardware threads of
    the host, and the share of it this process may use."""
    info = {"nproc": os.cpu_count(), "affinity": len(os.sched_getaffinity(0)),
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS"), "model": platform.processor() or None, "sockets": None}
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            k, _, v = line.partition(":")
            if k.strip() == "Model name":
                info["model"] = v.strip()
            elif k.strip() == "Socket(s)":
                info["sockets"] = int(v.strip())
    except (OSError, ValueError, subprocess.SubprocessError):
        pass
    return info


def cpu_threads(args):
    if args.cpu_threads > 0:
        return args.cpu_threads
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        return int(omp)            # the environment's default share (the GPU pool sets it per GPU)
    return len(os.sched_getaffinity(0))


def cgroup_cpu_quota():
    """The CPU bandwidth limit of this process's cgroup (cgroup v2 cpu.max, else
    v1 cfs quota/period) in CPUs, or None when unlimited / unreadable."""
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            return {"source": "cpu.max", "raw": f"{q} {p}", "cpus": int(q) / int(p)}
        return {"source": "cpu.max", "raw": "max", "cpus": None}
    except (OSError, ValueError):
        pass
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        p = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        return {"source": "cfs", "raw": f"{q} {p}", "cpus": q / p if q > 0 else None}
    except (OSError, ValueError):
        return None


def run_oracle(wl, first_frame, frames, row_step, threads, dump=None):
    exe = os.path.join(REPO, "oracle", "cpu_ref_bench")
    if not os.path.exists(exe):
        subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle")], check=True)
    env = dict(os.environ, OMP_NUM_THREADS=str(threads))
    cmd = [exe, "--cutoff", "--first", str(first_frame), "--row-step", str(row_step)]
    if dump:
        cmd += ["--dump", dump]
    if wl["scene"] == "c5":
        cmd += ["--variant", "1"]
    cmd += [os.path.join(REPO, "assets"), str(wl["width"]), str(wl["height"]), str(frames), "0", str(wl["height"]),
            str(wl["max_segments"]), str(threads)]
    out = subprocess.run(cmd, capture_output=True, text=True, env=env, check=True).stdout.strip().splitlines()[-1]
    return json.loads(out)


def check_rows(wl, first_frame, gpu_acc, step, threads):
    """The oracle's accumulator rows 0, step, 2 step, .. of the render's frames
    against the GPU's (H, W, 4) accumulator, bit for bit (and the per-pixel L2
    of north_star's tolerance).  Returns (the oracle run's JSON, parity)."""
    import numpy as np
    W, H, F = wl["width"], wl["height"], wl["spp"]
    with tempfile.TemporaryDirectory() as tmp:
        dump = os.path.join(tmp, "acc.f32")
        r = run_oracle(wl, first_frame, F, step, threads, dump)
        cpu_rows = np.fromfile(dump, dtype=np.float32).reshape(-1, W, 4)
    gpu_rows = gpu_acc[0::step]
    d = (gpu_rows[..., :3].astype(np.float64) - cpu_rows[..., :3].astype(np.float64)) / F
    per = np.sqrt((d ** 2).sum(-1))
    parity = {"rows": f"0:{H}:{step}", "frames": [first_frame, first_frame + F],
              "bitexact": bool(np.array_equal(gpu_rows.view(np.uint32), cpu_rows.view(np.uint32))),
              "rms_l2": float(np.sqrt((per ** 2).mean())), "max_l2": float(per.max()), "tolerance_l2": 1e-3}
    return r, parity


def cpu_baseline(args, wl, first_frame, gpu_acc):
    """Reference CPU algorithm (oracle restatement, OpenMP rows like
    renderer.cpp:163) timed twice on bounded samples of the last timed render:

    * at the environment's thread share (OMP_NUM_THREADS) over every
      cpu_row_step-th row and all spp frames -- its rows are compared bit for
      bit with the GPU's ("parity");
    * on the whole host (every CPU in the affinity mask) over EVERY row and the
      first spp/cpu_row_step frames -- the same number of samples, but 720+
      rows so that the row loop can feed 256 threads.

    The reported value is the faster of the two (the honest denominator of
    gpu_vs_cpu); both legs and the cgroup CPU quota are recorded."""
    W, H, F, step = wl["width"], wl["height"], wl["spp"], wl["cpu_row_step"]
    lease = cpu_threads(args)
    r, parity = check_rows(wl, first_frame, gpu_acc, step, lease)
    bounds = 'unbounded+RR' if wl['max_segments'] == 0 else 'max %d segments' % wl['max_segments']
    legs = {"lease": {"threads": r["threads"], "mrays_per_s": round(r["mrays_per_s"], 4), "seconds": r["seconds"],
                      "samples": r["samples"],
                      "sample": f"rows 0,{step},{2 * step},.. ({r['rows']} rows), frames {first_frame}..{first_frame + F - 1}"}}
    full = len(os.sched_getaffinity(0))
    quota = cgroup_cpu_quota()
    qcpus = quota.get("cpus") if quota else None
    if args.cpu_full_host == 1 and full > lease and qcpus is not None and qcpus <= lease:
        # the cgroup lets this process run on at most `lease` CPUs at a time: a
        # full-affinity run only adds throttling (measured on the GPU box: 256
        # threads under a 16-CPU quota 3.64 vs 5.87 Mrays/s, profiles/r3_cpu_baseline)
        legs["full_host"] = {"threads": full, "skipped": f"cgroup quota {qcpus:g} CPUs <= {lease} threads already used"}
    elif args.cpu_full_host and full > lease:
        ff = max(1, F // step)
        rf = run_oracle(wl, first_frame, ff, 1, full)
        legs["full_host"] = {"threads": rf["threads"], "mrays_per_s": round(rf["mrays_per_s"], 4),
                             "seconds": rf["seconds"], "samples": rf["samples"],
                             "sample": f"all {H} rows, frames {first_frame}..{first_frame + ff - 1}"}
    best = max((l for l in legs.values() if "mrays_per_s" in l), key=lambda l: l["mrays_per_s"])
    cpu = {"value": best["mrays_per_s"], "unit": "Mrays/s", "cores": best["threads"], "kind": "port",
           "sample": f"{W}x{H} {best['sample']} (1 spp each; the last timed render's frames), {bounds}, "
                     f"throughput cutoff on (as the GPU), oracle/cpu_ref_bench -O3, {best['seconds']:.2f} s",
           "seconds": best["seconds"], "samples": best["samples"], "legs": legs,
           "threads_full_host": full, "cgroup_quota": quota, "host": host_cpu_info(),
           "events": {k: r[k] for k in ("n_ext", "n_hit", "n_cont", "n_shadow", "n_acc", "n_unocc")}}
    return cpu, parity


def rocprof_summary(workload):
    """k_extend's rocprofv3 average and PMC traffic from the committed summary of this command."""
    path = next((p for p in (PMC_SUMMARY.format(r, workload.lower()) for r in PMC_ROUNDS) if os.path.exists(p)), None)
    if path is None:
        return None
    s = json.load(open(path))
    if s.get("workload", "C3") != workload:
        return None
    k = next((v for n, v in s.get("kernels", {}).items() if n.startswith("k_extend")), None)
    pmc = s.get("k_extend_pmc", {})
    return {"source": os.path.relpath(path, REPO), "avg_launch_ms": k["avg_us"] / 1e3 if k else None,
            "traffic": pmc.get("hbm_bytes_per_launch_corrected"), "issue": s.get("issue")}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch          # torch first: it loads the HIP runtime the library then binds to
    import torch.distributed as dist
    import surf_amd

    wl = dict(WORKLOADS[args.workload])
    for k in ("width", "height", "spp"):
        if getattr(args, k):
            wl[k] = getattr(args, k)
    if args.cpu_row_step:
        wl["cpu_row_step"] = args.cpu_row_step
    W, H, SPP, MAXSEG = wl["width"], wl["height"], wl["spp"], wl["max_segments"]

    dist_on = world > 1
    # SURF_BENCH_BACKEND=gloo: rehearsal of the N > 1 path on fewer GPUs than
    # ranks (rank -> device LOCAL_RANK % device count, gather through host
    # memory); the measured configuration is always nccl (RCCL), one GPU per rank
    backend = os.environ.get("SURF_BENCH_BACKEND", "nccl")
    if dist_on:
        if backend == "gloo":
            local = local % max(torch.cuda.device_count(), 1)
        torch.cuda.set_device(local)
        dist.init_process_group(backend, init_method="env://")
    dev = torch.device("cuda", local)
    coll_dev = dev if backend == "nccl" else torch.device("cpu")
    torch.cuda.init()

    surf_amd.load()
    tb = time.perf_counter()
    scene = surf_amd.Scene.indoor(variant=1 if wl["scene"] == "c5" else 0)
    scene_build_s = time.perf_counter() - tb
    spec = surf_amd.ShardSpec(rank, world, args.row_block if world > 1 else 0)
    r = surf_amd.Renderer(scene, W, H, device=local, shard=spec, pool_capacity=args.pool or None)
    if args.tail:
        r.set_tail_policy(*[int(x) for x in args.tail.split(",")])
    if args.tail_coop >= 0:
        r.set_tail_coop(args.tail_coop)
    rows = len(r.rows)
    gather = acc_dev = None
    if dist_on:
        from surf_amd.dist import RowGather
        acc_dev = torch.empty((rows, W, 4), dtype=torch.float32, device=dev)
        gather = RowGather(W, H, world, rank, args.row_block, coll_dev)

    def step(i):
        """One complete render: frames [i*SPP, (i+1)*SPP), drained; N > 1: one RCCL gather."""
        r.clear_accumulator()
        r.render(SPP, i * SPP, MAXSEG)
        r.synchronize()                   # every frame of the render accumulated
        if dist_on:
            r.copy_accumulator_to(acc_dev.data_ptr())
            gather.gather(acc_dev if coll_dev == dev else acc_dev.to(coll_dev))

    for w in range(args.warmup):
        step(w)
    # ---- timed region ----
    if dist_on:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(args.warmup + i)
    torch.cuda.synchronize(dev)
    if dist_on:
        dist.barrier()
    dt = time.perf_counter() - t0
    last_first = (args.warmup + args.steps - 1) * SPP
    st = r.stats()                        # the last render's counts (cleared per step)
    ev = {k: st[k] for k in ("n_ext", "n_hit", "n_cont", "n_shadow", "n_acc", "n_unocc", "iterations", "tail_paths",
                             "n_ext_wavefront")}
    if dist_on:
        t = torch.tensor([dt], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
        evt = torch.tensor([ev[k] for k in ev], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(evt)
        ev = {k: int(v) for k, v in zip(ev, evt.tolist())}
    gpu_acc = None
    if rank == 0 and not args.no_cpu:
        # N > 1: the frame assembled from the last step's gather (every rank's rows)
        gpu_acc = r.accumulator() if world == 1 else gather.assemble()
    samples_per_render = W * H * SPP
    value = samples_per_render * args.steps / dt / 1e6

    # ---- roofline of the dominant wavefront kernel (k_extend), HIP events on the render stream ----
    roof = kernel_ms = None
    if args.profile_pass > 0:
        r.set_profiling(True)
        for i in range(args.profile_pass):
            r.clear_accumulator()
            r.render(SPP, i * SPP, MAXSEG)
            r.synchronize()
        pe = r.stats()                    # the last profiled render
        r.set_profiling(False)
        launches = max(pe["launches_extend"], 1)
        rays_per_launch = pe["n_ext_wavefront"] / launches
        avg_ms = pe["ms_extend"] / launches
        per_rank = None
        if dist_on:
            # every rank profiles its own shard; the line reports the slowest
            # rank's k_extend (the one the max-over-ranks clock waits for)
            t = torch.zeros((world, 3), dtype=torch.float64, device=coll_dev)
            t[rank] = torch.tensor([avg_ms, rays_per_launch, launches], dtype=torch.float64)
            dist.all_reduce(t)
            per_rank = t.cpu().tolist()
            slow = max(range(world), key=lambda k: per_rank[k][0])
            avg_ms, rays_per_launch, launches = per_rank[slow][0], per_rank[slow][1], per_rank[slow][2]
        bytes_per_ray = EXTEND_BYTES_PER_RAY + (C5_SCENE_BYTES_PER_RAY if wl["scene"] == "c5" else 0.0)
        bytes_per_launch = bytes_per_ray * rays_per_launch
        achieved = bytes_per_launch / (avg_ms * 1e-3) / 1e9
        roof = {"bound": "hbm", "achieved": round(achieved, 3), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 6), "traffic": None,
                "kernel": "k_extend", "avg_launch_ms": round(avg_ms, 5), "launches": int(launches),
                "rays_per_launch": round(rays_per_launch, 1), "bytes_per_ray": round(bytes_per_ray, 1),
                "algorithmic_bytes_per_launch": round(bytes_per_launch, 1)}
        if per_rank:
            roof["rank"] = slow
            roof["per_rank_avg_launch_ms"] = [round(x[0], 5) for x in per_rank]
        # the committed rocprof/PMC summary is of the one-GPU command: an N > 1
        # line carries no traffic of its own (its ranks' kernels are not profiled)
        rp = rocprof_summary(args.workload) if not dist_on else None
        if rp:
            roof["traffic"] = round(rp["traffic"]) if rp["traffic"] else None
            if rp.get("issue"):
                # the issue-side bound next to the HBM one (SQ passes of the same command):
                # k_extend and the drain (k_tail_pair) per ray / per segment
                roof["issue"] = rp["issue"]
            roof["rocprof"] = {"source": rp["source"], "avg_launch_ms": rp["avg_launch_ms"],
                               "frac": round(bytes_per_launch / (rp["avg_launch_ms"] * 1e-3) / 1e9 / HBM_PEAK_GBS, 6)
                               if rp["avg_launch_ms"] else None}
        kernel_ms = {k: round(pe[k], 3) for k in ("ms_sort", "ms_extend", "ms_shade", "ms_connect", "ms_regen", "ms_tail", "ms_total")}
        kernel_ms["renders"] = args.profile_pass
        kernel_ms["tail_paths"] = int(pe["tail_paths"])

    cpu = parity = None
    if gpu_acc is not None and world == 1:
        try:
            cpu, parity = cpu_baseline(args, wl, last_first, gpu_acc)
        except Exception as e:  # reported, never silently replaced
            cpu = {"value": None, "unit": "Mrays/s", "cores": cpu_threads(args), "kind": "port", "sample": f"failed: {e}"}
    elif gpu_acc is not None:
        # N > 1 verifies its assembled frame too (the CPU leg is timed at N = 1 only):
        # a sparser row sample, on every CPU of the host
        try:
            _, parity = check_rows(wl, last_first, gpu_acc, wl["cpu_row_step"] * 4, len(os.sched_getaffinity(0)))
            parity["assembled_from_ranks"] = world
        except Exception as e:
            parity = {"bitexact": None, "error": str(e)}

    if rank == 0:
        per_sample = {k: round(ev[k] / samples_per_render, 4) for k in ("n_ext", "n_hit", "n_cont", "n_shadow", "n_acc", "n_unocc")}
        # SURVEY.md 8d whole-pipeline roofline: B_alg bytes per camera sample x samples/s against 8 TB/s
        b_alg = 48 + sum(B_EVENT[k] * ev[k] / samples_per_render for k in B_EVENT) + 20.0 / SPP
        if wl["scene"] == "c5":
            b_alg += C5_SCENE_BYTES_PER_RAY * ev["n_ext"] / samples_per_render
        pipeline = {"b_alg_per_sample": round(b_alg, 1), "achieved_gbs": round(value * 1e6 * b_alg / 1e9, 2),
                    "frac": round(value * 1e6 * b_alg / 1e9 / HBM_PEAK_GBS, 6)}
        out = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic camera samples of the bundled indoor scene (reference OBJ assets)",
            "config": {"workload": args.workload,
                       "scene": "bundled indoor (main.cpp:161-346)" if wl["scene"] == "indoor"
                                else "C5: indoor + 648 Suzannes in one 10.2M-triangle BLAS",
                       "width": W, "height": H, "spp": SPP, "renders": args.steps,
                       "step": f"one complete {SPP}-frame render including its drain",
                       "bounces": "unbounded + russian roulette" if MAXSEG == 0 else f"<= {MAXSEG} segments",
                       "zero_cutoff": True,
                       "parallelism": (f"row shards x{world} (rows interleaved in blocks of {args.row_block}) + one RCCL gather per render"
                                       if world > 1 else "single GPU")},
            "roofline": roof,
            "pipeline_roofline": pipeline,
            "cpu_baseline": cpu,
            "parity": parity,
            "gpu_vs_cpu": round(value / cpu["value"], 2) if cpu and cpu.get("value") else None,
            "events_per_sample": per_sample,
            "iterations_per_render": ev["iterations"],
            # the units of the issue-side roofline (tools/summarize_profile.py): rays k_extend traced and
            # segments the drain ran, summed over ranks at N > 1
            "events_per_render": {"n_ext": ev["n_ext"], "n_ext_wavefront": ev["n_ext_wavefront"],
                                  "drain_segments": ev["n_ext"] - ev["n_ext_wavefront"], "n_shadow": ev["n_shadow"],
                                  "iterations": ev["iterations"]},
            "tail_paths_per_render": ev["tail_paths"],
            "kernel_ms_profile_pass": kernel_ms,
            "scene_build_s": round(scene_build_s, 3),
        }
        print(json.dumps(out))
    if dist_on:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
