"""Benchmark: Mrays/s of the MI355X wavefront path tracer on BASELINE.json's
headline workload (C3: bundled indoor scene, 1280x720, unbounded bounces +
Russian roulette, 256 spp = 16 steps x 16 frames), next to the reference CPU
algorithm (oracle/cpu_ref_bench, OpenMP) timed on this host.

    python bench.py [--gpus N --steps K --warmup W]

One step = one batch of --frames-per-step frames (1 sample per pixel each) over
the full frame.  With N > 1 (torch.distributed.run, one rank per GPU) each rank
renders an interleaved 16-row shard of every frame and the float accumulator
is gathered to rank 0 over RCCL once per step; the total work is fixed, so
scaling is "strong".  Mrays/s = W*H*frames / seconds / 1e6 (main.cpp:431).

Prints ONE JSON line (rank 0).
"""
import argparse
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "surf-path-tracer_amd")
for p in (REPO, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

METRIC = "Mrays/s at 1280×720, 256 spp, indoor scene; 1/2/4/8 MI355X + CPU ref"
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
# Algorithmic HBM bytes per extension ray of k_extend (DESIGN.md "Roofline"):
# read ray o (16 B) + d (16 B), write hit (t,u,v,prim 16 B + inst 4 B).
EXTEND_BYTES_PER_RAY = 52
# rocprofv3 PMC summary of this bench command (tools/profile_round.sh + tools/summarize_profile.py):
# HBM bytes per k_extend launch, FETCH_SIZE x2 + WRITE_SIZE (MI355X_MICROARCH.md, HBM/rocprofv3 section).
PMC_SUMMARY = os.path.join(REPO, "profiles", "r1_s10", "summary.json")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=16)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--width", type=int, default=1280)
    ap.add_argument("--height", type=int, default=720)
    ap.add_argument("--frames-per-step", type=int, default=16)
    ap.add_argument("--max-segments", type=int, default=0, help="0 = unbounded + RR (C3); 8 = C2")
    ap.add_argument("--row-block", type=int, default=1,
                    help="rows per interleaved shard block (1 spreads the long-path-heavy rows over all GPUs)")
    ap.add_argument("--scene", choices=["indoor", "c5"], default="indoor",
                    help="indoor = bundled scene (C2/C3); c5 = +648-Suzanne 10.2M-triangle lattice BLAS (C5)")
    ap.add_argument("--cpu-frames", type=int, default=48, help="frames of the CPU baseline sample (full frame)")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--tail", type=str, default="", help="tuning: drain policy 'threshold,lanes_per_wave,stage_segments'")
    ap.add_argument("--tail-coop", type=int, default=-1, help="tuning: cooperative drain when <= N paths remain")
    ap.add_argument("--long", type=str, default="", help="tuning: long-path worker 'escape_segments,budget'")
    ap.add_argument("--persistent", type=int, default=-1, help="tuning: force the out-of-step traversal on (1) / off (0)")
    ap.add_argument("--profile-pass", type=int, default=-1,
                    help="steps re-run with per-kernel HIP events for the roofline (-1 = --steps, same composition as the timed run)")
    return ap.parse_args()


def workload(args):
    if args.scene == "c5":
        return "C5" if args.max_segments == 0 else f"C5-max{args.max_segments}seg"
    return {0: "C3", 8: "C2"}.get(args.max_segments, f"max{args.max_segments}seg")


def cpu_baseline(args):
    """Reference CPU algorithm (oracle restatement, OpenMP rows) on a bounded sample."""
    exe = os.path.join(REPO, "oracle", "cpu_ref_bench")
    if not os.path.exists(exe):
        subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle")], check=True)
    env = dict(os.environ, OMP_NUM_THREADS=str(args.cpu_threads))
    r0, r1, frames = 0, args.height, args.cpu_frames
    if args.scene == "c5":                # ~60x slower per sample: a centred row band, one frame
        r0, r1, frames = args.height // 2 - 32, args.height // 2 + 32, 1
    cmd = [exe, "--cutoff"] + (["--variant", "1"] if args.scene == "c5" else []) + [os.path.join(REPO, "assets"),
           str(args.width), str(args.height), str(frames), str(r0), str(r1), str(args.max_segments), str(args.cpu_threads)]
    out = subprocess.run(cmd, capture_output=True, text=True, env=env, check=True).stdout.strip().splitlines()[-1]
    r = json.loads(out)
    return {"value": round(r["mrays_per_s"], 4), "unit": "Mrays/s", "cores": r["threads"], "kind": "port",
            "sample": f"{args.width}x{args.height} rows {r0}..{r1 - 1}, frames 0..{frames - 1} (1 spp each), "
                      f"{'unbounded+RR' if args.max_segments == 0 else 'max %d segments' % args.max_segments}, "
                      f"throughput cutoff on (as the GPU), oracle/cpu_ref_bench, {r['seconds']:.2f} s",
            "seconds": r["seconds"], "samples": r["samples"],
            "events": {k: r[k] for k in ("n_ext", "n_hit", "n_cont", "n_shadow", "n_acc", "n_unocc")}}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch          # torch first: it loads the HIP runtime the library then binds to
    import torch.distributed as dist
    import numpy as np
    import surf_amd

    dist_on = world > 1
    if dist_on:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", init_method="env://")
    dev = torch.device("cuda", local)
    torch.cuda.init()

    surf_amd.load()
    W, H, F = args.width, args.height, args.frames_per_step
    tb = time.perf_counter()
    scene = surf_amd.Scene.indoor(variant=1 if args.scene == "c5" else 0)
    scene_build_s = time.perf_counter() - tb
    spec = surf_amd.ShardSpec(rank, world, args.row_block if world > 1 else 0)
    r = surf_amd.Renderer(scene, W, H, device=local, shard=spec)
    if args.tail:
        r.set_tail_policy(*[int(x) for x in args.tail.split(",")])
    if args.tail_coop >= 0:
        r.set_tail_coop(args.tail_coop)
    if args.long:
        r.set_long_paths(*[int(x) for x in args.long.split(",")])
    if args.persistent >= 0:
        r.set_persistent(bool(args.persistent))
    rows = len(r.rows)
    acc_dev = torch.empty((rows, W, 4), dtype=torch.float32, device=dev)
    gather = None
    if dist_on:
        from surf_amd.dist import RowGather
        gather = RowGather(W, H, world, rank, args.row_block, dev)

    def step(i):
        r.render(F, i * F, args.max_segments)
        if dist_on:                       # one RCCL gather of the accumulator per step
            r.copy_accumulator_to(acc_dev.data_ptr())
            gather.gather(acc_dev)

    for w in range(args.warmup):
        step(w)
    r.clear_accumulator()
    # ---- timed region ----
    if dist_on:
        dist.barrier()
    torch.cuda.synchronize(dev)
    r.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(i)
    r.synchronize()                       # drains the sample stream: every path finished
    torch.cuda.synchronize(dev)
    if dist_on:
        dist.barrier()
    dt = time.perf_counter() - t0
    st = r.stats()
    ev = {k: st[k] for k in ("n_ext", "n_hit", "n_cont", "n_shadow", "n_acc", "n_unocc", "iterations", "tail_paths")}
    if dist_on:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
        evt = torch.tensor([ev[k] for k in ev], dtype=torch.float64, device=dev)
        dist.all_reduce(evt)
        ev = {k: int(v) for k, v in zip(ev, evt.tolist())}
    samples = W * H * F * args.steps
    value = samples / dt / 1e6

    # ---- roofline of the dominant kernel (k_extend), HIP events on the render stream ----
    roof = None
    kernel_ms = None
    if args.profile_pass < 0:
        args.profile_pass = args.steps
    if args.profile_pass > 0:
        r.set_profiling(True)
        r.clear_accumulator()
        for i in range(args.profile_pass):
            r.render(F, i * F, args.max_segments)
        pe = r.stats()
        r.set_profiling(False)
        launches = max(pe["launches_extend"], 1)
        bytes_per_launch = EXTEND_BYTES_PER_RAY * pe["n_ext"] / launches
        avg_ms = pe["ms_extend"] / launches
        achieved = bytes_per_launch / (avg_ms * 1e-3) / 1e9
        traffic, traffic_src = None, None
        if os.path.exists(PMC_SUMMARY):
            pmc = json.load(open(PMC_SUMMARY)).get("k_extend_pmc", {})
            traffic = pmc.get("hbm_bytes_per_launch_corrected")
            traffic_src = os.path.relpath(PMC_SUMMARY, REPO)
        roof = {"bound": "hbm", "achieved": round(achieved, 3), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 6), "traffic": round(traffic) if traffic else None,
                "traffic_source": traffic_src,
                "kernel": "k_extend", "avg_launch_ms": round(avg_ms, 5), "launches": int(pe["launches_extend"]),
                "algorithmic_bytes_per_launch": round(bytes_per_launch, 1)}
        kernel_ms = {k: round(pe[k], 3) for k in ("ms_extend", "ms_shade", "ms_connect", "ms_regen", "ms_tail", "ms_total")}
        kernel_ms["steps"] = args.profile_pass
        kernel_ms["tail_paths"] = int(pe["tail_paths"])
        if dist_on:
            t = torch.tensor([achieved], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MIN)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        try:
            cpu = cpu_baseline(args)
        except Exception as e:  # reported, never silently replaced
            cpu = {"value": None, "unit": "Mrays/s", "cores": args.cpu_threads, "kind": "port", "sample": f"failed: {e}"}

    if rank == 0:
        per_sample = {k: round(ev[k] / samples, 4) for k in ("n_ext", "n_hit", "n_cont", "n_shadow", "n_acc", "n_unocc")}
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
            "config": {"workload": workload(args),
                       "scene": "bundled indoor (main.cpp:161-346)" if args.scene == "indoor"
                                else "C5: indoor + 648 Suzannes in one 10.2M-triangle BLAS",
                       "width": W, "height": H,
                       "spp": F * args.steps, "frames_per_step": F,
                       "bounces": "unbounded + russian roulette" if args.max_segments == 0 else f"<= {args.max_segments} segments",
                       "parallelism": f"row-shard x{world} (16-row interleave) + RCCL gather" if world > 1 else "single GPU"},
            "roofline": roof,
            "cpu_baseline": cpu,
            "gpu_vs_cpu": round(value / cpu["value"], 2) if cpu and cpu.get("value") else None,
            "events_per_sample": per_sample,
            "iterations": ev["iterations"],
            "tail_paths": ev["tail_paths"],
            "kernel_ms_profile_pass": kernel_ms,
            "scene_build_s": round(scene_build_s, 3),
        }
        print(json.dumps(out))
    if dist_on:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
