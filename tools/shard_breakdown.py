"""Where one row shard's render time goes (diagnostics): shard k of G of the
C3 workload, one profiled render (per-kernel HIP events; phases launched one
by one) and one unprofiled render, with the drain's share.
    python tools/shard_breakdown.py [G [k]]"""
import json
import sys
import time
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/surf-path-tracer_amd")
import torch  # noqa: F401
import surf_amd

G = int(sys.argv[1]) if len(sys.argv) > 1 else 8
K = int(sys.argv[2]) if len(sys.argv) > 2 else 1
W, H, F = 1280, 720, 256
scene = surf_amd.Scene.indoor()
r = surf_amd.Renderer(scene, W, H, shard=surf_amd.ShardSpec(K, G, 1 if G > 1 else 0))
r.render(16, 0, 0)
r.synchronize()
for prof in (False, True, False):
    r.clear_accumulator()
    r.set_profiling(prof)
    t = time.perf_counter()
    r.render(F, 16, 0)
    r.synchronize()
    dt = (time.perf_counter() - t) * 1e3
    st = r.stats()
    out = {"G": G, "shard": K, "profiled": prof, "wall_ms": round(dt, 2), "iterations": st["iterations"],
           "tail_paths": st["tail_paths"], "max_seg": st["max_segments"]}
    if prof:
        out.update({k: round(st[k], 2) for k in ("ms_sort", "ms_extend", "ms_shade", "ms_connect", "ms_regen", "ms_tail", "ms_total")})
    print(json.dumps(out), flush=True)
