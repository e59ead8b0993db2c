"""Projected strong scaling on one GPU: renders each row shard of G (16-row
interleave) of the C3 workload (1280x720, 256 frames, unbounded + RR) on
device 0 one after another and reports the slowest shard's time, i.e. what an
N=G run takes per GPU without the gather.  Diagnostics only."""
import json
import sys
import time
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/surf-path-tracer_amd")
import torch  # noqa: F401
import os
import surf_amd

W, H, F, STEPS = 1280, 720, 16, 16
gs = [int(x) for x in sys.argv[1].split(",")] if len(sys.argv) > 1 else [1, 2, 4, 8]
SHARDS = os.environ.get("SHARDS")   # "all" (default) or a count: only the first n shards of each G
scene = surf_amd.Scene.indoor()
base = None
for G in gs:
    times = []
    for k in range(G if not SHARDS else min(G, int(SHARDS))):
        r = surf_amd.Renderer(scene, W, H, shard=surf_amd.ShardSpec(k, G, int(os.environ.get("ROWBLOCK", "16")) if G > 1 else 0),
                              pool_capacity=int(os.environ["CAP"]) if os.environ.get("CAP") else None)
        if os.environ.get("LONG"):
            r.set_long_paths(*[int(x) for x in os.environ["LONG"].split(",")])
        if os.environ.get("TAIL"):
            r.set_tail_policy(*[int(x) for x in os.environ["TAIL"].split(",")])
        if os.environ.get("COOP"):
            r.set_tail_coop(int(os.environ["COOP"]))
        r.render(F, 0, 0); r.synchronize(); r.clear_accumulator()
        t0 = time.perf_counter()
        for i in range(STEPS):
            r.render(F, i * F, 0)
        r.synchronize()
        times.append(time.perf_counter() - t0)
        st = r.stats()
        r.close()
        if G == 1 or k == 0 or os.environ.get("VERBOSE"):
            print(json.dumps({"G": G, "shard": k, "ms": round(times[-1] * 1e3, 1), "tail_paths": st["tail_paths"],
                              "max_seg": st.get("max_segments"), "iters": st["iterations"]}), flush=True)
    t = max(times)
    base = base or t
    print(json.dumps({"cfg": {k: os.environ.get(k) for k in ("LONG", "TAIL", "COOP", "CAP") if os.environ.get(k)}, "G": G, "slowest_ms": round(t * 1e3, 1), "mean_ms": round(sum(times) / len(times) * 1e3, 1),
                      "projected_Mrays": round(W * H * F * STEPS / t / 1e6, 1), "speedup": round(base / t, 2)}), flush=True)
