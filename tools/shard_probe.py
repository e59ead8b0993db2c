"""Projected strong scaling on one GPU: renders each row shard of G of a
workload on device 0 one after another and reports the slowest shard's time,
i.e. what an N = G run takes per GPU before the gather.  Diagnostics only.

    python tools/shard_probe.py [G,G,...]
    env: W H (frame size, default 1280x720), F (frames per render, default 256),
         STEPS (timed renders per shard, default 1), ROWBLOCK (rows per
         interleave block, default 1), TAIL / COOP (drain policy knobs),
         POOL (paths in flight per shard, default: the library's ~4 full frames),
         ONLY (comma list: render only these shards of each G, e.g. for a profile)

Each shard: one untimed 16-frame warm-up render, then STEPS complete renders
of F frames (frames 16.., each drained), timed together."""
import json
import os
import sys
import time
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/surf-path-tracer_amd")
import torch  # noqa: F401
import surf_amd

W, H = int(os.environ.get("W", 1280)), int(os.environ.get("H", 720))
F, STEPS = int(os.environ.get("F", 256)), int(os.environ.get("STEPS", 1))
ROWBLOCK = int(os.environ.get("ROWBLOCK", "1"))
gs = [int(x) for x in sys.argv[1].split(",")] if len(sys.argv) > 1 else [1, 2, 4, 8]
scene = surf_amd.Scene.indoor()
base = None
for G in gs:
    times, maxseg = [], []
    only = [int(x) for x in os.environ["ONLY"].split(",")] if os.environ.get("ONLY") else range(G)
    for k in only:
        r = surf_amd.Renderer(scene, W, H, shard=surf_amd.ShardSpec(k, G, ROWBLOCK if G > 1 else 0),
                              pool_capacity=int(os.environ["POOL"]) if os.environ.get("POOL") else None)
        if os.environ.get("TAIL"):
            r.set_tail_policy(*[int(x) for x in os.environ["TAIL"].split(",")])
        if os.environ.get("COOP"):
            r.set_tail_coop(int(os.environ["COOP"]))
        r.render(16, 0, 0); r.synchronize(); r.clear_accumulator()
        t0 = time.perf_counter()
        for i in range(STEPS):
            r.clear_accumulator()
            r.render(F, 16 + i * F, 0)
            r.synchronize()
        times.append(time.perf_counter() - t0)
        st = r.stats()
        maxseg.append(st.get("max_segments"))
        r.close()
        print(json.dumps({"G": G, "shard": k, "ms": round(times[-1] * 1e3, 1), "tail_paths": st["tail_paths"], "tail_ms": st.get("ms_tail"),
                          "max_seg": st.get("max_segments"), "iters": st["iterations"]}), flush=True)
    t = max(times)
    base = base or t
    print(json.dumps({"W": W, "H": H, "F": F, "steps": STEPS, "rowblock": ROWBLOCK, "G": G,
                      "slowest_ms": round(t * 1e3, 1), "mean_ms": round(sum(times) / len(times) * 1e3, 1),
                      "slowest_shard": int(times.index(t)), "projected_Mrays": round(W * H * F * STEPS / t / 1e6, 1),
                      "speedup_vs_first_G": round(base / t, 2)}), flush=True)
