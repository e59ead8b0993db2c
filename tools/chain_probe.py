"""Per-segment latency of one long path in each drain engine: renders the
image row holding the longest path of frame 0 (pixel 630758, 3086 segments at
1280x720, oracle.path_lengths) with the whole stream handed to the tail, and
divides the render time by that path's segment count.
usage: SURF_TAIL_PAIR=0|1 python tools/chain_probe.py"""
import sys, time, json, os
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/surf-path-tracer_amd")
import torch  # noqa: F401
import surf_amd
W, H, P = 1280, 720, 630758
row = P // W
s = surf_amd.Scene.indoor()
r = surf_amd.Renderer(s, W, H, shard=surf_amd.ShardSpec(row, H, 1))
r.set_tail_policy(1 << 30, 0, 16)
r.set_tail_coop(1 << 30)
for rep in range(3):
    r.clear_accumulator()
    t = time.perf_counter()
    r.render(1, 0, 0)
    r.synchronize()
    dt = time.perf_counter() - t
    st = r.stats()
    print(json.dumps({"pair": os.environ.get("SURF_TAIL_PAIR", "1"), "s": round(dt, 4), "max_seg": st["max_segments"],
                      "us_per_segment": round(dt / max(st["max_segments"], 1) * 1e6, 2), "n_ext": st["n_ext"]}), flush=True)
