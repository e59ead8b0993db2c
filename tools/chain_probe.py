"""Per-segment latency of one long path: renders the single image row that
holds the longest path of frame 0 (pixel 630758, 3086 segments at 1280x720,
oracle.path_lengths) and times the drain in lane mode and cooperative mode."""
import sys, time, json
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/surf-path-tracer_amd")
import torch  # noqa: F401
import surf_amd
W, H, P = 1280, 720, 630758
row = P // W
s = surf_amd.Scene.indoor()
r = surf_amd.Renderer(s, W, H, shard=surf_amd.ShardSpec(row, H, 1))
for stage in (0, 64, 0, 64):
    r.set_tail_policy(0, 0, stage)
    r.clear_accumulator()
    t = time.perf_counter()
    r.render(1, 0, 0)
    r.synchronize()
    dt = time.perf_counter() - t
    st = r.stats()
    print(json.dumps({"mode": "coop" if stage else "lane", "s": round(dt, 4), "max_seg": st["max_segments"],
                      "us_per_segment": round(dt / max(st["max_segments"], 1) * 1e6, 2), "n_ext": st["n_ext"]}), flush=True)
