"""Throughput of the drain modes on one full frame (921,600 paths, ~5.2 M
segments): wavefront to the end vs one tail launch from the start vs staged."""
import sys, time, json
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/surf-path-tracer_amd")
import torch  # noqa: F401
import surf_amd
W, H = 1280, 720
s = surf_amd.Scene.indoor()
r = surf_amd.Renderer(s, W, H)
r.render(1, 0, 0); r.synchronize()
for name, (th, lpw, stage) in {"wavefront-only": (1, 0, 0), "tail-all lpw auto": (1 << 30, 0, 0),
                               "tail-all lpw 64": (1 << 30, 64, 0), "tail-all staged64": (1 << 30, 0, 64),
                               "default": (0, 0, 64), "default-1stage": (0, 0, 0)}.items():
    r.set_tail_policy(th, lpw, stage)
    for rep in range(2):
        r.clear_accumulator()
        t = time.perf_counter()
        r.render(1, rep + 1, 0)
        r.synchronize()
        dt = time.perf_counter() - t
    st = r.stats()
    print(json.dumps({"mode": name, "ms": round(dt * 1e3, 2), "Msegs/s": round(st["n_ext"] / dt / 1e6, 1),
                      "iters": st["iterations"], "tail_paths": st["tail_paths"], "max_seg": st["max_segments"]}), flush=True)
