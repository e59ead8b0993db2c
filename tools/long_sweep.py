"""Long-path worker sweep: C3 256 frames wall time per (escape length, budget)."""
import sys, time, json
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/surf-path-tracer_amd")
import torch  # noqa: F401
import surf_amd
W, H, F, STEPS = 1280, 720, 16, 16
s = surf_amd.Scene.indoor()
r = surf_amd.Renderer(s, W, H)
r.render(F, 0, 0); r.synchronize()
cfgs = [tuple(int(x) for x in a.split(",")) for a in sys.argv[1:]] or [(0, 64), (64, 64), (64, 32), (128, 64), (32, 64)]
for esc, bud in cfgs:
    r.set_long_paths(esc, bud)
    r.clear_accumulator()
    t = time.perf_counter()
    for i in range(STEPS):
        r.render(F, i * F, 0)
    t1 = time.perf_counter()
    r.synchronize()
    dt = time.perf_counter() - t
    st = r.stats()
    print(json.dumps({"escape": esc, "budget": bud, "mrays": round(W * H * F * STEPS / dt / 1e6, 2), "s": round(dt, 3),
                      "drain_s": round(time.perf_counter() - t1, 3), "iters": st["iterations"], "tail_paths": st["tail_paths"],
                      "n_ext": st["n_ext"], "max_seg": st["max_segments"]}), flush=True)
