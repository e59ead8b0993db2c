"""Pool-capacity sweep: C3 256 frames wall time, long-path worker on/off."""
import sys, time, json
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/surf-path-tracer_amd")
import torch  # noqa: F401
import surf_amd
W, H, F, STEPS = 1280, 720, 16, 16
s = surf_amd.Scene.indoor()
caps = [int(a) for a in sys.argv[1:]] or [524288, 1048576, 2097152, 3686400]
for cap in caps:
    for esc in (0, 64):
        r = surf_amd.Renderer(s, W, H, pool_capacity=cap)
        r.set_long_paths(esc, 32)
        r.render(F, 0, 0); r.synchronize()
        r.clear_accumulator()
        t = time.perf_counter()
        for i in range(STEPS):
            r.render(F, i * F, 0)
        t1 = time.perf_counter()
        r.synchronize()
        dt = time.perf_counter() - t
        st = r.stats()
        print(json.dumps({"capacity": cap, "escape": esc, "mrays": round(W * H * F * STEPS / dt / 1e6, 2), "s": round(dt, 3),
                          "drain_s": round(time.perf_counter() - t1, 3), "iters": st["iterations"], "tail_paths": st["tail_paths"]}),
              flush=True)
        r.close()
