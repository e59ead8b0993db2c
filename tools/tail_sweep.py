"""Drain-policy sweep: wall time of C3 (256 frames) per tail threshold / lanes."""
import sys, time, json
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/surf-path-tracer_amd")
import torch  # noqa: F401  (HIP runtime first)
import surf_amd
W, H, F, STEPS = 1280, 720, 16, 16
s = surf_amd.Scene.indoor()
r = surf_amd.Renderer(s, W, H)
r.render(F, 0, 0); r.synchronize()
pols = [(0, 0), (16384, 0), (65536, 0), (262144, 0), (921600, 0), (1, 0), (65536, 16), (65536, 64), (230400, 16)]
if len(sys.argv) > 1:
    pols = [tuple(int(x) for x in a.split(",")) for a in sys.argv[1:]]
for th, lpw in pols:
    r.set_tail_policy(th, lpw)
    r.clear_accumulator()
    t = time.perf_counter()
    for i in range(STEPS):
        r.render(F, i * F, 0)
    r.synchronize()
    dt = time.perf_counter() - t
    st = r.stats()
    r.set_profiling(True); r.clear_accumulator()
    for i in range(2):
        r.render(F, i * F, 0)
    r.synchronize()
    pe = r.stats(); r.set_profiling(False)
    print(json.dumps({"threshold": th, "lpw": lpw, "mrays": round(W * H * F * STEPS / dt / 1e6, 2), "s": round(dt, 3),
                      "iters": st["iterations"], "tail_paths": st["tail_paths"], "max_seg": st["max_segments"],
                      "prof_ms_tail": round(pe["ms_tail"], 1), "prof_ms_total": round(pe["ms_total"], 1),
                      "prof_max_seg": pe["max_segments"]}), flush=True)
