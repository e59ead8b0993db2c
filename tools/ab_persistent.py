"""A/B of the persistent (out-of-step) traversal: C3 wall time and per-kernel
profile-pass times with the variant on and off."""
import sys, time, json
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/surf-path-tracer_amd")
import torch  # noqa: F401
import surf_amd
W, H, F, STEPS = 1280, 720, 16, 16
s = surf_amd.Scene.indoor()
r = surf_amd.Renderer(s, W, H)
for on in (False, True, False, True):
    r.set_persistent(on)
    r.render(F, 0, 0); r.synchronize()
    r.clear_accumulator()
    t = time.perf_counter()
    for i in range(STEPS):
        r.render(F, i * F, 0)
    r.synchronize()
    dt = time.perf_counter() - t
    st = r.stats()
    r.set_profiling(True); r.clear_accumulator()
    for i in range(4):
        r.render(F, i * F, 0)
    r.synchronize()
    pe = r.stats(); r.set_profiling(False)
    print(json.dumps({"persistent": on, "mrays": round(W * H * F * STEPS / dt / 1e6, 2), "n_ext": st["n_ext"],
                      "prof": {k: round(pe[k], 1) for k in ("ms_extend", "ms_shade", "ms_connect", "ms_tail")},
                      "launches": pe["launches_extend"]}), flush=True)
