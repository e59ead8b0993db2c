"""The drop-in loop (the reference's interactive main.cpp:381-446: one frame per
Renderer::render call) on a long stream, against the same frames in one call
and against a larger fixed ring.  Diagnostics only (a stream
longer than the default 256-slot window issues frame f + 256 only once frame
f is accumulated, i.e. once its longest Russian-roulette path ended).

    python tools/dropin_loop.py
    env: W H (default 1280x720, C3), N (frames, default 1024),
         WINDOWS (comma list of frame windows, 0 = library default; default "0,2048")

Per window: a 16-frame warm-up stream, then N frames one per call (timed up
to the final synchronize), then the same N frames in one call."""
import json
import os
import sys
import time
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/surf-path-tracer_amd")
import torch  # noqa: F401
import surf_amd

W, H, N = int(os.environ.get("W", 1280)), int(os.environ.get("H", 720)), int(os.environ.get("N", 1024))
windows = [int(x) for x in os.environ.get("WINDOWS", "0,2048").split(",")]
scene = surf_amd.Scene.indoor()
for win in windows:
    r = surf_amd.Renderer(scene, W, H, frame_batch=win or None)
    r.render(16, 0, 0); r.synchronize()
    r.clear_accumulator()
    t0 = time.perf_counter()
    for f in range(N):
        r.render(1, 16 + f, 0)          # the stream continues: no drain between calls
        if f % 256 == 255:
            print(json.dumps({"window": win, "frames_issued": f + 1, "s": round(time.perf_counter() - t0, 2)}), flush=True)
    r.synchronize()
    t_loop = time.perf_counter() - t0
    a_loop = r.accumulator()
    r.clear_accumulator()
    t0 = time.perf_counter()
    r.render(N, 16 + N + 7, 0)      # a gap: a fresh stream (its default window grows to N)
    r.synchronize()
    t_one = time.perf_counter() - t0
    st = r.stats()
    r.close()
    print(json.dumps({"W": W, "H": H, "frames": N, "window": win or "default",
                      "loop_ms_per_frame": round(t_loop * 1e3 / N, 3), "one_call_ms_per_frame": round(t_one * 1e3 / N, 3),
                      "loop_Mrays": round(W * H * N / t_loop / 1e6, 1), "one_call_Mrays": round(W * H * N / t_one / 1e6, 1),
                      "loop_samples_ok": bool((a_loop[..., 3] == N).all()), "max_seg": st.get("max_segments")}), flush=True)
