"""Does cooperative-drain work overlap with the wavefront stream?  Diagnostics
only.  Renders a C3 stream on context A while context B (a small image whose
every path runs through the one-path-per-wave drain kernel) renders in a
second thread on its own stream; compares A's time and B's segment rate with
each alone.

    python tools/overlap_probe.py        env: BW BH (B's image, default 32x32), BF (frames per B call, 2)
"""
import json
import os
import sys
import threading
import time
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/surf-path-tracer_amd")
import torch  # noqa: F401
import surf_amd

BW, BH, BF = int(os.environ.get("BW", 32)), int(os.environ.get("BH", 32)), int(os.environ.get("BF", 2))
scene = surf_amd.Scene.indoor()
A = surf_amd.Renderer(scene, 1280, 720)
B = surf_amd.Renderer(scene, BW, BH)
B.set_tail_policy(1 << 30, 0, 0)
B.set_tail_coop(1 << 30)
A.render(16, 0, 0); A.synchronize()
B.render(BF, 0, 0); B.synchronize()


def run_a(first):
    A.clear_accumulator()
    t0 = time.perf_counter()
    A.render(256, first, 0)
    A.synchronize()
    return time.perf_counter() - t0


def b_loop(stop, out):
    n0 = B.stats()["n_ext"]
    t0 = time.perf_counter()
    f = 1000
    calls = 0
    while not stop.is_set():
        B.render(BF, f, 0)
        B.synchronize()
        f += BF
        calls += 1
    out["dt"] = time.perf_counter() - t0
    out["seg"] = B.stats()["n_ext"] - n0
    out["calls"] = calls


res = {}
res["a_alone_ms"] = [round(run_a(16 + 256 * i) * 1e3, 1) for i in range(2)]
stop, out = threading.Event(), {}
th = threading.Thread(target=b_loop, args=(stop, out)); th.start()
time.sleep(1.0); stop.set(); th.join()
res["b_alone_seg_per_s"] = out["seg"] / out["dt"]
res["b_alone_calls_per_s"] = out["calls"] / out["dt"]
for i in range(2):
    stop, out = threading.Event(), {}
    th = threading.Thread(target=b_loop, args=(stop, out)); th.start()
    time.sleep(0.05)
    ta = run_a(16 + 256 * (2 + i))
    stop.set(); th.join()
    b_equiv = out["seg"] / res["b_alone_seg_per_s"]
    res[f"together_{i}"] = {"a_ms": round(ta * 1e3, 1), "b_seg": out["seg"], "b_dt_ms": round(out["dt"] * 1e3, 1),
                            "b_alone_equiv_ms": round(b_equiv * 1e3, 1)}
print(json.dumps(res), flush=True)
