"""Does a second independent sample stream on the same GPU hide the kernel
tails of the first?  K row-shard contexts on device 0, each driven by its own
host thread (ctypes releases the GIL), 256 frames of 1280x720; reports Mrays/s
for K = 1, 2, 3, 4."""
import sys
import threading
import time
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/surf-path-tracer_amd")
import torch  # noqa: F401
import surf_amd

W, H, F, STEPS = 1280, 720, 16, 16
scene = surf_amd.Scene.indoor()
for K in (1, 2, 3, 4):
    rs = [surf_amd.Renderer(scene, W, H, shard=surf_amd.ShardSpec(k, K, 16)) for k in range(K)]
    for r in rs:                      # warm-up (graph build, first stream)
        r.render(F, 0, 0)
        r.synchronize()
        r.clear_accumulator()

    def run(r):
        for i in range(STEPS):
            r.render(F, i * F, 0)
        r.synchronize()

    t0 = time.perf_counter()
    th = [threading.Thread(target=run, args=(r,)) for r in rs]
    for t in th:
        t.start()
    for t in th:
        t.join()
    dt = time.perf_counter() - t0
    print(f"K={K}: {W * H * F * STEPS / dt / 1e6:.1f} Mrays/s ({dt * 1e3:.0f} ms)", flush=True)
    for r in rs:
        r.close()
