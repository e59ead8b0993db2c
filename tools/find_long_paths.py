"""Diagnostics: render C3 with a segment cap and report which samples hit it."""
import sys, time
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/surf-path-tracer_amd")
import numpy as np
import surf_amd
W, H = 1280, 720
frames = int(sys.argv[1]) if len(sys.argv) > 1 else 64
cap = int(sys.argv[2]) if len(sys.argv) > 2 else 20000
s = surf_amd.Scene.indoor()
r = surf_amd.Renderer(s, W, H)
t = time.time()
for f in range(0, frames, 16):
    r.render(16, f, cap)
r.synchronize()
dt = time.time() - t
n, ids = r.debug_capped()
st = r.stats()
print(f"frames {frames} cap {cap}: {dt:.2f}s, capped {n}, n_ext {st['n_ext']}, iters {st['iterations']}, tail {st['tail_paths']}")
npx = W * H
for sid in ids:
    slot, p = divmod(int(sid), npx)
    print(f"  frame {slot} pixel {p} (x={p % W}, y={p // W})")
