"""Long-path worker parity probe (diagnostics): GPU vs oracle for escape/lifetime combos."""
import sys
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/surf-path-tracer_amd")
import numpy as np
import torch  # noqa: F401
import oracle
import surf_amd
W, H, F = 128, 96, 6
ps = surf_amd.Scene.indoor()
os_ = oracle.OracleScene()
oracle.set_zero_cutoff(True)
c, cnt, _ = os_.render(W, H, F)
for esc, life, split in [(4, 0, 1), (2, 300, 1), (24, 300, 1), (4, 300, 0), (4, 300, 1), (4, 100000, 1)]:
    r = surf_amd.Renderer(ps, W, H, pool_capacity=8192)
    r.set_long_paths(esc, life)
    if split:
        r.render(2, 0, 0); r.render(F - 2, 2, 0)
    else:
        r.render(F, 0, 0)
    g = r.accumulator(); st = r.stats()
    bad = (g.view(np.uint32) != c.view(np.uint32)).any(-1)
    cbad = {k: (st[k], cnt[k]) for k in ("n_ext", "n_hit", "n_cont", "n_shadow", "n_acc", "n_unocc") if st[k] != cnt[k]}
    print(esc, life, split, "bad px", int(bad.sum()), "long", st["long_paths"], "alpha ok", bool((g[..., 3] == F).all()),
          "counts", cbad, flush=True)
    if bad.any():
        ys, xs = np.nonzero(bad)
        print("  first", list(zip(ys[:5], xs[:5])), "g", g[ys[0], xs[0]], "c", c[ys[0], xs[0]])
    r.close()
