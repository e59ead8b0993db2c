import sys, numpy as np
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/surf-path-tracer_amd")
import surf_amd, oracle
s = surf_amd.Scene.indoor()
W, H = 80, 60
o = oracle.OracleScene()
for F in (1, 2, 3):
    c, cnt, _ = o.render(W, H, F)
    for kw in ({}, {"frame_batch": 1}):
        r = surf_amd.Renderer(s, W, H, **kw); r.render(F); a = r.accumulator(); st = r.stats()
        bad = (a.view(np.uint32) != c.view(np.uint32)).any(-1)
        print(F, kw, "bad", int(bad.sum()), "alpha", np.unique(a[..., 3]), "n_ext", st["n_ext"], cnt["n_ext"], "tail", st["tail_paths"], "iters", st["iterations"], flush=True)
        if bad.any():
            # per-frame: compare with single-frame renders
            for f in range(F):
                cf, _, _ = o.render(W, H, 1, first_frame=f)
                print("   frame", f, "sum oracle", float(cf[..., :3].sum()))
            print("   sum gpu", float(a[..., :3].sum()), "sum oracle", float(c[..., :3].sum()))
# window 1 frame by frame in separate calls
r = surf_amd.Renderer(s, W, H, frame_batch=1)
for f in range(3):
    r.render(1, f)
a = r.accumulator(); c, _, _ = o.render(W, H, 3)
print("separate calls w1 bad", int((a.view(np.uint32) != c.view(np.uint32)).any(-1).sum()))
