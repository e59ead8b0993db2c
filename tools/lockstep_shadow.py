"""Shadow rays on the lock-step traversal model (tools/lockstep_sim.cpp with
LOCKSTEP_ANY=1): records C3's NEE shadow rays of 40 rows of frame 7 with the
oracle, orders them by target light x origin octant cell (the shadow key's
shape), and prints the model's wave steps, lanes per step and triangle tests per
TLAS instance -- where k_connect's work goes.
usage: python tools/lockstep_shadow.py"""
import os, subprocess, sys, tempfile
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import oracle as O
exe = os.path.join(tempfile.gettempdir(), "lockstep_sim")
subprocess.run(["g++", "-O2", "-std=c++17", "-msse4.1", "-ffp-contract=off", "-fopenmp", "-I" + os.path.join(REPO, "oracle"),
                os.path.join(REPO, "tools", "lockstep_sim.cpp"), "-o", exe, "-lz"], check=True)
O.load()
S = O.OracleScene()
W = 1280
_, (so, sd, st) = S.record_rays(W, 720, 7, 300 * W, 340 * W, max_ext=1 << 21, max_shadow=1 << 21)
n = len(so)
end = so + sd * st[:, None]
light = (end[:, 0] > 0).astype(np.int64)
lo, hi = so.min(0), so.max(0)
cell = (((so - lo) / (hi - lo + 1e-6)) * 2).astype(np.int64).clip(0, 1)
key = light * 8 + cell[:, 0] * 4 + cell[:, 1] * 2 + cell[:, 2]
order = np.argsort(key * n + np.arange(n), kind="stable")
fn = os.path.join(tempfile.mkdtemp(), "sh.bin")
with open(fn, "wb") as f:
    np.array([n], np.uint32).tofile(f)
    np.concatenate([so[order], sd[order], st[order, None]], axis=1).astype(np.float32).tofile(f)
env = dict(os.environ, SURF_ASSETS=os.path.join(REPO, "assets"), LOCKSTEP_ANY="1")
print("shadow rays", n)
print(subprocess.run([exe, fn], capture_output=True, text=True, check=True, env=env).stdout)
