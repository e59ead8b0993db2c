"""C3 pool-key candidates on the lock-step traversal model (tools/lockstep_sim.cpp):
the recorded extension rays of rows 300..339 of frame 7 ordered by the current key
(heavy mask descending x quadrant) and by finer origin cells / direction signs;
prints the model's visit steps per 64 rays for each.  usage: python tools/lockstep_keys_c3.py"""
import os, subprocess, sys, tempfile, time
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import oracle as O
exe = os.path.join(tempfile.gettempdir(), "lockstep_sim")
subprocess.run(["g++", "-O2", "-std=c++17", "-msse4.1", "-ffp-contract=off", "-fopenmp", "-I" + os.path.join(REPO, "oracle"),
                os.path.join(REPO, "tools", "lockstep_sim.cpp"), "-o", exe, "-lz"], check=True)
O.load()
t = time.time()
S = O.OracleScene()
W = 1280
(eo, ed), _ = S.record_rays(W, 720, 7, 300 * W, 340 * W, max_ext=1 << 21, max_shadow=1 << 21)
n = len(eo); print("rays", n, round(time.time() - t, 1), flush=True)
primary = np.abs(eo[:, 2] + 7.0) < 0.6
env = dict(os.environ, SURF_ASSETS=os.path.join(REPO, "assets"))
d = tempfile.mkdtemp()
def write(order, fn):
    with open(fn, "wb") as f:
        np.array([n], np.uint32).tofile(f)
        np.concatenate([eo[order], ed[order]], axis=1).astype(np.float32).tofile(f)
pos = np.arange(n)
write(pos, os.path.join(d, "raw.bin"))
subprocess.run([exe, os.path.join(d, "raw.bin"), "mask", os.path.join(d, "mask.bin")], check=True, env=env)
m = np.fromfile(os.path.join(d, "mask.bin"), dtype=np.uint32)
heavy = ((m >> 3) & 7).astype(np.int64)
quad = ((eo[:, 0] >= 0) + 2 * (eo[:, 2] >= 0)).astype(np.int64)
lo, hi = eo.min(0), eo.max(0)
def cell(k, axes=(0, 1, 2)):
    c = (((eo - lo) / (hi - lo + 1e-6)) * k).astype(np.int64).clip(0, k - 1)
    r = np.zeros(n, np.int64)
    for a in axes: r = r * k + c[:, a]
    return r
dsign = (ed[:, 1] > 0).astype(np.int64)
keys = {
    "current (7-mask)x quad": np.where(primary, 1 << 20, (7 - heavy) * 4 + quad),
    "(7-mask) x octant": np.where(primary, 1 << 20, (7 - heavy) * 8 + cell(2)),
    "(7-mask) x quad x dy": np.where(primary, 1 << 20, ((7 - heavy) * 4 + quad) * 2 + dsign),
    "(7-mask) x cell4xz": np.where(primary, 1 << 20, (7 - heavy) * 16 + cell(4, (0, 2))),
    "(7-mask) x cell4^3": np.where(primary, 1 << 20, (7 - heavy) * 64 + cell(4)),
    "(7-mask) x cell8^3": np.where(primary, 1 << 20, (7 - heavy) * 512 + cell(8)),
}
for name, key in keys.items():
    o = np.argsort(key * n + pos, kind="stable")
    fn = os.path.join(d, "k.bin"); write(o, fn)
    out = subprocess.run([exe, fn], capture_output=True, text=True, check=True, env=env).stdout.splitlines()
    print(name, "|", [l for l in out if l.startswith("groups")][0], flush=True)
