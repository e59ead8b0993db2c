"""C5 ray orders on the lock-step traversal model (tools/lockstep_sim.cpp on the
C5 scene, SCENE_VARIANT=1): records the extension rays of 12 rows of frame 7
with the oracle and prints the model's wave steps per 64 rays for the record
order, the quadrant key and spatial origin-cell keys (64 to 4096 bins).
usage: python tools/lockstep_c5_keys.py"""
import os, subprocess, sys, tempfile, time
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import oracle as O
exe = os.path.join(tempfile.gettempdir(), "lockstep_sim")
subprocess.run(["g++", "-O2", "-std=c++17", "-msse4.1", "-ffp-contract=off", "-fopenmp", "-I" + os.path.join(REPO, "oracle"),
                os.path.join(REPO, "tools", "lockstep_sim.cpp"), "-o", exe, "-lz"], check=True)
O.load()
t=time.time()
S = O.OracleScene(variant=1)
print('scene', time.time()-t, flush=True)
W = 1280
(eo, ed), _ = S.record_rays(W, 720, 7, 340 * W, 352 * W, max_ext=1 << 21, max_shadow=1 << 20)
n = len(eo); print('rays', n, time.time()-t, flush=True)
env = dict(os.environ, SURF_ASSETS=os.path.join(REPO, "assets"), SCENE_VARIANT="1")
d = tempfile.mkdtemp()
def write(order, fn):
    with open(fn, "wb") as f:
        np.array([n], np.uint32).tofile(f)
        np.concatenate([eo[order], ed[order]], axis=1).astype(np.float32).tofile(f)
pos = np.arange(n)
quad = (eo[:, 0] >= 0) + 2 * (eo[:, 2] >= 0)
lo, hi = eo.min(0), eo.max(0)
def cell(k):
    c = (((eo - lo) / (hi - lo + 1e-6)) * k).astype(np.int64).clip(0, k - 1)
    return c[:, 0] * k * k + c[:, 1] * k + c[:, 2]
octant = (ed[:, 0] >= 0) * 4 + (ed[:, 1] >= 0) * 2 + (ed[:, 2] >= 0)
keys = {'pool order (unsorted)': pos, 'quadrant': quad * n + pos, 'cell4^3 (64 bins)': cell(4) * n + pos,
        'cell2^3 x octant (64)': (cell(2) * 8 + octant) * n + pos, 'cell8^3 (512)': cell(8) * n + pos,
        'cell16^3 (4096)': cell(16) * n + pos}
for name, key in keys.items():
    o = np.argsort(key, kind='stable')
    fn = os.path.join(d, 'k.bin'); write(o, fn)
    out = subprocess.run([exe, fn], capture_output=True, text=True, check=True, env=env).stdout.splitlines()
    line = [l for l in out if l.startswith('groups')][0]
    print(f'{name:26s} {line}', flush=True)
